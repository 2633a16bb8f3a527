"""CPU oracle (test infrastructure only) for GraphService's typed path queries.

A restatement of the three Cypher reads of the reference's GraphService over a plain edge
list -- no CSR, no device -- so the drop-in's device traversals (egr_snapshot_typed_neighbors,
egraph_dropin/graph_service.py) can be checked against it:
  * related_changes     <- find_related_changes, /root/reference/src/database/neo4j.py:205-229
  * affected_by_node    <- find_affected_by_node, neo4j.py:232-252
  * service_dependencies <- get_service_dependencies, neo4j.py:255-279
Semantics restated from the Cypher text (parity unpinned: there is no Neo4j here and the
reference's tests hold no fixture for these queries):
  * MATCH binds one row per matching path; `(a)<-[:T*]-(b)` is a variable-length path of >= 1
    T relationships, none used twice in one path;
  * `c.changed_at >= datetime() - duration(...)` holds only for a timezone-aware datetime
    property (a Neo4j DATETIME): a string, a naive datetime (LOCAL DATETIME) or a missing value
    compares to null and drops the row; ORDER BY ... DESC keeps ties in match order;
  * OPTIONAL MATCH yields one row with null when nothing matches; collect(DISTINCT x) keeps the
    first occurrence of each node.
Graph input: `labels[v]`, `ids[v]`, `edges` = [(src, dst, type name)], `props[(label, id)]`.
"""
from __future__ import annotations

import datetime as _dt

# OWNS* is expanded without a depth bound, as Cypher does: relationships are unique within a
# path (one relationship per ordered vertex pair and type -- the reference MERGEs them), so the
# expansion ends.


def _props(labels, ids, props, v):
    return dict(props.get((labels[v], ids[v]), {"id": ids[v]}))


def _adj(edges):
    out, inn = {}, {}
    for s, d, t in edges:
        out.setdefault((s, t), []).append(d)
        inn.setdefault((d, t), []).append(s)
    return out, inn


def _find(labels, ids, props, label, **want):
    hits = []
    for v in range(len(ids)):
        if labels[v] != label:
            continue
        p = props.get((label, ids[v]), {"id": ids[v]})
        if all(k in p and p[k] == x for k, x in want.items()):
            hits.append(v)
    return hits


def related_changes(labels, ids, edges, props, incident_id, window_minutes=30, now=None):
    out, inn = _adj(edges)
    now = now or _dt.datetime.now(_dt.timezone.utc)
    cutoff = now - _dt.timedelta(minutes=window_minutes)
    rows = []
    for i in _find(labels, ids, props, "Incident", id=incident_id):
        for s in out.get((i, "AFFECTS"), []):
            for c in inn.get((s, "APPLIES_TO"), []):
                if labels[c] != "ChangeEvent":
                    continue
                p = _props(labels, ids, props, c)
                t = p.get("changed_at")
                if isinstance(t, _dt.datetime) and t.tzinfo is not None and t >= cutoff:
                    rows.append(p)
    rows.sort(key=lambda p: p["changed_at"], reverse=True)
    return rows


def affected_by_node(labels, ids, edges, props, node_name):
    out, inn = _adj(edges)
    rows = []
    for n in _find(labels, ids, props, "Node", name=node_name):
        for p in inn.get((n, "SCHEDULED_ON"), []):
            if labels[p] != "Pod":
                continue
            # every path (p)<-[:OWNS*]-(d:Deployment), relationships unique within a path
            deps = []
            stack = [(p, frozenset(), 0)]
            while stack:
                cur, used, depth = stack.pop()
                nxt = []
                for u in inn.get((cur, "OWNS"), []):
                    if (u, cur) in used:
                        continue
                    if labels[u] == "Deployment":
                        deps.append(u)
                    nxt.append((u, used | {(u, cur)}, depth + 1))
                stack.extend(reversed(nxt))        # (depth first, in neighbour order)
            for d in deps:
                svcs = [s for s in inn.get((d, "SELECTS"), []) if labels[s] == "Service"]
                for s in svcs or [None]:
                    rows.append({"pod": _props(labels, ids, props, p),
                                 "deployment": _props(labels, ids, props, d),
                                 "service": _props(labels, ids, props, s) if s is not None else None})
    return rows


def service_dependencies(labels, ids, edges, props, service_name, namespace):
    out, inn = _adj(edges)
    hits = _find(labels, ids, props, "Service", name=service_name, namespace=namespace)
    if not hits:
        return {"service": None, "downstream": [], "upstream": []}
    s = hits[0]

    def distinct(vs):
        seen, keep = set(), []
        for v in vs:
            if labels[v] == "Service" and v not in seen:
                seen.add(v)
                keep.append(v)
        return [_props(labels, ids, props, v) for v in keep]
    return {"service": _props(labels, ids, props, s),
            "downstream": distinct(out.get((s, "CALLS"), [])),
            "upstream": distinct(inn.get((s, "CALLS"), []))}
