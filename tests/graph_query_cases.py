"""Known-answer graphs for GraphService's typed path queries (neo4j.py:205-279) and the helpers
the CPU (oracle) and GPU (drop-in) tests share.  Results there are "parity unpinned": no Neo4j
runs here and the reference holds no fixture for these queries; the known answers below are
written from the Cypher text (oracle/graph_queries.py states the semantics)."""
from __future__ import annotations

import datetime as dt

NOW = dt.datetime(2026, 10, 18, 12, 0, 0, tzinfo=dt.timezone.utc)


def _ago(minutes: float) -> dt.datetime:
    return NOW - dt.timedelta(minutes=minutes)


def known_answer_world():
    """(entities, relations, expected) -- entities as (id, label, properties) and relations as
    (source, target, type), in creation order; expected answers of the three queries."""
    E = []

    def ent(i, lab, **p):
        E.append((i, lab, dict(p)))
    ent("incident:i1", "Incident", title="CrashLoop")
    ent("incident:i2", "Incident", title="unrelated")
    ent("node:node-a", "Node", name="node-a")
    ent("node:node-b", "Node", name="node-b")
    for p in ("p1", "p2", "p3", "p4"):
        ent(f"pod:ns:{p}", "Pod", name=p, namespace="ns")
    ent("deployment:ns:d1", "Deployment", name="d1", namespace="ns")
    ent("deployment:ns:d2", "Deployment", name="d2", namespace="ns")
    ent("replicaset:ns:rs1", "ReplicaSet", name="rs1", namespace="ns")
    ent("service:ns:api", "Service", name="api", namespace="ns")
    ent("service:ns:web", "Service", name="web", namespace="ns")
    ent("service:ns:cron", "Service", name="cron", namespace="ns")
    ent("service:other:api", "Service", name="api", namespace="other")
    ent("database:ns:db", "Database", name="db", namespace="ns")
    # change events: tz-aware datetimes inside / outside the window, an ISO string (Neo4j: a
    # STRING never compares with a DATETIME), a naive datetime (LOCAL DATETIME: null too)
    ent("change:c1", "ChangeEvent", revision="1", changed_at=_ago(5))
    ent("change:c2", "ChangeEvent", revision="2", changed_at=_ago(60))
    ent("change:c3", "ChangeEvent", revision="3", changed_at=_ago(3).isoformat())
    ent("change:c4", "ChangeEvent", revision="4", changed_at=_ago(1).replace(tzinfo=None))
    ent("change:c5", "ChangeEvent", revision="5", changed_at=_ago(10))
    ent("change:c6", "ChangeEvent", revision="6", changed_at=_ago(2))
    ent("change:c7", "ChangeEvent", revision="7", changed_at=_ago(4))          # on i2's target
    ent("change:c8", "ChangeEvent", revision="8")                              # no changed_at
    R = [("incident:i1", "pod:ns:p1", "AFFECTS"), ("incident:i1", "pod:ns:p2", "AFFECTS"),
         ("incident:i1", "deployment:ns:d1", "AFFECTS"), ("incident:i2", "pod:ns:p4", "AFFECTS"),
         ("change:c1", "deployment:ns:d1", "APPLIES_TO"), ("change:c2", "deployment:ns:d1", "APPLIES_TO"),
         ("change:c3", "deployment:ns:d1", "APPLIES_TO"), ("change:c4", "pod:ns:p1", "APPLIES_TO"),
         ("change:c5", "pod:ns:p1", "APPLIES_TO"), ("change:c6", "pod:ns:p2", "APPLIES_TO"),
         ("change:c7", "pod:ns:p4", "APPLIES_TO"), ("change:c8", "pod:ns:p2", "APPLIES_TO"),
         # a change that also applies to a second affected target: two rows
         ("change:c5", "deployment:ns:d1", "APPLIES_TO"),
         ("pod:ns:p1", "node:node-a", "SCHEDULED_ON"), ("pod:ns:p2", "node:node-a", "SCHEDULED_ON"),
         ("pod:ns:p3", "node:node-a", "SCHEDULED_ON"), ("pod:ns:p4", "node:node-b", "SCHEDULED_ON"),
         # p1: owned by d1 directly and through rs1 (two OWNS* paths), p2 by d2, p3 by nothing
         ("deployment:ns:d1", "pod:ns:p1", "OWNS"), ("replicaset:ns:rs1", "pod:ns:p1", "OWNS"),
         ("deployment:ns:d1", "replicaset:ns:rs1", "OWNS"), ("deployment:ns:d2", "pod:ns:p2", "OWNS"),
         ("deployment:ns:d2", "pod:ns:p4", "OWNS"),
         ("service:ns:api", "deployment:ns:d1", "SELECTS"), ("service:ns:web", "deployment:ns:d1", "SELECTS"),
         ("service:ns:api", "service:ns:web", "CALLS"), ("service:ns:web", "service:ns:api", "CALLS"),
         ("service:ns:cron", "service:ns:api", "CALLS"), ("service:ns:api", "database:ns:db", "CALLS"),
         ("service:other:api", "service:ns:api", "CALLS")]
    props = {i: dict(p, id=i) for i, _, p in E}
    expected = {
        "related_changes": [props[c] for c in ("change:c6", "change:c1", "change:c5", "change:c5")],
        "affected_by_node": sorted(
            [(("pod:ns:p1",), "deployment:ns:d1", s) for s in ("service:ns:api", "service:ns:web")] * 2
            + [(("pod:ns:p2",), "deployment:ns:d2", None)], key=str),
        "service_dependencies": {"service": "service:ns:api", "downstream": ["service:ns:web"],
                                 "upstream": sorted(["service:ns:web", "service:ns:cron",
                                                     "service:other:api"])},
    }
    return E, R, expected


def affected_key(rows):
    """affected_by_node rows as a sorted list of ((pod id,), deployment id, service id or None):
    Neo4j leaves their order unspecified."""
    return sorted((((r["pod"]["id"],), r["deployment"]["id"], r["service"]["id"] if r["service"] else None)
                   for r in rows), key=str)


def deps_key(out):
    return {"service": out["service"]["id"] if out["service"] else None,
            "downstream": sorted(d["id"] for d in out["downstream"]),
            "upstream": sorted(u["id"] for u in out["upstream"])}
