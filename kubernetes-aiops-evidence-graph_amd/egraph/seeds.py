"""Evidence rows -> propagation seeds (DESIGN.md §5 "attachment").

A row's seed value is its `signal_strength`, set by the collectors' scoring functions
(kubernetes_collector.py:255-288, :409-420, :479-485, :532, :601-602; logs_collector.py:220-240;
metrics_collector.py:246-328; deploy_diff_collector.py:205-219, :385, :448).  The row attaches to
the first of its candidate vertex ids present in the graph, following the collectors' id scheme
(kubernetes_collector.py:93-314, deploy_diff_collector.py:246-269); rows with no candidate in the
graph, or with a non-positive strength, seed nothing.
"""
from __future__ import annotations

import numpy as np

def attach_ids(ev: dict) -> list[str]:
    """Candidate vertex ids of an evidence row, most specific first."""
    t, ns, name = ev.get("evidence_type"), ev.get("entity_namespace"), ev.get("entity_name")
    data = ev.get("data") or {}
    if t == "kubernetes_pod":
        return [f"pod:{ns}:{name}"]
    if t in ("kubernetes_deployment", "deploy_change", "image_change"):
        return [f"deployment:{ns}:{name}"]
    if t == "kubernetes_node":
        return [f"node:{name}"]
    if t == "kubernetes_hpa":
        return [f"hpa:{ns}:{name}"]
    if t == "config_change":
        return [f"configmap:{ns}:{name}"]
    if t == "kubernetes_event":
        obj = data.get("involved_object") or {}
        kind = str(obj.get("kind", "")).lower()
        ids = [f"event:{ns}:{name}"]
        if kind == "node":
            ids.append(f"node:{obj.get('name')}")
        elif kind:
            ids.append(f"{kind}:{obj.get('namespace', ns)}:{obj.get('name')}")
        return ids
    if t == "log_signal":
        return [f"logpattern:{ns}:{name}", f"service:{ns}:{name}", f"deployment:{ns}:{name}"]
    if t == "metric_signal":
        return [f"metric:{ns}:{name}"]
    return []


def seeds_for_batch(graph, evidence_lists: list[list[dict]], pending: list | None = None):
    """(vertex u32, column u32, strength f32) triples for a batch: each row attaches to the
    first of its candidate ids present in the graph; unattached rows are dropped.
    `pending` (optional, a list) receives per column the set of candidate ids ranked before the
    one attached (all of them for an unattached row): the vertices whose later creation would
    re-attach a row -- the alert storm's re-rank trigger (egraph/storm.py)."""
    flat, count, col, val = [], [], [], []
    for b, evs in enumerate(evidence_lists):
        for ev in evs:
            ids = attach_ids(ev)
            s = float(ev.get("signal_strength", 0.5))
            if not ids or s <= 0:
                continue
            flat.extend(ids)
            count.append(len(ids))
            col.append(b)
            val.append(s)
    if pending is not None:
        pending[:] = [set() for _ in evidence_lists]
    if not flat:
        return np.zeros(0, np.uint32), np.zeros(0, np.uint32), np.zeros(0, np.float32)
    found = graph.lookup(flat)
    chosen = np.full(len(count), -1, np.int64)
    pos = 0
    for r, n in enumerate(count):
        for j, v in enumerate(found[pos:pos + n]):
            if v >= 0:
                chosen[r] = v
                if pending is not None and j:
                    pending[col[r]].update(flat[pos:pos + j])
                break
        else:
            if pending is not None:
                pending[col[r]].update(flat[pos:pos + n])
        pos += n
    keep = chosen >= 0
    return (chosen[keep].astype(np.uint32), np.asarray(col, np.uint32)[keep],
            np.asarray(val, np.float32)[keep])
