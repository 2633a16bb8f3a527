"""Alert-storm pipeline (BASELINE config C5: ~100k alerts/min streamed
through dedup, incremental CSR update and re-ranking).  One `tick` per batch of alerts (e.g. one
second of the stream):

  1. fingerprints of the alert keys                       GPU  egr_fingerprint
  2. the webhook loop: duplicates vs new incidents        GPU  egr_dedup_ingest
       (reference src/services/ingestion/main.py:141-170 + deduplicator.py, TTL 4 h)
  3. the new incidents' entities / relations MERGEd       host egr_graph_merge_* (id interning)
       (+ any topology delta of the tick, e.g. new Events)
  4. the device snapshot brought up to date               GPU  egr_snapshot_update
  5. affected incidents: BFS `hops` deep from every vertex the update touched
                                                          GPU  egr_snapshot_within
     An open incident is re-ranked iff a touched vertex lies within `hops` of its incident
     vertex or of one of its seed vertices (the only places its reach set and its propagated
     scores can change: a score at v sums walks of length <= hops from the seeds, and an entry's
     value changes only when its column's degree does), or a vertex one of its evidence rows
     would now attach to was created (seeds.seeds_for_batch `pending`).
  6. re-rank new + affected incidents                     GPU  egr_frontier_run
Every cached ranking therefore equals a from-scratch ranking of the current graph
(tests/test_storm_gpu.py checks it tick by tick).
"""
from __future__ import annotations

import time
from dataclasses import dataclass, field
from typing import Callable

import numpy as np
import torch

from egraph.alerts import DedupTable, fingerprints
from egraph.device import to_device
from egraph.graph import EvidenceGraph
from egraph.seeds import seeds_for_batch

NO_NODE = 0xFFFFFFFF


@dataclass
class StormCase:
    """What opening an incident adds: its id, the entities / relations it MERGEs and its
    evidence rows (Evidence dicts)."""
    incident_id: str
    entities: list          # [(id, label)]
    relations: list         # [(source_id, target_id, type)]
    evidence: list


@dataclass
class OpenIncident:
    handle: int
    incident_id: str
    evidence: list
    vertex: int = -1
    seeds: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint32))
    pending: set = field(default_factory=set)
    top_ids: np.ndarray | None = None      # [k] u32 vertex ids, NO_NODE padded
    top_scores: np.ndarray | None = None   # [k] f32
    ranked_at: int = -1                    # tick of the last re-rank


class StormEngine:
    COL_BUCKETS = (64, 256, 1024, 4096)

    def __init__(self, graph: EvidenceGraph, *, device=None, hops: int = 3, k: int = 10,
                 ttl_ms: int = 4 * 3600 * 1000, dedup_capacity: int = 1 << 16, weights=None):
        self.g = graph
        self.snap = graph.snapshot(weights, device)
        self.dev = self.snap.dev
        self.hops, self.k, self.ttl_ms = hops, k, ttl_ms
        self.table = DedupTable(dedup_capacity, self.dev)
        self.incidents: list[OpenIncident] = []
        self._pending: dict[str, set[int]] = {}
        self._frontiers: dict[int, object] = {}
        self.ticks = 0

    # ---- frontier per column bucket, grown / recreated as needed ---------------------------
    def _frontier(self, n_cols: int, n_seeds: int):
        b = next((c for c in self.COL_BUCKETS if c >= n_cols), None)
        if b is None:
            raise ValueError(f"{n_cols} columns exceed the largest bucket {self.COL_BUCKETS[-1]}")
        fr = self._frontiers.get(b)
        if fr is None or fr.max_seeds < n_seeds or fr.max_vertices < self.snap.n_vertices:
            cap = max(n_seeds, 64 * b, fr.max_seeds * 2 if fr is not None else 0)
            fr = self.snap.frontier(b, max_seeds=cap, k=self.k)
            self._frontiers[b] = fr
        return fr

    def _rank(self, handles: list[int]) -> None:
        inc_label = self.g.labels().index("Incident") if "Incident" in self.g.labels() else -1
        top = self.COL_BUCKETS[-1]
        for lo in range(0, len(handles), top):
            part = [self.incidents[h] for h in handles[lo:lo + top]]
            pend: list = []
            sv, sc, ss = seeds_for_batch(self.g, [x.evidence for x in part], pending=pend)
            fr = self._frontier(len(part), len(sv))
            src = np.full(fr.B, NO_NODE, np.uint32)
            src[: len(part)] = [x.vertex if x.vertex >= 0 else NO_NODE for x in part]
            fr.set_seeds(to_device(sv, self.dev), to_device(sc, self.dev), to_device(ss, self.dev))
            ids, scores = fr.run(to_device(src, self.dev), hops=self.hops, exclude_label=inc_label)
            ids = ids.cpu().numpy().view(np.uint32)
            scores = scores.cpu().numpy()
            order = np.argsort(sc, kind="stable")
            bounds = np.searchsorted(sc[order], np.arange(len(part) + 1))
            for j, x in enumerate(part):
                x.top_ids, x.top_scores = ids[j].copy(), scores[j].copy()
                x.seeds = np.unique(sv[order[bounds[j]:bounds[j + 1]]])
                for pid in x.pending:
                    s = self._pending.get(pid)
                    if s is not None:
                        s.discard(x.handle)
                x.pending = pend[j]
                for pid in x.pending:
                    self._pending.setdefault(pid, set()).add(x.handle)
                x.ranked_at = self.ticks

    def tick(self, keys: list[str], now_ms: int, make_case: Callable[[int, int], StormCase],
             topology: tuple | None = None) -> dict:
        """One batch of alerts.  `keys`: the alerts' fingerprint keys, in arrival order
        (normalizer.py:217 strings).  `make_case(handle, alert_index)` builds the incident an
        alert opens.  `topology`: optional (vertex ids, labels, edge src, dst, types) MERGEd in
        the same tick.  Returns counts and per-stage wall times (ms)."""
        t = [time.perf_counter()]
        fp, _ = fingerprints(keys, self.dev)
        dup, inc, n_new = self.table.ingest(fp, now_ms, self.ttl_ms)     # synchronises
        dup_h = dup.cpu().numpy()
        inc_h = inc.cpu().numpy()
        t.append(time.perf_counter())
        # host MERGE of the new incidents and the tick's topology
        openers = np.flatnonzero(~dup_h)
        ids, labels, es, ed, et = [], [], [], [], []
        new_handles = []
        t_collect = 0.0
        for i in openers:
            h = int(inc_h[i])
            tc = time.perf_counter()
            case = make_case(h, int(i))
            t_collect += time.perf_counter() - tc
            assert h == len(self.incidents), "incident handles are dense and ordered"
            self.incidents.append(OpenIncident(h, case.incident_id, case.evidence))
            new_handles.append(h)
            for vid, lab in case.entities:
                ids.append(vid)
                labels.append(lab)
            for s, d, ty in case.relations:
                es.append(s)
                ed.append(d)
                et.append(ty)
        if topology is not None:
            tv, tl, ts, td, tt = topology
            ids += list(tv)
            labels += list(tl)
            es += list(ts)
            ed += list(td)
            et += list(tt)
        V0, E0 = self.snap.n_vertices, self.snap.synced_edges
        if ids:
            self.g.merge_nodes(ids, labels)
        if es:
            self.g.merge_edges(es, ed, et)
        for x in (self.incidents[h] for h in new_handles):
            x.vertex = int(self.g.lookup([f"incident:{x.incident_id}"])[0])
        t.append(time.perf_counter())
        n_v, n_e = self.snap.sync(self.g)                                 # GPU CSR update
        t.append(time.perf_counter())
        # affected incidents
        affected = set(new_handles)
        old = [x for x in self.incidents[: len(self.incidents) - len(new_handles)]]
        if (n_v or n_e) and old:
            s2, d2, _ = self.g.export_edges(E0, n_e)
            touched = np.unique(np.concatenate([np.arange(V0, V0 + n_v, dtype=np.int64),
                                                s2.astype(np.int64), d2.astype(np.int64)]))
            dist = self.snap.within(to_device(touched.astype(np.uint32), self.dev), self.hops)
            # incident vertices and seed vertices of every old incident, on the device
            verts = np.concatenate([np.array([max(x.vertex, 0) for x in old], np.int64)] +
                                   [x.seeds.astype(np.int64) for x in old])
            owner = np.concatenate([np.arange(len(old), dtype=np.int64)] +
                                   [np.full(len(x.seeds), j, np.int64) for j, x in enumerate(old)])
            hit = (dist[to_device(verts, self.dev)] != 255).to(torch.int32)
            flag = torch.zeros(len(old), dtype=torch.int32, device=self.dev)
            flag.scatter_reduce_(0, to_device(owner, self.dev), hit, reduce="amax")
            for j in np.flatnonzero(flag.cpu().numpy()):
                affected.add(old[j].handle)
            # rows that would now attach to a newly created vertex
            for v in range(V0, V0 + n_v):
                hs = self._pending.get(self.g.vertex_id(v))
                if hs:
                    affected.update(hs)
        t.append(time.perf_counter())
        self._rank(sorted(affected))
        torch.cuda.synchronize(self.dev)
        t.append(time.perf_counter())
        self.ticks += 1
        ms = [(b - a) * 1e3 for a, b in zip(t, t[1:])]
        ms[1] -= t_collect * 1e3          # the incidents' evidence comes from the collectors
        return {"alerts": len(keys), "duplicates": int(dup_h.sum()), "new_incidents": n_new,
                "new_vertices": n_v, "new_edges": n_e, "affected": len(affected),
                "open_incidents": len(self.incidents),
                "ms": dict(zip(("fingerprint_dedup", "merge_host", "csr_update", "affected", "rerank"), ms)),
                "collect_ms": t_collect * 1e3}

    def rankings(self) -> list[tuple[np.ndarray, np.ndarray]]:
        return [(x.top_ids, x.top_scores) for x in self.incidents]
