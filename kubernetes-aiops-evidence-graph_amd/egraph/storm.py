"""Alert-storm pipeline (BASELINE config C5: ~100k alerts/min streamed
through dedup, incremental CSR update and re-ranking).  One `tick` per batch of alerts (e.g. one
second of the stream):

  1. fingerprints of the alert keys                       GPU  egr_fingerprint
  2. the webhook loop: duplicates vs new incidents        GPU  egr_dedup_ingest
       (reference src/services/ingestion/main.py:141-170 + deduplicator.py, TTL 4 h)
  3. the new incidents' entities / relations MERGEd       host egr_graph_merge_* (id interning)
       (+ any topology delta of the tick, e.g. new Events)
  4. the device snapshot brought up to date               GPU  egr_snapshot_update
  5. affected incidents: BFS `hops - 1` deep from every vertex the update touched (a new
     vertex or an endpoint of a new edge)                 GPU  egr_snapshot_within
     An open incident is re-ranked iff a touched vertex lies within hops-1 of its incident
     vertex or of one of its seed vertices, or a vertex one of its evidence rows would now
     attach to was created (seeds.seeds_for_batch `pending`).  Why that suffices: a score is a
     sum over walks seed = x0 -> ... -> xL = v (L <= hops) of products of entry values
     w / deg(x_i), i < L; such a walk changes only if some x_i with i <= L-1 <= hops-1 is
     touched (its degree changed, or a new edge leaves it).  The candidate set (vertices within
     `hops` of the incident) grows only through a new edge with an endpoint within hops-1 of
     the incident vertex.
  6. re-rank new + affected incidents                     GPU  egr_frontier_run
     (seed triples are cached per incident and recomputed only for new incidents and those
     whose pending ids appeared)
Every cached ranking therefore equals a from-scratch ranking of the current graph
(tests/test_storm_gpu.py checks it tick by tick).

Across GPUs (`comm` given: one process per GPU, BASELINE C5 "across 8xMI355X"):
  * the dedup table is sharded by fingerprint range (egraph.alerts.ShardedDedup): each rank
    fingerprints the alerts that arrived at it, routes them to their owners (all-to-all) and
    every rank receives the whole tick's decisions, numbered as one table would;
  * the graph is replicated: every rank MERGEs every new incident and the topology delta in
    the same order and updates its own device CSR (the delta is small; the host MERGE is the
    part that does not shrink with more ranks);
  * incident h is owned by rank h % world: only the owner keeps its seeds and ranking, checks
    whether it is affected and re-ranks it.
The union of the owners' rankings equals the single-GPU engine's (tests/test_storm_gpu.py).
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Callable

import numpy as np
import torch

from egraph.alerts import DedupTable, ShardedDedup, fingerprints
from egraph.device import to_device
from egraph.graph import EvidenceGraph
from egraph.seeds import SeedCandidates

NO_NODE = 0xFFFFFFFF


@dataclass
class StormCase:
    """What opening an incident adds: its id, the entities / relations it MERGEs and its
    evidence rows (Evidence dicts)."""
    incident_id: str
    entities: list          # [(id, label)]
    relations: list         # [(source_id, target_id, type)]
    evidence: list


class OpenIncident:
    """One open incident: its handle and id, its incident vertex, its evidence rows (released
    once its candidates are extracted unless keep_evidence) and its attachment candidates; its
    seeds and ranking live in the engine's arrays (SeedStore, RankStore), read by handle."""
    __slots__ = ("handle", "incident_id", "evidence", "cand", "store", "seeds", "vtx")

    def __init__(self, handle: int, incident_id: str, evidence: list | None, store=None,
                 seeds: "SeedStore | None" = None, vtx: "np.ndarray | None" = None):
        self.handle, self.incident_id, self.evidence = handle, incident_id, evidence
        self.cand = None           # SeedCandidates, or (keyed batch, column) until sliced
        self.store, self.seeds, self.vtx = store, seeds, vtx

    @property
    def vertex(self) -> int:                     # incident vertex (-1: not in the graph)
        return int(self.vtx.a[self.handle]) if self.vtx is not None else -1

    @property
    def sv(self) -> np.ndarray:                  # seed vertices
        return self.seeds.get(self.handle)[0] if self.seeds is not None else np.zeros(0, np.uint32)

    @property
    def ss(self) -> np.ndarray:                  # seed strengths
        return self.seeds.get(self.handle)[1] if self.seeds is not None else np.zeros(0, np.float32)

    # its ranking, read from the engine's arrays (a re-rank writes them in one step per launch)
    @property
    def top_ids(self) -> np.ndarray | None:      # [k] u32 vertex ids, NO_NODE padded
        return self.store.row(self.handle)[0] if self.store is not None else None

    @property
    def top_scores(self) -> np.ndarray | None:   # [k] f32
        return self.store.row(self.handle)[1] if self.store is not None else None

    @property
    def ranked_at(self) -> int:                  # tick of the last re-rank (-1: never)
        return self.store.row(self.handle)[2] if self.store is not None else -1


class _Grow:
    """A numpy array indexed by handle, grown geometrically (fill value for new slots)."""

    def __init__(self, dtype, fill):
        self.a = np.full(0, fill, dtype)
        self.fill = fill

    def ensure(self, n: int) -> None:
        if n > len(self.a):
            m = max(n, 2 * len(self.a), 1024)
            self.a = np.concatenate([self.a, np.full(m - len(self.a), self.fill, self.a.dtype)])


def ranges(start: np.ndarray, length: np.ndarray) -> np.ndarray:
    """Concatenated index ranges [start[i], start[i] + length[i]) (int64)."""
    length = np.asarray(length, np.int64)
    tot = int(length.sum())
    if not tot:
        return np.zeros(0, np.int64)
    ex = np.cumsum(length) - length
    return np.repeat(np.asarray(start, np.int64) - ex, length) + np.arange(tot, dtype=np.int64)


class SeedStore:
    """Every incident's seed triples in two pooled arrays (vertex u32, strength f32), a slice
    per handle: setting an incident's seeds appends a new slice (the old one becomes garbage,
    compacted away once it dominates), and gathering many incidents' seeds is one vectorised
    index -- no per-incident Python objects or loops."""

    def __init__(self):
        self.v = np.zeros(0, np.uint32)
        self.s = np.zeros(0, np.float32)
        self.n = 0                                   # used length of the pools
        self.start = _Grow(np.int64, 0)
        self.len = _Grow(np.int64, 0)
        self.live = 0

    def set(self, handles: np.ndarray, sv: np.ndarray, ss: np.ndarray, counts: np.ndarray) -> None:
        """Incident handles[j] gets the next counts[j] entries of (sv, ss), in order."""
        handles = np.asarray(handles, np.int64)
        counts = np.asarray(counts, np.int64)
        if not len(handles):
            return
        top = int(handles.max()) + 1
        self.start.ensure(top)
        self.len.ensure(top)
        self.live -= int(self.len.a[handles].sum())
        m = len(sv)
        if self.n + m > len(self.v):
            cap = max(self.n + m, 2 * len(self.v), 4096)
            self.v = np.concatenate([self.v[: self.n], np.zeros(cap - self.n, np.uint32)])
            self.s = np.concatenate([self.s[: self.n], np.zeros(cap - self.n, np.float32)])
        self.v[self.n:self.n + m] = sv
        self.s[self.n:self.n + m] = ss
        self.start.a[handles] = self.n + np.cumsum(counts) - counts
        self.len.a[handles] = counts
        self.n += m
        self.live += m
        if self.n > 4096 and 2 * self.live < self.n:
            self._compact()

    def _compact(self) -> None:
        hs = np.flatnonzero(self.len.a)
        idx = ranges(self.start.a[hs], self.len.a[hs])
        self.v, self.s = self.v[idx].copy(), self.s[idx].copy()
        self.start.a[hs] = np.cumsum(self.len.a[hs]) - self.len.a[hs]
        self.n = self.live = len(idx)

    def counts(self, handles: np.ndarray) -> np.ndarray:
        h = np.asarray(handles, np.int64)
        out = np.zeros(len(h), np.int64)
        ok = h < len(self.len.a)
        out[ok] = self.len.a[h[ok]]
        return out

    def gather(self, handles: np.ndarray) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
        """(vertices, strengths, per-handle counts) of these incidents, in handle order."""
        h = np.asarray(handles, np.int64)
        cnt = self.counts(h)
        st = np.zeros(len(h), np.int64)
        ok = h < len(self.start.a)
        st[ok] = self.start.a[h[ok]]
        idx = ranges(st, cnt)
        return self.v[idx], self.s[idx], cnt

    def get(self, h: int) -> tuple[np.ndarray, np.ndarray]:
        v, s, _ = self.gather(np.array([h], np.int64))
        return v, s


class RankStore:
    """Every incident's latest top-k, by handle: [n, k] ids and scores and the tick each was
    ranked at; a row is None until its incident is first ranked."""

    def __init__(self, k: int):
        self.k = k
        self.ids = np.full((0, k), NO_NODE, np.uint32)
        self.scores = np.zeros((0, k), np.float32)
        self.tick = np.full(0, -1, np.int64)

    def put(self, handles: np.ndarray, ids: np.ndarray, scores: np.ndarray, tick: int) -> None:
        top = int(handles.max()) + 1 if len(handles) else 0
        if top > len(self.tick):
            n = max(top, 2 * len(self.tick), 1024)
            self.ids = np.concatenate([self.ids, np.full((n - len(self.tick), self.k), NO_NODE, np.uint32)])
            self.scores = np.concatenate([self.scores, np.zeros((n - len(self.tick), self.k), np.float32)])
            self.tick = np.concatenate([self.tick, np.full(n - len(self.tick), -1, np.int64)])
        self.ids[handles] = ids
        self.scores[handles] = scores
        self.tick[handles] = tick

    def row(self, h: int):
        if h >= len(self.tick) or self.tick[h] < 0:
            return None, None, -1
        return self.ids[h].copy(), self.scores[h].copy(), int(self.tick[h])


class PendingIndex:
    """The storm's pending-id index: (hash of a candidate id ranked before a row's attached one,
    incident handle, generation) entries, searchable by hash.  Entries arrive as hash-sorted
    runs, one per tick; a query binary-searches every run.  Runs are merged (and retired
    generations dropped) once there are more than MAX_RUNS of them, so an insert costs the size
    of the tick's own entries, not of the whole index (np.insert into one sorted array copied
    every resident entry on every tick)."""
    MAX_RUNS = 8

    def __init__(self):
        self.runs: list[tuple[np.ndarray, np.ndarray, np.ndarray]] = []

    def __len__(self) -> int:
        return sum(len(r[0]) for r in self.runs)

    def insert(self, h: np.ndarray, o: np.ndarray, g: np.ndarray, gen: np.ndarray) -> None:
        order = np.argsort(h, kind="stable")
        self.runs.append((h[order], o[order], g[order]))
        if len(self.runs) > self.MAX_RUNS:
            hh = np.concatenate([r[0] for r in self.runs])
            oo = np.concatenate([r[1] for r in self.runs])
            gg = np.concatenate([r[2] for r in self.runs])
            live = gg == gen[oo]
            hh, oo, gg = hh[live], oo[live], gg[live]
            order = np.argsort(hh, kind="stable")
            self.runs = [(hh[order], oo[order], gg[order])]

    def hits(self, q: np.ndarray, gen: np.ndarray) -> set:
        """Handles with a live entry whose hash is one of q's: per run, the runs of equal hashes
        found by binary search."""
        out = []
        for rh, ro, rg in self.runs:
            lo = np.searchsorted(rh, q, "left")
            n = np.searchsorted(rh, q, "right") - lo
            tot = int(n.sum())
            if not tot:
                continue
            ix = np.repeat(lo - (np.cumsum(n) - n), n) + np.arange(tot)
            o = ro[ix]
            out.append(o[rg[ix] == gen[o]])
        return set(np.unique(np.concatenate(out)).tolist()) if out else set()


class StormEngine:
    COL_BUCKETS = (64, 256, 1024, 4096)

    def __init__(self, graph: EvidenceGraph, *, device=None, hops: int = 3, k: int = 10,
                 ttl_ms: int = 4 * 3600 * 1000, dedup_capacity: int = 1 << 16, weights=None,
                 comm=None, rank: int = 0, keep_evidence: bool = False):
        self.g = graph
        # an incident's evidence rows are read once, to extract its attachment candidates
        # (SeedCandidates): afterwards only the candidates are kept (and other ranks' incidents
        # never keep them), so the open incidents hold no per-row Python objects
        self.keep_evidence = keep_evidence
        self.snap = graph.snapshot(weights, device)
        self.dev = self.snap.dev
        self.hops, self.k, self.ttl_ms = hops, k, ttl_ms
        self.table = DedupTable(dedup_capacity, self.dev)
        # comm (egraph.shard.TorchComm): fingerprint-sharded table, incidents owned round-robin
        self.rank, self.world = (rank, comm.P) if comm is not None else (0, 1)
        self.dedup = ShardedDedup(self.table, comm, rank) if comm is not None else None
        self.incidents: list[OpenIncident] = []
        # pending-id index: (hash of a candidate id ranked before a row's attached one, incident
        # handle, generation); an entry is live while its generation is the incident's current
        # one.  A hash match only ever adds an incident to the re-attached set (a spurious
        # match re-attaches and re-ranks it exactly: harmless).
        self._pending = PendingIndex()
        self._gen = np.zeros(0, np.int64)
        self._frontiers: dict[int, object] = {}
        self.ranks = RankStore(k)
        self.seeds = SeedStore()                  # every incident's seed triples, by handle
        self.vtx = _Grow(np.int64, -1)           # every incident's vertex, by handle
        self.ticks = 0
        self.last_reseed: dict = {}
        # (vertex, incident) pairs the affected test reads: incident vertices and seed vertices
        self._chk_v = torch.zeros(0, dtype=torch.int64, device=self.dev)
        self._chk_o = torch.zeros(0, dtype=torch.int64, device=self.dev)
        self._stale = 0
        # objects the tick is done with (the new incidents' evidence rows once their candidates
        # are extracted, the incident cases once MERGEd): freed at the end of the tick, in a
        # stage of their own (release_host: ~0.4 us per evidence row on the GPU box)
        self._drop: list = []

    # ---- frontier per column bucket, grown / recreated as needed ---------------------------
    def _frontier(self, n_cols: int, n_seeds: int):
        b = next((c for c in self.COL_BUCKETS if c >= n_cols), None)
        if b is None:
            raise ValueError(f"{n_cols} columns exceed the largest bucket {self.COL_BUCKETS[-1]}")
        fr = self._frontiers.get(b)
        if fr is None or fr.max_seeds < n_seeds or fr.max_vertices < self.snap.n_vertices:
            cap = max(n_seeds, 64 * b, fr.max_seeds * 2 if fr is not None else 0)
            fr = self.snap.frontier(b, max_seeds=cap, k=self.k, pool_entries=-1)
            self._frontiers[b] = fr
        return fr

    def _reseed(self, handles: list[int]) -> None:
        """(Re)attach the evidence rows of these incidents to the current graph: their
        candidate ids are extracted once per incident (native, egraph/seeds.py; the incidents
        without them in ONE pass) and all of them are looked up and attached in ONE batch."""
        t0 = time.perf_counter()
        xs = [self.incidents[h] for h in handles]
        need = [x for x in xs if x.cand is None]
        batch = None
        if need:
            # one keyed batch for the tick's new incidents; an incident keeps (batch, column) and
            # is sliced out of it only if it is ever re-attached together with other incidents
            batch = SeedCandidates.keyed_batch([x.evidence for x in need])
            for j, x in enumerate(need):
                x.cand = (batch, j)
                if not self.keep_evidence:
                    self._drop.append(x.evidence)     # (freed at the end of the tick)
                    x.evidence = None
        t1 = time.perf_counter()
        if not xs:
            return
        if batch is not None and len(need) == len(xs):
            cand = batch                       # (xs are exactly the new incidents, in order)
        else:
            cand = SeedCandidates.combine([self._cand(x) for x in xs], with_flat=False)
        blob, off, hashes = cand.keys
        found = self.g.lookup_blob(blob, off) if cand.n_flat else np.zeros(0, np.int64)
        sv, col, ss, before, bcol = cand.attach_found_idx(found)
        hs = np.asarray(handles, np.int64)
        cut = np.searchsorted(col, np.arange(len(xs) + 1, dtype=np.uint32))
        self.seeds.set(hs, sv, ss, np.diff(cut))          # (rows come in column order)
        t2 = time.perf_counter()
        # the incidents' pending ids: their earlier entries retire (generation bump)
        top = int(hs.max()) + 1
        if top > len(self._gen):
            self._gen = np.concatenate([self._gen, np.zeros(max(top - len(self._gen), 1024), np.int64)])
        self._gen[hs] += 1
        if len(before):
            oh = hs[bcol.astype(np.int64)]
            self._pending.insert(hashes[before], oh, self._gen[oh], self._gen)
        self.last_reseed = {"incidents": len(xs), "new": len(need), "candidates_ms": (t1 - t0) * 1e3,
                            "attach_ms": (t2 - t1) * 1e3, "pending_ms": (time.perf_counter() - t2) * 1e3}

    @staticmethod
    def _cand(x: "OpenIncident") -> SeedCandidates:
        """x's own candidates (a column of the keyed batch it arrived in)."""
        if isinstance(x.cand, tuple):
            x.cand = x.cand[0].column(x.cand[1])
        return x.cand

    def _pending_hit(self, ids: list) -> set:
        """Incidents with a live pending entry whose hash matches one of these ids."""
        if not ids or not len(self._pending):
            return set()
        from egraph import _lib
        q = np.frombuffer(_lib.pyhost.hash_ids(ids), np.int64)    # (seed_keys' id hashes)
        return self._pending.hits(q, self._gen)

    def _check_parts(self, handles) -> tuple[torch.Tensor, torch.Tensor]:
        """(vertex, incident) pairs of these incidents: each incident vertex, then every seed
        vertex (SeedStore order)."""
        hs = np.asarray(handles, np.int64)
        self.vtx.ensure(int(hs.max()) + 1 if len(hs) else 0)
        sv, _, cnt = self.seeds.gather(hs)
        v = np.concatenate([np.maximum(self.vtx.a[hs], 0), sv.astype(np.int64)])
        o = np.concatenate([hs, np.repeat(hs, cnt)])
        return to_device(v, self.dev), to_device(o, self.dev)

    def owns(self, handle: int) -> bool:
        return handle % self.world == self.rank

    def _rebuild_check(self) -> None:
        self._chk_v, self._chk_o = self._check_parts(
            np.arange(self.rank, len(self.incidents), self.world, dtype=np.int64))

    def _append_check(self, handles: list[int]) -> None:
        if handles:
            v, o = self._check_parts(handles)
            self._chk_v = torch.cat([self._chk_v, v])
            self._chk_o = torch.cat([self._chk_o, o])

    def _rank(self, handles: list[int]) -> None:
        """Re-rank these incidents from their cached seeds (one frontier launch per 4096)."""
        inc_label = self.g.labels().index("Incident") if "Incident" in self.g.labels() else -1
        top = self.COL_BUCKETS[-1]
        hs_all = np.asarray(handles, np.int64)
        for lo in range(0, len(hs_all), top):
            hs = hs_all[lo:lo + top]
            n = len(hs)
            sv, ss, cnt = self.seeds.gather(hs)
            sc = np.repeat(np.arange(n, dtype=np.uint32), cnt)
            fr = self._frontier(n, len(sv))
            src = np.full(fr.B, NO_NODE, np.uint32)
            vx = self.vtx.a[hs]
            src[:n] = np.where(vx >= 0, vx, NO_NODE).astype(np.uint32)
            fr.set_seeds(to_device(sv, self.dev), to_device(sc, self.dev), to_device(ss, self.dev))
            ids, scores = fr.run(to_device(src, self.dev), hops=self.hops, exclude_label=inc_label)
            ids = ids.cpu().numpy().view(np.uint32)
            scores = scores.cpu().numpy()
            fr.adapt()              # overflowing columns: the wide-table retry from the next call on
            # the launch's rows into the engine's arrays, one step for all of them
            self.ranks.put(hs, ids[:n], scores[:n], self.ticks)

    def tick(self, keys: list[str], now_ms: int, make_case: Callable[[int, int], StormCase],
             topology: tuple | None = None, seq=None) -> dict:
        """One batch of alerts.  `keys`: the alerts' fingerprint keys, in arrival order
        (normalizer.py:217 strings).  `make_case(handle, alert_index)` builds the incident an
        alert opens.  `topology`: optional (vertex ids, labels, edge src, dst, types) MERGEd in
        the same tick.  Across GPUs `keys` are the alerts that arrived at this rank and `seq`
        their numbers in the tick's global arrival order (alert_index refers to that order;
        make_case and topology must be the same on every rank).  Returns counts and per-stage
        wall times (ms)."""
        t = [time.perf_counter()]
        fp, _ = fingerprints(keys, self.dev)
        if self.dedup is None:
            dup, inc, n_new = self.table.ingest(fp, now_ms, self.ttl_ms)     # synchronises
            dup_h = dup.cpu().numpy()
            inc_h = inc.cpu().numpy()
        else:
            if seq is None:
                raise ValueError("a sharded tick needs the alerts' global arrival numbers (seq)")
            dup_h, inc_h, n_new = self.dedup.ingest(
                fp, torch.as_tensor(np.asarray(seq, np.int64)), now_ms, self.ttl_ms)
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
            self._drop.append(case)
            self.incidents.append(OpenIncident(h, case.incident_id, case.evidence
                                               if self.keep_evidence or self.owns(h) else None,
                                               store=self.ranks, seeds=self.seeds, vtx=self.vtx))
            new_handles.append(h)
            if case.entities:                      # (column-wise, in C: zip(*) per case)
                a, b = zip(*case.entities)
                ids += a
                labels += b
            if case.relations:
                a, b, c = zip(*case.relations)
                es += a
                ed += b
                et += c
        if topology is not None:
            tv, tl, ts, td, tt = topology
            ids += list(tv)
            labels += list(tl)
            es += list(ts)
            ed += list(td)
            et += list(tt)
        V0, E0 = self.snap.n_vertices, self.snap.synced_edges
        new_ids: list[str] = []
        if ids:
            vix = self.g.merge_nodes(ids, labels)
            new_ids = [ids[i] for i in np.flatnonzero(vix >= V0)]
        if es:
            self.g.merge_edges(es, ed, et)
        if new_handles:
            vs = self.g.lookup([f"incident:{self.incidents[h].incident_id}" for h in new_handles])
            self.vtx.ensure(new_handles[-1] + 1)
            self.vtx.a[np.asarray(new_handles, np.int64)] = vs
        t.append(time.perf_counter())
        n_v, n_e = self.snap.sync(self.g)                                 # GPU CSR update
        t.append(time.perf_counter())
        # affected incidents (before the new incidents join the check arrays); only this
        # rank's own incidents are checked and re-ranked
        n_old = len(self.incidents) - len(new_handles)
        new_handles = [h for h in new_handles if self.owns(h)]
        affected = set(new_handles)
        reseed = set()
        if n_old:                                        # rows that would attach differently now
            reseed = {h for h in self._pending_hit(new_ids) if h < n_old}
        if (n_v or n_e) and n_old and self.hops >= 1:
            s2, d2, _ = self.g.export_edges(E0, n_e)
            touched = np.unique(np.concatenate([np.arange(V0, V0 + n_v, dtype=np.int64),
                                                s2.astype(np.int64), d2.astype(np.int64)]))
            dist = self.snap.within(to_device(touched.astype(np.uint32), self.dev), self.hops - 1)
            hit = (dist[self._chk_v] != 255).to(torch.int32)
            flag = torch.zeros(n_old, dtype=torch.int32, device=self.dev)
            flag.scatter_reduce_(0, self._chk_o, hit, reduce="amax")
            affected.update(np.flatnonzero(flag.cpu().numpy()).tolist())
        affected |= reseed
        t.append(time.perf_counter())
        # seeds: new incidents and re-attached ones
        self._reseed(sorted(set(new_handles) | reseed))
        # re-attached incidents: append their new seed vertices; the old entries stay (a
        # superset only re-ranks more) until they make up half the arrays
        self._append_check(sorted(set(new_handles) | reseed))
        if reseed:
            self._stale += int(self.seeds.counts(np.fromiter(reseed, np.int64, len(reseed))).sum()) + len(reseed)
        if self._stale * 2 > self._chk_v.numel():
            self._rebuild_check()
            self._stale = 0
        t.append(time.perf_counter())
        self._rank(sorted(affected))
        torch.cuda.synchronize(self.dev)
        t.append(time.perf_counter())
        self._drop.clear()
        t.append(time.perf_counter())
        self.ticks += 1
        ms = [(b - a) * 1e3 for a, b in zip(t, t[1:])]
        ms[1] -= t_collect * 1e3          # the incidents' evidence comes from the collectors
        return {"alerts": len(dup_h), "duplicates": int(dup_h.sum()), "new_incidents": n_new,
                "new_vertices": n_v, "new_edges": n_e, "affected": len(affected),
                "open_incidents": len(self.incidents),
                "ms": dict(zip(("fingerprint_dedup", "merge_host", "csr_update", "affected", "seeds_host",
                               "rerank", "release_host"), ms)),
                "collect_ms": t_collect * 1e3, "reseed": dict(self.last_reseed)}

    def rankings(self) -> list[tuple[np.ndarray, np.ndarray]]:
        """(top ids, top scores) of every incident (None for those another rank owns)."""
        return [(x.top_ids, x.top_scores) for x in self.incidents]
