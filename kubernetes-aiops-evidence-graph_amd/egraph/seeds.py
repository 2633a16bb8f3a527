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


def _row(ev) -> tuple[list, float]:
    """One row's candidates and strength, in the order the statement below evaluates them."""
    return attach_ids(ev), float(ev.get("signal_strength", 0.5))


def candidates_py(evidence_lists: list[list[dict]]) -> tuple[list, list, list, list]:
    """(flat candidate ids, per-row counts, columns, strengths) of every row that seeds:
    the Python statement of the native pyhost.seed_candidates (tests compare the two)."""
    flat, count, col, val = [], [], [], []
    for b, evs in enumerate(evidence_lists):
        for ev in evs:
            ids, s = _row(ev)
            if not ids or s <= 0:
                continue
            flat.extend(ids)
            count.append(len(ids))
            col.append(b)
            val.append(s)
    return flat, count, col, val


class SeedCandidates:
    """The attachment candidates of a batch's evidence rows, computed once (string work, in
    native code: csrc/pyhost.c seed_candidates, with _row as its hand-over for rows whose values
    are not plain built-ins) and re-attached cheaply against a growing graph (`attach`): flat
    candidate ids, per-row candidate counts, columns and strengths."""

    def __init__(self, evidence_lists: list[list[dict]]):
        from . import _lib
        flat, count, col, val = _lib.pyhost.seed_candidates(evidence_lists, _row)
        self.n_cols = len(evidence_lists)
        self.flat = flat
        self.keys = None
        # (no seeding row at all: the native call returns None for the empty buffers)
        self.count = np.frombuffer(count or b"", np.int64)
        self.col = np.frombuffer(col or b"", np.uint32)
        self.val = np.frombuffer(val or b"", np.float64).astype(np.float32)

    @classmethod
    def _of(cls, n_cols: int, flat: list | None, count, col, val, keys=None) -> "SeedCandidates":
        o = cls.__new__(cls)
        o.n_cols, o.flat, o.count, o.col, o.val = n_cols, flat, count, col, val
        o.keys = keys
        return o

    @property
    def n_flat(self) -> int:
        return len(self.flat) if self.flat is not None else len(self.keys[2])

    def _flat_keys(self):
        """(utf-8 blob, int64 offsets [n+1], int64 hashes of the ids' bytes [n]) of the flat ids:
        what a blob graph lookup and the storm's pending index read (pyhost.hash_ids)."""
        from . import _lib
        from .graph import str_blob
        b, o = str_blob(self.flat)
        return b, o, np.frombuffer(_lib.pyhost.hash_ids(self.flat), np.int64)

    @classmethod
    def per_column(cls, evidence_lists: list[list[dict]], keys: bool = False) -> list["SeedCandidates"]:
        """One SeedCandidates per evidence list, from ONE native pass over all of them.  With
        `keys`, each also carries its ids' blob / offsets / hashes (for combine(with_flat=False))
        and drops the per-id str list."""
        n = len(evidence_lists)
        if not keys:
            sc = cls(evidence_lists)
            rb = np.searchsorted(sc.col, np.arange(n + 1, dtype=np.uint32))   # rows per column
            fb = np.concatenate([[0], np.cumsum(sc.count)])[rb]               # flat ids per column
            return [cls._of(1, sc.flat[fb[b]:fb[b + 1]], sc.count[rb[b]:rb[b + 1]],
                            np.zeros(rb[b + 1] - rb[b], np.uint32), sc.val[rb[b]:rb[b + 1]])
                    for b in range(n)]
        batch = cls.keyed_batch(evidence_lists)
        return [batch.column(b) for b in range(n)]

    @classmethod
    def keyed_batch(cls, evidence_lists: list[list[dict]]) -> "SeedCandidates":
        """The keyed candidates of a whole batch (columns = the lists' positions) from one native
        pass that emits the ids as a blob + offsets + hashes directly (csrc/pyhost.c seed_keys;
        no Python str per id).  column(b) is list b's own SeedCandidates, sliced on demand."""
        from . import _lib
        from .encode import encode_threads
        blob, off, hs, count, col, val = _lib.pyhost.seed_keys(evidence_lists, _row, encode_threads())
        off, hs = np.frombuffer(off, np.int64), np.frombuffer(hs, np.int64)
        return cls._of(len(evidence_lists), None, np.frombuffer(count, np.int64),
                       np.frombuffer(col, np.uint32), np.frombuffer(val, np.float32), (blob, off, hs))

    def column(self, b: int) -> "SeedCandidates":
        """Column b of a keyed batch as a one-column SeedCandidates (keys re-based)."""
        cut = getattr(self, "_cut", None)
        if cut is None:
            rb = np.searchsorted(self.col, np.arange(self.n_cols + 1, dtype=np.uint32))
            cut = self._cut = (rb, np.concatenate([[0], np.cumsum(self.count)])[rb])
        rb, fb = cut
        blob, off, hs = self.keys
        f0, f1, r0, r1 = fb[b], fb[b + 1], rb[b], rb[b + 1]
        k = (blob[off[f0]:off[f1]], off[f0:f1 + 1] - off[f0], hs[f0:f1])
        return self._of(1, None, self.count[r0:r1], np.zeros(r1 - r0, np.uint32), self.val[r0:r1], k)

    @classmethod
    def combine(cls, parts: list["SeedCandidates"], with_flat: bool = True) -> "SeedCandidates":
        """The single-column candidates `parts` as the columns 0..len(parts)-1 of one batch.
        with_flat=False joins the parts' keys (per_column(keys=True)) instead of their id lists."""
        rows = [len(p.count) for p in parts]
        count = np.concatenate([p.count for p in parts]) if parts else np.zeros(0, np.int64)
        col = np.repeat(np.arange(len(parts), dtype=np.uint32), rows)
        val = np.concatenate([p.val for p in parts]) if parts else np.zeros(0, np.float32)
        if with_flat:
            return cls._of(len(parts), [i for p in parts for i in p.flat], count, col, val)
        if not parts:
            return cls._of(0, None, count, col, val, (b"", np.zeros(1, np.int64), np.zeros(0, np.int64)))
        lens = np.array([len(p.keys[0]) for p in parts], np.int64)
        base = np.concatenate([[0], np.cumsum(lens)[:-1]])
        off = np.concatenate([np.zeros(1, np.int64)] + [p.keys[1][1:] + base[j] for j, p in enumerate(parts)])
        keys = (b"".join(p.keys[0] for p in parts), off, np.concatenate([p.keys[2] for p in parts]))
        return cls._of(len(parts), None, count, col, val, keys)

    def attach(self, graph, pending: list | None = None):
        """(vertex u32, column u32, strength f32) triples: each row attaches to its first
        candidate present in `graph`.  `pending` (optional list) receives per column the
        candidate ids ranked before the attached one (all, for an unattached row)."""
        if pending is not None:
            pending[:] = [set() for _ in range(self.n_cols)]
        if not self.n_flat:
            return np.zeros(0, np.uint32), np.zeros(0, np.uint32), np.zeros(0, np.float32)
        if self.flat is None:
            return self.attach_found(graph.lookup_blob(*self.keys[:2]), pending)
        return self.attach_found(graph.lookup(self.flat), pending)

    def attach_found_idx(self, found: np.ndarray):
        """attach_found's triples plus, as flat candidate indices and their columns, the
        candidates ranked before each row's attached one (all of an unattached row's) -- the
        ids whose creation would re-attach a row (egraph/storm.py indexes them by hash)."""
        if not self.n_flat:
            z = np.zeros(0, np.int64)
            return (np.zeros(0, np.uint32), np.zeros(0, np.uint32), np.zeros(0, np.float32), z,
                    np.zeros(0, np.uint32))
        from . import _lib
        found = np.ascontiguousarray(found, np.int64)
        sv, ok, before, brow = _lib.pyhost.attach_idx(found, np.ascontiguousarray(self.count, np.int64))
        ok = np.frombuffer(ok, np.bool_)
        before = np.frombuffer(before, np.int64)
        return (np.frombuffer(sv, np.uint32), self.col[ok], self.val[ok], before,
                self.col[np.frombuffer(brow, np.int64)])

    def attach_found(self, found: np.ndarray, pending: list | None = None):
        """attach() with the graph lookup of self.flat already done (callers batch it)."""
        if pending is not None:
            pending[:] = [set() for _ in range(self.n_cols)]
        if not self.n_flat:
            return np.zeros(0, np.uint32), np.zeros(0, np.uint32), np.zeros(0, np.float32)
        if pending is not None and self.flat is None:
            raise ValueError("pending id sets need the id list (combine(with_flat=True))")
        found = np.asarray(found).astype(np.int64)
        n = len(self.flat)
        starts = np.concatenate([[0], np.cumsum(self.count)[:-1]])
        pos = np.where(found >= 0, np.arange(n), n)
        first = np.minimum.reduceat(pos, starts)            # flat index of the attached id
        ok = first < n
        if pending is not None:
            row_of = np.repeat(np.arange(len(self.count)), self.count)
            before = np.arange(n) < np.repeat(np.where(ok, first, n), self.count)
            for i in np.flatnonzero(before):
                pending[self.col[row_of[i]]].add(self.flat[i])
        return (found[first[ok]].astype(np.uint32), self.col[ok], self.val[ok])


def attach_native(graph, evidence_lists: list[list[dict]], threads: int | None = None):
    """SeedCandidates(evidence_lists).attach(graph) in one native pass (csrc/pyhost.c
    seed_attach): candidate ids are formatted as bytes and resolved by egr_graph_find, on the
    encoder's worker pool for large batches, with no Python str built per id.  Rows whose values
    are not plain built-ins are handed to `_row` (the Python statement), in row order."""
    import ctypes as C

    from . import _lib
    from .encode import encode_threads
    find = C.cast(_lib.lib.egr_graph_find, C.c_void_p).value
    v, c, s = _lib.pyhost.seed_attach(evidence_lists, _row, find, graph.handle.value,
                                      encode_threads() if threads is None else threads)
    return (np.frombuffer(v, np.uint32).copy(), np.frombuffer(c, np.uint32).copy(),
            np.frombuffer(s, np.float32).copy())


def seeds_for_batch(graph, evidence_lists: list[list[dict]], pending: list | None = None):
    """(vertex u32, column u32, strength f32) triples for a batch: each row attaches to the
    first of its candidate ids present in the graph; unattached rows are dropped.
    `pending` (optional, a list) receives per column the set of candidate ids ranked before the
    one attached (all of them for an unattached row): the vertices whose later creation would
    re-attach a row -- the alert storm's re-rank trigger (egraph/storm.py).  Without `pending`
    the attachment runs in one native pass (attach_native)."""
    if pending is None:
        return attach_native(graph, evidence_lists)
    return SeedCandidates(evidence_lists).attach(graph, pending)
