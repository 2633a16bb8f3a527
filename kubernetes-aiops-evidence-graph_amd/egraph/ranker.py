"""GPU ranker for arbitrary hypothesis lists (HypothesisRanker.rank, hypothesis_ranker.py:13-80).

The host gathers the four numbers the reference reads from each dict (with its defaults and
its TypeErrors); egr_rank computes final_score with Python-exact float64 rounding and the
stable descending order of every list in one launch, over persistent pinned / device buffers
(one packed copy each way; zero-copy mapped host memory for small lists), so a single small
list costs one kernel round trip.

Fused ranks.  egr_rules_eval already ranks every hypothesis list it generates (the ranker's
score and order are fused into the rules kernel, csrc/rules.hip).  The workflow ranks exactly
those lists in its next activity (activities.py:124-170), so the rules path registers each
generated list here (keyed by its hypothesis ids; bounded, least recently used first out) and
rank() reuses the kernel's final scores and order when the list it gets has the same ids, in the
same order, with the four inputs the ranker reads unchanged -- verified field by field, so the
result is exactly what egr_rank would compute.  Any other list (edited, reordered, foreign)
goes to egr_rank.
"""
from __future__ import annotations

import math
import threading
from collections import OrderedDict

import numpy as np
import torch

from . import _lib as L
from .catalog import CATEGORY_WEIGHTS
from .device import MappedBuffer, require_device


def _num(x, what: str) -> float:
    if not isinstance(x, (int, float)):
        raise TypeError(f"unsupported operand type(s) for {what}: '{type(x).__name__}'")
    return float(x)


def gather(hyps: list[dict]) -> tuple[list, list, list, list]:
    """Per-dict inputs with the reference's defaults (:46-59)."""
    conf, catw, sup, strength = [], [], [], []
    for h in hyps:
        c = h.get("confidence", 0.5)
        w = CATEGORY_WEIGHTS.get(h.get("category", "unknown"), 1.0)
        s = h.get("support_count", 0)
        g = h.get("signal_strength", 0)
        conf.append(_num(c, "*="))
        catw.append(w)
        sup.append(_num(s, ">"))
        strength.append(_num(g, "*"))
    for v in (*conf, *sup, *strength):
        if math.isnan(v):
            raise ValueError("NaN hypothesis scores are not supported (Python's sort order "
                             "with NaN keys is unspecified)")
    return conf, catw, sup, strength


class _RankRunner:
    """egr_rank over persistent device / pinned host buffers on its own stream: one packed
    host-to-device copy, the kernel, one packed device-to-host copy, one event wait."""

    ZERO_COPY_ENTRIES = 4096     # lists with up to this many hypotheses in total: mapped memory

    def __init__(self, dev: torch.device):
        self.dev = dev
        self.stream = torch.cuda.Stream(dev)
        self.event = torch.cuda.Event()
        self.cap = 0
        self.lock = threading.Lock()
        self.mapped = None

    def _layout(self, n: int, nl: int):
        ino = 32 * n
        in_bytes = ino + 8 * (nl + 1)
        fo = (in_bytes + 7) // 8 * 8                      # final f64 [n], then order i32 [n]
        oo = fo + 8 * n
        return ino, in_bytes, fo, oo, oo + 4 * n

    def _fill(self, h, cols, off, n, nl, ino) -> None:
        f64 = h[: 8 * (4 * n + nl + 1)].view(np.float64)
        for j, col in enumerate(cols):
            f64[j * n:(j + 1) * n] = col
        h[ino: ino + 8 * (nl + 1)].view(np.int64)[:] = off

    def run(self, cols, off):
        n, nl = len(cols[0]), len(off) - 1
        need = 8 * (5 * n + nl + 1) + 4 * n + 64
        with self.lock:
            if n <= self.ZERO_COPY_ENTRIES:
                # zero-copy: the kernel reads the columns from and writes the results to mapped
                # host memory -- one launch, no DMA copies
                if self.mapped is None:
                    self.mapped = MappedBuffer(1 << 20)
                h, base = self.mapped.np, self.mapped.dev
                ino, _, fo, oo, end = self._layout(n, nl)
                self._fill(h, cols, off, n, nl, ino)
                L.check(L.lib.egr_rank(base, base + 8 * n, base + 16 * n, base + 24 * n, base + ino,
                                       nl, base + fo, base + oo, self.stream.cuda_stream), "egr_rank")
                self.event.record(self.stream)
                self.event.synchronize()
                return h[fo:oo].view(np.float64).copy(), h[oo:end].view(np.int32).copy()
            if need > self.cap:
                self.cap = max(need, 2 * self.cap, 1 << 16)
                self.dbuf = torch.empty(self.cap, dtype=torch.uint8, device=self.dev)
                self.hbuf = torch.empty(self.cap, dtype=torch.uint8).pin_memory()
                self.hnp = self.hbuf.numpy()
            h = self.hnp
            ino, in_bytes, fo, oo, end = self._layout(n, nl)
            self._fill(h, cols, off, n, nl, ino)
            base = self.dbuf.data_ptr()
            with torch.cuda.stream(self.stream):
                self.dbuf[:in_bytes].copy_(self.hbuf[:in_bytes], non_blocking=True)
                L.check(L.lib.egr_rank(base, base + 8 * n, base + 16 * n, base + 24 * n, base + ino,
                                       nl, base + fo, base + oo, self.stream.cuda_stream), "egr_rank")
                self.hbuf[fo:end].copy_(self.dbuf[fo:end], non_blocking=True)
                self.event.record(self.stream)
            self.event.synchronize()
            return h[fo:oo].view(np.float64).copy(), h[oo:end].view(np.int32).copy()


_RUNNERS: dict = {}


class FusedRanks:
    """The rules kernel's ranking of the lists it generated, for rank() to reuse (module doc).
    A launch's fields are packed once into one bytes block (row j = list j: the slot order, the
    kernel's order, confidence, signal strength and final score per slot); a record keeps the
    list's hypothesis ids, the block and its row, and is built in native code
    (csrc/pyhost.c fused_records), so registering a launch's lists runs no Python loop."""

    def __init__(self, capacity: int = 1 << 16):
        self.capacity = capacity
        self.recs: OrderedDict = OrderedDict()
        self.lock = threading.Lock()
        self.hits = self.misses = 0

    @staticmethod
    def pack(res, sel) -> bytes:
        """The block of rows `sel` of a launch's results (csrc/pyhost.c's fused-rank layout)."""
        S = res.confidence.shape[1]
        a8 = (2 * S + 7) // 8 * 8
        buf = np.zeros((len(sel), a8 + 24 * S), np.uint8)
        buf[:, :S] = res.order_conf[sel]
        buf[:, S:2 * S] = res.order_rank[sel]
        for k, a in enumerate((res.confidence, res.strength, res.final_score)):
            buf[:, a8 + 8 * S * k:a8 + 8 * S * (k + 1)] = \
                np.ascontiguousarray(a[sel], np.float64).view(np.uint8)
        return buf.tobytes()

    def register(self, cat, res, lists: list[list[dict]], rows) -> None:
        """lists[j] = the unranked dicts of result row rows[j] (confidence order)."""
        rows = list(rows)
        if not rows:
            return
        blk = self.pack(res, np.asarray(rows, np.int64))
        u = cat.unknown
        # what the native check (pyhost.fused_apply) compares against, read from the catalog
        # now as apply() would read it
        ncat = (cat.n_rules, tuple(r["category"] for r in cat.rules),
                tuple(len(r["conditions"]) for r in cat.rules),
                (u["confidence"], u["category"], u["support_count"], u["signal_strength"]))
        recs = L.pyhost.fused_records(lists if type(lists) is list else list(lists), blk, cat, ncat)
        with self.lock:
            self.recs.update(recs)
            while len(self.recs) > self.capacity:
                self.recs.popitem(last=False)

    def apply(self, hyps: list) -> list | None:
        """Rank `hyps` from its record if it is exactly a registered list; else None."""
        if type(hyps) is list:
            # lookup, checks and writes in native code (csrc/pyhost.c fused_rank); None: a value
            # it leaves to the Python statements below
            r = L.pyhost.fused_rank(self.recs, hyps)
            if r is not None:
                if type(r) is int:                 # 0: a miss; 1: not a candidate (not counted)
                    if r == 0:
                        self.misses += 1
                    return None
                self.hits += 1
                return r
        if not hyps or not isinstance(hyps[0], dict):
            return None
        # (one C-level get: atomic under the GIL against register()'s locked updates)
        rec = self.recs.get(hyps[0].get("id"))
        if rec is None or len(hyps) != len(rec[0]):
            self.misses += 1
            return None
        ids, cat, blk, row, _ = rec
        R, rules, u = cat.n_rules, cat.rules, cat.unknown
        S = R + 1
        a8 = (2 * S + 7) // 8 * 8
        rb = np.frombuffer(blk, np.uint8, a8 + 24 * S, row * (a8 + 24 * S))
        slots, orank = rb[:len(hyps)].tolist(), rb[S:S + len(hyps)].tolist()
        conf, strength, final = (rb[a8 + 8 * S * k:a8 + 8 * S * (k + 1)].view(np.float64).tolist()
                                 for k in range(3))
        for h, hid, slot in zip(hyps, ids, slots):
            if not isinstance(h, dict) or h.get("id") != hid:
                self.misses += 1
                return None
            # the (confidence, category, support_count, signal_strength) the kernel emitted
            if slot == R:
                c, catg, sup, st = u["confidence"], u["category"], u["support_count"], u["signal_strength"]
            else:
                r = rules[slot]
                c, catg, sup, st = conf[slot], r["category"], len(r["conditions"]), strength[slot]
            if h.get("confidence", 0.5) != c or h.get("category", "unknown") != catg or \
                    h.get("support_count", 0) != sup or h.get("signal_strength", 0) != st:
                self.misses += 1
                return None
        self.hits += 1
        pos = {}
        for p, (h, slot) in enumerate(zip(hyps, slots)):
            h["final_score"] = final[slot]
            pos[slot] = p
        out = [hyps[pos[s]] for s in orank]
        for q, h in enumerate(out, 1):
            h["rank"] = q
        return out


FUSED = FusedRanks()


def rank_lists(lists: list[list[dict]], device=None, fused: bool = True) -> list[list[dict]]:
    """Rank every list in one launch; mutates and returns the dicts like the reference.  Lists
    the rules kernel generated and already ranked are served from FUSED (`fused=False`: the
    caller already asked it)."""
    out: list = [FUSED.apply(hyps) for hyps in lists] if fused else [None] * len(lists)
    todo = [j for j, r in enumerate(out) if r is None]
    if not todo:
        return out                     # (every list was a kernel-ranked one: no device call)
    dev = require_device(device)
    cols = ([], [], [], [])
    off = [0]
    for j in todo:
        hyps = lists[j]
        for acc, vals in zip(cols, gather(hyps)):
            acc.extend(vals)
        off.append(off[-1] + len(hyps))
    n = off[-1]
    if n == 0:
        for j in todo:
            out[j] = []
        return out
    r = _RUNNERS.get(dev)
    if r is None:
        r = _RUNNERS[dev] = _RankRunner(dev)
    final_h, order_h = r.run(cols, off)
    for t, j in enumerate(todo):
        hyps, b = lists[j], off[t]
        for i, h in enumerate(hyps):
            h["final_score"] = float(final_h[b + i])
        ranked = [hyps[int(order_h[b + p])] for p in range(len(hyps))]
        for p, h in enumerate(ranked):
            h["rank"] = p + 1
        out[j] = ranked
    return out
