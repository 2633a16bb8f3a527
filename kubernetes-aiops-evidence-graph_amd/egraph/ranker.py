"""GPU ranker for arbitrary hypothesis lists (HypothesisRanker.rank, hypothesis_ranker.py:13-80).

The host gathers the four numbers the reference reads from each dict (with its defaults and
its TypeErrors); egr_rank computes final_score with Python-exact float64 rounding and the
stable descending order of every list in one launch, over persistent pinned / device buffers
(one packed copy each way), so a single small list costs one kernel round trip.
"""
from __future__ import annotations

import math
import threading

import numpy as np
import torch

from . import _lib as L
from .catalog import CATEGORY_WEIGHTS
from .device import require_device


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

    def __init__(self, dev: torch.device):
        self.dev = dev
        self.stream = torch.cuda.Stream(dev)
        self.event = torch.cuda.Event()
        self.cap = 0
        self.lock = threading.Lock()

    def run(self, cols, off):
        n, nl = len(cols[0]), len(off) - 1
        need = 8 * (5 * n + nl + 1) + 4 * n + 64
        with self.lock:
            if need > self.cap:
                self.cap = max(need, 2 * self.cap, 1 << 16)
                self.dbuf = torch.empty(self.cap, dtype=torch.uint8, device=self.dev)
                self.hbuf = torch.empty(self.cap, dtype=torch.uint8).pin_memory()
                self.hnp = self.hbuf.numpy()
            h = self.hnp
            f64 = h[: 8 * (4 * n + nl + 1)].view(np.float64)
            for j, col in enumerate(cols):
                f64[j * n:(j + 1) * n] = col
            ino = 32 * n
            h[ino: ino + 8 * (nl + 1)].view(np.int64)[:] = off
            in_bytes = ino + 8 * (nl + 1)
            fo = (in_bytes + 7) // 8 * 8                      # final f64 [n], then order i32 [n]
            oo = fo + 8 * n
            end = oo + 4 * n
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


def rank_lists(lists: list[list[dict]], device=None) -> list[list[dict]]:
    """Rank every list in one launch; mutates and returns the dicts like the reference."""
    dev = require_device(device)
    cols = ([], [], [], [])
    off = [0]
    for hyps in lists:
        for acc, vals in zip(cols, gather(hyps)):
            acc.extend(vals)
        off.append(off[-1] + len(hyps))
    n = off[-1]
    if n == 0:
        return [[] for _ in lists]
    r = _RUNNERS.get(dev)
    if r is None:
        r = _RUNNERS[dev] = _RankRunner(dev)
    final_h, order_h = r.run(cols, off)
    out = []
    for j, hyps in enumerate(lists):
        b = off[j]
        for i, h in enumerate(hyps):
            h["final_score"] = float(final_h[b + i])
        ranked = [hyps[int(order_h[b + p])] for p in range(len(hyps))]
        for p, h in enumerate(ranked):
            h["rank"] = p + 1
        out.append(ranked)
    return out
