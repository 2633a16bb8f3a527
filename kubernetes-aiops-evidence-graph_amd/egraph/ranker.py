"""GPU ranker for arbitrary hypothesis lists (HypothesisRanker.rank, hypothesis_ranker.py:13-80).

The host gathers the four numbers the reference reads from each dict (with its defaults and
its TypeErrors); egr_rank computes final_score with Python-exact float64 rounding and the
stable descending order of every list in one launch.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib as L
from .catalog import CATEGORY_WEIGHTS
from .device import require_device, to_device


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
    with torch.cuda.device(dev):
        c, w, s, g = (to_device(np.asarray(x, np.float64), dev) for x in cols)
        o = to_device(np.asarray(off, np.int64), dev)
        final = torch.empty(n, dtype=torch.float64, device=dev)
        order = torch.empty(n, dtype=torch.int32, device=dev)
        L.check(L.lib.egr_rank(L.ptr(c), L.ptr(w), L.ptr(s), L.ptr(g), L.ptr(o), len(lists),
                               L.ptr(final), L.ptr(order), L.stream_handle(dev)), "egr_rank")
        final_h = final.cpu().numpy()
        order_h = order.cpu().numpy()
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
