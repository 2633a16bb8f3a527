"""Diagnostic (GPU box): how well do cheap per-column proxies predict a frontier column's time,
and what would longest-first column ordering save?  Runs the bench's C3 batch in profile mode,
reads each column's start/end stamps, its member count and two a-priori proxies (seed count,
sum of seed-vertex degrees), and simulates list scheduling of the columns over 512 slots
(2 workgroups x 256 CUs) in launch order vs sorted by each proxy."""
from __future__ import annotations

import heapq
import os
import sys
from pathlib import Path

os.environ["EGRAPH_FRONTIER_PROFILE"] = "1"
REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "kubernetes-aiops-evidence-graph_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def makespan(times, order, slots=512):
    h = [0.0] * slots
    heapq.heapify(h)
    end = 0.0
    for c in order:
        t = heapq.heappop(h) + times[c]
        end = max(end, t)
        heapq.heappush(h, t)
    return end


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = bench.setup("C3", 1024, 10, 0, dev)
    for _ in range(3):
        bench.step_frontier(ctx, 3)
    torch.cuda.synchronize()
    ph = ctx["frontier"].phase_times().astype(np.float64) * 10.0 / 1000.0
    t = ph[:, :, 0]
    used = int((t[0, :24] > 0).sum())
    total = t[:, used - 1] - t[:, 0]
    start = t[:, 0] - t[:, 0].min()
    fr = ctx["frontier"]
    B = fr.B
    members = np.array([len(fr.members(b)[0]) for b in range(B)], np.float64)
    sv, sc, ss = ctx["seed_host"]
    csr = ctx["graph"].csr()
    deg = np.diff(csr["row_ptr"].astype(np.int64))
    nseed = np.bincount(sc, minlength=B).astype(np.float64)
    degsum = np.bincount(sc, weights=deg[sv], minlength=B)
    # unique seed vertices per column and their degree sum (duplicates max-combine)
    key = np.unique(sc.astype(np.int64) * (1 << 32) + sv)
    ucol, uv = key >> 32, key & 0xFFFFFFFF
    udeg = np.bincount(ucol, weights=deg[uv], minlength=B)
    d2 = np.zeros(B)
    rp = csr["row_ptr"].astype(np.int64)
    col = csr["col"].astype(np.int64)
    for b in range(B):   # 2-hop degree mass of the unique seeds
        vs = uv[ucol == b]
        nb = np.concatenate([col[rp[v]:rp[v + 1]] for v in vs]) if len(vs) else np.zeros(0, np.int64)
        d2[b] = deg[nb].sum()
    print(f"column time: mean {total.mean():.1f} p50 {np.median(total):.1f} max {total.max():.1f} us;"
          f" start span {start.max():.1f}; last end {(start + total).max():.1f}")
    for name, p in (("members", members), ("seeds", nseed), ("seed_deg", degsum),
                    ("useed_deg", udeg), ("2hop_deg", d2)):
        r = np.corrcoef(p, total)[0, 1]
        ms = makespan(total, np.argsort(-p, kind="stable"))
        print(f"{name:>10}: corr {r:+.3f}  LPT-by-proxy makespan {ms:.1f} us")
    print(f"launch order makespan {makespan(total, np.arange(B)):.1f} us; "
          f"oracle LPT {makespan(total, np.argsort(-total)):.1f} us; ideal {total.sum() / 512:.1f} us")


if __name__ == "__main__":
    main()
