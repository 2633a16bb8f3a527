"""Launch-order predictors against measured column durations (CPU; diagnostic).

Reads the per-column start / duration / member arrays frontier_profile.py --out saved next to
its JSON (a GPU run of the headline launch: C3, 1024 x 20 distinct batches), rebuilds the same
world on the host and prints the Spearman correlation of each candidate cost predictor with the
measured durations -- the grid's drain tail is as long as the last-started columns, so the
launch order wants a predictor that ranks durations well.
Usage: python scripts/launch_order_study.py gpurun_out/r05drain/prof.npz [--merge 20]
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "kubernetes-aiops-evidence-graph_amd"))

import numpy as np  # noqa: E402

import bench  # noqa: E402


def rank(x):
    r = np.empty(len(x), np.float64)
    r[np.argsort(x, kind="stable")] = np.arange(len(x))
    return r


def spearman(a, b):
    return float(np.corrcoef(rank(a), rank(b))[0, 1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("npz")
    ap.add_argument("--config", default="C3")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--merge", type=int, default=20)
    args = ap.parse_args()
    d = np.load(args.npz)
    total, members = d["total"], d["members"]
    g, batches = bench.make_world(args.config, args.batch, args.merge, seed0=1000)
    sv, sc, ss, src = bench.merge_batches([b[1:] for b in batches], args.batch)
    csr = g.csr()
    rp = csr["row_ptr"].astype(np.int64)
    col = csr["col"].astype(np.int64)
    V = len(rp) - 1
    deg = rp[1:] - rp[:-1]
    # 2-hop weight: sum over v's neighbours of (1 + their degree)
    w2 = np.add.reduceat(np.concatenate([1 + deg[col], [0]]), rp[:-1]) if len(col) else np.zeros(V)
    w2[deg == 0] = 0
    # 3-hop weight (with repeats), capped per neighbour
    w3 = np.add.reduceat(np.concatenate([w2[col], [0]]), rp[:-1])
    w3[deg == 0] = 0
    Bm = args.batch * args.merge
    sc = np.asarray(sc, np.int64)
    sv = np.asarray(sv, np.int64)
    ok = sv < V

    def per_col(w):
        out = np.zeros(Bm, np.float64)
        np.add.at(out, sc[ok], w[sv[ok]])
        return out

    preds = {
        "seeds": per_col(np.ones(V)),
        "current: sum(1 + deg)": per_col(1 + deg),
        "sum w2 (2-hop)": per_col(1 + deg + w2),
        "sum w3 (3-hop)": per_col(w3),
        "sum sqrt(w3)": per_col(np.sqrt(w3)),
        "sum log1p(w2)": per_col(np.log1p(w2)),
        "measured members": members.astype(np.float64),
    }
    for name, p in preds.items():
        print(f"{name:>24}: Spearman with duration {spearman(p, total):.3f}")
    # the drain under each order: a list schedule of the measured durations on S slots
    S = 1792
    import heapq
    for name, p in preds.items():
        order = np.argsort(-p, kind="stable")
        h = [0.0] * S
        for c in order:
            t = heapq.heappop(h)
            heapq.heappush(h, t + total[c])
        print(f"{name:>24}: simulated makespan {max(h):.1f} us (mean load {total.sum() / S:.1f})")


if __name__ == "__main__":
    main()
