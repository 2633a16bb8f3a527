"""Per-phase timing of the frontier kernel on the bench workload (diagnostic, GPU box).

Creates the frontier with $EGRAPH_FRONTIER_PROFILE=1 so every column's workgroup stamps
s_memrealtime (100 MHz) at its phase boundaries, runs the bench's C3 batch a few times and
prints the mean / p50 / p99 duration of each phase and the spread of column start times.
Usage: python scripts/frontier_profile.py [--config C3] [--batch 1024]
"""
from __future__ import annotations

import argparse
import json
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C3")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--hops", type=int, default=3)
    ap.add_argument("--out", default="")
    ap.add_argument("--pool", action="store_true", help="keep the member pool (no last-pull pruning)")
    ap.add_argument("--merge", type=int, default=1,
                    help="batches per launch, as bench.py --merge (20 = the headline's launch of "
                         "20 different incident sets)")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = bench.setup(args.config, args.batch, 10, 0, dev, pool_entries=0 if args.pool else -1,
                      merge=args.merge)
    bench.step_frontier(ctx, args.hops)
    torch.cuda.synchronize()
    ctx["frontier"].adapt(ctx["frontier"].stats())   # as bench.py's warm-up (C4: mid-first)
    for _ in range(3 * args.merge):
        bench.step_frontier(ctx, args.hops)
    torch.cuda.synchronize()
    raw = ctx["frontier"].phase_times()
    cont = np.nonzero(raw[:, 39, 0] > 0)[0]     # columns finished in a continuation region
    if len(cont):
        # their first stamp was moved to slot 38 (run_column restamped the phases)
        t0 = np.where(raw[:, 39, 0] > 0, raw[:, 38, 0], raw[:, 0, 0]).astype(np.float64)
        base = t0.min()
        cs, ce = raw[cont, 39, 0].astype(np.float64), raw[cont, 39, 1].astype(np.float64)
        ends = raw[:, :20, 0].max(1).astype(np.float64)
        span = (np.maximum(ends.max(), ce.max()) - base) / 100.0
        st = (t0[cont] - base) / 100.0
        print(f"continued columns: {len(cont)}; start (us after the first column) p50 "
              f"{np.percentile(st, 50):.1f} max {st.max():.1f}; narrow attempt mean "
              f"{((cs - t0[cont]) / 100.0).mean():.1f} us; continuation mean "
              f"{((ce - cs) / 100.0).mean():.1f} max {((ce - cs) / 100.0).max():.1f} us; last "
              f"continuation end {(ce.max() - base) / 100.0:.1f} us of a {span:.1f}-us launch; "
              f"members p50 {np.percentile(raw[cont, 20, 0], 50):.0f} max {raw[cont, 20, 0].max()}")
        raw = raw.copy()
        raw[cont, 0, 0] = raw[cont, 38, 0]
    members = raw[:, 20, 0].astype(np.int64)
    full = raw.astype(np.float64) * 10.0 / 1000.0   # -> us
    full[:, 20, 0] = 0
    t = full[:, :, 0]
    wv = full[:, :, 1:]
    H = args.hops
    names = ["seeds", "seed-grow"]
    for h in range(H):
        names += [f"pull{h}", f"copy+seed{h}"]
    names += ["topk(wave)", "merge+pool", "end"]
    used = int((t[0, :20] > 0).sum())
    d = np.diff(t[:, : used], axis=1)
    rep = {}
    for i in range(used - 1):
        nm = names[i] if i < len(names) else f"slot{i}"
        col = d[:, i]
        rep[nm] = {"mean_us": float(col.mean()), "p50_us": float(np.percentile(col, 50)),
                   "p99_us": float(np.percentile(col, 99)), "max_us": float(col.max())}
        print(f"{nm:>12}: mean {col.mean():8.2f}  p50 {np.percentile(col, 50):8.2f}  "
              f"p99 {np.percentile(col, 99):8.2f}  max {col.max():8.2f} us")
    # per phase: spread of the waves' finish times before the barrier (imbalance) and the
    # barrier's own latency after the last wave
    print("wave finish spread (max - min over waves) / last-wave-to-barrier-exit:")
    for i in range(1, used):
        w = wv[:, i, :]
        if (w > 0).all():
            spread = w.max(1) - w.min(1)
            exitlat = t[:, i] - w.max(1)
            nm = names[i - 1] if i - 1 < len(names) else f"slot{i}"
            print(f"{nm:>12}: spread mean {spread.mean():7.2f} p99 {np.percentile(spread, 99):7.2f}"
                  f"  barrier-exit mean {exitlat.mean():6.2f} us")
    sub = wv[:, 24:36, :]
    if (sub > 0).any():
        print("last pull, per-wave sums (us): member+row_ptr / light rows (rest) / hub rows (rest)"
              " / store / light loads / light probes / light chain / light inserts / hub loads / "
              "hub probes / hub chain / hub inserts:",
              " / ".join(f"{sub[:, k, :].mean():.2f}" for k in range(12)))
    tk = wv[:, 36:38, :]
    if (tk > 0).any():
        print("top-k, per wave (us): candidate keys (LDS) %.2f / k wave-max rounds %.2f"
              % (tk[:, 0, :].mean(), tk[:, 1, :].mean()))
    q = np.percentile(members, [50, 90, 99, 99.9, 100])
    print("members per column: mean %.0f p50 %d p90 %d p99 %d p99.9 %d max %d; > 768: %.1f %%, "
          "> 1024: %.1f %%" % (members.mean(), *q, 100 * (members > 768).mean(),
                               100 * (members > 1024).mean()))
    total = t[:, used - 1] - t[:, 0]
    start = t[:, 0] - t[:, 0].min()
    end = t[:, used - 1] - t[:, 0].min()
    print(f"column total: mean {total.mean():.1f} p50 {np.percentile(total, 50):.1f} "
          f"max {total.max():.1f} us; starts span {start.max():.1f} us; last end {end.max():.1f} us")
    # the grid's drain: column slots busy over time (a slot = one resident workgroup; the
    # narrow geometry holds 7 per CU), and how well the launch order predicted the durations
    slots = 7 * torch.cuda.get_device_properties(dev).multi_processor_count
    mk = end.max()
    busy = total.sum() / (slots * mk)
    last_start = start.max()
    order = ctx["lanes"][0]["order"] if ctx["lanes"][0].get("order") is not None else None
    pos = np.empty(len(start), np.int64)
    pos[np.argsort(start, kind="stable")] = np.arange(len(start))
    q10 = np.percentile(end, [90, 99])
    tail_cols = total[start >= np.percentile(start, 95)]
    rk = np.corrcoef(pos, np.argsort(np.argsort(-total)))[0, 1]
    print(f"drain: slot occupancy {busy:.3f} over a {mk:.1f}-us makespan ({slots} slots); the "
          f"last column starts at {last_start:.1f} us ({mk - last_start:.1f} us before the end); "
          f"90 / 99 % of columns ended by {q10[0]:.1f} / {q10[1]:.1f} us; the last 5 % of starts "
          f"last {tail_cols.mean():.1f} us (all {total.mean():.1f}); rank correlation of start "
          f"order with duration order {rk:.3f}")
    hist = np.histogram(end, bins=20, range=(0, mk))[0]
    running = [int(((start <= x) & (end > x)).sum()) for x in np.linspace(0, mk, 41)[1:-1]]
    print("columns running at 2.5 % steps of the makespan:", running)
    rep["drain"] = {"slot_occupancy": float(busy), "makespan_us": float(mk),
                    "last_start_us": float(last_start), "running": running,
                    "ends_hist": hist.tolist(), "order_rank_corr": float(rk)}
    del order
    if args.out:
        # per column (index = column id): start / duration (us) and members, for offline
        # predictor studies (scripts/launch_order_study.py)
        np.savez(Path(args.out).with_suffix(".npz"), start=start, total=total, members=members)
    rep["column_total"] = {"mean_us": float(total.mean()), "max_us": float(total.max())}
    rep["start_span_us"] = float(start.max())
    rep["makespan_us"] = float(end.max())
    rep["work"] = ctx["frontier"].stats()
    print(json.dumps(rep["work"]))
    if args.out:
        Path(args.out).write_text(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
