"""Calibrate the CPU baseline's stand-in for the reference's Python rules path (this container
only: it imports /root/reference, which never travels to the GPU box).

bench.py's `cpu_baseline.python_rules_path` times oracle/rca_oracle.py -- the pure-Python
restatement of RulesEngine.generate_hypotheses + HypothesisRanker.rank (rules_engine.py:199-478,
hypothesis_ranker.py:13-80), pinned bit for bit to the reference's outputs by
tests/test_oracle_golden.py -- because the reference cannot run on the GPU box.  This script
times the REAL reference path beside the restatement on the same incidents, in this container,
and records how much slower the reference is (ratio > 1: the stand-in is conservative, and the
GPU's speed-up over the reference is that much larger than the bench line states).

Reference modules are loaded by path with the shims of oracle/gen_golden.py (a no-op structlog
stub -- the reference logs one `info` line per matched rule, which real structlog would format
and write; the stub makes the reference faster, so the ratio is a lower bound -- and
datetime.UTC on Python 3.10); no bytecode is written.  Both paths run the per-incident pattern of
the reference's activity (activities.py:124-170): `ranker.rank(await engine.generate_hypotheses(
incident, evidence))`, one event loop, one core.  ONE statistic: per interleaved pair of rounds
(reference round, then stand-in round: adjacent in time, so host-speed drift cancels) the ratio
of their times; the median of the REPS pair ratios, with its distribution-free 95 % confidence
interval (order statistics of the binomial(REPS, 1/2) -- no normality assumed).

Workloads: C1 (the reference simulator's CrashLoop scenario rendered as ~100 collector rows,
egraph.synth.c1_world), C3-shaped incidents (the bench's generator, 200 incidents of ~89 rows)
and the reference-recorded golden rule cases (tests/golden/rules_cases.json, ~12 rows each).
Writes profiles/r06_standin_calibration.json (bench.py reads its C3 ratio and interval for
cpu_baseline.speedup_vs_reference).

Usage: python oracle/calibrate_standin.py [--ref /root/reference] [--reps 61]
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import platform
import sys
import time
from pathlib import Path
from types import SimpleNamespace

sys.dont_write_bytecode = True
REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "oracle"))
sys.path.insert(0, str(REPO / "kubernetes-aiops-evidence-graph_amd"))

import gen_golden  # noqa: E402  (its shims and by-path loader)
import rca_oracle  # noqa: E402


def workloads() -> dict[str, list[list[dict]]]:
    from egraph import synth
    _, c1 = synth.c1_world()
    cl = synth.build_cluster(synth.CONFIGS["C3"])
    c3 = synth.make_incidents(cl, 200, seed=1000)
    gold = json.loads((REPO / "tests" / "golden" / "rules_cases.json").read_text())
    cases = gold["cases"] if isinstance(gold, dict) and "cases" in gold else gold
    return {"C1": [c1.evidence] * 50,
            "C3": [x.evidence for x in c3],
            "golden": [c["evidence"] for c in cases]}


def time_paths(engine, ranker, evs: list[list[dict]], reps: int) -> dict:
    incs = [SimpleNamespace(id=f"inc-{i}") for i in range(len(evs))]

    async def ref_round():
        t0 = time.perf_counter()
        for inc, ev in zip(incs, evs):
            ranker.rank(await engine.generate_hypotheses(inc, ev))
        return time.perf_counter() - t0

    async def standin_round():
        t0 = time.perf_counter()
        for inc, ev in zip(incs, evs):
            rca_oracle.rca(inc.id, ev)
        return time.perf_counter() - t0

    async def go():
        ref, sta = [], []
        await ref_round()
        await standin_round()
        for _ in range(reps):                      # interleaved rounds
            ref.append(await ref_round())
            sta.append(await standin_round())
        return ref, sta
    ref, sta = asyncio.run(go())
    n = len(evs)
    pair = sorted(r / s for r, s in zip(ref, sta))
    lo, hi = median_ci(len(pair))
    med = (pair[(len(pair) - 1) // 2] + pair[len(pair) // 2]) / 2
    return {"incidents": n, "rows_per_incident": sum(map(len, evs)) / n, "pairs": len(pair),
            "reference_over_standin_time": med,
            "reference_over_standin_time_ci95": [pair[lo], pair[hi]],
            "pair_ratio_min_max": [pair[0], pair[-1]],
            "reference_per_s_median": n / sorted(ref)[len(ref) // 2],
            "standin_per_s_median": n / sorted(sta)[len(sta) // 2]}


def median_ci(n: int, conf: float = 0.95) -> tuple[int, int]:
    """0-based order-statistic indices (lo, hi) of a distribution-free `conf` interval for the
    median of n samples: the largest symmetric k with P(k <= Binomial(n, 1/2) <= n - 1 - k)
    >= conf, i.e. the interval [x_(k), x_(n-1-k)]."""
    from math import comb
    pmf = [comb(n, i) / 2 ** n for i in range(n + 1)]
    best = 0
    for k in range(n // 2):
        if sum(pmf[k + 1:n - k]) >= conf:     # P(k < X <= n - 1 - k): x_(k) <= median <= x_(n-1-k)
            best = k
        else:
            break
    return best, n - 1 - best


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--reps", type=int, default=61)
    args = ap.parse_args()
    ref = Path(args.ref)
    gen_golden._install_shims()
    re_mod = gen_golden._load(ref / "src/services/rca/rules_engine.py", "ref_rules_engine")
    rk_mod = gen_golden._load(ref / "src/services/rca/hypothesis_ranker.py", "ref_hypothesis_ranker")
    engine, ranker = re_mod.RulesEngine(), rk_mod.HypothesisRanker()
    out = {"what": "the reference's Python rules path (RulesEngine.generate_hypotheses + "
                   "HypothesisRanker.rank, loaded from /root/reference) against its restatement "
                   "oracle/rca_oracle.py, the stand-in bench.py times as cpu_baseline."
                   "python_rules_path on the GPU box; one core; statistic: the median over "
                   "interleaved pairs of rounds of (reference round time / stand-in round time), "
                   "with its distribution-free 95 % interval",
           "script": "oracle/calibrate_standin.py", "host": platform.processor() or platform.machine(),
           "cpus": os.cpu_count(), "python": platform.python_version(), "reps": args.reps,
           "workloads": {}}
    for name, evs in workloads().items():
        r = time_paths(engine, ranker, evs, args.reps)
        out["workloads"][name] = r
        ci = r["reference_over_standin_time_ci95"]
        print(f"{name}: {r['incidents']} incidents x {r['rows_per_incident']:.1f} rows, {r['pairs']} "
              f"pairs: the reference takes {r['reference_over_standin_time']:.3f}x the stand-in's "
              f"time (95 % CI {ci[0]:.3f} .. {ci[1]:.3f})", flush=True)
    c3 = out["workloads"]["C3"]
    out["bench_workload_ratio"] = c3["reference_over_standin_time"]
    out["bench_workload_ratio_ci95"] = c3["reference_over_standin_time_ci95"]
    out["note"] = ("bench.py's python_rules_path runs C3-shaped incidents: the reference path "
                   f"takes {c3['reference_over_standin_time']:.3f}x the stand-in's time there, so "
                   "the reference's own rate on the GPU box is the bench's python_rules_path value "
                   "/ that ratio (cpu_baseline.speedup_vs_reference)")
    path = REPO / "profiles" / "r06_standin_calibration.json"
    path.write_text(json.dumps(out, indent=1))
    print(f"wrote {path}")


if __name__ == "__main__":
    main()
