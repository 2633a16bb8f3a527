"""Host microbenchmark (no GPU): the alert storm's candidate extraction (pyhost.seed_keys) over
real storm evidence rows at 1..16 worker threads, and the cost of dropping the rows afterwards.
Run on the GPU box's CPU share to see how the native pool scales there."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "kubernetes-aiops-evidence-graph_amd"))
import numpy as np  # noqa: E402
from egraph import _lib, synth  # noqa: E402
from egraph.seeds import _row  # noqa: E402

c = synth.build_cluster(synth.CONFIGS["C3"])
wl = synth.StormWorkload(c, n_keys=10000, seed=9, events_per_incident=8)
cases = []
for t in range(12):
    wl.alerts(1666)
    cases += [wl.make_case(len(cases), i) for i in range(0, 1666, 9)]
ev = [x.evidence for x in cases]
rows = sum(len(e) for e in ev)
print(f"{len(ev)} incidents, {rows} rows; cpus {len(os.sched_getaffinity(0))}")
for th in (1, 2, 4, 8, 16):
    best = 1e9
    for _ in range(3):
        t0 = time.perf_counter()
        _lib.pyhost.seed_keys(ev, _row, th)
        best = min(best, time.perf_counter() - t0)
    print(f"seed_keys threads {th:2d}: {best * 1e3:7.2f} ms  {best / rows * 1e9:6.1f} ns/row")
part = ev[:177]
t0 = time.perf_counter()
_lib.pyhost.seed_keys(part, _row, 16)
t1 = time.perf_counter()
print(f"one tick's 177 incidents ({sum(len(e) for e in part)} rows): {1e3 * (t1 - t0):.2f} ms")
t0 = time.perf_counter()
del part, ev
for x in cases:
    x.evidence = None
print(f"dropping all rows: {(time.perf_counter() - t0) * 1e9 / rows:.1f} ns/row")
