"""The native rules encoder's time by worker count (host only; diagnostic): encode_batch over the
bench's C3 batch (1024 incidents, ~91k evidence rows), best of 9 per thread count.
  python scripts/encode_scaling.py"""
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "kubernetes-aiops-evidence-graph_amd"))
from egraph import catalog, synth  # noqa: E402
from egraph.encode import encode_batch  # noqa: E402

cl = synth.build_cluster(synth.CONFIGS["C3"])
ev = [x.evidence for x in synth.make_incidents(cl, 1024, seed=1000)]
cat = catalog.default()
print("rows", sum(len(e) for e in ev))
for thr in (1, 2, 4, 8, 16):
    ts = []
    for _ in range(9):
        t = time.perf_counter()
        encode_batch(ev, cat, threads=thr)
        ts.append(time.perf_counter() - t)
    print(f"{thr:2d} threads: best {min(ts) * 1e3:.3f} ms, median {sorted(ts)[4] * 1e3:.3f} ms")
