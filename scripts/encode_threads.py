"""Native evidence encoder on the C3 bench batch (1024 incidents, ~91k rows) at several worker
thread counts: best / median ms of 7 runs each; every result checked against the 1-thread one.
Usage: python scripts/encode_threads.py [threads ...]"""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "kubernetes-aiops-evidence-graph_amd"))
from egraph import catalog, synth  # noqa: E402
from egraph.encode import encode_batch, encode_threads  # noqa: E402

cl = synth.build_cluster(synth.CONFIGS["C3"])
ev = [c.evidence for c in synth.make_incidents(cl, 1024, seed=1000)]
cat = catalog.default()
ref = encode_batch(ev, cat, threads=1)
print(f"rows {ref.n_rows}, default threads {encode_threads()}")
for th in [int(a) for a in sys.argv[1:]] or [1, 2, 4, 8, 16]:
    ts = []
    for _ in range(7):
        t0 = time.perf_counter()
        e = encode_batch(ev, cat, threads=th)
        ts.append(time.perf_counter() - t0)
    same = all(np.array_equal(getattr(e, k).view(np.uint8), getattr(ref, k).view(np.uint8))
               for k in ("flags", "vocab", "node", "err", "seg_off")) and e.evidence_ids == ref.evidence_ids
    print(f"{th:3d} threads: best {min(ts) * 1e3:7.2f} ms  median {np.median(ts) * 1e3:7.2f} ms  same={same}",
          flush=True)
