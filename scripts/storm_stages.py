"""Wall time of the alert-storm tick's host helpers (bench.py --workload storm at its defaults,
one GPU), per tick: wraps the functions behind the seed stage with timers.
Usage: python scripts/storm_stages.py [ticks]"""
import sys
import time
from collections import defaultdict
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.argv = [sys.argv[0], "--workload", "storm", "--steps", sys.argv[1] if len(sys.argv) > 1 else "12",
            "--warmup", "3"]
import bench  # noqa: E402

from egraph import graph, seeds, storm  # noqa: E402

acc = defaultdict(float)
calls = defaultdict(int)


def wrap(owner, name, label):
    f = owner.__dict__[name]
    raw = f.__func__ if isinstance(f, classmethod) else f

    def g(*a, **kw):
        t = time.perf_counter()
        try:
            return raw(*a, **kw)
        finally:
            acc[label] += time.perf_counter() - t
            calls[label] += 1
    if isinstance(f, classmethod):
        setattr(owner, name, classmethod(g))
    else:
        setattr(owner, name, g)


wrap(seeds.SeedCandidates, "per_column", "per_column")
wrap(seeds.SeedCandidates, "combine", "combine")
wrap(seeds.SeedCandidates, "attach_found_idx", "attach_found_idx")
wrap(graph.EvidenceGraph, "lookup_blob", "lookup_blob")
wrap(storm.StormEngine, "_reseed", "_reseed")
wrap(storm.StormEngine, "_append_check", "_append_check")
wrap(storm.StormEngine, "_rebuild_check", "_rebuild_check")
wrap(storm.StormEngine, "_pending_hit", "_pending_hit")
wrap(storm.StormEngine, "tick", "tick")
bench.main()
n = calls["tick"]
for k in sorted(acc, key=acc.get, reverse=True):
    print(f"{k:18s} {acc[k] / n * 1e3:8.3f} ms/tick  ({calls[k]} calls)", file=sys.stderr)
