"""cProfile of the alert-storm tick (bench.py --workload storm at its defaults, one GPU): the
host functions behind the per-stage times.  Usage: python scripts/storm_profile.py [ticks]"""
import cProfile
import io
import pstats
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.argv = [sys.argv[0], "--workload", "storm", "--steps", sys.argv[1] if len(sys.argv) > 1 else "12",
            "--warmup", "3"]
import bench  # noqa: E402

from egraph import storm  # noqa: E402

prof = cProfile.Profile()
real_tick = storm.StormEngine.tick


def tick(self, *a, **kw):
    prof.enable()
    try:
        return real_tick(self, *a, **kw)
    finally:
        prof.disable()


storm.StormEngine.tick = tick
bench.main()
s = io.StringIO()
pstats.Stats(prof, stream=s).sort_stats("cumulative").print_stats(35)
print(s.getvalue(), file=sys.stderr)
