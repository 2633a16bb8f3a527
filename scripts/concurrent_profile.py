"""Host-side profile of the drop-in's concurrent single calls (CPU only, no GPU).

Every incident of a C3-sized batch is its own RulesEngine.generate_hypotheses +
HypothesisRanker.rank call, all in flight at once (the Temporal activities' pattern); the
batcher coalesces them into launches.  Here the launch itself is replaced by the C oracle's
orc_rules_eval on the same encoded columns (a test stand-in: only the host path is measured),
so the host overheads -- per-call bookkeeping, the coalesced encode, dict assembly and the
ranker's fused reuse -- can be profiled and tuned without a GPU.
  python scripts/concurrent_profile.py [n_incidents] [--cprofile] [--gpu]"""
import asyncio
import cProfile
import gc
import pstats
import sys
import time
from pathlib import Path
from types import SimpleNamespace

REPO = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "kubernetes-aiops-evidence-graph_amd"), str(REPO / "oracle"),
                str(REPO / "tests")]
import numpy as np  # noqa: E402

import oracle  # noqa: E402
from egraph import batcher as B  # noqa: E402
from egraph.rca import RulesResult  # noqa: E402


class CpuRunner:
    """RulesRunner's interface with the kernel replaced by orc_rules_eval (stand-in)."""
    SMALL_ROWS = 128
    ZERO_COPY_ROWS = 16384

    def __init__(self, cat, device=None):
        self.cat = cat
        self.res = None

    def input_views(self, rows, n):
        return (np.empty(rows, np.uint32), np.empty(rows, np.uint32), np.empty(rows, np.uint32),
                np.empty(rows, np.float64), np.empty(n + 1, np.int64))

    async def run(self, enc):
        o = oracle.rules_eval(self.cat.table, enc.flags, enc.vocab, enc.node, enc.err, enc.seg_off)
        await asyncio.sleep(0)
        return RulesResult(o["mask"], o["n_hyp"], o["order_conf"], o["order_rank"], o["confidence"],
                           o["final_score"], o["strength"])


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 1024
    if "--gpu" not in sys.argv:                      # (--gpu: the real launches, on a GPU box)
        B.RulesRunner = CpuRunner
        import egraph.ranker as R
        R.require_device = lambda device=None: None  # every list is served by the fused ranks
    from egraph import synth
    from src.services.rca import rules_engine as RE
    from src.services.rca.hypothesis_ranker import HypothesisRanker
    # --heap: also build the C3 evidence graph, as bench.py's process holds it (229k vertices,
    # their id tuples and property dicts: a much larger set of GC-tracked objects)
    keep = None
    if "--heap" in sys.argv:
        keep = synth.build_graph(synth.build_cluster(synth.CONFIGS["C3"]))
    cl = synth.build_cluster(synth.CONFIGS["C3"])
    cases = synth.make_incidents(cl, n, seed=1000)
    ev = [x.evidence for x in cases]
    incs = [SimpleNamespace(id=f"inc-{i}") for i in range(n)]
    eng = RE.RulesEngine()
    ranker = HypothesisRanker()

    async def one(i):
        return ranker.rank(await eng.generate_hypotheses(incs[i], ev[i]))

    async def rounds(k):
        b = RE._batcher(eng.catalog, eng.device)
        ts = []
        for _ in range(k):
            gc.collect()
            t0 = time.perf_counter()
            await asyncio.gather(*[one(i) for i in range(n)])
            ts.append(time.perf_counter() - t0)
        return ts, b.launches

    asyncio.run(rounds(1))
    if "--cprofile" in sys.argv:
        pr = cProfile.Profile()
        pr.enable()
        ts, launches = asyncio.run(rounds(3))
        pr.disable()
        pstats.Stats(pr).sort_stats(sys.argv[-1] if sys.argv[-1] in ("tottime", "cumulative") else "cumulative").print_stats(30)
    else:
        ts, launches = asyncio.run(rounds(5))
    print(f"{n} concurrent calls: best {min(ts) * 1e3:.2f} ms -> {n / min(ts):,.0f} incidents/s "
          f"({launches} launches in the timed rounds' loop)")


if __name__ == "__main__":
    main()
