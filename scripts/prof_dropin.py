"""Host profile of the drop-in paths on a GPU box (cProfile; not a benchmark): the concurrent
pattern (every incident its own generate_hypotheses + rank call, the batcher coalescing them)
and rank_root_causes_batch with its stage split.  Prints the top functions by own time."""
import asyncio
import cProfile
import gc
import io
import pstats
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402
import torch  # noqa: E402


def top(pr, n=28):
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(n)
    print("\n".join(s.getvalue().splitlines()[:n + 12]))


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = bench.setup("C3", 1024, 10, 0, dev, 1, pool_entries=-1, merge=1)
    for _ in range(3):
        bench.step_frontier(ctx, 3)
    torch.cuda.synchronize(dev)
    from types import SimpleNamespace
    from src.services.rca import rules_engine as RE
    from src.services.rca.hypothesis_ranker import HypothesisRanker
    ev = ctx["evidence"]
    incs = [SimpleNamespace(id=f"inc-{i}") for i in range(len(ev))]
    eng = RE.RulesEngine(device=dev)
    ranker = HypothesisRanker()

    async def one(i):
        return ranker.rank(await eng.generate_hypotheses(incs[i], ev[i]))

    async def conc(rounds, pr=None):
        ts = []
        for _ in range(rounds):
            gc.collect()
            if pr:
                pr.enable()
            t0 = time.perf_counter()
            await asyncio.gather(*[one(i) for i in range(len(ev))])
            ts.append(time.perf_counter() - t0)
            if pr:
                pr.disable()
        return ts

    async def run():
        await conc(2)
        ts = await conc(5)
        print("concurrent ms (unprofiled):", [round(t * 1e3, 2) for t in ts])
        pr = cProfile.Profile()
        await conc(3, pr)
        top(pr)
        # the pieces alone: generate_hypotheses only; rank only
        hy = await asyncio.gather(*[eng.generate_hypotheses(incs[i], ev[i]) for i in range(len(ev))])
        t0 = time.perf_counter()
        await asyncio.gather(*[eng.generate_hypotheses(incs[i], ev[i]) for i in range(len(ev))])
        t1 = time.perf_counter()
        for h in hy:
            ranker.rank(h)
        t2 = time.perf_counter()
        print(f"generate_hypotheses x{len(ev)} concurrent: {1e3 * (t1 - t0):.2f} ms; "
              f"rank x{len(ev)} serial: {1e3 * (t2 - t1):.2f} ms")
    asyncio.run(run())
    r = bench.dropin_graph(ctx, dev, 3, 10)
    print("dropin_graph", round(r["value"]), "incidents/s", round(r["ms_per_batch"], 2), "ms;",
          {k: round(v, 3) for k, v in r["stages_ms"].items()})
    from src.database import GraphService
    from src.services.workflow import activities
    GraphService.reset()
    GraphService._graph, GraphService._snapshot, GraphService.device = ctx["graph"], ctx["snap"], dev
    data = [{"incident": {"id": i}, "evidence": {"evidence": e}, "k": 10}
            for i, e in zip(ctx["incident_ids"], ev)]
    pr = cProfile.Profile()

    async def g(n):
        for _ in range(n):
            await activities.rank_root_causes_batch(data)
    asyncio.run(g(2))
    pr.enable()
    asyncio.run(g(5))
    pr.disable()
    top(pr)


if __name__ == "__main__":
    main()
