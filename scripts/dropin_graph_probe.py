"""Where the drop-in graph half's time goes between its stages and the activity call (GPU box):
rank_root_causes_sync called directly, through asyncio.to_thread in one event loop, and
activities.rank_root_causes_batch, each the best of 7 calls after warm-up."""
import asyncio
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402
import torch  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    ctx = bench.setup("C3", 1024, 10, 0, dev, 1, pool_entries=-1, merge=1)
    bench.step_frontier(ctx, 3)
    torch.cuda.synchronize(dev)
    from src.database import GraphService
    from src.services.workflow import activities
    GraphService.reset()
    GraphService._graph, GraphService._snapshot, GraphService.device = ctx["graph"], ctx["snap"], dev
    ids = list(ctx["incident_ids"])
    ev = ctx["evidence"]
    data = [{"incident": {"id": i}, "evidence": {"evidence": e}, "k": 10} for i, e in zip(ids, ev)]

    def best(f, n=7):
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            f()
            ts.append(time.perf_counter() - t0)
        return min(ts) * 1e3, sorted(ts)[len(ts) // 2] * 1e3

    GraphService.rank_root_causes_sync(ids, ev, 3, 10)
    print("direct sync: best %.2f ms, median %.2f ms" % best(lambda: GraphService.rank_root_causes_sync(ids, ev, 3, 10)))

    async def run_all():
        loop = asyncio.get_running_loop()
        await asyncio.to_thread(GraphService.rank_root_causes_sync, ids, ev, 3, 10)
        ts = []
        for _ in range(7):
            t0 = time.perf_counter()
            await asyncio.to_thread(GraphService.rank_root_causes_sync, ids, ev, 3, 10)
            ts.append(time.perf_counter() - t0)
        print("to_thread: best %.2f ms, median %.2f ms" % (min(ts) * 1e3, sorted(ts)[3] * 1e3))
        ts = []
        for _ in range(7):
            t0 = time.perf_counter()
            await activities.rank_root_causes_batch(data)
            ts.append(time.perf_counter() - t0)
        print("activity: best %.2f ms, median %.2f ms" % (min(ts) * 1e3, sorted(ts)[3] * 1e3))
        stages: dict = {}
        t0 = time.perf_counter()
        GraphService.rank_root_causes_sync(ids, ev, 3, 10, stages=stages)
        print("staged call %.2f ms:" % ((time.perf_counter() - t0) * 1e3),
              {k: round(v * 1e3, 3) for k, v in stages.items()})
    asyncio.run(run_all())


if __name__ == "__main__":
    main()
