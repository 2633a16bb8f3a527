"""bench.py's multi-rank contract on CPU (gloo, world size 2): the timed region
(bench.timed_steps: barrier + sync, exactly K steps, sync + barrier, MAX over ranks) with the
incident-sharded step -- every rank ranks its own batch of incidents (bench.setup's
seed 1000 + rank) on its replicated graph; here a CPU engine (the C oracle's frontier) stands in
for the GPU frontier.  Checks: every rank gets the same, maximal elapsed time (the slow rank's),
the ranks' batches are different incidents, and each rank's top-k equals the oracle's dense
recurrence on its own batch."""
from __future__ import annotations

import os
import socket

import numpy as np


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), EGRAPH_BENCH_BACKEND="gloo")
    import time

    import torch
    import torch.distributed as dist

    import bench
    import oracle
    from egraph import synth
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        B, k = 16, 5
        cl = synth.build_cluster(synth.ClusterConfig(pods=600, namespaces=3, nodes=12,
                                                     deployments=60, services=40, seed=7))
        cases = synth.make_incidents(cl, B, seed=1000 + rank)     # bench.setup's per-rank batch
        synth.add_incidents(cl, cases)
        g = synth.build_graph(cl)
        sv, sc, ss = synth.seeds_for_batch(g, [x.evidence for x in cases])
        src = g.lookup([f"incident:{x.incident['id']}" for x in cases]).astype(np.uint32)
        csr = g.csr()
        vl, _, _, _ = g.export()
        inc = g.labels().index("Incident")
        out = {}

        def step():                         # the CPU stand-in for one frontier pass
            out["r"] = oracle.frontier(csr["row_ptr"], csr["col"], csr["val"], vl, sv, sc, ss,
                                       src, 3, inc, k)
            if rank == 1:
                time.sleep(0.05)            # the slow rank sets the time
        steps = 3
        elapsed = bench.timed_steps(step, steps, dist, rank, lambda: None, torch.device("cpu"))
        exp = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, B, 3)
        er = oracle.reach(csr["row_ptr"], csr["col"], src, 3)
        e_ids, e_sc = oracle.topk(exp, er, vl, inc, k)
        ids, scores, _ = out["r"]
        q.put((rank, elapsed, [x.incident["id"] for x in cases], bool((ids == e_ids).all()),
               scores.tobytes() == e_sc.tobytes(), world * B / (elapsed / steps)))
    finally:
        dist.destroy_process_group()


def test_incident_sharded_timed_region_gloo_world_size_2():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, e0, ids0, ok0, sc0, v0), (r1, e1, ids1, ok1, sc1, v1) = res
    assert e0 == e1 and e0 >= 3 * 0.05                 # MAX over ranks, every rank has it
    assert v0 == v1 and v0 > 0                          # value = all ranks' incidents / time
    assert not set(ids0) & set(ids1)                    # each rank its own incidents
    assert ok0 and ok1 and sc0 and sc1                  # each rank's top-k = the oracle's


def test_gpus_flag_must_match_world_size(monkeypatch):
    """`--gpus N` under a launcher with another world size is refused before any GPU call."""
    import sys

    import pytest

    import bench
    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert "WORLD_SIZE=1" in str(e.value.code)


def test_gpus_flag_launches_ranks(monkeypatch):
    """`bench.py --gpus N` with no launcher starts N ranks under torch.distributed.run (child
    process, 127.0.0.1 rendezvous) and exits with its status."""
    import subprocess
    import sys

    import pytest

    import bench
    calls = []
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "7"])
    monkeypatch.setattr(subprocess, "call", lambda cmd: calls.append(cmd) or 3)
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 3
    (cmd,) = calls
    assert cmd[1:4] == ["-m", "torch.distributed.run", "--nnodes=1"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "7"] and cmd[-5].endswith("bench.py")


def test_merge_batches_offsets_columns_and_launch_groups():
    """--merge M: batch i's seed columns move to i*B.., sources concatenate in batch order; the
    step functions enqueue on the first call of every group of M and on no other."""
    import bench
    b0 = (np.array([5, 6], np.uint32), np.array([0, 1], np.uint32), np.array([1.0, 2.0], np.float32),
          np.array([10, 11], np.uint32))
    b1 = (np.array([7], np.uint32), np.array([1], np.uint32), np.array([3.0], np.float32),
          np.array([12, 13], np.uint32))
    sv, sc, ss, src = bench.merge_batches([b0, b1], 2)
    assert sv.tolist() == [5, 6, 7] and sc.tolist() == [0, 1, 3] and sc.dtype == np.uint32
    assert ss.tolist() == [1.0, 2.0, 3.0] and src.tolist() == [10, 11, 12, 13]
    ctx = {"merge": 3, "sub": 0}
    assert [bench._launch_due(ctx) for _ in range(7)] == [True, False, False, True, False, False, True]
    assert all(bench._launch_due({"merge": 1, "sub": 0}) for _ in range(3))
