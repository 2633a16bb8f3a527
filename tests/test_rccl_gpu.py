"""The RCCL code paths (backend "nccl" = RCCL on ROCm) on the one GPU of a test box: a process
group of world size 1 over RCCL runs every collective the multi-GPU paths use -- TorchComm's
device-side all_gather_into_tensor and all_to_all_single (egraph/shard.py), the partitioned
plan's halo exchange and top-k merge, ShardedDedup's routing and decision gather
(egraph/alerts.py) and the storm engine with a comm -- and each must equal the no-collective
path bit for bit.  (RCCL refuses two ranks on one device, so the 2-rank protocols are covered by
the gloo tests: tests/test_shard.py, tests/test_storm_dist.py, tests/test_storm_gpu.py.)  Runs
in a child process so the RCCL communicator never lives in the pytest process."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _main(port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    out = {}
    try:
        from egraph import shard, synth
        from egraph.alerts import DedupTable, ShardedDedup, fingerprints
        from egraph.graph import EvidenceGraph, Snapshot
        from egraph.storm import StormEngine
        comm = shard.TorchComm()
        out["backend"] = dist.get_backend()
        out["gloo"] = comm.gloo
        # collectives on device tensors
        x = torch.arange(7, dtype=torch.int64, device=dev)
        (g,) = comm.all_gather([x])
        out["all_gather"] = g.cpu().tolist() == list(range(7))
        ((r, rc),) = comm.all_to_all_v([(x * 3, [7])])
        out["all_to_all_v"] = r.cpu().tolist() == [3 * i for i in range(7)] and rc == [7]
        # the partitioned plan at P = 1 over RCCL equals the plain plan
        cfg = synth.ClusterConfig(pods=1500, namespaces=6, nodes=30, deployments=150,
                                  services=100, attach_fraction=0.3, seed=5)
        c = synth.build_cluster(cfg)
        cases = synth.make_incidents(c, 48, seed=6)
        synth.add_incidents(c, cases)
        gr = EvidenceGraph()
        gr.merge_nodes(c.ids, c.labels)
        gr.merge_edges(c.src, c.dst, c.types)
        sv, sc, ss = synth.seeds_for_batch(gr, [k.evidence for k in cases])
        src = gr.lookup([f"incident:{k.incident['id']}" for k in cases]).astype(np.uint32)
        csr = gr.csr()
        vl, _, _, _ = gr.export()
        V, B, kk = gr.num_vertices, len(cases), 8
        inc = gr.labels().index("Incident")
        owner = shard.partition_vertices(csr["row_ptr"], vl, gr.labels(), 1)
        lg = shard.build_local(csr, vl, owner, 0, 1)
        snap = Snapshot.from_csr(lg.row_ptr, lg.col, lg.meta, lg.val, lg.vlabel, gr.labels(), dev)

        def t(a):
            return torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        lv, lc, ls = shard.local_seeds(lg, V, sv, sc, ss)
        plan = snap.plan(B, max_seeds=max(len(lv), 1), k=kk)
        plan.set_seeds(t(lv), t(lc), t(ls))
        plan.set_sources(t(shard.local_sources(lg, V, src)))
        run = shard.RankRun(lg, plan, dev)
        ((ids, sco),) = shard.run_partitioned([run], comm, 3, inc, kk)
        ref = gr.snapshot(device=dev).plan(B, max_seeds=max(len(sv), 1), k=kk)
        ref.set_seeds(t(sv), t(sc), t(ss))
        ref.set_sources(t(src))
        e_ids, e_sc = ref.run(3, inc)
        got = ids.cpu().numpy()
        want = e_ids.cpu().numpy().view(np.uint32).astype(np.int64).reshape(got.shape)
        out["partitioned"] = bool((got == want).all()) and \
            sco.cpu().numpy().tobytes() == e_sc.cpu().numpy().reshape(sco.shape).tobytes()
        # ShardedDedup over RCCL equals the plain table, decision for decision
        keys = [f"alertmanager:A{i % 37}:ns:svc{i % 11}" for i in range(400)]
        fp, _ = fingerprints(keys, dev)
        plain = DedupTable(4096, dev)
        d0, i0, n0 = plain.ingest(fp, 1_000_000, 60_000)
        sd = ShardedDedup(DedupTable(4096, dev), comm, 0)
        d1, i1, n1 = sd.ingest(fp, torch.arange(len(keys), dtype=torch.int64), 1_000_000, 60_000)
        out["dedup"] = (np.asarray(d1).tolist() == d0.cpu().numpy().tolist()
                        and np.asarray(i1).tolist() == i0.cpu().numpy().tolist() and n1 == n0)
        # the storm engine with an RCCL comm equals the engine without one
        wl_a = synth.StormWorkload(c, n_keys=300, seed=9, events_per_incident=8)
        wl_b = synth.StormWorkload(c, n_keys=300, seed=9, events_per_incident=8)
        g_a = synth.build_graph(c)
        g_b = synth.build_graph(c)
        e_a = StormEngine(g_a, device=dev, hops=3, k=8, dedup_capacity=4096)
        e_b = StormEngine(g_b, device=dev, hops=3, k=8, dedup_capacity=4096, comm=comm, rank=0)
        now, same = 1_000_000, True
        for tick in range(4):
            now += 1000
            ka, kb = wl_a.alerts(40), wl_b.alerts(40)
            sa = e_a.tick(ka, now, wl_a.make_case, topology=wl_a.topology(3))
            sb = e_b.tick(kb, now, wl_b.make_case, topology=wl_b.topology(3),
                          seq=np.arange(len(kb)))
            same &= (sa["new_incidents"], sa["duplicates"]) == (sb["new_incidents"], sb["duplicates"])
        for xa, xb in zip(e_a.incidents, e_b.incidents):
            same &= bool(np.array_equal(xa.top_ids, xb.top_ids)) and \
                xa.top_scores.tobytes() == xb.top_scores.tobytes()
        out["storm"] = same and len(e_a.incidents) == len(e_b.incidents) > 0
    finally:
        dist.destroy_process_group()
    q.put(out)


def test_rccl_world_size_one_paths_equal_local():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_main, args=(_port(), q))
    p.start()
    out = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert out.pop("backend") == "nccl" and out.pop("gloo") is False
    assert all(out.values()), out
