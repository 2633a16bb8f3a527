"""The partitioned-graph path on the GPU with the HIP plan (egraph/shard.py): P partitions of
one graph, each its own local snapshot + plan on cuda:0, halo exchanges through the pack /
unpack kernels (LocalComm concatenates the ranks' buffers where RCCL all-gathers them).  Owned
scores are bit-identical to the unpartitioned oracle recurrence, and the merged top-k and the
reach sets equal the unpartitioned ones.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu


def _graph(B, seed, pods):
    from egraph import synth
    from egraph.graph import EvidenceGraph
    cfg = synth.ClusterConfig(pods=pods, namespaces=8, nodes=40, deployments=pods // 10,
                              services=pods // 15, attach_fraction=0.3, seed=seed)
    c = synth.build_cluster(cfg)
    cases = synth.make_incidents(c, B, seed=seed + 1)
    synth.add_incidents(c, cases)
    g = EvidenceGraph()
    g.merge_nodes(c.ids, c.labels)
    g.merge_edges(c.src, c.dst, c.types)
    sv, sc, ss = synth.seeds_for_batch(g, [x.evidence for x in cases])
    src = g.lookup([f"incident:{x.incident['id']}" for x in cases]).astype(np.uint32)
    return g, sv, sc, ss, src


def _dev(a):
    from egraph.device import to_device
    return to_device(np.ascontiguousarray(a), torch.device("cuda", 0))


@pytest.mark.parametrize("P,B,sparse,overlap", [(2, 40, True, None), (3, 130, True, None),
                                                (4, 70, True, None), (2, 40, False, None),
                                                (4, 70, False, None), (3, 130, True, False)])
def test_partitioned_plan_equals_unpartitioned(P, B, sparse, overlap):
    """(overlap None: the reach chain on its own stream, the default for device engines;
    False: every kernel on one stream.)"""
    from egraph import shard
    from egraph.graph import Snapshot
    g, sv, sc, ss, src = _graph(B, seed=80 + P, pods=2500)
    csr = g.csr()
    vl, _, _, _ = g.export()
    V, k = g.num_vertices, 8
    inc = g.labels().index("Incident")
    owner = shard.partition_vertices(csr["row_ptr"], vl, g.labels(), P)
    runs = []
    for r in range(P):
        lg = shard.build_local(csr, vl, owner, r, P)
        snap = Snapshot.from_csr(lg.row_ptr, lg.col, lg.meta, lg.val, lg.vlabel, g.labels())
        lv, lc, ls = shard.local_seeds(lg, V, sv, sc, ss)
        plan = snap.plan(B, max_seeds=max(len(lv), 1), k=k)
        plan.set_seeds(_dev(lv), _dev(lc), _dev(ls))
        plan.set_sources(_dev(shard.local_sources(lg, V, src)))
        runs.append(shard.RankRun(lg, plan, torch.device("cuda", 0)))
        runs[-1].snap = snap
    out = shard.run_partitioned(runs, shard.LocalComm(), 3, inc, k, sparse=sparse, overlap=overlap)
    for run in runs:                 # 2 hops x (scores + reach) exchanged
        dense = 2 * run.halo_bytes_per_hop
        assert run.sent_bytes == dense if not sparse else run.sent_bytes < dense
    exp = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, B, 3)
    er = oracle.reach(csr["row_ptr"], csr["col"], src, 3)
    e_ids, e_sc = oracle.topk(exp, er, vl, inc, k)
    for run, (ids, scores) in zip(runs, out):
        lg = run.lg
        got = run.eng.read_scores().cpu().numpy()[: lg.n_owned]
        assert got.tobytes() == exp[lg.gid[: lg.n_owned]].tobytes()        # bit-identical
        reach = run.eng.read_reach().cpu().numpy().view(np.uint64)[:, : lg.n_owned]
        np.testing.assert_array_equal(reach, er[:, lg.gid[: lg.n_owned]])
        np.testing.assert_array_equal(ids.cpu().numpy(), e_ids.astype(np.int64))
        np.testing.assert_array_equal(scores.cpu().numpy(), e_sc)


def _rank_main(rank, P, port, q):
    import os

    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=P)
    try:
        from egraph import shard
        from egraph.graph import Snapshot
        B, k = 48, 6
        g, sv, sc, ss, src = _graph(B, seed=91, pods=1800)
        csr = g.csr()
        vl, _, _, _ = g.export()
        V = g.num_vertices
        owner = shard.partition_vertices(csr["row_ptr"], vl, g.labels(), P)
        lg = shard.build_local(csr, vl, owner, rank, P)
        snap = Snapshot.from_csr(lg.row_ptr, lg.col, lg.meta, lg.val, lg.vlabel, g.labels())
        lv, lc, ls = shard.local_seeds(lg, V, sv, sc, ss)
        plan = snap.plan(B, max_seeds=max(len(lv), 1), k=k)
        plan.set_seeds(_dev(lv), _dev(lc), _dev(ls))
        plan.set_sources(_dev(shard.local_sources(lg, V, src)))
        run = shard.RankRun(lg, plan, torch.device("cuda", 0))
        (ids, scores), = shard.run_partitioned([run], shard.TorchComm(), 3,
                                               g.labels().index("Incident"), k)
        own = plan.read_scores().cpu().numpy()[: lg.n_owned]
        q.put((rank, lg.gid[: lg.n_owned], own, ids.cpu().numpy(), scores.cpu().numpy()))
    finally:
        dist.destroy_process_group()


def test_partitioned_two_processes_one_gpu():
    """Two processes, one partition each, exchanging through torch.distributed (gloo staged
    through host memory: RCCL needs one GPU per rank)."""
    import socket

    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    B, k = 48, 6
    g, sv, sc, ss, src = _graph(B, seed=91, pods=1800)
    csr = g.csr()
    vl, _, _, _ = g.export()
    exp = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, B, 3)
    er = oracle.reach(csr["row_ptr"], csr["col"], src, 3)
    e_ids, e_sc = oracle.topk(exp, er, vl, g.labels().index("Incident"), k)
    for rank, gids, own, ids, scores in res:
        assert own.tobytes() == exp[gids].tobytes()
        np.testing.assert_array_equal(ids, e_ids.astype(np.int64))
        np.testing.assert_array_equal(scores, e_sc)


def test_partitioned_c4_eight_partitions():
    """BASELINE C4 (the 1.09M-vertex graph with its dense Event / LogPattern / MetricAnomaly
    links, ~10M CSR entries) edge-cut into 8 partitions in one process: the 8-GPU layout of
    bench.py --shard graph.  Owned scores bit-identical to the unpartitioned oracle recurrence,
    merged top-k equal to the unpartitioned top-k."""
    from egraph import shard, synth
    from egraph.graph import Snapshot
    P, B, k = 8, 16, 8
    c = synth.build_cluster(synth.CONFIGS["C4"])
    cases = synth.make_incidents(c, B, seed=1000)
    synth.add_incidents(c, cases)
    g = synth.build_graph(c)
    sv, sc, ss = synth.seeds_for_batch(g, [x.evidence for x in cases])
    src = g.lookup([f"incident:{x.incident['id']}" for x in cases]).astype(np.uint32)
    csr = g.csr()
    vl = g.vertex_labels()
    V = g.num_vertices
    assert V > 1_000_000 and len(csr["col"]) > 9_000_000
    inc = g.labels().index("Incident")
    owner = shard.partition_vertices(csr["row_ptr"], vl, g.labels(), P)
    runs = []
    for r in range(P):
        lg = shard.build_local(csr, vl, owner, r, P)
        snap = Snapshot.from_csr(lg.row_ptr, lg.col, lg.meta, lg.val, lg.vlabel, g.labels())
        lv, lc, ls = shard.local_seeds(lg, V, sv, sc, ss)
        plan = snap.plan(B, max_seeds=max(len(lv), 1), k=k)
        plan.set_seeds(_dev(lv), _dev(lc), _dev(ls))
        plan.set_sources(_dev(shard.local_sources(lg, V, src)))
        runs.append(shard.RankRun(lg, plan, torch.device("cuda", 0)))
        runs[-1].snap = snap
    out = shard.run_partitioned(runs, shard.LocalComm(), 3, inc, k, sparse=True)
    exp = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, B, 3)
    er = oracle.reach(csr["row_ptr"], csr["col"], src, 3)
    e_ids, e_sc = oracle.topk(exp, er, vl, inc, k)
    assert sum(r.lg.n_owned for r in runs) == V
    for run, (ids, scores) in zip(runs, out):
        lg = run.lg
        got = run.eng.read_scores().cpu().numpy()[: lg.n_owned]
        assert got.tobytes() == exp[lg.gid[: lg.n_owned]].tobytes()        # bit-identical
        np.testing.assert_array_equal(ids.cpu().numpy(), e_ids.astype(np.int64))
        np.testing.assert_array_equal(scores.cpu().numpy(), e_sc)


@pytest.mark.parametrize("P,B", [(3, 130), (2, 40)])
def test_partitioned_plan_reruns_with_new_seeds(P, B):
    """The same partition plans run three times with different seed sets (A, B, A): the sparse
    unpack's tile-flag clearing (only the halo tiles the previous scatter wrote, after one full
    clear per buffer) leaves no stale halo entry -- owned scores, reach and the merged top-k equal
    the unpartitioned oracle on every run.  B = 130 runs 128-column tiles, B = 40 16-column ones."""
    from egraph import shard
    from egraph.graph import Snapshot
    g, sv, sc, ss, src = _graph(B, seed=90 + P, pods=2500)
    rng = np.random.default_rng(P)
    # a second seed set: the same rows moved to other columns, strengths rescaled
    perm = rng.permutation(B).astype(np.uint32)
    sets = [(sv, sc, ss), (sv, perm[sc], (ss * 1.5).astype(np.float32)), (sv, sc, ss)]
    csr = g.csr()
    vl, _, _, _ = g.export()
    V, k = g.num_vertices, 8
    inc = g.labels().index("Incident")
    owner = shard.partition_vertices(csr["row_ptr"], vl, g.labels(), P)
    runs = []
    for r in range(P):
        lg = shard.build_local(csr, vl, owner, r, P)
        snap = Snapshot.from_csr(lg.row_ptr, lg.col, lg.meta, lg.val, lg.vlabel, g.labels())
        plan = snap.plan(B, max_seeds=max(len(sv), 1), k=k)
        runs.append(shard.RankRun(lg, plan, torch.device("cuda", 0)))
        runs[-1].snap = snap
    er = oracle.reach(csr["row_ptr"], csr["col"], src, 3)
    for t, (a, b, c) in enumerate(sets):
        for run in runs:
            lv, lc, ls = shard.local_seeds(run.lg, V, a, b, c)
            run.eng.set_seeds(_dev(lv), _dev(lc), _dev(ls))
            run.eng.set_sources(_dev(shard.local_sources(run.lg, V, src)))
        out = shard.run_partitioned(runs, shard.LocalComm(), 3, inc, k, sparse=True)
        exp = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], a, b, c, B, 3)
        e_ids, e_sc = oracle.topk(exp, er, vl, inc, k)
        for run, (ids, scores) in zip(runs, out):
            lg = run.lg
            got = run.eng.read_scores().cpu().numpy()[: lg.n_owned]
            assert got.tobytes() == exp[lg.gid[: lg.n_owned]].tobytes(), f"run {t}"
            reach = run.eng.read_reach().cpu().numpy().view(np.uint64)[:, : lg.n_owned]
            np.testing.assert_array_equal(reach, er[:, lg.gid[: lg.n_owned]])
            np.testing.assert_array_equal(ids.cpu().numpy(), e_ids.astype(np.int64), err_msg=f"run {t}")
            np.testing.assert_array_equal(scores.cpu().numpy(), e_sc, err_msg=f"run {t}")


@pytest.mark.parametrize("P,B", [(2, 40), (3, 130), (4, 70)])
def test_partitioned_fixed_slots_equal_oracle(P, B):
    """The fixed-capacity halo exchange (egr_plan_pack_sparse_cap / unpack_sparse_cap: device
    counts and overflow flag, equal-split all-to-all, no host read per exchange): a calibrating
    pass over the host-count path, passes on the fixed slots with other seed sets, and a pass
    whose slots are forced too small -- it overflows, recalibrates and re-runs
    (run_partitioned_retry).  Every pass: owned scores, reach and merged top-k equal the oracle."""
    from egraph import shard
    from egraph.graph import Snapshot
    g, sv, sc, ss, src = _graph(B, seed=120 + P, pods=2500)
    rng = np.random.default_rng(P)
    perm = rng.permutation(B).astype(np.uint32)
    sets = [(sv, sc, ss), (sv, perm[sc], (ss * 1.5).astype(np.float32)), (sv, sc, ss), (sv, sc, ss)]
    csr = g.csr()
    vl, _, _, _ = g.export()
    V, k = g.num_vertices, 8
    inc = g.labels().index("Incident")
    owner = shard.partition_vertices(csr["row_ptr"], vl, g.labels(), P)
    runs = []
    for r in range(P):
        lg = shard.build_local(csr, vl, owner, r, P)
        snap = Snapshot.from_csr(lg.row_ptr, lg.col, lg.meta, lg.val, lg.vlabel, g.labels())
        plan = snap.plan(B, max_seeds=max(len(sv), 1), k=k)
        runs.append(shard.RankRun(lg, plan, torch.device("cuda", 0)))
        runs[-1].snap = snap
    er = oracle.reach(csr["row_ptr"], csr["col"], src, 3)
    for t, (a, b, c) in enumerate(sets):
        def reset():
            for run in runs:
                lv, lc, ls = shard.local_seeds(run.lg, V, a, b, c)
                run.eng.set_seeds(_dev(lv), _dev(lc), _dev(ls))
                run.eng.set_sources(_dev(shard.local_sources(run.lg, V, src)))
        reset()
        if t == 3:
            for run in runs:
                run.cap = {"scores": 1, "reach": 1}
        fixed_before = all(run.cap for run in runs)
        out = shard.run_partitioned_retry(runs, shard.LocalComm(), 3, inc, k, reset)
        assert fixed_before == (t > 0)
        assert all(run.cap["scores"] >= 1024 for run in runs)       # (re)calibrated
        exp = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], a, b, c, B, 3)
        e_ids, e_sc = oracle.topk(exp, er, vl, inc, k)
        for run, (ids, scores) in zip(runs, out):
            lg = run.lg
            got = run.eng.read_scores().cpu().numpy()[: lg.n_owned]
            assert got.tobytes() == exp[lg.gid[: lg.n_owned]].tobytes(), f"run {t}"
            reach = run.eng.read_reach().cpu().numpy().view(np.uint64)[:, : lg.n_owned]
            np.testing.assert_array_equal(reach, er[:, lg.gid[: lg.n_owned]])
            np.testing.assert_array_equal(ids.cpu().numpy(), e_ids.astype(np.int64), err_msg=f"run {t}")
            np.testing.assert_array_equal(scores.cpu().numpy(), e_sc, err_msg=f"run {t}")
