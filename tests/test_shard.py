"""The partitioned-graph path (egraph/shard.py) on CPU.

* Host maps: every owned row of every rank equals its global row with the entries remapped
  (CSR order kept), halo rows are empty, and the all-to-all routing (rank r sends q the rows q reads, grouped
  by reader) lands every halo row on the right received row.
* The whole protocol at world size 2 under gloo (two processes, torch.distributed all_gather of
  CPU tensors): per-hop halo exchange of scores and reach words, then the top-k merge -- with
  the CPU engine (tests/shard_cpu_engine.py, the C oracle's single-hop step) in place of the
  HIP plan.  Scores of the owned rows are bit-identical to the unpartitioned oracle recurrence
  and the merged top-k equals the unpartitioned top-k.
The same protocol on the GPU with the HIP plan: tests/test_shard_gpu.py.
"""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch

import oracle


def _graph(B=24, seed=71, pods=900):
    from egraph import synth
    from egraph.graph import EvidenceGraph
    cfg = synth.ClusterConfig(pods=pods, namespaces=6, nodes=24, deployments=pods // 10,
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


@pytest.mark.parametrize("P", [1, 2, 3, 5])
def test_local_graphs_cover_the_global_csr(P):
    from egraph import shard
    g, *_ = _graph()
    csr = g.csr()
    vl, _, _, _ = g.export()
    owner = shard.partition_vertices(csr["row_ptr"], vl, g.labels(), P)
    assert owner.min() >= 0 and owner.max() < P
    rp = csr["row_ptr"].astype(np.int64)
    locs = [shard.build_local(csr, vl, owner, r, P) for r in range(P)]
    assert sum(lg.n_owned for lg in locs) == g.num_vertices
    sent = {}
    for lg in locs:
        lrp = lg.row_ptr.astype(np.int64)
        for lv in range(lg.n_owned):
            v = int(lg.gid[lv])
            glob = csr["col"][rp[v]:rp[v + 1]]
            loc = lg.gid[lg.col[lrp[lv]:lrp[lv + 1]]]
            assert (loc == glob).all()
            assert (lg.val[lrp[lv]:lrp[lv + 1]] == csr["val"][rp[v]:rp[v + 1]]).all()
        assert (lrp[lg.n_owned:] == lrp[lg.n_owned]).all()          # halo rows are empty
        assert (owner[lg.gid[: lg.n_owned]] == lg.rank).all()
        assert (owner[lg.gid[lg.n_owned:]] != lg.rank).all()
        assert sum(lg.send_counts) == len(lg.send_rows) and lg.send_counts[lg.rank] == 0
        assert (lg.send_rows < lg.n_owned).all()
        off = np.concatenate([[0], np.cumsum(lg.send_counts)])
        for q in range(P):
            sent[(lg.rank, q)] = lg.gid[lg.send_rows[off[q]:off[q + 1]].astype(np.int64)]
    # routing: what q receives from r is what r sends to q; halo sources pick the right rows
    for lg in locs:
        assert all(lg.recv_counts[r] == len(sent[(r, lg.rank)]) for r in range(P))
        recv = np.concatenate([sent[(r, lg.rank)] for r in range(P)])
        assert len(recv) == len(lg.halo_rows)
        assert (recv[lg.halo_src.astype(np.int64)] == lg.gid[lg.n_owned:]).all()
        # every halo vertex is read by an owned row, and no boundary row is sent twice to q
        for r in range(P):
            assert len(np.unique(sent[(r, lg.rank)])) == len(sent[(r, lg.rank)])


def _rank_main(rank, P, port, q, sparse=True, fixed=False):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=P)
    try:
        from egraph import shard
        from shard_cpu_engine import CpuEngine
        g, sv, sc, ss, src = _graph()
        csr = g.csr()
        vl, _, _, _ = g.export()
        V, B = g.num_vertices, len(src)
        owner = shard.partition_vertices(csr["row_ptr"], vl, g.labels(), P)
        lg = shard.build_local(csr, vl, owner, rank, P)
        eng = CpuEngine(lg, B, k=6)
        eng.set_seeds(*shard.local_seeds(lg, V, sv, sc, ss))
        eng.set_sources(shard.local_sources(lg, V, src))
        run = shard.RankRun(lg, eng, torch.device("cpu"))
        inc = g.labels().index("Incident")
        if fixed:
            # calibrating pass, a pass on the fixed slots, then one whose slots are forced too
            # small: it overflows, grows them and re-runs (run_partitioned_retry)
            def reset():
                eng.set_seeds(*shard.local_seeds(lg, V, sv, sc, ss))
                eng.set_sources(shard.local_sources(lg, V, src))
            comm = shard.TorchComm()
            shard.run_partitioned_retry([run], comm, 3, inc, 6, reset)
            assert run.cap["scores"] >= 1024
            reset()
            c0 = comm.calls
            shard.run_partitioned_retry([run], comm, 3, inc, 6, reset)
            # a steady-state pass: one all-to-all per exchange (2 score + 2 reach) and the
            # candidates' all-gather, which also carries the overflow flags -- 5 collectives
            assert comm.calls - c0 == 5, comm.calls - c0
            run.cap = {"scores": 2, "reach": 2}
            reset()
            (ids, scores), = shard.run_partitioned_retry([run], comm, 3, inc, 6, reset)
            assert run.cap["scores"] >= 1024           # recalibrated by the re-run
        else:
            (ids, scores), = shard.run_partitioned([run], shard.TorchComm(), 3, inc, 6,
                                                   sparse=sparse)
        q.put((rank, lg.gid[: lg.n_owned], eng.scores_owned(), ids.numpy(), scores.numpy(),
               run.sent_bytes, 2 * run.halo_bytes_per_hop))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("P,sparse,fixed", [(2, True, False), (2, False, False), (8, True, False),
                                            (2, True, True), (4, True, True)])
def test_partitioned_protocol_gloo_world_size_2(P, sparse, fixed):
    """(P = 8: the 8-GPU layout of the edge-cut path, every peer pair exchanging.  fixed: the
    fixed-capacity slot exchange, calibrated, then overflowed and re-run.)"""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, P, port, q, sparse, fixed)) for r in range(P)]
    for p in procs:
        p.start()
    res = [q.get(timeout=240) for _ in range(P)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g, sv, sc, ss, src = _graph()
    csr = g.csr()
    B = len(src)
    exp = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, B, 3)
    er = oracle.reach(csr["row_ptr"], csr["col"], src, 3)
    vl, _, _, _ = g.export()
    e_ids, e_sc = oracle.topk(exp, er, vl, g.labels().index("Incident"), 6)
    covered = 0
    for rank, gids, owned_scores, ids, scores, sent, dense in res:
        # 2 exchanges (scores + reach) x 2 hops; the sparse one sends only non-zero entries
        if not fixed:
            assert sent == dense if not sparse else 0 < sent < dense
        assert owned_scores.tobytes() == exp[gids].tobytes()          # bit-identical rows
        covered += len(gids)
        got = ids.astype(np.int64)
        want = e_ids.astype(np.int64)
        np.testing.assert_array_equal(got, want)                      # merged top-k, every rank
        np.testing.assert_array_equal(scores, e_sc)
    assert covered == g.num_vertices
