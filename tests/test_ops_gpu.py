"""The registered custom ops (torch.ops.egraph.*, csrc/torch_ops.cpp over the C-ABI) against the
oracle: rules_eval vs orc_rules_eval (bit-exact float64), frontier_run vs orc_frontier, propagate
vs orc_propagate (bit-identical), reach vs orc_reach, topk over the op outputs vs orc_topk --
and the drop-in services, which call them, stay equal to the reference restatement."""
from __future__ import annotations

import random

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu


def _dev(a):
    from egraph.device import to_device
    return to_device(np.ascontiguousarray(a), torch.device("cuda", 0))


def _world(B=96, seed=131):
    from egraph import synth
    cfg = synth.ClusterConfig(pods=3000, namespaces=6, nodes=60, deployments=300, services=200,
                              attach_fraction=0.3, seed=seed)
    c = synth.build_cluster(cfg)
    cases = synth.make_incidents(c, B, seed=seed + 1)
    synth.add_incidents(c, cases)
    g = synth.build_graph(c)
    sv, sc, ss = synth.seeds_for_batch(g, [x.evidence for x in cases])
    src = g.lookup([f"incident:{x.incident['id']}" for x in cases]).astype(np.uint32)
    return g, cases, sv, sc, ss, src


def test_rules_eval_op():
    import evidence_fuzz
    from egraph import catalog, ops
    from egraph.encode import encode_batch
    rng = random.Random(5)
    cat = catalog.default()
    enc = encode_batch([evidence_fuzz.random_evidence(rng) for _ in range(500)], cat)
    outs = ops.rules_eval(_dev(enc.flags), _dev(enc.vocab), _dev(enc.node), _dev(enc.err),
                          _dev(enc.seg_off), ops.rule_table_tensor(cat))
    mask, n_hyp, oc, orank, conf, fin, st = (t.cpu().numpy() for t in outs)
    exp = oracle.rules_eval(cat.table, enc.flags, enc.vocab, enc.node, enc.err, enc.seg_off)
    np.testing.assert_array_equal(mask.view(np.uint32), exp["mask"])
    np.testing.assert_array_equal(n_hyp, exp["n_hyp"])
    np.testing.assert_array_equal(oc, exp["order_conf"])
    np.testing.assert_array_equal(orank, exp["order_rank"])
    assert conf.tobytes() == exp["confidence"].tobytes()
    assert fin.tobytes() == exp["final_score"].tobytes()
    assert st.tobytes() == exp["strength"].tobytes()


def test_graph_ops_match_oracle():
    from egraph import ops
    g, _, sv, sc, ss, src = _world()
    B, k, hops = len(src), 10, 3
    inc = g.labels().index("Incident")
    snap = g.snapshot()
    csr = g.csr()
    vl, _, _, _ = g.export()
    # frontier_run (top-k only frontier, as GraphService runs it)
    fr = snap.frontier(B, max_seeds=len(sv), k=k, pool_entries=-1)
    ids, sco = ops.frontier_run(fr, _dev(sv), _dev(sc), _dev(ss), _dev(src), hops, inc)
    e_ids, e_sc, _ = oracle.frontier(csr["row_ptr"], csr["col"], csr["val"], vl, sv, sc, ss, src,
                                     hops, inc, k)
    np.testing.assert_array_equal(ids.cpu().numpy().view(np.uint32), e_ids)
    assert sco.cpu().numpy().tobytes() == e_sc.tobytes()
    # propagate / reach / topk through the dense plan's ops
    plan = snap.plan(B, max_seeds=len(sv), k=k)
    scores = ops.propagate(plan, _dev(sv), _dev(sc), _dev(ss), hops)
    bits = ops.reach(plan, _dev(src), hops)
    exp = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, B, hops)
    er = oracle.reach(csr["row_ptr"], csr["col"], src, hops)
    assert scores.shape == (g.num_vertices, B)
    assert scores.cpu().numpy().tobytes() == exp.tobytes()
    np.testing.assert_array_equal(bits.cpu().numpy().view(np.uint64), er)
    for kk, ex in ((k, inc), (16, -1), (1, inc)):
        t_ids, t_sc = ops.topk(snap, scores, bits, kk, ex)
        o_ids, o_sc = oracle.topk(exp, er, vl, ex, kk)
        np.testing.assert_array_equal(t_ids.cpu().numpy().view(np.uint32), o_ids)
        assert t_sc.cpu().numpy().tobytes() == o_sc.tobytes()


def test_ops_reject_bad_inputs():
    from egraph import ops
    g, _, sv, sc, ss, src = _world(B=8, seed=137)
    snap = g.snapshot()
    fr = snap.frontier(8, max_seeds=len(sv), k=5, pool_entries=-1)
    with pytest.raises(ValueError):                          # seed arrays differ in length
        ops.frontier_run(fr, _dev(sv), _dev(sc[:-1]), _dev(ss), _dev(src))
    with pytest.raises(ValueError):                          # wrong dtype
        torch.ops.egraph.topk(ops._h(snap), torch.zeros((g.num_vertices, 8), device="cuda"),
                              torch.zeros((1, g.num_vertices), dtype=torch.int32, device="cuda"),
                              5, -1)
    with pytest.raises(NotImplementedError):                 # no CPU kernel: no fallback
        torch.ops.egraph.topk(ops._h(snap), torch.zeros((g.num_vertices, 8)),
                              torch.zeros((1, g.num_vertices), dtype=torch.int64), 5, -1)
