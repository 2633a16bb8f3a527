"""Parity at the configurations the numbers come from (BASELINE.json configs C2, C3, C4).

* C3, the exact bench configuration (bench.py defaults): the 100k-pod graph, B = 1024 incidents
  per batch, top-k-only frontiers (pool_entries = -1: the pruned narrow-table kernel), three
  frontier + rules states in flight on their own streams, rules on each lane's side stream.
  Six batches with DIFFERENT incidents are interleaved over the three lanes exactly as
  bench.step_frontier does; every batch's top-k ids / scores are checked against the CPU
  frontier oracle (orc_frontier, itself pinned to the dense oracle in
  tests/test_oracle_frontier.py) and its rule outputs against orc_rules_eval.
* C2 (10k pods, 1k concurrent mixed incidents): the rules kernel, the drop-in dicts (against
  the reference restatement rca_oracle, itself pinned to the reference's goldens) and the
  frontier top-k against both oracles.
* C4 (the 1M-vertex graph, ~10M CSR entries): the frontier engine at B = 256 against
  orc_frontier, and the edge-cut partitioned plan at P = 2 and P = 4 (one process) against the
  unpartitioned oracle: owned scores bit-identical, merged top-k equal.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu


def _dev(a):
    from egraph.device import to_device
    return to_device(np.ascontiguousarray(a), torch.device("cuda", 0))


def _world(config: str, batches: list[int], seed0: int = 1000):
    """The config's cluster with len(batches) incident batches added; per batch its cases."""
    from egraph import synth
    cl = synth.build_cluster(synth.CONFIGS[config])
    out = []
    for j, B in enumerate(batches):
        cases = synth.make_incidents(cl, B, seed=seed0 + j)
        synth.add_incidents(cl, cases)
        out.append(cases)
    return synth.build_graph(cl), out


def _batch_inputs(g, cases):
    from egraph import synth
    ev = [x.evidence for x in cases]
    sv, sc, ss = synth.seeds_for_batch(g, ev)
    src = g.lookup([f"incident:{x.incident['id']}" for x in cases]).astype(np.uint32)
    return ev, sv, sc, ss, src


def _oracle_topk(g, csr, vl, sv, sc, ss, src, k=10, hops=3):
    inc = g.labels().index("Incident")
    ids, sco, _ = oracle.frontier(csr["row_ptr"], csr["col"], csr["val"], vl, sv, sc, ss, src,
                                  hops, inc, k, threads=16)
    return ids, sco


def _check_rules(res, enc):
    from egraph import catalog
    exp = oracle.rules_eval(catalog.default().table, enc.flags, enc.vocab, enc.node, enc.err, enc.seg_off)
    np.testing.assert_array_equal(res.mask, exp["mask"])
    np.testing.assert_array_equal(res.n_hyp, exp["n_hyp"])
    np.testing.assert_array_equal(res.order_rank, exp["order_rank"])
    np.testing.assert_array_equal(res.order_conf, exp["order_conf"])
    assert res.final_score.tobytes() == exp["final_score"].tobytes()
    assert res.confidence.tobytes() == exp["confidence"].tobytes()


@pytest.mark.parametrize("seed_input", ["device", "order", None])
def test_bench_config_c3_pipelined_lanes(seed_input, monkeypatch):
    """bench.py's C3 step exactly: three lanes, six different batches, seeds as grouped input
    with the launch order computed on the device (the default) or on the host, or sorted on the
    device (--seed-input sort)."""
    import bench
    monkeypatch.setattr(bench, "GROUPED", seed_input)
    from egraph import catalog
    from egraph.encode import encode_batch
    from egraph.rca import RulesDeviceBatch
    B, k, hops, P, n_batches = 1024, 10, 3, 3, 6
    g, batches = _world("C3", [B] * n_batches)
    dev = torch.device("cuda", 0)
    inc = g.labels().index("Incident")
    inputs = []
    for cases in batches:
        ev, sv, sc, ss, src = _batch_inputs(g, cases)
        enc = encode_batch(ev, catalog.default())
        inputs.append(dict(enc=enc, host=(sv, sc, ss, src),
                           seeds=(_dev(sv), _dev(sc), _dev(ss)), sources=_dev(src),
                           rules=RulesDeviceBatch(enc, catalog.default(), dev)))
    max_seeds = max(len(x["host"][0]) for x in inputs)
    snap = g.snapshot(device=dev)
    lanes = bench.build_lanes(snap, B, max_seeds, k, P, -1, dev,
                              [(None, x["rules"], x["seeds"], x["sources"]) for x in inputs[:P]])
    assert all(ln["frontier"].pool_entries == -1 for ln in lanes)
    ctx = dict(lanes=lanes, tick=0, inc_label=inc)
    row_ptr = g.csr()["row_ptr"]
    got = [(torch.empty(B * k, dtype=torch.int32, device=dev),
            torch.empty(B * k, dtype=torch.float32, device=dev)) for _ in range(n_batches)]
    for i, x in enumerate(inputs):                  # bench.step_frontier, one batch per step
        lane = ctx["lanes"][ctx["tick"] % P]
        lane.update(sources=x["sources"], rules=x["rules"])
        bench.set_lane_seeds(lane, x["seeds"], B, snap, dev, row_ptr)
        lane = bench.step_frontier(ctx, hops)
        with torch.cuda.stream(lane["main"]):       # the lane's outputs before its next batch
            got[i][0].copy_(lane["frontier"].out_ids)
            got[i][1].copy_(lane["frontier"].out_scores)
    torch.cuda.synchronize()
    csr = g.csr()
    vl, _, _, _ = g.export()
    for i, x in enumerate(inputs):
        sv, sc, ss, src = x["host"]
        e_ids, e_sc = _oracle_topk(g, csr, vl, sv, sc, ss, src, k, hops)
        np.testing.assert_array_equal(got[i][0].cpu().numpy().view(np.uint32).reshape(B, k), e_ids,
                                      err_msg=f"batch {i}")
        assert got[i][1].cpu().numpy().reshape(B, k).tobytes() == e_sc.tobytes(), f"batch {i}"
        _check_rules(x["rules"].fetch(), x["enc"])
    st = lanes[0]["frontier"].stats()
    assert st["overflowed"] == 0 and st["members"] > 0


@pytest.mark.parametrize("inline", [True, False])
def test_bench_config_c3_graph_replay(inline):
    """bench.py's default timed loop: each lane's batch captured as a HIP graph (rules inline on
    the lane's stream -- the default -- or forked to its side stream, seed prep, frontier,
    overflow grid) and replayed in turn.  Three lanes with different batches, two rounds of
    replays: every lane's outputs equal the oracle's."""
    import bench
    from egraph import catalog
    from egraph.encode import encode_batch
    from egraph.rca import RulesDeviceBatch
    B, k, hops, P = 1024, 10, 3, 3
    g, batches = _world("C3", [B] * P, seed0=3000)
    dev = torch.device("cuda", 0)
    inputs = []
    for cases in batches:
        ev, sv, sc, ss, src = _batch_inputs(g, cases)
        enc = encode_batch(ev, catalog.default())
        inputs.append(dict(enc=enc, host=(sv, sc, ss, src), seeds=(_dev(sv), _dev(sc), _dev(ss)),
                           sources=_dev(src), rules=RulesDeviceBatch(enc, catalog.default(), dev)))
    snap = g.snapshot(device=dev)
    lanes = bench.build_lanes(snap, B, max(len(x["host"][0]) for x in inputs), k, P, -1, dev,
                              [(None, x["rules"], x["seeds"], x["sources"]) for x in inputs])
    ctx = dict(lanes=lanes, tick=0, inc_label=g.labels().index("Incident"))
    bench.capture_lanes(ctx, hops, inline_rules=inline)
    for ln in lanes:                    # poison the outputs: the replays must rewrite them
        ln["frontier"].out_ids.fill_(-7)
        ln["rules"].mask.fill_(-7)
    torch.cuda.synchronize()
    for _ in range(2 * P):
        bench.step_graph(ctx, hops)
    torch.cuda.synchronize()
    csr = g.csr()
    vl, _, _, _ = g.export()
    for ln, x in zip(lanes, inputs):
        sv, sc, ss, src = x["host"]
        e_ids, e_sc = _oracle_topk(g, csr, vl, sv, sc, ss, src, k, hops)
        np.testing.assert_array_equal(ln["frontier"].out_ids.cpu().numpy().view(np.uint32).reshape(B, k), e_ids)
        assert ln["frontier"].out_scores.cpu().numpy().reshape(B, k).tobytes() == e_sc.tobytes()
        _check_rules(x["rules"].fetch(), x["enc"])


def test_bench_config_c3_merged_launch():
    """bench.py --merge 3: three different C3 batches in one lane's launch (columns at their
    batch's offset, one costliest-first order across all 3072), captured and replayed twice:
    every batch's slice of the outputs equals the oracle's ranking of that batch alone, and the
    rules over the three batches' rows equal the oracle's."""
    import bench
    monkey = bench.GROUPED
    bench.GROUPED = "device"
    try:
        from egraph import catalog
        from egraph.encode import encode_batch
        from egraph.rca import RulesDeviceBatch
        B, k, hops, M = 1024, 10, 3, 3
        g, batches = _world("C3", [B] * M, seed0=5000)
        dev = torch.device("cuda", 0)
        hosts, evs = [], []
        for cases in batches:
            ev, sv, sc, ss, src = _batch_inputs(g, cases)
            hosts.append((sv, sc, ss, src))
            evs += ev
        msv, msc, mss, msrc = bench.merge_batches(hosts, B)
        enc = encode_batch(evs, catalog.default())
        rules = RulesDeviceBatch(enc, catalog.default(), dev)
        snap = g.snapshot(device=dev)
        lanes = bench.build_lanes(snap, B * M, len(msv), k, 1, -1, dev,
                                  [(None, rules, (_dev(msv), _dev(msc), _dev(mss)), _dev(msrc))])
        ctx = dict(lanes=lanes, tick=0, inc_label=g.labels().index("Incident"), merge=M, sub=0)
        bench.capture_lanes(ctx, hops)
        lanes[0]["frontier"].out_ids.fill_(-7)
        torch.cuda.synchronize()
        for _ in range(2 * M):
            bench.step_graph(ctx, hops)
        torch.cuda.synchronize()
        csr = g.csr()
        vl, _, _, _ = g.export()
        ids = lanes[0]["frontier"].out_ids.cpu().numpy().view(np.uint32).reshape(M, B, k)
        sco = lanes[0]["frontier"].out_scores.cpu().numpy().reshape(M, B, k)
        for i, (sv, sc, ss, src) in enumerate(hosts):
            e_ids, e_sc = _oracle_topk(g, csr, vl, sv, sc, ss, src, k, hops)
            np.testing.assert_array_equal(ids[i], e_ids, err_msg=f"batch {i}")
            assert sco[i].tobytes() == e_sc.tobytes(), f"batch {i}"
        _check_rules(rules.fetch(), enc)
    finally:
        bench.GROUPED = monkey


def test_bench_headline_launch_m20():
    """The exact launch the headline times (bench.py --steps 20 --warmup 5, the driver's run):
    bench.setup("C3", B=1024, merge=20) -- 20 DIFFERENT incident sets, 20,480 columns in one
    launch, the locality layout, the launch order computed on the device -- warmed up as main()
    does (bench.warm_up: eager steps, Frontier.adapt() switching the overflow handling on for the
    columns that overflow the 7-per-CU narrow table -- continuation regions, the wide retry
    behind them -- then, at M = 20, eager launches: main() captures HIP graphs only below
    bench.GRAPH_MERGE_MAX batches per launch), then launched once more with poisoned outputs.  Every one of the 20,480 columns' top-k ids and
    score bytes equals orc_frontier's on the same merged input, the rules over all 20 batches'
    rows equal orc_rules_eval's, and some columns did overflow the narrow table and were
    finished in continuation regions inside the grid (none reached the global-memory variant)."""
    import bench
    saved = bench.GROUPED
    bench.GROUPED = "device"
    try:
        dev = torch.device("cuda", 0)
        B, k, hops, M = 1024, 10, 3, 20
        ctx = bench.setup("C3", B, k, 0, dev, pool_entries=-1, merge=M)
        assert ctx["distinct_batches"] == M and ctx["merge"] == M
        graphs = M < bench.GRAPH_MERGE_MAX          # (as main(): eager launches at M = 20)
        step = bench.warm_up(ctx, hops, 5, dev, graphs=graphs)
        assert step is (bench.step_graph if graphs else bench.step_frontier)
        lane = ctx["lanes"][0]
        fr = lane["frontier"]
        assert fr.retry_blocks > 0 and fr.wide_first == fr.FIRST_NARROW, "C3 runs narrow + retry"
        fr.out_ids.fill_(-7)
        fr.out_scores.fill_(float("nan"))
        lane["rules"].mask.fill_(-7)
        torch.cuda.synchronize()
        ctx["sub"] = 0
        for _ in range(M):                  # one timed-region's worth: a single launch of M batches
            step(ctx, hops)
        torch.cuda.synchronize()
        st = fr.stats()
        assert st["overflowed"] > 0, "the headline launch retries its overflowing columns"
        assert st["global_columns"] == 0
        if fr.CONTINUATION_REGIONS > 0:      # ... each finished in its own workgroup, in a region
            assert fr.continuation_regions > 0 and st["continued"] == st["overflowed"], st
        g = ctx["graph"]
        csr = g.csr()
        vl, _, _, _ = g.export()
        sv, sc, ss, src = ctx["lane_host"]
        assert len(src) == B * M
        e_ids, e_sc = _oracle_topk(g, csr, vl, sv, sc, ss, src, k, hops)
        ids = fr.out_ids.cpu().numpy().view(np.uint32).reshape(B * M, k)
        sco = fr.out_scores.cpu().numpy().reshape(B * M, k)
        for i in range(M):
            sl = slice(i * B, (i + 1) * B)
            np.testing.assert_array_equal(ids[sl], e_ids[sl], err_msg=f"batch {i}")
            assert sco[sl].tobytes() == e_sc[sl].tobytes(), f"batch {i}"
        _check_rules(lane["rules"].fetch(), ctx["lane_enc"])
    finally:
        bench.GROUPED = saved


@pytest.mark.parametrize("mid_cont", [False, True])
def test_c4_launch_m20(mid_cont, monkeypatch):
    """C4 through the replicated frontier as bench.py --config C4 --steps 20 times it: 20
    different incident sets in one launch of 20,480 columns, warmed up as main() does -- the
    narrow table overflows, adapt() starts every column in the mid table, whose overflowing
    columns take the wide retry (the default) or, with $EGRAPH_FRONTIER_MID_CONT, continue
    inside the grid, each in a region adapt()'s second look sized for all of them (no serial
    wide retry, no global-memory variant).  Every column's top-k ids and score bytes equal
    orc_frontier's."""
    import bench
    from egraph.graph import Frontier
    if mid_cont:
        monkeypatch.setenv("EGRAPH_FRONTIER_MID_CONT", "1")        # (read at frontier creation)
        monkeypatch.setattr(Frontier, "MID_CONTINUATION", True)
    saved = bench.GROUPED
    bench.GROUPED = "device"
    try:
        dev = torch.device("cuda", 0)
        B, k, hops, M = 1024, 10, 3, 20
        ctx = bench.setup("C4", B, k, 0, dev, pool_entries=-1, merge=M)
        step = bench.warm_up(ctx, hops, 5, dev, graphs=M < bench.GRAPH_MERGE_MAX)
        lane = ctx["lanes"][0]
        fr = lane["frontier"]
        assert fr.wide_first == fr.FIRST_MID and fr.retry_blocks > 0
        fr.out_ids.fill_(-7)
        fr.out_scores.fill_(float("nan"))
        torch.cuda.synchronize()
        ctx["sub"] = 0
        for _ in range(M):
            step(ctx, hops)
        torch.cuda.synchronize()
        st = fr.stats()
        assert st["overflowed"] > 0 and st["global_columns"] == 0, st
        if mid_cont:
            assert fr.continuation_regions >= st["overflowed"] and st["continued"] == st["overflowed"], st
        else:
            assert st["continued"] == 0, st
        g = ctx["graph"]
        csr = g.csr()
        vl, _, _, _ = g.export()
        sv, sc, ss, src = ctx["lane_host"]
        e_ids, e_sc = _oracle_topk(g, csr, vl, sv, sc, ss, src, k, hops)
        ids = fr.out_ids.cpu().numpy().view(np.uint32).reshape(B * M, k)
        sco = fr.out_scores.cpu().numpy().reshape(B * M, k)
        for i in range(M):
            sl = slice(i * B, (i + 1) * B)
            np.testing.assert_array_equal(ids[sl], e_ids[sl], err_msg=f"batch {i}")
            assert sco[sl].tobytes() == e_sc[sl].tobytes(), f"batch {i}"
    finally:
        bench.GROUPED = saved


def test_c2_rules_dropin_and_frontier():
    import asyncio
    from types import SimpleNamespace

    import rca_oracle
    from egraph import catalog
    from egraph.encode import encode_batch
    from egraph.rca import RulesDeviceBatch
    from helpers import record
    from src.services.rca.rules_engine import RulesEngine
    B = 1000
    g, (cases,) = _world("C2", [B])
    assert {x.scenario for x in cases} >= {"crashloop", "crashloop_deploy", "oom", "imagepull"}
    ev, sv, sc, ss, src = _batch_inputs(g, cases)
    enc = encode_batch(ev, catalog.default())
    rb = RulesDeviceBatch(enc, catalog.default(), torch.device("cuda", 0))
    rb.launch()
    _check_rules(rb.fetch(), enc)
    # the drop-in batch API against the reference restatement, every incident
    incs = [SimpleNamespace(id=x.incident["id"]) for x in cases]
    out = asyncio.run(RulesEngine().rank_incidents_batch(incs, ev))
    for x, hyps in zip(cases, out):
        assert record(hyps) == record(rca_oracle.rca(x.incident["id"], x.evidence))
    # frontier (pruned, top-k only) against orc_frontier and the dense oracle
    snap = g.snapshot()
    fr = snap.frontier(B, max_seeds=len(sv), k=10, pool_entries=-1)
    fr.set_seeds(_dev(sv), _dev(sc), _dev(ss))
    inc = g.labels().index("Incident")
    ids, sco = fr.run(_dev(src), hops=3, exclude_label=inc)
    csr = g.csr()
    vl, _, _, _ = g.export()
    e_ids, e_sc = _oracle_topk(g, csr, vl, sv, sc, ss, src)
    np.testing.assert_array_equal(ids.cpu().numpy().view(np.uint32), e_ids)
    assert sco.cpu().numpy().tobytes() == e_sc.tobytes()
    dense = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, B, 3, 16)
    reach = oracle.reach(csr["row_ptr"], csr["col"], src, 3, 16)
    d_ids, d_sc = oracle.topk(dense, reach, vl, inc, 10)
    np.testing.assert_array_equal(d_ids, e_ids)
    assert d_sc.tobytes() == e_sc.tobytes()


@pytest.fixture(scope="module")
def c4():
    g, (cases,) = _world("C4", [256], seed0=2000)
    ev, sv, sc, ss, src = _batch_inputs(g, cases)
    csr = g.csr()
    vl, _, _, _ = g.export()
    assert len(csr["col"]) > 9_000_000 and g.num_vertices > 1_000_000
    return g, csr, vl, sv, sc, ss, src


def test_c4_frontier_b256(c4):
    """C4's larger neighbourhoods overflow the narrow table: the first run sends those columns
    to the global-memory variant, adapt() turns the wide-table retry on with the mid table first,
    and the rerun takes the columns through the mid table (its overflows through the persistent
    wide grid) -- the same top-k every time, and in the wide-first and narrow-first modes too
    (bench.py's C4 path)."""
    g, csr, vl, sv, sc, ss, src = c4
    B = len(src)
    fr = g.snapshot().frontier(B, max_seeds=len(sv), k=10, pool_entries=-1)
    e_ids, e_sc = _oracle_topk(g, csr, vl, sv, sc, ss, src)
    for run in range(2):
        fr.set_seeds(_dev(sv), _dev(sc), _dev(ss))
        ids, sco = fr.run(_dev(src), hops=3, exclude_label=g.labels().index("Incident"))
        np.testing.assert_array_equal(ids.cpu().numpy().view(np.uint32), e_ids, err_msg=f"run {run}")
        assert sco.cpu().numpy().tobytes() == e_sc.tobytes()
        if run == 0:
            assert fr.stats()["overflowed"] > 0 and fr.adapt() and fr.retry_blocks > 0
    # most C4 columns overflow the narrow table: adapt() chose mid-first (the 2.8k-slot table,
    # then the wide grid for what overflows it), and most fit that table, so its second look
    # keeps it; wide-first and narrow-then-retry give the same top-k
    assert fr.wide_first == fr.FIRST_MID
    st = fr.stats()
    assert st["overflowed"] <= B // 2 and st["global_columns"] == 0
    assert not fr.adapt(st) and fr.wide_first == fr.FIRST_MID
    for mode, name in ((fr.FIRST_WIDE, "wide-first"), (fr.FIRST_NARROW, "narrow + retry")):
        fr.set_wide_first(mode)
        fr.set_seeds(_dev(sv), _dev(sc), _dev(ss))
        ids, sco = fr.run(_dev(src), hops=3, exclude_label=g.labels().index("Incident"))
        np.testing.assert_array_equal(ids.cpu().numpy().view(np.uint32), e_ids, err_msg=name)
        assert sco.cpu().numpy().tobytes() == e_sc.tobytes()


@pytest.mark.parametrize("P", [2, 4])
def test_c4_partitioned_plan(c4, P):
    from egraph import shard
    from egraph.graph import Snapshot
    g, csr, vl, sv, sc, ss, src = c4
    B, k = 64, 10
    keep = sc < B
    sv, sc, ss, src = sv[keep], sc[keep], ss[keep], src[:B]
    V = g.num_vertices
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
    out = shard.run_partitioned(runs, shard.LocalComm(), 3, inc, k)
    e_ids, e_sc = _oracle_topk(g, csr, vl, sv, sc, ss, src, k)
    exp = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, B, 3, 16)
    for run, (ids, scores) in zip(runs, out):
        lg = run.lg
        own = run.eng.read_scores().cpu().numpy()[: lg.n_owned]
        assert own.tobytes() == exp[lg.gid[: lg.n_owned]].tobytes()        # bit-identical
        np.testing.assert_array_equal(ids.cpu().numpy(), e_ids.astype(np.int64))
        np.testing.assert_array_equal(scores.cpu().numpy(), e_sc)


def test_simulator_scenarios_and_c1_through_the_dropin():
    """The four reference-simulator scenarios and C1 (tests/golden/simulator_cases.json, judged
    by the reference) through the drop-in RulesEngine; C1's graph through GraphService (the
    activities' build_evidence_graph + rank_root_causes) against the oracle."""
    import asyncio
    import json
    from types import SimpleNamespace

    from conftest import REPO
    from egraph import synth
    from helpers import golden_record, record
    from src.database import GraphService
    from src.models import GraphEntity, GraphRelation
    from src.services.rca.hypothesis_ranker import HypothesisRanker
    from src.services.rca.rules_engine import RulesEngine
    sim = json.loads((REPO / "tests" / "golden" / "simulator_cases.json").read_text())
    eng = RulesEngine()
    out = asyncio.run(eng.rank_incidents_batch([SimpleNamespace(id=c["incident_id"]) for c in sim["cases"]],
                                               [c["evidence"] for c in sim["cases"]]))
    for c, hyps in zip(sim["cases"], out):
        assert record(hyps) == golden_record(c["expected"]), c["name"]
    c1 = next(c for c in sim["cases"] if c["name"] == "C1")
    one = HypothesisRanker().rank(asyncio.run(eng.generate_hypotheses(SimpleNamespace(id=c1["incident_id"]),
                                                                      c1["evidence"])))
    assert record(one) == golden_record(c1["expected"])
    assert one[0]["rule_id"] == "crashloop_recent_deploy"
    # C1's evidence graph through the drop-in GraphService
    cl, case = synth.c1_world()
    GraphService.reset()
    try:
        asyncio.run(GraphService.create_entities_batch([GraphEntity(id=i, type=lab)
                                                        for i, lab in zip(cl.ids, cl.labels)]))
        asyncio.run(GraphService.create_relations_batch([GraphRelation(source_id=s, target_id=d, relation_type=t)
                                                         for s, d, t in zip(cl.src, cl.dst, cl.types)]))
        got = asyncio.run(GraphService.rank_root_causes([case.incident["id"]], [case.evidence], hops=3, k=10))[0]
        g = GraphService.graph()
        sv, sc, ss = synth.seeds_for_batch(g, [case.evidence])
        src = g.lookup([f"incident:{case.incident['id']}"]).astype(np.uint32)
        csr = g.csr()
        vl, _, _, _ = g.export()
        e_ids, e_sc = _oracle_topk(g, csr, vl, sv, sc, ss, src)
        want = [(g.vertex_id(int(v)), float(s)) for v, s in zip(e_ids[0], e_sc[0]) if v != 0xFFFFFFFF]
        assert [(r["id"], r["score"]) for r in got] == want and len(want) == 10
        sub = asyncio.run(GraphService.get_incident_graph(f"incident:{case.incident['id']}"))
        assert 90 <= len(sub["nodes"]) <= g.num_vertices
    finally:
        GraphService.reset()
