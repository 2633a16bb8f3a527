"""GPU parity of the frontier engine (egr_frontier_*, csrc/frontier.hip).

The frontier engine must give exactly what the dense plan gives: scores bit-identical to the
C oracle's dense recurrence (oracle/egraph_oracle.c orc_propagate, fmaf in CSR order), reach
sets equal to the per-column BFS (orc_reach), top-k ids and scores equal to orc_topk.  Cases
cover the LDS table, the global-memory fallback (columns whose members overflow the LDS table),
both mixed in one batch, empty / invalid sources and seeds, duplicate seeds (max-combined), a
member pool too small to keep every column, and several hop counts.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu

NO_NODE = 0xFFFFFFFF


def _dev(a):
    from egraph.device import to_device
    return to_device(np.ascontiguousarray(a), torch.device("cuda", 0))


def _world(B, seed=11, pods=3000, nodes=60):
    from egraph import synth
    from egraph.graph import EvidenceGraph
    cfg = synth.ClusterConfig(pods=pods, namespaces=6, nodes=nodes, deployments=pods // 10,
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


def _check(g, sv, sc, ss, src, B, hops=3, k=10, exclude=None, pool_entries=0, scores=True):
    from egraph.graph import group_seeds, launch_order
    snap = g.snapshot()
    fr = snap.frontier(B, max_seeds=max(len(sv), 1), k=k, pool_entries=pool_entries)
    fr.set_seeds(_dev(sv), _dev(sc), _dev(ss))
    inc = g.labels().index("Incident") if exclude is None else exclude
    ids, sco = fr.run(_dev(src), hops=hops, exclude_label=inc)
    got_ids = ids.cpu().numpy().view(np.uint32).copy()
    got_sc = sco.cpu().numpy().copy()
    csr = g.csr()
    exp = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, B, hops)
    er = oracle.reach(csr["row_ptr"], csr["col"], src, hops)
    vl, _, _, _ = g.export()
    e_ids, e_sc = oracle.topk(exp, er, vl, inc, k)
    np.testing.assert_array_equal(got_ids, e_ids)
    np.testing.assert_array_equal(got_sc, e_sc)
    # the same triples grouped by column on the host (egr_frontier_run_grouped: no device sort)
    gp, gv, gs = group_seeds(sv, sc, ss, B)
    fg = snap.frontier(B, max_seeds=max(len(gv), 1), k=k, pool_entries=pool_entries)
    g_ids, g_sc = fg.run_grouped(_dev(gp), _dev(gv), _dev(gs), _dev(src), hops=hops, exclude_label=inc)
    np.testing.assert_array_equal(g_ids.cpu().numpy().view(np.uint32), e_ids)
    assert g_sc.cpu().numpy().tobytes() == e_sc.tobytes()
    # ... started costliest-first (a caller-given launch order changes no bit)
    order = launch_order(gp, gv, g.csr()["row_ptr"])
    assert sorted(order.tolist()) == list(range(B))
    g_ids, g_sc = fg.run_grouped(_dev(gp), _dev(gv), _dev(gs), _dev(src), hops=hops, exclude_label=inc,
                                 order=_dev(order))
    np.testing.assert_array_equal(g_ids.cpu().numpy().view(np.uint32), e_ids)
    assert g_sc.cpu().numpy().tobytes() == e_sc.tobytes()
    st = fr.stats()
    assert 0 <= st["continued"] <= st["overflowed"]
    if scores:
        assert fr.read_scores().cpu().numpy().tobytes() == exp.tobytes()     # bit-identical
        np.testing.assert_array_equal(fr.read_reach().cpu().numpy().view(np.uint64), er)
    return fr


@pytest.mark.parametrize("B", [1, 7, 64, 130, 600])
def test_frontier_equals_oracle(B):
    g, sv, sc, ss, src = _world(B)
    fr = _check(g, sv, sc, ss, src, B)
    st = fr.stats()
    assert st["overflowed"] == 0 and st["members"] > 0 and st["pull_entries"] > 0


@pytest.mark.parametrize("hops", [1, 2, 4])
def test_frontier_hops(hops):
    g, sv, sc, ss, src = _world(40, seed=21, pods=1500)
    _check(g, sv, sc, ss, src, 40, hops=hops, k=7)


@pytest.mark.parametrize("k", [1, 16])
def test_frontier_k_and_no_exclusion(k):
    g, sv, sc, ss, src = _world(33, seed=23, pods=1200)
    _check(g, sv, sc, ss, src, 33, k=k, exclude=-1)


def test_frontier_matches_dense_plan():
    B = 300
    g, sv, sc, ss, src = _world(B, seed=5, pods=6000, nodes=100)
    snap = g.snapshot()
    inc = g.labels().index("Incident")
    plan = snap.plan(B, max_seeds=len(sv), k=10)
    plan.set_seeds(_dev(sv), _dev(sc), _dev(ss))
    plan.set_sources(_dev(src))
    d_ids, d_sc = plan.run(hops=3, exclude_label=inc)
    fr = snap.frontier(B, max_seeds=len(sv), k=10)
    fr.set_seeds(_dev(sv), _dev(sc), _dev(ss))
    f_ids, f_sc = fr.run(_dev(src), hops=3, exclude_label=inc)
    assert torch.equal(d_ids, f_ids) and torch.equal(d_sc, f_sc)
    assert torch.equal(plan.read_scores(), fr.read_scores())
    assert torch.equal(plan.read_reach(), fr.read_reach())


def _hub_world(n_leaves=9000, n_cols=6):
    """A star (hub + leaves, each leaf with a private tail vertex) plus a small ring: a column
    seeded at the hub touches every vertex (> the LDS table's 6144 members) and takes the
    global-memory fallback; a column seeded on the ring stays in LDS."""
    from egraph.graph import EvidenceGraph
    ids = ["hub"] + [f"leaf{i}" for i in range(n_leaves)] + [f"tail{i}" for i in range(n_leaves)]
    ids += [f"ring{i}" for i in range(50)] + [f"inc{c}" for c in range(n_cols)]
    labels = ["Node"] + ["Pod"] * (2 * n_leaves) + ["Service"] * 50 + ["Incident"] * n_cols
    src = ["hub"] * n_leaves + [f"leaf{i}" for i in range(n_leaves)]
    dst = [f"leaf{i}" for i in range(n_leaves)] + [f"tail{i}" for i in range(n_leaves)]
    typ = ["SCHEDULED_ON"] * n_leaves + ["HAS_EVENT"] * n_leaves
    src += [f"ring{i}" for i in range(50)]
    dst += [f"ring{(i + 1) % 50}" for i in range(50)]
    typ += ["CALLS"] * 50
    for c in range(n_cols):
        src.append(f"inc{c}")
        dst.append("hub" if c % 2 == 0 else f"ring{c}")
        typ.append("AFFECTS")
    g = EvidenceGraph()
    g.merge_nodes(ids, labels)
    g.merge_edges(src, dst, typ)
    look = g.lookup
    sv = np.concatenate([look(["hub", "leaf3", "tail7"]), look(["ring1", "ring2"]),
                         look(["hub"]), look(["ring5"])]).astype(np.uint32)
    sc = np.array([0, 0, 0, 1, 1, 2, 3], np.uint32)
    ss = np.array([0.9, 0.5, 0.7, 0.8, 0.6, 0.95, 0.4], np.float32)
    srcv = look([f"inc{c}" for c in range(n_cols)]).astype(np.uint32)
    return g, sv, sc, ss, srcv


def test_frontier_overflow_fallback_mixed():
    g, sv, sc, ss, src = _hub_world()
    fr = _check(g, sv, sc, ss, src, len(src), k=12)
    st = fr.stats()
    assert st["overflowed"] >= 1             # the hub columns went through the fallback
    assert st["overflowed"] < len(src)       # the ring columns did not


@pytest.mark.parametrize("mode", ["pool", "pruned", "pruned_wide_retry", "narrow_unpruned",
                                  "retry_grid_7", "retry_grid_7_big_hubs", "continue_64",
                                  "continue_64_big_hubs", "continue_5"])
def test_frontier_global_table_reuse(mode, monkeypatch):
    """More overflowing columns than global-variant workgroups (32): each workgroup reuses its
    table across columns and must leave it clean (wide table with a pool, narrow table pruned,
    the same with the wide-table retry on its default 512-block grid, narrow table with pruning
    switched off).  retry_grid_7: the wide retry on a 7-block persistent grid, so each block
    takes ~21 of the 150 hub columns in turn (its LDS table reused); _big_hubs: hubs past the
    wide table's 4608 members, so the retry hands every one of them on to the global variant.
    continue_64: the retry on with 64 continuation regions -- each of the first 64 overflowing
    hub columns finishes in its own workgroup, in a global-memory region, the rest go to the
    global variant; the runs repeat, so every region is reused from the state its last column
    left; _big_hubs: ~6000 members per hub column, at a region's 6144-member limit;
    continue_5: 5 regions, most hub columns find none left."""
    if mode == "narrow_unpruned":
        monkeypatch.setenv("EGRAPH_FRONTIER_NO_PRUNE", "1")
    if mode == "pruned_wide_retry":
        monkeypatch.setenv("EGRAPH_FRONTIER_WIDE_RETRY", "1")
    # retry_grid_7: ~2000 members per hub column (over the narrow table's 1152, within the
    # wide 4608); otherwise ~6000 (past both LDS tables)
    leaves = 1000 if mode in ("retry_grid_7", "continue_64", "continue_5") else 3000
    g, sv, sc, ss, src = _hub_world(n_leaves=leaves, n_cols=300)   # 150 hub columns
    if mode.startswith(("retry_grid", "continue")):
        from egraph.graph import Frontier
        real_run = Frontier.run

        def run(self, *a, **kw):                    # the retry switched on before the run
            self.set_retry(7)
            self.set_continuation(int(mode.split("_")[1]) if mode.startswith("continue") else 0)
            return real_run(self, *a, **kw)
        monkeypatch.setattr(Frontier, "run", run)
    fr = _check(g, sv, sc, ss, src, len(src), k=10, pool_entries=0 if mode == "pool" else -1,
                scores=mode == "pool")
    st = fr.stats()
    assert st["overflowed"] >= 33
    if mode == "continue_64":
        assert st["continued"] == 64 and st["global_columns"] == st["overflowed"] - 64, st
    if mode == "continue_5":
        assert st["continued"] == 5 and st["global_columns"] == st["overflowed"] - 5, st
    if mode == "continue_64_big_hubs":       # (each column ends in a region or the global variant)
        assert st["continued"] + st["global_columns"] == st["overflowed"], st


def test_frontier_edge_inputs():
    """Empty column (no source), out-of-range seeds and columns, duplicate seeds."""
    g, sv, sc, ss, src = _world(20, seed=41, pods=1000)
    V = g.num_vertices
    src = src.copy()
    src[3] = NO_NODE
    src[7] = V + 5                                  # out of range: no reach set
    sv = np.concatenate([sv, [V + 1, 0, sv[0], sv[0]]]).astype(np.uint32)
    sc = np.concatenate([sc, [0, 25, sc[0], sc[0]]]).astype(np.uint32)        # col 25 >= B
    ss = np.concatenate([ss, [0.5, 0.5, 0.01, 0.99]]).astype(np.float32)      # max-combined
    fr = _check(g, sv, sc, ss, src, 20)
    ids = fr.out_ids.view(20, 10).cpu().numpy().view(np.uint32)
    assert (ids[3] == NO_NODE).all() and (ids[7] == NO_NODE).all()


def test_frontier_no_seeds():
    g, sv, sc, ss, src = _world(9, seed=43, pods=800)
    e = np.zeros(0, np.uint32)
    _check(g, e, e, np.zeros(0, np.float32), src, 9)


def test_frontier_small_pool_still_ranks():
    """A pool too small for every column's members: top-k stays exact."""
    g, sv, sc, ss, src = _world(50, seed=47, pods=2000)
    fr = _check(g, sv, sc, ss, src, 50, pool_entries=3000, scores=False)
    assert fr.stats()["pool_used"] > 3000


def test_frontier_without_pool_ranks_identically():
    """pool_entries=-1 (top-k only): same top-k, and the read functions refuse."""
    from egraph import _lib as L
    g, sv, sc, ss, src = _world(70, seed=53, pods=1800)
    fr = _check(g, sv, sc, ss, src, 70, pool_entries=-1, scores=False)
    with pytest.raises(L.EgraphError, match="without a member pool"):
        fr.read_scores()
    with pytest.raises(L.EgraphError, match="without a member pool"):
        fr.members(0)


@pytest.mark.parametrize("hops,k,exclude", [(1, 7, None), (2, 10, None), (3, 16, -1), (4, 5, None)])
def test_frontier_pruned_last_pull_exact(hops, k, exclude):
    """Without a pool the last pull skips every member outside the candidate set and the
    expansion before it inserts no new member (reach runs two walks ahead, so the candidate
    set is final by then): top-k stays bit-identical to the oracle and fewer CSR entries are
    pulled."""
    g, sv, sc, ss, src = _world(64, seed=59, pods=2500)
    full = _check(g, sv, sc, ss, src, 64, hops=hops, k=k, exclude=exclude)
    pr = _check(g, sv, sc, ss, src, 64, hops=hops, k=k, exclude=exclude, pool_entries=-1,
                scores=False)
    fs, ps = full.stats(), pr.stats()
    # the expansion before the last pull inserts nothing new: fewer members, fewer rows
    assert ps["members"] <= fs["members"] and ps["rows"] <= fs["rows"]
    assert ps["pull_entries"] < fs["pull_entries"] if hops >= 2 else ps["pull_entries"] <= fs["pull_entries"]


def test_frontier_pruned_overflow_and_edges():
    """The pruned last pull in the global-memory variant and on empty / invalid columns."""
    g, sv, sc, ss, src = _hub_world()
    fr = _check(g, sv, sc, ss, src, len(src), k=12, pool_entries=-1, scores=False)
    assert fr.stats()["overflowed"] >= 1
    g, sv, sc, ss, src = _world(20, seed=41, pods=1000)
    src = src.copy()
    src[3] = NO_NODE
    src[7] = g.num_vertices + 5
    _check(g, sv, sc, ss, src, 20, pool_entries=-1, scores=False)


def test_frontier_bad_arguments():
    g, sv, sc, ss, src = _world(4, seed=49, pods=400)
    snap = g.snapshot()
    with pytest.raises(ValueError):
        snap.frontier(0, 10)
    with pytest.raises(ValueError):
        snap.frontier(4, 10, k=17)
    fr = snap.frontier(4, max_seeds=len(sv), k=3)
    with pytest.raises(RuntimeError):          # seeds not set (EGR_ESTATE)
        fr.run(_dev(src))
    fr.set_seeds(_dev(sv), _dev(sc), _dev(ss))
    with pytest.raises(ValueError):
        fr.run(_dev(src), hops=0)
    with pytest.raises(ValueError):
        fr.set_seeds(_dev(np.zeros(len(sv) + 1, np.uint32)), _dev(np.zeros(len(sv) + 1, np.uint32)),
                     _dev(np.zeros(len(sv) + 1, np.float32)))


def test_graph_service_rank_root_causes():
    """GraphService.rank_root_causes (drop-in API, entities / relations as the collectors emit
    them) against the oracle's propagation + reach + top-k over the same graph."""
    import asyncio

    from egraph import synth
    from egraph.seeds import seeds_for_batch
    from src.database import GraphService
    from src.services.workflow import activities
    cfg = synth.ClusterConfig(pods=1500, namespaces=5, nodes=40, deployments=150, services=100,
                              attach_fraction=0.3, seed=61)
    c = synth.build_cluster(cfg)
    cases = synth.make_incidents(c, 12, seed=62)
    synth.add_incidents(c, cases)
    GraphService.reset()
    try:
        ents = [{"id": i, "type": lab} for i, lab in zip(c.ids, c.labels)]
        rels = [{"source_id": s, "target_id": d, "relation_type": t}
                for s, d, t in zip(c.src, c.dst, c.types)]
        from src.models import GraphEntity, GraphRelation
        asyncio.run(GraphService.create_entities_batch([GraphEntity(**e) for e in ents]))
        asyncio.run(GraphService.create_relations_batch([GraphRelation(**r) for r in rels]))
        ids = [x.incident["id"] for x in cases]
        evs = [x.evidence for x in cases]
        got = asyncio.run(GraphService.rank_root_causes(ids, evs, hops=3, k=5))
        g = GraphService.graph()
        sv, sc, ss = seeds_for_batch(g, evs)
        src = g.lookup([f"incident:{i}" for i in ids]).astype(np.uint32)
        csr = g.csr()
        exp = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, len(ids), 3)
        er = oracle.reach(csr["row_ptr"], csr["col"], src, 3)
        vl, _, _, _ = g.export()
        e_ids, e_sc = oracle.topk(exp, er, vl, g.labels().index("Incident"), 5)
        for b in range(len(ids)):
            want = [(g.vertex_id(int(v)), float(s)) for v, s in zip(e_ids[b], e_sc[b])
                    if v != NO_NODE]
            assert [(r["id"], r["score"]) for r in got[b]] == want
            assert [r["rank"] for r in got[b]] == list(range(1, len(want) + 1))
        # the additive activity returns the same list for one incident
        one = asyncio.run(activities.rank_root_causes(
            {"incident": cases[3].incident, "evidence": {"evidence": evs[3]}, "k": 5}))
        assert one == got[3]
    finally:
        GraphService.reset()


def test_frontier_narrow_unpruned_world(monkeypatch):
    """The narrow table with pruning switched off (an A/B knob): many columns overflow into the
    global-memory variant, results stay exact."""
    monkeypatch.setenv("EGRAPH_FRONTIER_NO_PRUNE", "1")
    g, sv, sc, ss, src = _world(300, seed=61, pods=6000, nodes=100)
    _check(g, sv, sc, ss, src, 300, pool_entries=-1, scores=False)


def test_graph_service_concurrent_calls():
    """Concurrent rank_root_causes calls (Temporal runs activities concurrently; the ranking
    runs in worker threads) interleaved with writes on the event loop: every call returns its
    own incident's ranking, equal to the same call made alone (the shared frontier's
    seeds and output buffers were not serialised)."""
    import asyncio

    from egraph import synth
    from src.database import GraphService
    from src.models import GraphEntity, GraphRelation
    cfg = synth.ClusterConfig(pods=1200, namespaces=4, nodes=30, deployments=120, services=80,
                              attach_fraction=0.3, seed=71)
    c = synth.build_cluster(cfg)
    cases = synth.make_incidents(c, 16, seed=72)
    synth.add_incidents(c, cases)
    GraphService.reset()
    try:
        asyncio.run(GraphService.create_entities_batch(
            [GraphEntity(id=i, type=lab) for i, lab in zip(c.ids, c.labels)]))
        asyncio.run(GraphService.create_relations_batch(
            [GraphRelation(source_id=s, target_id=d, relation_type=t)
             for s, d, t in zip(c.src, c.dst, c.types)]))
        ids = [x.incident["id"] for x in cases]
        evs = [x.evidence for x in cases]
        alone = [GraphService.rank_root_causes_sync([i], [e], hops=3, k=5)[0] for i, e in zip(ids, evs)]

        async def go():
            calls = [GraphService.rank_root_causes([i], [e], hops=3, k=5) for i, e in zip(ids, evs)]
            # writes of an unconnected component between the calls: the rankings cannot change,
            # but every write forces a snapshot sync under the readers
            writes = [GraphService.create_entities_batch([GraphEntity(id=f"iso-{j}", type="Service")])
                      for j in range(8)]
            out = await asyncio.gather(*calls, *writes)
            return out[:len(calls)]
        for _ in range(3):
            got = asyncio.run(go())
            assert [g_[0] for g_ in got] == alone
    finally:
        GraphService.reset()
