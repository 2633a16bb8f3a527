"""GPU parity of the graph stages: reach (A8), propagation (A9), top-k.

Reach sets are exact against a per-column BFS (oracle) and hand-built known answers of
APOC subgraphAll semantics; propagated scores are compared BIT-FOR-BIT with the C oracle (both
accumulate with fmaf in CSR order), which is far inside the north star's 1e-5 relative bar;
top-k ids and scores are exact.
"""
from __future__ import annotations

import asyncio

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu


def _small_world(B, seed=11, pods=3000):
    from egraph import synth
    from egraph.graph import EvidenceGraph
    cfg = synth.ClusterConfig(pods=pods, namespaces=6, nodes=60, deployments=300, services=200,
                              attach_fraction=0.3, seed=seed)
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


# B spans every reach row width: RG = 1 (B <= 128), 2, 4, 8, 16, 32 and 64 lanes x 16 B
@pytest.mark.parametrize("B", [1, 5, 16, 37, 64, 130, 257, 600, 1100, 2100, 4200])
def test_propagation_reach_topk_equal_oracle(B):
    g, sv, sc, ss, src = _small_world(B, pods=3000 if B <= 600 else 800)
    snap = g.snapshot()
    plan = snap.plan(B, max_seeds=len(sv), k=10)
    plan.set_seeds(_dev(sv), _dev(sc), _dev(ss))
    plan.set_sources(_dev(src))
    inc_label = g.labels().index("Incident")
    ids, scores = plan.run(hops=3, exclude_label=inc_label)
    got_scores = plan.read_scores().cpu().numpy()
    got_reach = plan.read_reach().cpu().numpy().view(np.uint64)
    torch.cuda.synchronize()
    csr = g.csr()
    exp_scores = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, B, 3)
    assert got_scores.tobytes() == exp_scores.tobytes()           # bit-identical
    exp_reach = oracle.reach(csr["row_ptr"], csr["col"], src, 3)
    np.testing.assert_array_equal(got_reach, exp_reach)
    vl, _, _, _ = g.export()
    e_ids, e_sc = oracle.topk(exp_scores, exp_reach, vl, inc_label, 10)
    np.testing.assert_array_equal(ids.cpu().numpy().view(np.uint32), e_ids)
    np.testing.assert_array_equal(scores.cpu().numpy(), e_sc)


@pytest.mark.parametrize("B", [37, 600])
def test_zero_tile_skip_off_is_bit_identical(B, monkeypatch):
    """The hop's zero-tile skip (live-entry compaction by the input's tile flags, and by the
    seed tile masks in the first hop) against the full gather ($EGRAPH_HOP_NO_SKIP=1, read at
    plan creation): the same scores bit for bit, both equal to the oracle."""
    g, sv, sc, ss, src = _small_world(B, seed=5, pods=1500)
    snap = g.snapshot()
    got = []
    for off in (False, True):
        if off:
            monkeypatch.setenv("EGRAPH_HOP_NO_SKIP", "1")
        plan = snap.plan(B, max_seeds=len(sv), k=5)
        plan.set_seeds(_dev(sv), _dev(sc), _dev(ss))
        plan.set_sources(_dev(src))
        plan.run(hops=4)
        got.append(plan.read_scores().cpu().numpy())
    csr = g.csr()
    exp = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, B, 4)
    assert got[0].tobytes() == exp.tobytes() and got[1].tobytes() == exp.tobytes()


def _hub_world(n=5000):
    from egraph.graph import EvidenceGraph
    g = EvidenceGraph()
    g.merge_nodes([f"p{i}" for i in range(n)] + ["hub", "inc"], ["Pod"] * n + ["Node", "Incident"])
    g.merge_edges([f"p{i}" for i in range(n)] + ["inc"], ["hub"] * n + ["p0"],
                  ["SCHEDULED_ON"] * n + ["AFFECTS"])
    return g


@pytest.mark.parametrize("world", ["small", "hub"])
def test_reused_plan_reads_no_stale_tiles(world):
    """The hop does not store a row tile that came out all +0 (and holds no seed of the row):
    such a tile keeps whatever an earlier run left in it, and every reader goes through the tile
    flags.  A plan run first with seeds in every tile, then with seeds in the first tile only,
    must give the second run's scores, top-k (candidate lists and full scan) and packed rows
    exactly as a fresh plan / the oracle do -- including the hub row longer than the 2048-entry
    LDS stage, whose gathers are not compacted ("hub")."""
    B = 300                                                     # three 128-column tiles
    rng = np.random.default_rng(7)
    if world == "small":
        g, sv, sc, ss, src = _small_world(B, seed=17, pods=1500)
    else:
        g = _hub_world()
        n = 5000
        sv = rng.integers(0, n, 4000).astype(np.uint32)
        sc = rng.integers(0, B, 4000).astype(np.uint32)
        ss = rng.random(4000).astype(np.float32)
        src = np.full(B, n + 1, np.uint32)
    first = sc < 128                                            # the second run: tile 0 only
    sv2, sc2, ss2 = sv[first], sc[first], ss[first]
    assert len(sv2) and (~first).any()
    snap = g.snapshot()
    plan = snap.plan(B, max_seeds=len(sv), k=6)
    assert plan.tile_width == 128
    for vv, cc, s_ in ((sv, sc, ss), (sv2, sc2, ss2)):
        plan.set_seeds(_dev(vv), _dev(cc), _dev(s_))
        plan.set_sources(_dev(src))
        ids, scores = plan.run(hops=3)
    csr = g.csr()
    exp = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv2, sc2, ss2, B, 3)
    assert plan.read_scores().cpu().numpy().tobytes() == exp.tobytes()
    er = oracle.reach(csr["row_ptr"], csr["col"], src, 3)
    vl, _, _, _ = g.export()
    eids, esc = oracle.topk(exp, er, vl, -1, 6)
    np.testing.assert_array_equal(ids.cpu().numpy().view(np.uint32), eids)
    np.testing.assert_array_equal(scores.cpu().numpy(), esc)
    inc = g.labels().index("Incident")
    ids2, sc_2 = plan.topk(exclude_label=inc)                   # (no lists for it: the full scan)
    eids2, esc2 = oracle.topk(exp, er, vl, inc, 6)
    np.testing.assert_array_equal(ids2.cpu().numpy().view(np.uint32), eids2)
    np.testing.assert_array_equal(sc_2.cpu().numpy(), esc2)
    rows = np.sort(rng.choice(exp.shape[0], size=64, replace=False)).astype(np.uint32)
    out = torch.empty((64, 384), dtype=torch.float32, device="cuda")
    plan.pack_scores(_dev(rows), out)
    torch.cuda.synchronize()
    packed = out.cpu().numpy()[:, :B]
    assert packed.tobytes() == np.ascontiguousarray(exp[rows]).tobytes()


@pytest.mark.parametrize("tw", [4, 16, 64, 128])
def test_tile_width_override(tw, monkeypatch):
    B = 200
    monkeypatch.setenv("EGRAPH_TILE_WIDTH", str(tw))
    g, sv, sc, ss, src = _small_world(B, seed=31, pods=1500)
    plan = g.snapshot().plan(B, max_seeds=len(sv), k=6)
    assert plan.tile_width == tw
    plan.set_seeds(_dev(sv), _dev(sc), _dev(ss))
    plan.set_sources(_dev(src))
    inc = g.labels().index("Incident")
    ids, scores = plan.run(hops=3, exclude_label=inc)
    csr = g.csr()
    exp = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, B, 3)
    assert plan.read_scores().cpu().numpy().tobytes() == exp.tobytes()
    er = oracle.reach(csr["row_ptr"], csr["col"], src, 3)
    np.testing.assert_array_equal(plan.read_reach().cpu().numpy().view(np.uint64), er)
    vl, _, _, _ = g.export()
    eids, esc = oracle.topk(exp, er, vl, inc, 6)
    np.testing.assert_array_equal(ids.cpu().numpy().view(np.uint32), eids)
    np.testing.assert_array_equal(scores.cpu().numpy(), esc)
    # the full-scan top-k path (no candidate lists) must agree too
    ids2, sc2 = plan.topk(exclude_label=-1)
    eids2, esc2 = oracle.topk(exp, er, vl, -1, 6)
    np.testing.assert_array_equal(ids2.cpu().numpy().view(np.uint32), eids2)
    np.testing.assert_array_equal(sc2.cpu().numpy(), esc2)


@pytest.mark.parametrize("B", [64, 128])
def test_step_equals_hop_plus_reach_hop(B):
    g, sv, sc, ss, src = _small_world(B, seed=21, pods=2000)
    csr = g.csr()
    exp = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, B, 3)
    exp_r = oracle.reach(csr["row_ptr"], csr["col"], src, 3)
    snap = g.snapshot()
    for fused in (False, True):
        plan = snap.plan(B, max_seeds=len(sv), k=4)
        plan.set_seeds(_dev(sv), _dev(sc), _dev(ss))
        plan.set_sources(_dev(src))
        for _ in range(3):
            if fused:
                plan.step()
            else:
                plan.hop()
                plan.reach_hop()
        assert plan.read_scores().cpu().numpy().tobytes() == exp.tobytes()
        np.testing.assert_array_equal(plan.read_reach().cpu().numpy().view(np.uint64), exp_r)


@pytest.mark.parametrize("exclude", [-1, "Incident", "Pod"])
def test_candidates_entry_point_and_exclusions(exclude):
    """hop/reach_hop driven by the caller, then candidates() + topk(): same as the oracle for
    every exclusion (candidate lists are rebuilt when the exclusion changes)."""
    B = 150
    g, sv, sc, ss, src = _small_world(B, seed=41, pods=1200)
    ex = g.labels().index(exclude) if isinstance(exclude, str) else exclude
    plan = g.snapshot().plan(B, max_seeds=len(sv), k=7)
    plan.set_seeds(_dev(sv), _dev(sc), _dev(ss))
    plan.set_sources(_dev(src))
    for _ in range(3):
        plan.hop()
        plan.reach_hop()
    plan.candidates(ex)
    ids, scores = plan.topk(ex)
    csr = g.csr()
    exp = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, B, 3)
    er = oracle.reach(csr["row_ptr"], csr["col"], src, 3)
    vl, _, _, _ = g.export()
    eids, esc = oracle.topk(exp, er, vl, ex, 7)
    np.testing.assert_array_equal(ids.cpu().numpy().view(np.uint32), eids)
    np.testing.assert_array_equal(scores.cpu().numpy(), esc)
    # a different exclusion than the lists were built for falls back to the full scan
    other = -1 if ex != -1 else g.labels().index("Incident")
    ids2, sc2 = plan.topk(other)
    eids2, esc2 = oracle.topk(exp, er, vl, other, 7)
    np.testing.assert_array_equal(ids2.cpu().numpy().view(np.uint32), eids2)
    np.testing.assert_array_equal(sc2.cpu().numpy(), esc2)


def test_hub_rows_longer_than_the_lds_stage():
    """A vertex whose CSR row exceeds the 2048 staged entries takes the global-read path."""
    n = 5000
    g = _hub_world(n)
    B = 64
    rng = np.random.default_rng(0)
    sv = rng.integers(0, n, 3000).astype(np.uint32)
    sc = rng.integers(0, B, 3000).astype(np.uint32)
    ss = rng.random(3000).astype(np.float32)
    src = np.full(B, n + 1, np.uint32)
    plan = g.snapshot().plan(B, max_seeds=len(sv), k=8)
    plan.set_seeds(_dev(sv), _dev(sc), _dev(ss))
    plan.set_sources(_dev(src))
    ids, _ = plan.run(hops=3)
    csr = g.csr()
    exp = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, B, 3)
    assert plan.read_scores().cpu().numpy().tobytes() == exp.tobytes()
    er = oracle.reach(csr["row_ptr"], csr["col"], src, 3)
    vl, _, _, _ = g.export()
    eids, _ = oracle.topk(exp, er, vl, -1, 8)
    np.testing.assert_array_equal(ids.cpu().numpy().view(np.uint32), eids)


@pytest.mark.parametrize("hops", [1, 2, 4])
def test_hop_counts(hops):
    B = 20
    g, sv, sc, ss, src = _small_world(B, seed=3, pods=1500)
    plan = g.snapshot().plan(B, max_seeds=len(sv), k=5)
    plan.set_seeds(_dev(sv), _dev(sc), _dev(ss))
    plan.set_sources(_dev(src))
    plan.run(hops=hops)
    csr = g.csr()
    exp = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, B, hops)
    assert plan.read_scores().cpu().numpy().tobytes() == exp.tobytes()
    np.testing.assert_array_equal(plan.read_reach().cpu().numpy().view(np.uint64),
                                  oracle.reach(csr["row_ptr"], csr["col"], src, hops))


def test_duplicate_and_invalid_seeds_are_max_combined():
    from egraph.graph import EvidenceGraph
    g = EvidenceGraph()
    g.merge_nodes(["a", "b", "c"], ["Pod", "Pod", "Node"])
    g.merge_edges(["a", "b"], ["c", "c"], ["SCHEDULED_ON", "SCHEDULED_ON"])
    sv = np.array([0, 0, 1, 7, 2], np.uint32)          # vertex 7 does not exist: dropped
    sc = np.array([0, 0, 1, 0, 9], np.uint32)          # column 9 >= B: dropped
    ss = np.array([0.25, 0.75, 0.5, 1.0, 1.0], np.float32)
    plan = g.snapshot().plan(2, max_seeds=5, k=3)
    plan.set_seeds(_dev(sv), _dev(sc), _dev(ss))
    plan.set_sources(_dev(np.array([0, 1], np.uint32)))
    plan.run(hops=2)
    csr = g.csr()
    exp = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, 2, 2)
    assert plan.read_scores().cpu().numpy().tobytes() == exp.tobytes()


def test_reach_known_answers_apoc_semantics():
    """subgraphAll(maxLevel=3): undirected, all types, start node included, shared pods link
    incidents (Incident -> Pod <- Incident' -> Pod')."""
    from egraph.graph import EvidenceGraph
    g = EvidenceGraph()
    g.create_entities_batch([
        {"id": "incident:1", "type": "Incident"}, {"id": "incident:2", "type": "Incident"},
        {"id": "pod:p1", "type": "Pod"}, {"id": "pod:p2", "type": "Pod"},
        {"id": "pod:p3", "type": "Pod"}, {"id": "node:n1", "type": "Node"},
        {"id": "deployment:d", "type": "Deployment"}, {"id": "change:c", "type": "ChangeEvent"}])
    g.create_relations_batch([
        {"source_id": "incident:1", "target_id": "pod:p1", "relation_type": "AFFECTS"},
        {"source_id": "incident:2", "target_id": "pod:p1", "relation_type": "AFFECTS"},
        {"source_id": "incident:2", "target_id": "pod:p2", "relation_type": "AFFECTS"},
        {"source_id": "pod:p2", "target_id": "node:n1", "relation_type": "SCHEDULED_ON"},
        {"source_id": "pod:p3", "target_id": "node:n1", "relation_type": "SCHEDULED_ON"},
        {"source_id": "deployment:d", "target_id": "change:c", "relation_type": "HAS_RECENT_CHANGE"},
        {"source_id": "pod:p3", "target_id": "node:missing", "relation_type": "SCHEDULED_ON"}])
    plan = g.snapshot().plan(2, max_seeds=0, k=1)
    plan.set_sources(_dev(g.lookup(["incident:1", "incident:2"]).astype(np.uint32)))
    for _ in range(3):
        plan.reach_hop()
    bits = plan.read_reach().cpu().numpy().view(np.uint64)[0]
    members = lambda b: {g.vertex_id(v) for v in range(g.num_vertices) if bits[v] >> b & 1}  # noqa
    assert members(0) == {"incident:1", "pod:p1", "incident:2", "pod:p2"}
    assert members(1) == {"incident:2", "pod:p1", "pod:p2", "incident:1", "node:n1", "pod:p3"}


def test_graph_service_get_incident_graph():
    from src.database import GraphService
    from src.models import GraphEntity, GraphRelation
    GraphService.reset()
    ents = [GraphEntity(id="incident:42", type="Incident", properties={"id": "42", "title": "t"}),
            GraphEntity(id="pod:ns:a", type="Pod", properties={"phase": "Running"}),
            GraphEntity(id="node:n", type="Node", properties={"ready": False}),
            GraphEntity(id="pod:ns:b", type="Pod"), GraphEntity(id="pod:ns:far", type="Pod"),
            GraphEntity(id="deployment:ns:x", type="Deployment")]
    rels = [GraphRelation(source_id="incident:42", target_id="pod:ns:a", relation_type="AFFECTS"),
            GraphRelation(source_id="pod:ns:a", target_id="node:n", relation_type="SCHEDULED_ON",
                          properties={"w": 1}),
            GraphRelation(source_id="pod:ns:b", target_id="node:n", relation_type="SCHEDULED_ON"),
            GraphRelation(source_id="deployment:ns:x", target_id="pod:ns:b", relation_type="OWNS"),
            GraphRelation(source_id="deployment:ns:x", target_id="pod:ns:far", relation_type="OWNS")]
    assert asyncio.run(GraphService.create_entities_batch(ents)) == 6
    assert asyncio.run(GraphService.create_relations_batch(rels)) == 5
    out = asyncio.run(GraphService.get_incident_graph("incident:42", depth=3))
    assert {n["id"] for n in out["nodes"]} == {"incident:42", "pod:ns:a", "node:n", "pod:ns:b"}
    inc = next(n for n in out["nodes"] if n["id"] == "incident:42")
    assert inc["labels"] == ["Incident"] and inc["properties"]["title"] == "t"
    assert {(r["type"], r["source"], r["target"]) for r in out["relationships"]} == {
        ("AFFECTS", "incident:42", "pod:ns:a"), ("SCHEDULED_ON", "pod:ns:a", "node:n"),
        ("SCHEDULED_ON", "pod:ns:b", "node:n")}
    assert asyncio.run(GraphService.get_incident_graph("42")) == {"nodes": [], "relationships": []}
    assert len(asyncio.run(GraphService.get_incident_graph("42", resolve_bare_uuid=True))["nodes"]) == 4
    d4 = asyncio.run(GraphService.get_incident_graph("incident:42", depth=4))
    assert {n["id"] for n in d4["nodes"]} == {"incident:42", "pod:ns:a", "node:n", "pod:ns:b",
                                              "deployment:ns:x"}
    GraphService.reset()
