"""Incremental snapshot updates on the GPU (csrc/update.hip, egr_snapshot_update): after every
MERGE batch the device CSR -- row order, columns, types, values -- is bit-identical to the CSR a
full rebuild of the grown host graph produces (egr_graph_csr), propagation over the updated
snapshot equals the oracle, and bad deltas are rejected with the snapshot unchanged."""
from __future__ import annotations

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu


def _base(seed=5, pods=600):
    from egraph import synth
    from egraph.graph import EvidenceGraph
    cfg = synth.ClusterConfig(pods=pods, namespaces=6, nodes=20, deployments=pods // 10,
                              services=pods // 15, attach_fraction=0.3, seed=seed)
    c = synth.build_cluster(cfg)
    g = EvidenceGraph()
    g.merge_nodes(c.ids, c.labels)
    g.merge_edges(c.src, c.dst, c.types)
    return g, c


def _assert_same_csr(snap, g):
    d = snap.download()
    h = g.csr()
    vl, _, _, _ = g.export()
    assert snap.n_vertices == g.num_vertices and snap.n_entries == 2 * g.num_edges
    np.testing.assert_array_equal(d["row_ptr"], h["row_ptr"])
    np.testing.assert_array_equal(d["col"], h["col"])
    np.testing.assert_array_equal(d["meta"], h["meta"])
    assert d["val"].tobytes() == h["val"].tobytes()
    np.testing.assert_array_equal(d["vlabel"], vl)


def _random_batch(rng, g, n_new, n_edges, tag, new_types=("CALLS",)):
    ids = g.vertex_ids()
    labels = ["Incident", "Pod", "Event", "LogPattern"]
    new = [f"{tag}:{i}" for i in range(n_new)]
    nl = [labels[i % len(labels)] for i in range(n_new)]
    pool = ids + new
    # hubs get a share of the new edges (degree changes ripple into many rows' values)
    hubs = ids[:5]
    src, dst, typ = [], [], []
    types = ["OWNS", "SELECTS", "RUNS_ON", "HAS_EVENT", "AFFECTS", *new_types]
    for _ in range(n_edges):
        a = pool[rng.integers(len(pool))] if rng.random() < 0.8 else hubs[rng.integers(len(hubs))]
        b = pool[rng.integers(len(pool))]
        src.append(a)
        dst.append(b)
        typ.append(types[rng.integers(len(types))])
    # repeat some existing edges: MERGE must not create them again
    _, es, ed, et = g.export()
    rt = g.rel_types()
    for e in rng.integers(0, len(es), size=min(20, len(es))):
        src.append(ids[es[e]])
        dst.append(ids[ed[e]])
        typ.append(rt[et[e]])
    return new, nl, src, dst, typ


def test_update_matches_full_rebuild_over_many_batches():
    g, _ = _base()
    snap = g.snapshot()
    rng = np.random.default_rng(1)
    plans = []
    for it, (nn, ne) in enumerate([(0, 50), (40, 0), (30, 400), (1, 1), (200, 3000), (0, 1),
                                   (500, 20), (10, 5000)]):
        new, nl, src, dst, typ = _random_batch(rng, g, nn, ne, f"u{it}",
                                               new_types=("CALLS", f"T{it}") if it % 3 == 0 else ())
        g.merge_nodes(new, nl)
        g.merge_edges(src, dst, typ)
        v0 = snap.version
        snap.sync(g)
        assert snap.version == v0 + 1
        _assert_same_csr(snap, g)
    # a self loop and an edge to a brand-new vertex in the same batch
    g.merge_nodes(["solo"], ["Pod"])
    g.merge_edges(["solo", "solo"], ["solo", g.vertex_ids()[0]], ["CALLS", "CALLS"])
    snap.sync(g)
    _assert_same_csr(snap, g)
    del plans


def test_propagation_over_updated_snapshot_matches_oracle():
    from egraph import synth
    g, c = _base(seed=9, pods=800)
    snap = g.snapshot()
    B, k = 48, 8
    fr = snap.frontier(B, max_seeds=1 << 16, k=k)
    # the incident batch arrives as a MERGE delta (incident vertices + their evidence edges)
    cases = synth.make_incidents(c, B, seed=33)
    n0 = len(c.ids)
    e0 = len(c.src)
    synth.add_incidents(c, cases)
    g.merge_nodes(c.ids[n0:], c.labels[n0:])
    g.merge_edges(c.src[e0:], c.dst[e0:], c.types[e0:])
    snap.sync(g)
    _assert_same_csr(snap, g)
    sv, sc, ss = synth.seeds_for_batch(g, [x.evidence for x in cases])
    src = g.lookup([f"incident:{x.incident['id']}" for x in cases]).astype(np.uint32)
    from egraph.device import to_device
    dev = snap.dev
    fr.set_seeds(to_device(sv, dev), to_device(sc, dev), to_device(ss, dev))
    ids, scores = fr.run(to_device(src, dev), hops=3, exclude_label=g.labels().index("Incident"))
    csr = g.csr()
    vl, _, _, _ = g.export()
    exp = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, B, 3)
    er = oracle.reach(csr["row_ptr"], csr["col"], src, 3)
    e_ids, e_sc = oracle.topk(exp, er, vl, g.labels().index("Incident"), k)
    np.testing.assert_array_equal(ids.cpu().numpy().view(np.uint32), e_ids)
    assert scores.cpu().numpy().tobytes() == e_sc.tobytes()


def test_plans_refuse_after_update_and_frontier_outgrows():
    from egraph import _lib as L
    g, _ = _base(seed=3, pods=300)
    snap = g.snapshot()
    plan = snap.plan(8, max_seeds=16, k=4)
    fr = snap.frontier(8, max_seeds=16, k=4)
    g.merge_nodes(["x1"], ["Pod"])
    snap.sync(g)
    z = torch.zeros(1, dtype=torch.int32, device=snap.dev)
    with pytest.raises(L.EgraphError, match="updated after this plan"):
        plan.set_seeds(z, z, z.float())
    fr.set_seeds(z, z, z.float())          # within the frontier's headroom: still valid
    grow = fr.max_vertices - snap.n_vertices + 1
    g.merge_nodes([f"y{i}" for i in range(grow)], ["Pod"] * grow)
    snap.sync(g)
    with pytest.raises(L.EgraphError, match="grew past"):
        fr.set_seeds(z, z, z.float())


def test_bad_deltas_are_rejected_and_leave_the_snapshot_unchanged():
    from egraph.device import to_device
    g, _ = _base(seed=4, pods=300)
    snap = g.snapshot()
    before = snap.download()
    dev = snap.dev
    _, es, ed, et = g.export()
    w = g.weight_array()
    u8 = lambda a: to_device(np.asarray(a, np.uint8), dev)       # noqa: E731
    u32 = lambda a: to_device(np.asarray(a, np.uint32), dev)     # noqa: E731
    # an edge already in the snapshot
    with pytest.raises(ValueError, match="already in the snapshot"):
        snap.update(u8([]), u32([es[3]]), u32([ed[3]]), u8([et[3]]), w)
    # the same new edge twice in one delta
    with pytest.raises(ValueError, match="already in the snapshot"):
        snap.update(u8([]), u32([0, 0]), u32([1, 1]), u8([60, 60]), w)
    # endpoint beyond the grown vertex count
    with pytest.raises(ValueError, match="out of range"):
        snap.update(u8([1]), u32([0]), u32([snap.n_vertices + 1]), u8([0]), w)
    after = snap.download()
    for k in before:
        assert before[k].tobytes() == after[k].tobytes()
    assert snap.version == 0


def test_graph_service_reads_after_writes_use_incremental_sync():
    """Writes after the first read reach the device by incremental updates of the same
    snapshot; ranking afterwards equals the oracle over the grown graph."""
    import asyncio

    from egraph import synth
    from egraph.seeds import seeds_for_batch
    from src.database.graph import GraphService as GS
    from src.models import GraphEntity, GraphRelation
    cfg = synth.ClusterConfig(pods=900, namespaces=4, nodes=30, deployments=90, services=60,
                              attach_fraction=0.3, seed=71)
    c = synth.build_cluster(cfg)
    GS.reset()
    run = asyncio.run
    try:
        def write(lo_n, lo_e):
            run(GS.create_entities_batch([GraphEntity(id=i, type=t)
                                          for i, t in zip(c.ids[lo_n:], c.labels[lo_n:])]))
            run(GS.create_relations_batch([GraphRelation(source_id=s_, target_id=d, relation_type=t)
                                           for s_, d, t in zip(c.src[lo_e:], c.dst[lo_e:], c.types[lo_e:])]))
        write(0, 0)
        first = synth.make_incidents(c, 6, seed=72)
        n0, e0 = len(c.ids), len(c.src)
        synth.add_incidents(c, first)
        write(n0, e0)
        ids1 = [x.incident["id"] for x in first]
        GS.rank_root_causes_sync(ids1, [x.evidence for x in first], k=5)
        snap = GS._snapshot
        v0 = snap.version
        second = synth.make_incidents(c, 10, seed=73)
        n1, e1 = len(c.ids), len(c.src)
        synth.add_incidents(c, second)
        write(n1, e1)
        cases = first + second
        ids = [x.incident["id"] for x in cases]
        evs = [x.evidence for x in cases]
        got = GS.rank_root_causes_sync(ids, evs, k=5)
        assert GS._snapshot is snap and snap.version == v0 + 1
        g = GS.graph()
        _assert_same_csr(snap, g)
        sv, sc, ss = seeds_for_batch(g, evs)
        src = g.lookup([f"incident:{i}" for i in ids]).astype(np.uint32)
        csr = g.csr()
        exp = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, len(ids), 3)
        er = oracle.reach(csr["row_ptr"], csr["col"], src, 3)
        vl, _, _, _ = g.export()
        e_ids, e_sc = oracle.topk(exp, er, vl, g.labels().index("Incident"), 5)
        for b in range(len(ids)):
            want = [(g.vertex_id(int(v)), float(s_)) for v, s_ in zip(e_ids[b], e_sc[b])
                    if v != 0xFFFFFFFF]
            assert [(r["id"], r["score"]) for r in got[b]] == want
        nodes = GS.get_incident_graphs([f"incident:{ids[-1]}"], 1)[0]["nodes"]
        assert any(n["properties"]["id"] == f"incident:{ids[-1]}" for n in nodes)
    finally:
        GS.reset()


def test_snapshot_file_roundtrip_from_the_device(tmp_path):
    """Checkpoint an updated device snapshot (egraph/snapfile.py), upload it elsewhere without
    the host graph: identical CSR; restore the host graph: identical again after a sync."""
    from egraph import snapfile
    g, _ = _base(seed=6, pods=500)
    snap = g.snapshot()
    rng = np.random.default_rng(2)
    new, nl, src, dst, typ = _random_batch(rng, g, 50, 600, "ck")
    g.merge_nodes(new, nl)
    g.merge_edges(src, dst, typ)
    snap.sync(g)
    p = tmp_path / "ck.egrsnap"
    snapfile.save(p, g, snapshot=snap)
    loaded = snapfile.load_snapshot(p)
    a, b = snap.download(), loaded.download()
    for k in a:
        assert a[k].tobytes() == b[k].tobytes()
    g2 = snapfile.load_graph(p)
    s2 = g2.snapshot()
    c = s2.download()
    for k in a:
        assert a[k].tobytes() == c[k].tobytes()
