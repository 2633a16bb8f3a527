"""The frontier engine's locality layout (csrc/layout.hip): a snapshot lays its frontier arrays
out in egr_locality_order's vertex order, and every frontier result must be bit-identical to the
canonical layout ($EGRAPH_FRONTIER_LAYOUT=0) and to the oracle -- top-k ids (original ids,
original-id tie order) and scores, member pools, reach -- also after incremental snapshot
updates (new vertices appended to the layout) and for partition-local snapshots."""
from __future__ import annotations

import numpy as np
import pytest
import torch

import oracle

pytestmark = pytest.mark.gpu


def _dev(a):
    from egraph.device import to_device
    return to_device(np.ascontiguousarray(a), torch.device("cuda", 0))


def _world(pods=4000, B=96, seed=31):
    from egraph import synth
    cfg = synth.ClusterConfig(pods=pods, namespaces=8, nodes=60, deployments=pods // 10,
                              services=pods // 20, attach_fraction=0.35, seed=seed)
    c = synth.build_cluster(cfg)
    cases = synth.make_incidents(c, B, seed=seed + 1)
    synth.add_incidents(c, cases)
    g = synth.build_graph(c)
    sv, sc, ss = synth.seeds_for_batch(g, [x.evidence for x in cases])
    src = g.lookup([f"incident:{x.incident['id']}" for x in cases]).astype(np.uint32)
    return c, g, cases, sv, sc, ss, src


def _snap(g, monkeypatch, on: bool):
    monkeypatch.setenv("EGRAPH_FRONTIER_LAYOUT", "1" if on else "0")
    return g.snapshot()


def _run(snap, sv, sc, ss, src, inc, pool=-1, k=10):
    fr = snap.frontier(len(src), max_seeds=max(len(sv), 1), k=k, pool_entries=pool)
    fr.set_seeds(_dev(sv), _dev(sc), _dev(ss))
    ids, sco = fr.run(_dev(src), hops=3, exclude_label=inc)
    return fr, ids.cpu().numpy().view(np.uint32).copy(), sco.cpu().numpy().copy()


@pytest.mark.parametrize("pool", [-1, 0])
def test_layout_equals_canonical_and_oracle(monkeypatch, pool):
    _, g, _, sv, sc, ss, src = _world()
    inc = g.labels().index("Incident")
    on = _snap(g, monkeypatch, True)
    off = _snap(g, monkeypatch, False)
    fa, ia, sa = _run(on, sv, sc, ss, src, inc, pool)
    fb, ib, sb = _run(off, sv, sc, ss, src, inc, pool)
    np.testing.assert_array_equal(ia, ib)
    assert sa.tobytes() == sb.tobytes()
    csr = g.csr()
    vl, _, _, _ = g.export()
    e_ids, e_sc, _ = oracle.frontier(csr["row_ptr"], csr["col"], csr["val"], vl, sv, sc, ss, src,
                                     3, inc, 10)
    np.testing.assert_array_equal(ia.reshape(e_ids.shape), e_ids)
    assert sa.reshape(e_sc.shape).tobytes() == e_sc.tobytes()
    if pool == 0:
        # member pools: the same (original) vertices with the same scores and depths
        for b in range(0, len(src), 7):
            va, xa, da = fa.members(b)
            vb, xb, db = fb.members(b)
            oa, ob = np.argsort(va), np.argsort(vb)
            np.testing.assert_array_equal(va[oa], vb[ob])
            assert xa[oa].tobytes() == xb[ob].tobytes()
            np.testing.assert_array_equal(da[oa], db[ob])
        assert torch.equal(fa.read_reach(), fb.read_reach())


@pytest.mark.parametrize("per", [20, 300])
def test_layout_follows_snapshot_updates(monkeypatch, per):
    """After incremental updates (new incidents, vertices and edges MERGEd on the host and synced
    to the device) the laid-out frontier still equals a fresh snapshot and the oracle.  per=20:
    the new vertices are appended to the order (their perm / iperm filled on the device);
    per=300: the graph grows by more than a quarter, so the update recomputes the locality order
    from the current CSR and uploads it whole."""
    from egraph import synth
    # (per=300: a small cluster, so its incidents' new vertices are more than a quarter of it)
    c, g, cases, sv, sc, ss, src = _world(pods=3000 if per == 20 else 300, B=64, seed=41)
    inc = g.labels().index("Incident")
    snap = _snap(g, monkeypatch, True)
    v_start = g.num_vertices
    more = synth.make_incidents(c, 2 * per, seed=99)
    for j in range(2):
        part = more[per * j: per * j + per]
        for case in part:
            g.merge_nodes([e["id"] for e in case.entities], [e["type"] for e in case.entities])
            g.merge_edges([r["source_id"] for r in case.relations],
                          [r["target_id"] for r in case.relations],
                          [r["relation_type"] for r in case.relations])
        nv, ne = snap.sync(g)
        assert nv > 0 and ne > 0
        allc = cases + more[: per * j + per]
        if per == 300 and j == 0:
            assert g.num_vertices > 1.25 * v_start, "the re-order path needs a quarter's growth"
        sv2, sc2, ss2 = synth.seeds_for_batch(g, [x.evidence for x in allc])
        src2 = g.lookup([f"incident:{x.incident['id']}" for x in allc]).astype(np.uint32)
        _, ia, sa = _run(snap, sv2, sc2, ss2, src2, inc)
        fresh = _snap(g, monkeypatch, False)
        _, ib, sb = _run(fresh, sv2, sc2, ss2, src2, inc)
        np.testing.assert_array_equal(ia, ib, err_msg=f"update {j}")
        assert sa.tobytes() == sb.tobytes()
        csr = g.csr()
        vl, _, _, _ = g.export()
        e_ids, e_sc, _ = oracle.frontier(csr["row_ptr"], csr["col"], csr["val"], vl, sv2, sc2,
                                         ss2, src2, 3, inc, 10)
        np.testing.assert_array_equal(ia.reshape(e_ids.shape), e_ids)


def test_layout_on_partition_local_snapshot(monkeypatch):
    """Snapshot.from_csr (partition-local graphs, snapshot files) lays its frontier out too."""
    from egraph.graph import Snapshot
    _, g, _, sv, sc, ss, src = _world(pods=2500, B=48, seed=51)
    inc = g.labels().index("Incident")
    csr = g.csr()
    vl, _, _, _ = g.export()
    monkeypatch.setenv("EGRAPH_FRONTIER_LAYOUT", "1")
    s1 = Snapshot.from_csr(csr["row_ptr"], csr["col"], csr["meta"], csr["val"], vl, g.labels())
    _, ia, sa = _run(s1, sv, sc, ss, src, inc)
    e_ids, e_sc, _ = oracle.frontier(csr["row_ptr"], csr["col"], csr["val"], vl, sv, sc, ss, src,
                                     3, inc, 10)
    np.testing.assert_array_equal(ia.reshape(e_ids.shape), e_ids)
    assert sa.reshape(e_sc.shape).tobytes() == e_sc.tobytes()
