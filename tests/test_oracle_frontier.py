"""The per-column CPU frontier oracle (oracle/egraph_oracle.c orc_frontier) against the dense
restatement (orc_propagate + orc_reach + orc_topk): bit-identical top-k ids and scores.  It is
bench.py's CPU baseline and the checker of the large-config GPU tests, so it is pinned here
first (CPU only)."""
from __future__ import annotations

import numpy as np
import pytest

import oracle


def _world(B, seed, pods=1500, nodes=40, scenario=None):
    from egraph import synth
    from egraph.graph import EvidenceGraph
    cfg = synth.ClusterConfig(pods=pods, namespaces=5, nodes=nodes, deployments=pods // 10,
                              services=pods // 15, attach_fraction=0.3, seed=seed)
    c = synth.build_cluster(cfg)
    cases = synth.make_incidents(c, B, seed=seed + 1, scenario=scenario)
    synth.add_incidents(c, cases)
    g = EvidenceGraph()
    g.merge_nodes(c.ids, c.labels)
    g.merge_edges(c.src, c.dst, c.types)
    sv, sc, ss = synth.seeds_for_batch(g, [x.evidence for x in cases])
    src = g.lookup([f"incident:{x.incident['id']}" for x in cases]).astype(np.uint32)
    return g, sv, sc, ss, src


def _dense(g, sv, sc, ss, src, hops, exclude, k):
    csr = g.csr()
    B = len(src)
    sco = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, B, hops)
    reach = oracle.reach(csr["row_ptr"], csr["col"], src, hops)
    vl, _, _, _ = g.export()
    return oracle.topk(sco, reach, vl, exclude, k)


def _sparse(g, sv, sc, ss, src, hops, exclude, k, threads=0, prune=True):
    csr = g.csr()
    vl, _, _, _ = g.export()
    return oracle.frontier(csr["row_ptr"], csr["col"], csr["val"], vl, sv, sc, ss, src, hops,
                           exclude, k, threads, prune)


@pytest.mark.parametrize("B,hops,k", [(1, 3, 10), (37, 3, 10), (64, 1, 5), (64, 2, 16), (50, 4, 7)])
def test_frontier_oracle_equals_dense(B, hops, k):
    g, sv, sc, ss, src = _world(B, seed=100 + B + hops)
    inc = g.labels().index("Incident")
    for exclude in (inc, -1):
        e_ids, e_sc = _dense(g, sv, sc, ss, src, hops, exclude, k)
        works = []
        for prune in (False, True):
            ids, sco, work = _sparse(g, sv, sc, ss, src, hops, exclude, k, threads=4, prune=prune)
            np.testing.assert_array_equal(ids, e_ids)
            assert sco.tobytes() == e_sc.tobytes()
            assert work[0] > 0 and work[1] > 0
            works.append(work)
        assert works[1][0] <= works[0][0]          # the pruned last hop reads fewer entries


def test_frontier_oracle_edge_inputs():
    """No source / out-of-range source, out-of-range seeds and columns, duplicates, no seeds."""
    g, sv, sc, ss, src = _world(20, seed=7, pods=800)
    V = g.num_vertices
    src = src.copy()
    src[3] = 0xFFFFFFFF
    src[7] = V + 5
    sv = np.concatenate([sv, [V + 1, 0, sv[0], sv[0]]]).astype(np.uint32)
    sc = np.concatenate([sc, [0, 25, sc[0], sc[0]]]).astype(np.uint32)
    ss = np.concatenate([ss, [0.5, 0.5, 0.01, 0.99]]).astype(np.float32)
    inc = g.labels().index("Incident")
    e_ids, e_sc = _dense(g, sv, sc, ss, src, 3, inc, 10)
    ids, sco, _ = _sparse(g, sv, sc, ss, src, 3, inc, 10)
    np.testing.assert_array_equal(ids, e_ids)
    assert sco.tobytes() == e_sc.tobytes()
    e = np.zeros(0, np.uint32)
    e_ids, e_sc = _dense(g, e, e, np.zeros(0, np.float32), src, 3, inc, 10)
    ids, sco, _ = _sparse(g, e, e, np.zeros(0, np.float32), src, 3, inc, 10)
    np.testing.assert_array_equal(ids, e_ids)
    assert sco.tobytes() == e_sc.tobytes()


def test_frontier_oracle_thread_count_invariant():
    g, sv, sc, ss, src = _world(96, seed=31, pods=3000, nodes=60)
    inc = g.labels().index("Incident")
    a = _sparse(g, sv, sc, ss, src, 3, inc, 10, threads=1)
    b = _sparse(g, sv, sc, ss, src, 3, inc, 10, threads=8)
    np.testing.assert_array_equal(a[0], b[0])
    assert a[1].tobytes() == b[1].tobytes() and a[2] == b[2]
