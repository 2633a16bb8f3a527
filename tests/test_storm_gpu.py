"""The alert-storm pipeline (egraph/storm.py) on the GPU, tick by tick: dedup decisions equal the
oracle's webhook loop (restating src/services/ingestion/main.py:141-170 with Redis TTL), and
after every tick EVERY open incident's cached ranking is bit-identical to a from-scratch ranking
of the current graph -- so re-ranking only the affected incidents loses nothing."""
from __future__ import annotations

import numpy as np
import pytest

import alerts_oracle as AO
import oracle

pytestmark = pytest.mark.gpu


def _fresh_rankings(g, incidents, hops, k):
    from egraph.device import to_device
    from egraph.seeds import seeds_for_batch
    snap = g.snapshot()
    B = len(incidents)
    sv, sc, ss = seeds_for_batch(g, [x.evidence for x in incidents])
    fr = snap.frontier(B, max_seeds=max(len(sv), 1), k=k)
    src = np.array([x.vertex for x in incidents], np.uint32)
    fr.set_seeds(to_device(sv, snap.dev), to_device(sc, snap.dev), to_device(ss, snap.dev))
    ids, scores = fr.run(to_device(src, snap.dev), hops=hops, exclude_label=g.labels().index("Incident"))
    return ids.cpu().numpy().view(np.uint32), scores.cpu().numpy(), (sv, sc, ss, src)


def test_storm_ticks_match_full_recompute_and_oracle():
    from egraph import synth
    from egraph.graph import EvidenceGraph
    from egraph.storm import StormEngine
    # sparse enough (5 pods per node) that a tick's 3-hop neighbourhood leaves incidents out
    cfg = synth.ClusterConfig(pods=3000, namespaces=10, nodes=600, deployments=600, services=300,
                              attach_fraction=0.2, seed=77)
    c = synth.build_cluster(cfg)
    g = EvidenceGraph()
    g.merge_nodes(c.ids, c.labels)
    g.merge_edges(c.src, c.dst, c.types)
    wl = synth.StormWorkload(c, n_keys=900, seed=5, events_per_incident=10)
    ttl_s = 20
    eng = StormEngine(g, hops=3, k=8, ttl_ms=ttl_s * 1000, dedup_capacity=4096)
    store = AO.TTLStore()
    now = 1_000_000
    saw_partial = False
    log = []
    for tick in range(14):
        now += [1000, 1000, 7000, 25_000][tick % 4]
        keys = wl.alerts(60 if tick < 2 else 12)
        topo = wl.topology(4)
        before = len(eng.incidents)
        st = eng.tick(keys, now, wl.make_case, topology=topo)
        # dedup decisions = the reference's loop over a TTL store
        dup, inc, n_new = AO.webhook_loop(store, [AO.fingerprint(k_) for k_ in keys], now, ttl_s, before)
        assert st["new_incidents"] == n_new and st["duplicates"] == sum(dup)
        assert len(eng.incidents) == before + n_new
        saw_partial |= st["affected"] < st["open_incidents"]
        log.append((st["new_incidents"], st["affected"], st["open_incidents"]))
        # every cached ranking equals a full recompute on the current graph
        ids, scores, _ = _fresh_rankings(g, eng.incidents, 3, 8)
        for j, x in enumerate(eng.incidents):
            np.testing.assert_array_equal(x.top_ids, ids[j], err_msg=f"tick {tick} incident {j}")
            assert x.top_scores.tobytes() == scores[j].tobytes()
    assert saw_partial, f"expected ticks that re-rank only part of the open incidents: {log}"
    # and the full recompute equals the oracle
    ids, scores, (sv, sc, ss, src) = _fresh_rankings(g, eng.incidents, 3, 8)
    csr = g.csr()
    vl, _, _, _ = g.export()
    B = len(eng.incidents)
    exp = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, B, 3)
    er = oracle.reach(csr["row_ptr"], csr["col"], src, 3)
    e_ids, e_sc = oracle.topk(exp, er, vl, g.labels().index("Incident"), 8)
    np.testing.assert_array_equal(ids, e_ids)
    assert scores.tobytes() == e_sc.tobytes()
