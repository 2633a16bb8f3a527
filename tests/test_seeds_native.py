"""The native seed-candidate extraction (csrc/pyhost.c seed_candidates behind
egraph.seeds.SeedCandidates) against its Python statement (egraph.seeds.candidates_py): the same
candidate ids, counts, columns and strengths on collector-shaped evidence and on edge rows, and
the same exception where the statement raises."""
from __future__ import annotations

import math
import random

import numpy as np
import pytest


def _both(lists):
    from egraph import _lib
    from egraph.seeds import _row, candidates_py
    f, c, o, v = _lib.pyhost.seed_candidates(lists, _row)
    a = (f, np.frombuffer(c, np.int64).tolist(), np.frombuffer(o, np.uint32).tolist(),
         np.frombuffer(v, np.float64).tolist())
    b = candidates_py(lists)
    return a, b


def _same(a, b):
    fa, ca, cola, va = a
    fb, cb, colb, vb = b
    assert fa == fb and ca == cb and cola == colb
    assert len(va) == len(vb)
    for x, y in zip(va, vb):
        assert (math.isnan(x) and math.isnan(y)) or x == y


class _D(dict):
    pass


EDGE = [
    {"evidence_type": "kubernetes_event", "entity_namespace": "ns", "entity_name": "e",
     "data": {"involved_object": {"kind": "Node", "name": "n1"}}},
    {"evidence_type": "kubernetes_event", "entity_namespace": "ns", "entity_name": "e",
     "data": {"involved_object": {"kind": "Pod", "name": "p", "namespace": "other"}}},
    {"evidence_type": "kubernetes_event", "entity_namespace": "ns", "entity_name": "e",
     "data": {"involved_object": {"kind": None}}},
    {"evidence_type": "kubernetes_event", "entity_namespace": "ns", "entity_name": "e",
     "data": {"involved_object": {}}},
    {"evidence_type": "kubernetes_event", "entity_namespace": "ns", "entity_name": "e", "data": {}},
    {"evidence_type": "kubernetes_event", "entity_namespace": "ns", "entity_name": "e", "data": None},
    {"evidence_type": "kubernetes_event", "entity_namespace": "ns", "entity_name": "e",
     "data": {"involved_object": {"kind": 7, "name": 3, "namespace": None}}},
    {"evidence_type": "kubernetes_event", "entity_name": "e", "data": {"involved_object": None}},
    {"evidence_type": "kubernetes_event", "entity_namespace": "ns", "entity_name": "e",
     "data": {"involved_object": _D(kind="Deployment", name="d")}},
    {"evidence_type": "kubernetes_event", "entity_namespace": "ns", "entity_name": "e", "data": ""},
    {"evidence_type": "kubernetes_pod", "entity_namespace": None, "entity_name": 5},
    {"evidence_type": "kubernetes_pod", "entity_namespace": "ns", "entity_name": "p",
     "signal_strength": 0},
    {"evidence_type": "kubernetes_pod", "entity_namespace": "ns", "entity_name": "p",
     "signal_strength": -0.5},
    {"evidence_type": "kubernetes_pod", "entity_namespace": "ns", "entity_name": "p",
     "signal_strength": float("nan")},
    {"evidence_type": "kubernetes_pod", "entity_namespace": "ns", "entity_name": "p",
     "signal_strength": "0.7"},
    {"evidence_type": "kubernetes_pod", "entity_namespace": "ns", "entity_name": "p",
     "signal_strength": True},
    {"evidence_type": "kubernetes_pod", "entity_namespace": "ns", "entity_name": "p",
     "signal_strength": 2},
    {"evidence_type": "log_signal", "entity_namespace": "ns", "entity_name": "svc"},
    {"evidence_type": "metric_signal", "entity_namespace": 1.5, "entity_name": False},
    {"evidence_type": "kubernetes_node", "entity_name": "n"},
    {"evidence_type": "kubernetes_hpa", "entity_namespace": "ns", "entity_name": "h"},
    {"evidence_type": "config_change", "entity_namespace": "ns", "entity_name": "c"},
    {"evidence_type": "image_change", "entity_namespace": "ns", "entity_name": "d"},
    {"evidence_type": "deploy_change", "entity_namespace": "ns", "entity_name": "d"},
    {"evidence_type": "kubernetes_deployment", "entity_namespace": "ns", "entity_name": "d"},
    {"evidence_type": "unknown_kind", "entity_namespace": "ns", "entity_name": "x"},
    {"entity_namespace": "ns", "entity_name": "x"},
    _D(evidence_type="kubernetes_pod", entity_namespace="ns", entity_name="sub"),
    {"evidence_type": "kubernetes_pod", "entity_namespace": ["l"], "entity_name": "p"},
]


def test_native_matches_python_on_collector_evidence():
    from egraph import synth
    c = synth.build_cluster(synth.ClusterConfig(pods=1500, namespaces=5, nodes=40,
                                                deployments=150, services=100, seed=9))
    lists = [x.evidence for x in synth.make_incidents(c, 120, seed=10)]
    a, b = _both(lists)
    _same(a, b)
    assert len(a[0]) > 5000


def test_native_matches_python_on_edge_rows():
    rng = random.Random(3)
    lists = [EDGE, [], EDGE[::-1]] + [rng.sample(EDGE, 8) for _ in range(20)]
    a, b = _both(lists)
    _same(a, b)


@pytest.mark.parametrize("threads", [2, 4, 7])
def test_seed_keys_all_rows_on_the_workers(threads):
    """Collector rows only (none handed over): seed_keys assembles its output by concatenating the
    workers' arrays -- the same blob, offsets, hashes, counts, columns and strengths as
    SeedCandidates, for job splits that cut the batch at different lists."""
    from egraph import _lib, synth
    from egraph.graph import str_blob
    from egraph.seeds import SeedCandidates, _row
    c = synth.build_cluster(synth.ClusterConfig(pods=1500, namespaces=5, nodes=40,
                                                deployments=150, services=100, seed=9))
    lists = [x.evidence for x in synth.make_incidents(c, 150, seed=11)]
    lists[3] = []                                   # an empty list inside a job
    sc = SeedCandidates(lists)
    blob, off, hs, count, col, val = _lib.pyhost.seed_keys(lists, _row, threads)
    b, o = str_blob(sc.flat)
    assert blob == b and np.array_equal(np.frombuffer(off, np.int64), o)
    assert np.array_equal(np.frombuffer(hs, np.int64), np.frombuffer(_lib.pyhost.hash_ids(sc.flat), np.int64))
    assert np.array_equal(np.frombuffer(count, np.int64), sc.count)
    assert np.array_equal(np.frombuffer(col, np.uint32), sc.col)
    assert np.array_equal(np.frombuffer(val, np.float32), sc.val, equal_nan=True)


@pytest.mark.parametrize("bad", [
    {"evidence_type": "kubernetes_pod", "entity_namespace": "ns", "entity_name": "p",
     "signal_strength": "x"},                                      # float("x"): ValueError
    {"evidence_type": "kubernetes_pod", "entity_namespace": "ns", "entity_name": "p",
     "signal_strength": None},                                     # float(None): TypeError
    {"evidence_type": "kubernetes_event", "entity_namespace": "ns", "entity_name": "e",
     "data": {"involved_object": ["x"]}},                          # list.get: AttributeError
    ["not", "a", "dict"],                                          # list.get: AttributeError
    {"evidence_type": "kubernetes_pod", "entity_namespace": "ns", "entity_name": "p",
     "signal_strength": 10 ** 400},                                # float(huge): OverflowError
])
def test_native_raises_like_python(bad):
    from egraph import _lib
    from egraph.seeds import _row, candidates_py
    with pytest.raises(Exception) as e1:
        candidates_py([[bad]])
    with pytest.raises(Exception) as e2:
        _lib.pyhost.seed_candidates([[bad]], _row)
    assert type(e1.value) is type(e2.value)


def test_seed_candidates_attach_unchanged():
    from egraph import synth
    from egraph.seeds import SeedCandidates, candidates_py
    c = synth.build_cluster(synth.ClusterConfig(pods=800, namespaces=4, nodes=20,
                                                deployments=80, services=60, seed=5))
    cases = synth.make_incidents(c, 30, seed=6)
    synth.add_incidents(c, cases)
    g = synth.build_graph(c)
    lists = [x.evidence for x in cases]
    sc = SeedCandidates(lists)
    flat, count, col, val = candidates_py(lists)
    assert sc.flat == flat and sc.count.tolist() == count
    p1, p2 = [], []
    a = sc.attach(g, p1)
    b = sc.attach_found(g.lookup(sc.flat), p2)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    assert p1 == p2


def test_per_column_and_combined_attach_match_one_incident_at_a_time():
    """The storm's batched reseed (egraph/storm.py _reseed): candidates of many incidents from
    one native pass (SeedCandidates.per_column) and one attach over all of them (combine) give
    each incident the seeds and pending ids of its own SeedCandidates([evidence]).attach."""
    import numpy as np
    from egraph import synth
    from egraph.seeds import SeedCandidates
    cl = synth.build_cluster(synth.ClusterConfig(pods=600, namespaces=4, nodes=12,
                                                 deployments=60, services=40, seed=3))
    lists = [c.evidence for c in synth.make_incidents(cl, 40, seed=5)] + [[]]
    per = SeedCandidates.per_column(lists)
    rng = np.random.default_rng(0)
    singles = [SeedCandidates([ev]) for ev in lists]
    for p, s in zip(per, singles):
        assert p.flat == s.flat and np.array_equal(p.count, s.count)
        assert np.array_equal(p.val, s.val) and np.array_equal(p.col, s.col)
    found_one = [rng.integers(-1, 50, len(s.flat)) for s in singles]   # -1 = not in the graph
    comb = SeedCandidates.combine(per)
    pend: list = []
    sv, col, ss = comb.attach_found(np.concatenate(found_one) if comb.flat else np.zeros(0, np.int64), pend)
    cut = np.searchsorted(col, np.arange(len(lists) + 1, dtype=np.uint32))
    for j, s in enumerate(singles):
        p1: list = []
        v1, _, s1 = s.attach_found(found_one[j], p1)
        assert np.array_equal(sv[cut[j]:cut[j + 1]], v1) and np.array_equal(ss[cut[j]:cut[j + 1]], s1)
        assert pend[j] == p1[0]


def test_attach_found_idx_matches_pending_sets():
    """The storm's hashed pending index is fed by attach_found_idx: its (flat index, column)
    pairs name exactly the candidate ids attach_found puts in each column's pending set."""
    import numpy as np
    from egraph import synth
    from egraph.seeds import SeedCandidates
    cl = synth.build_cluster(synth.ClusterConfig(pods=600, namespaces=4, nodes=12,
                                                 deployments=60, services=40, seed=3))
    lists = [c.evidence for c in synth.make_incidents(cl, 30, seed=9)]
    sc = SeedCandidates(lists)
    found = np.random.default_rng(1).integers(-1, 40, len(sc.flat))
    pend: list = []
    v1, c1, s1 = sc.attach_found(found, pend)
    v2, c2, s2, before, bcol = sc.attach_found_idx(found)
    assert np.array_equal(v1, v2) and np.array_equal(c1, c2) and np.array_equal(s1, s2)
    got = [set() for _ in lists]
    for i, c in zip(before, bcol):
        got[int(c)].add(sc.flat[int(i)])
    assert got == pend


def test_storm_pending_index_lookup():
    """StormEngine._pending_hit over the pending index (PendingIndex: hash-sorted runs, merged
    past MAX_RUNS) with duplicate hashes and retired generations (host logic only; no device)."""
    import types
    import numpy as np
    from egraph.storm import StormEngine
    rng = np.random.default_rng(4)
    ids = [f"pod/ns/p{i}" for i in range(300)]
    ent = [(ids[int(rng.integers(300))], int(rng.integers(40)), int(rng.integers(3))) for _ in range(2000)]
    gen = rng.integers(0, 3, 40)
    from egraph import _lib
    h = np.frombuffer(_lib.pyhost.hash_ids([e[0] for e in ent]), np.int64)
    o = np.array([e[1] for e in ent], np.int64)
    g = np.array([e[2] for e in ent], np.int64)
    from egraph.storm import PendingIndex
    for runs in (1, 5, 12):                   # one run; several; merged past MAX_RUNS
        idx = PendingIndex()
        for part in np.array_split(np.arange(len(ent)), runs):
            idx.insert(h[part], o[part], g[part], gen)
        assert len(idx.runs) <= PendingIndex.MAX_RUNS
        eng = types.SimpleNamespace(_pending=idx, _gen=gen)
        for q in ([], ids[:1], ids[::7], ["absent"], ids):
            want = {e[1] for e in ent if e[0] in set(q) and e[2] == gen[e[1]]}
            assert StormEngine._pending_hit(eng, q) == want


def test_keyed_candidates_match_flat_ones():
    """per_column(keys=True) + combine(with_flat=False) (the storm's reseed form: utf-8 blob,
    offsets and hashes instead of str lists) name the same ids in the same order, and attach
    identically, as the str-list form -- including non-ASCII names and empty columns."""
    import numpy as np
    from egraph import _lib, synth
    from egraph.graph import str_blob
    from egraph.seeds import SeedCandidates
    cl = synth.build_cluster(synth.ClusterConfig(pods=400, namespaces=3, nodes=8,
                                                 deployments=40, services=30, seed=5))
    lists = [c.evidence for c in synth.make_incidents(cl, 20, seed=2)]
    lists[3] = []
    lists[7] = [dict(lists[7][0], entity_name="pé-テ")] + lists[7][1:]
    flat = SeedCandidates.combine(SeedCandidates.per_column(lists))
    keyed = SeedCandidates.combine(SeedCandidates.per_column(lists, keys=True), with_flat=False)
    pick = [2, 0, 7, 3, 5]
    part_f = SeedCandidates.combine([SeedCandidates.per_column(lists)[i] for i in pick])
    part_k = SeedCandidates.combine([SeedCandidates.per_column(lists, keys=True)[i] for i in pick],
                                    with_flat=False)
    for f, k in ((flat, keyed), (part_f, part_k)):
        b, o = str_blob(f.flat)
        assert k.keys[0] == b and np.array_equal(k.keys[1], o)
        assert np.array_equal(k.keys[2], np.frombuffer(_lib.pyhost.hash_ids(f.flat), np.int64))
        assert k.n_flat == f.n_flat and np.array_equal(k.count, f.count)
        assert np.array_equal(k.col, f.col) and np.array_equal(k.val, f.val)
        found = np.random.default_rng(3).integers(-1, 30, f.n_flat)
        for a, c in zip(f.attach_found_idx(found), k.attach_found_idx(found)):
            assert np.array_equal(a, c)
    empty = SeedCandidates.combine([], with_flat=False)
    assert empty.n_flat == 0 and len(empty.attach_found_idx(np.zeros(0))[0]) == 0


def _attach_both(g, lists, threads):
    from egraph.seeds import SeedCandidates, attach_native
    a = attach_native(g, lists, threads)
    b = SeedCandidates(lists).attach(g)
    for x, y in zip(a, b):
        assert x.dtype == y.dtype and len(x) == len(y)
        if x.dtype == np.float32:
            assert np.array_equal(x, y, equal_nan=True)
        else:
            assert np.array_equal(x, y)
    return a


def _edge_graph():
    """A graph holding some of EDGE's candidate ids (and ids the workers must format: None,
    True, non-ASCII) so that first-present-wins is exercised on each candidate position."""
    from egraph.graph import EvidenceGraph
    g = EvidenceGraph()
    ids = ["pod:ns:p", "deployment:ns:d", "node:n1", "node:n", "hpa:ns:h", "configmap:ns:c",
           "event:ns:e", "pod:other:p", "service:ns:svc", "deployment:ns:svc", "metric:1.5:False",
           "pod:None:5", "deployment:None:d", "none:ns:None", "7:None:3", "pod:ns:pé-テ",
           "deployment:ns:sub"]
    g.merge_nodes(ids, ["X"] * len(ids))
    g.merge_nodes(["pod:ns:p"], ["Y"])              # a second vertex with the same id: first wins
    return g


@pytest.mark.parametrize("threads", [1, 4])
def test_attach_native_matches_python_on_collector_evidence(threads):
    """seeds_for_batch's native pass (csrc/pyhost.c seed_attach over egr_graph_find) attaches
    exactly like SeedCandidates.attach (str ids + egr_graph_lookup), on the worker pool
    (>= 4096 rows) and on the calling thread."""
    from egraph import synth
    c = synth.build_cluster(synth.ClusterConfig(pods=1500, namespaces=5, nodes=40,
                                                deployments=150, services=100, seed=9))
    cases = synth.make_incidents(c, 120, seed=10)
    synth.add_incidents(c, cases)
    g = synth.build_graph(c)
    lists = [x.evidence for x in cases]
    assert sum(map(len, lists)) >= 4096
    v, col, s = _attach_both(g, lists, threads)
    assert len(v) > 1000


@pytest.mark.parametrize("threads", [1, 4])
def test_attach_native_matches_python_on_edge_rows(threads):
    rng = random.Random(5)
    uni = [{"evidence_type": "kubernetes_pod", "entity_namespace": "ns", "entity_name": "pé-テ"},
           {"evidence_type": "kubernetes_event", "entity_namespace": "ns", "entity_name": "x",
            "data": {"involved_object": {"kind": "DÉPLOYMENT", "name": "d"}}},
           {"evidence_type": "kubernetes_event", "entity_namespace": "ns", "entity_name": "x",
            "data": {"involved_object": {"kind": "NODE", "name": "n1"}}},
           {"evidence_type": "kubernetes_pod", "entity_namespace": "ns", "entity_name": "p" * 600}]
    rows = EDGE + uni
    # pad past the parallel threshold so the worker pass runs with edge rows inside it
    lists = [rows, [], rows[::-1]] + [rng.sample(rows, 12) for _ in range(400)]
    _attach_both(_edge_graph(), lists, threads)


@pytest.mark.parametrize("threads", [2, 4, 7])
def test_seed_keys_all_rows_on_the_workers(threads):
    """Collector rows only (none handed over): seed_keys assembles its output by concatenating the
    workers' arrays -- the same blob, offsets, hashes, counts, columns and strengths as
    SeedCandidates, for job splits that cut the batch at different lists."""
    from egraph import _lib, synth
    from egraph.graph import str_blob
    from egraph.seeds import SeedCandidates, _row
    c = synth.build_cluster(synth.ClusterConfig(pods=1500, namespaces=5, nodes=40,
                                                deployments=150, services=100, seed=9))
    lists = [x.evidence for x in synth.make_incidents(c, 150, seed=11)]
    lists[3] = []                                   # an empty list inside a job
    sc = SeedCandidates(lists)
    blob, off, hs, count, col, val = _lib.pyhost.seed_keys(lists, _row, threads)
    b, o = str_blob(sc.flat)
    assert blob == b and np.array_equal(np.frombuffer(off, np.int64), o)
    assert np.array_equal(np.frombuffer(hs, np.int64), np.frombuffer(_lib.pyhost.hash_ids(sc.flat), np.int64))
    assert np.array_equal(np.frombuffer(count, np.int64), sc.count)
    assert np.array_equal(np.frombuffer(col, np.uint32), sc.col)
    assert np.array_equal(np.frombuffer(val, np.float32), sc.val, equal_nan=True)


@pytest.mark.parametrize("bad", [
    {"evidence_type": "kubernetes_pod", "entity_namespace": "ns", "entity_name": "p",
     "signal_strength": "x"},
    {"evidence_type": "kubernetes_event", "entity_namespace": "ns", "entity_name": "e",
     "data": {"involved_object": ["x"]}},
    ["not", "a", "dict"],
    {"evidence_type": "kubernetes_pod", "entity_namespace": "ns", "entity_name": "\ud800"},
])
def test_attach_native_raises_like_python(bad):
    from egraph.seeds import SeedCandidates, attach_native
    g = _edge_graph()
    lists = [[dict(EDGE[0])] * 5000, [bad]]
    with pytest.raises(Exception) as e1:
        SeedCandidates(lists).attach(g)
    for th in (1, 4):
        with pytest.raises(Exception) as e2:
            attach_native(g, lists, th)
        assert type(e1.value) is type(e2.value)


def test_graph_find_matches_lookup():
    from egraph import _lib
    g = _edge_graph()
    ids = ["pod:ns:p", "node:n1", "absent", "", "pod:ns:pé-テ", "deployment:ns:sub"]
    want = g.lookup(ids).tolist()
    got = [_lib.lib.egr_graph_find(g.handle, x.encode(), len(x.encode())) for x in ids]
    assert got == want and want[0] == 0 and want[2] == -1


@pytest.mark.parametrize("threads", [1, 4])
def test_seed_keys_match_seed_candidates(threads):
    """pyhost.seed_keys (the keyed per_column form, one native pass) names the same ids, counts,
    columns and strengths as SeedCandidates (str ids through the Python statement for the rows
    it hands over), with hash_ids' hashes -- on collector rows and on edge rows, both thread
    modes (the worker pool runs from 4096 rows)."""
    from egraph import _lib, synth
    from egraph.graph import str_blob
    from egraph.seeds import SeedCandidates, _row
    c = synth.build_cluster(synth.ClusterConfig(pods=1500, namespaces=5, nodes=40,
                                                deployments=150, services=100, seed=9))
    lists = [x.evidence for x in synth.make_incidents(c, 120, seed=10)]
    rng = random.Random(7)
    lists += [EDGE, [], EDGE[::-1]] + [rng.sample(EDGE, 8) for _ in range(30)]
    lists[5] = [dict(lists[5][0], entity_name="pé-テ")] + lists[5][1:]
    sc = SeedCandidates(lists)
    blob, off, hs, count, col, val = _lib.pyhost.seed_keys(lists, _row, threads)
    b, o = str_blob(sc.flat)
    assert blob == b and np.array_equal(np.frombuffer(off, np.int64), o)
    assert np.array_equal(np.frombuffer(hs, np.int64), np.frombuffer(_lib.pyhost.hash_ids(sc.flat), np.int64))
    assert np.array_equal(np.frombuffer(count, np.int64), sc.count)
    assert np.array_equal(np.frombuffer(col, np.uint32), sc.col)
    assert np.array_equal(np.frombuffer(val, np.float32), sc.val, equal_nan=True)


@pytest.mark.parametrize("threads", [2, 4, 7])
def test_seed_keys_all_rows_on_the_workers(threads):
    """Collector rows only (none handed over): seed_keys assembles its output by concatenating the
    workers' arrays -- the same blob, offsets, hashes, counts, columns and strengths as
    SeedCandidates, for job splits that cut the batch at different lists."""
    from egraph import _lib, synth
    from egraph.graph import str_blob
    from egraph.seeds import SeedCandidates, _row
    c = synth.build_cluster(synth.ClusterConfig(pods=1500, namespaces=5, nodes=40,
                                                deployments=150, services=100, seed=9))
    lists = [x.evidence for x in synth.make_incidents(c, 150, seed=11)]
    lists[3] = []                                   # an empty list inside a job
    sc = SeedCandidates(lists)
    blob, off, hs, count, col, val = _lib.pyhost.seed_keys(lists, _row, threads)
    b, o = str_blob(sc.flat)
    assert blob == b and np.array_equal(np.frombuffer(off, np.int64), o)
    assert np.array_equal(np.frombuffer(hs, np.int64), np.frombuffer(_lib.pyhost.hash_ids(sc.flat), np.int64))
    assert np.array_equal(np.frombuffer(count, np.int64), sc.count)
    assert np.array_equal(np.frombuffer(col, np.uint32), sc.col)
    assert np.array_equal(np.frombuffer(val, np.float32), sc.val, equal_nan=True)


@pytest.mark.parametrize("bad", [
    {"evidence_type": "kubernetes_pod", "entity_namespace": "ns", "entity_name": "p",
     "signal_strength": "x"},
    ["not", "a", "dict"],
])
def test_seed_keys_raise_like_python(bad):
    from egraph import _lib
    from egraph.seeds import _row, candidates_py
    lists = [[dict(EDGE[0])] * 5000, [bad]]
    with pytest.raises(Exception) as e1:
        candidates_py(lists)
    for th in (1, 4):
        with pytest.raises(Exception) as e2:
            _lib.pyhost.seed_keys(lists, _row, th)
        assert type(e1.value) is type(e2.value)


def test_storm_rank_store_rows():
    """StormEngine's RankStore (host logic): rows by handle, grown on demand, None / -1 until an
    incident is first ranked, later puts overwrite, and OpenIncident reads its row through it."""
    import numpy as np
    from egraph.storm import OpenIncident, RankStore
    st = RankStore(4)
    x = OpenIncident(7, "i7", None, store=st)
    assert x.top_ids is None and x.top_scores is None and x.ranked_at == -1
    ids = np.arange(8, dtype=np.uint32).reshape(2, 4)
    sc = np.linspace(0, 1, 8, dtype=np.float32).reshape(2, 4)
    st.put(np.array([7, 2000]), ids, sc, 3)
    assert np.array_equal(x.top_ids, ids[0]) and x.top_scores.tobytes() == sc[0].tobytes()
    assert x.ranked_at == 3 and st.row(2000)[2] == 3 and st.row(5)[0] is None
    st.put(np.array([7]), ids[1:], sc[1:], 4)
    assert np.array_equal(x.top_ids, ids[1]) and x.ranked_at == 4
    got = x.top_ids
    got[0] = 99                                   # a copy: the store is not written through
    assert st.row(7)[0][0] == ids[1][0]


def test_storm_seed_store():
    """StormEngine's SeedStore (host logic): per-handle slices of pooled arrays; a reset of an
    incident's seeds replaces its slice, gathers follow the requested handle order, unknown and
    empty handles gather nothing, and compaction keeps every live slice."""
    import numpy as np
    from egraph.storm import OpenIncident, SeedStore, ranges
    assert ranges(np.array([5, 0, 9]), np.array([2, 0, 3])).tolist() == [5, 6, 9, 10, 11]
    st = SeedStore()
    rng = np.random.default_rng(3)
    want = {}
    for it in range(300):
        hs = rng.choice(200, size=int(rng.integers(1, 20)), replace=False)
        cnt = rng.integers(0, 40, len(hs))
        sv = rng.integers(0, 1 << 20, int(cnt.sum())).astype(np.uint32)
        ss = rng.random(int(cnt.sum())).astype(np.float32)
        st.set(hs, sv, ss, cnt)
        o = 0
        for h, c in zip(hs.tolist(), cnt.tolist()):
            want[h] = (sv[o:o + c].copy(), ss[o:o + c].copy())
            o += c
        if it % 50 == 49:
            q = np.array(sorted(want, key=lambda _: rng.random()) + [5000], np.int64)
            v, s, c = st.gather(q)
            assert c[-1] == 0
            assert v.tolist() == [x for h in q[:-1].tolist() for x in want[h][0].tolist()]
            assert s.tobytes() == b"".join(want[h][1].tobytes() for h in q[:-1].tolist())
    assert st.n <= 2 * st.live + 4096                 # garbage was compacted
    x = OpenIncident(int(next(iter(want))), "i", None, seeds=st)
    assert x.sv.tolist() == want[x.handle][0].tolist()
    assert OpenIncident(7, "j", None).sv.size == 0 and OpenIncident(7, "j", None).vertex == -1
