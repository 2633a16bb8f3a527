"""The native host side of the rules boundary (csrc/pyhost.c), checked on the CPU.

* encode_rows (behind egraph.encode.encode_batch) must give the same columns, node keys and
  evidence ids as the all-Python encoder (encode_batch_py) on every input, and raise the same
  exception type wherever the Python encoder (and the reference, tests/golden/rules_errors.json)
  raises -- including rows of non-plain types that it hands to the Python row encoder.
* assemble (behind egraph.rca.hypothesis_lists) must build the same dicts, keys in the same
  order, as hypothesis_dicts, with a fresh uuid4 string id per hypothesis.
"""
from __future__ import annotations

import json
import math
import random
import uuid
from collections import OrderedDict

import numpy as np
import pytest

import evidence_fuzz
from conftest import REPO


def _same(a, b):
    for k in ("flags", "vocab", "node", "err", "seg_off"):
        x, y = getattr(a, k), getattr(b, k)
        assert x.dtype == y.dtype and x.shape == y.shape, k
        assert np.array_equal(x.view(np.uint8), y.view(np.uint8)), k   # bitwise (NaN, -0.0)
    assert a.evidence_ids == b.evidence_ids


def _encode_both(lists):
    from egraph import catalog
    from egraph.encode import encode_batch, encode_batch_py
    cat = catalog.default()
    return encode_batch(lists, cat), encode_batch_py(lists, cat)


def test_flag_bits_match_the_header():
    from egraph import _lib as L
    assert L.pyhost.flag_bits() == (
        L.F_RECENT_DEPLOY, L.F_IMAGE_CHANGED, L.F_MEMORY_HIGH, L.F_HPA_AT_MAX, L.F_LATENCY_HIGH,
        L.F_NODE_ISSUE, L.F_NOT_READY, L.F_READINESS_FAIL, L.F_ERR_FLOAT, L.EGR_NO_NODE)


def test_native_encoder_matches_python_on_fuzz_and_scenarios():
    rng = random.Random(11)
    lists = [evidence_fuzz.random_evidence(rng) for _ in range(600)]
    lists += [ev for _, ev in evidence_fuzz.scenario_cases()]
    lists += [[]]                                   # an incident without evidence
    a, b = _encode_both(lists)
    _same(a, b)
    assert a.n_rows > 5000


def test_native_encoder_matches_python_on_golden_rule_cases():
    cases = json.loads((REPO / "tests" / "golden" / "rules_cases.json").read_text())
    lists = [c["evidence"] for c in cases["cases"]]
    a, b = _encode_both(lists)
    _same(a, b)


def test_native_encoder_matches_python_on_synthetic_cluster_incidents():
    from egraph import synth
    cl = synth.build_cluster(synth.ClusterConfig(pods=600, namespaces=4, nodes=12,
                                                 deployments=60, services=40, seed=3))
    lists = [c.evidence for c in synth.make_incidents(cl, 64, seed=5)]
    a, b = _encode_both(lists)
    _same(a, b)


class _Dict(dict):
    """A dict subclass: the native encoder must hand such rows to Python."""


class _Truthy:
    def __bool__(self):
        return True


class _Weird:
    def __eq__(self, other):
        return other == "Ready"

    def __hash__(self):
        return hash("Ready")


def _edge_rows():
    pod = "kubernetes_pod"
    rows = [
        # missing / None / odd-typed fields that do not raise
        {"id": 1, "evidence_type": pod},
        {"id": 2, "evidence_type": pod, "data": {}},
        {"evidence_type": pod, "data": {"waiting_reason": "CrashLoopBackOff", "node_name": "n1"}},
        {"id": None, "evidence_type": pod, "data": {"terminated_reason": "OOMKilled",
                                                    "restart_count": 2.5, "node_name": 7}},
        {"id": "b", "evidence_type": pod, "data": {"restart_count": True, "node_name": "n1"}},
        {"id": "c", "evidence_type": pod, "data": {"restart_count": float("nan"), "node_name": "n2"}},
        {"id": "d", "evidence_type": pod, "data": {"restart_count": -3, "node_name": "n2",
                                                   "waiting_reason": ""}},
        {"id": "e", "evidence_type": pod, "data": {"waiting_reason": 5, "restart_count": 1,
                                                   "node_name": 1.0}},
        {"id": "f", "evidence_type": pod, "data": {
            "phase": "Running", "restart_count": 0,
            "conditions": [{"type": "PodScheduled"}, {"type": "Ready", "status": "False",
                                                      "reason": "ContainersNotReady"}, 5]}},
        {"id": "g", "evidence_type": pod, "data": {
            "phase": "Running", "conditions": [{"type": "Ready", "status": None}]}},
        {"id": "h", "evidence_type": pod, "data": {
            "phase": "Pending", "conditions": [{"type": "Ready", "status": "False"}]}},
        {"id": "i", "evidence_type": pod, "data": {
            "phase": "Running", "conditions": ({"type": "Ready", "status": "False"},)}},
        {"id": "j", "evidence_type": pod, "data": _Dict(waiting_reason="ImagePullBackOff",
                                                         restart_count=1, node_name="n3")},
        {"id": "k", "evidence_type": pod, "data": {
            "phase": "Running", "conditions": [{"type": _Weird(), "status": "False"}]}},
        {"id": "l", "evidence_type": pod, "data": {"waiting_reason": _Truthy(),
                                                   "restart_count": 0}},
        # deploy / image
        {"id": 10, "evidence_type": "deploy_change", "data": {"is_recent_change": 1}},
        {"id": 11, "evidence_type": "deploy_change", "data": {"is_recent_change": []}},
        {"id": 12, "evidence_type": "deploy_change"},
        {"id": 13, "evidence_type": "image_change", "data": {"image_changed": "yes"}},
        {"id": 14, "evidence_type": "image_change", "data": {"image_changed": _Truthy()}},
        # logs
        {"id": 20, "evidence_type": "log_signal", "data": {"patterns_found": ["network", "oom", 3],
                                                           "error_count": 12}},
        {"id": 21, "evidence_type": "log_signal", "data": {"error_count": 2.5}},
        {"id": 22, "evidence_type": "log_signal", "data": {"error_count": -0.0}},
        {"id": 23, "evidence_type": "log_signal", "data": {"error_count": float("inf")}},
        {"id": 24, "evidence_type": "log_signal", "data": {"error_count": 2 ** 31}},
        {"id": 25, "evidence_type": "log_signal", "data": {"error_count": -(2 ** 31)}},
        {"id": 26, "evidence_type": "log_signal", "data": {"error_count": 2 ** 70}},
        {"id": 27, "evidence_type": "log_signal", "data": {"error_count": True}},
        {"id": 28, "evidence_type": "log_signal", "data": {"patterns_found": "network"}},
        {"id": 29, "evidence_type": "log_signal", "data": {"patterns_found": ("network",),
                                                           "error_count": 3.0}},
        {"id": 30, "evidence_type": "log_signal", "data": {"error_count": float("nan")}},
        # metrics
        {"id": 40, "evidence_type": "metric_signal", "data": {"query_name": "memory_usage",
                                                              "is_anomalous": True,
                                                              "current_value": 95}},
        {"id": 41, "evidence_type": "metric_signal", "data": {"query_name": "memory_usage",
                                                              "is_anomalous": True,
                                                              "current_value": ""}},
        {"id": 42, "evidence_type": "metric_signal", "data": {"query_name": "memory",
                                                              "is_anomalous": 0,
                                                              "current_value": "high"}},
        {"id": 43, "evidence_type": "metric_signal", "data": {"query_name": "hpa_max_replicas",
                                                              "current_value": True}},
        {"id": 44, "evidence_type": "metric_signal", "data": {"query_name": "hpa_max",
                                                              "current_value": "1"}},
        {"id": 45, "evidence_type": "metric_signal", "data": {"query_name": "hpa_max",
                                                              "current_value": 1.0}},
        {"id": 46, "evidence_type": "metric_signal", "data": {"query_name": "p99_latency"}},
        {"id": 47, "evidence_type": "metric_signal", "data": {"query_name": "p99_latency",
                                                              "current_value": float("nan")}},
        {"id": 48, "evidence_type": "metric_signal", "data": {"query_name": ["latency"],
                                                              "current_value": 5}},
        {"id": 49, "evidence_type": "metric_signal", "data": {}},
        {"id": 50, "evidence_type": "metric_signal", "data": {"query_name": "memory",
                                                              "is_anomalous": True,
                                                              "current_value": float("nan")}},
        # nodes
        {"id": 60, "evidence_type": "kubernetes_node", "data": {"name": "n1"}},
        {"id": 61, "evidence_type": "kubernetes_node", "data": {
            "name": "n2", "conditions": {"Ready": {"status": "True"}}}},
        {"id": 62, "evidence_type": "kubernetes_node", "data": {
            "name": None, "conditions": {"Ready": {}}}},
        {"id": 63, "evidence_type": "kubernetes_node", "data": {
            "name": "n4", "conditions": OrderedDict(Ready={"status": "Unknown"})}},
        # unknown / odd types
        {"id": 70, "evidence_type": "kubernetes_event", "data": None},
        {"id": 71, "evidence_type": None, "data": 5},
        {"id": 72, "evidence_type": 3},
        {"id": 73},
        _Dict(id=74, evidence_type="deploy_change", data={"is_recent_change": True}),
    ]
    return rows


def test_native_encoder_edge_rows_match_python():
    rows = _edge_rows()
    # one row per incident, then all in one incident, then shuffled batches of six
    lists = [[r] for r in rows] + [rows]
    rng = random.Random(2)
    for _ in range(20):
        lists.append(rng.sample(rows, 6))
    a, b = _encode_both(lists)
    _same(a, b)
    assert any(math.isnan(x) for x in a.err)
    # the plain rows stay native, the others are handed to the Python row encoder
    from egraph import _lib as L
    from egraph import catalog
    from egraph.encode import _columns, _RowEncoder
    e = _RowEncoder(catalog.default())
    _, n_slow = L.pyhost.encode_rows([rows], e.waiting, e.terminated, e.patterns, e.node_keys,
                                     e.row, *_columns([rows]))
    assert 5 <= n_slow <= 20


def _encode_threads(lists, threads):
    from egraph import catalog
    from egraph.encode import encode_batch
    return encode_batch(lists, catalog.default(), threads=threads)


@pytest.mark.parametrize("threads", [2, 7])
def test_parallel_row_pass_matches_python(threads):
    """The worker threads' read-only row pass (csrc/pyhost.c): fuzz rows, the edge rows (dict
    subclasses, non-str keys, objects with __eq__ / __bool__, NaN, huge ints, odd types) spread
    over a batch past the pass's 4096-row minimum, and synthetic cluster incidents -- bit for bit
    the Python encoder, with the same node-key numbering and ids."""
    from egraph import catalog, synth
    from egraph.encode import encode_batch_py
    cat = catalog.default()
    rng = random.Random(23)
    edge = _edge_rows()
    lists = [evidence_fuzz.random_evidence(rng) for _ in range(400)]
    for _ in range(300):
        lists.append(rng.sample(edge, 5) + evidence_fuzz.random_evidence(rng, 4))
    cl = synth.build_cluster(synth.ClusterConfig(pods=600, namespaces=4, nodes=12,
                                                 deployments=60, services=40, seed=3))
    lists += [c.evidence for c in synth.make_incidents(cl, 40, seed=5)]
    lists += [[]]
    rng.shuffle(lists)
    a = _encode_threads(lists, threads)
    assert a.n_rows > 4096
    _same(a, encode_batch_py(lists, cat))
    _same(a, _encode_threads(lists, 1))


def test_parallel_pass_fast_completion_matches_python():
    """A batch of plain rows only (no row for the serial encoder, every node name a str): the
    parallel pass completes without the serial loop -- node numbering in first-seen order over
    the worker rows, segment offsets and the first five ids per incident written directly.  Bit
    for bit the Python encoder, incidents with fewer than five rows, rows without an id and
    empty incidents included."""
    from egraph import catalog, synth
    from egraph.encode import encode_batch_py
    cat = catalog.default()
    cl = synth.build_cluster(synth.ClusterConfig(pods=900, namespaces=4, nodes=9,
                                                 deployments=80, services=50, seed=8))
    lists = [c.evidence for c in synth.make_incidents(cl, 60, seed=9)]
    rng = random.Random(31)
    short = []
    for ev in lists[:20]:                            # 1-4 rows, some without an id
        rows = [dict(r) for r in rng.sample(ev, rng.randint(1, 4))]
        if rng.random() < 0.5:
            rows[0].pop("id", None)
        short.append(rows)
    lists += short + [[], []]
    rng.shuffle(lists)
    for threads in (3, 16):
        a = _encode_threads(lists, threads)
        assert a.n_rows > 4096
        _same(a, encode_batch_py(lists, cat))
        _same(a, _encode_threads(lists, 1))
    assert (a.node != 0xFFFFFFFF).sum() > 100           # node names numbered


BAD_ROWS = [
    ({"evidence_type": "kubernetes_pod", "data": {"restart_count": None}}, TypeError),
    ({"evidence_type": "kubernetes_pod", "data": {"restart_count": "3"}}, TypeError),
    ({"evidence_type": "kubernetes_pod", "data": {"waiting_reason": ["x"]}}, TypeError),
    ({"evidence_type": "kubernetes_pod", "data": {"waiting_reason": "x", "node_name": ["n"]}},
     TypeError),
    ({"evidence_type": "kubernetes_pod", "data": {"conditions": None}}, TypeError),
    ({"evidence_type": "kubernetes_pod", "data": {"conditions": ["Ready"]}}, AttributeError),
    ({"evidence_type": "kubernetes_pod", "data": None}, AttributeError),
    ({"evidence_type": "log_signal", "data": {"patterns_found": None}}, TypeError),
    ({"evidence_type": "log_signal", "data": {"patterns_found": [["network"]]}}, TypeError),
    ({"evidence_type": "log_signal", "data": {"error_count": None}}, TypeError),
    ({"evidence_type": "metric_signal", "data": {"query_name": None}}, TypeError),
    ({"evidence_type": "metric_signal", "data": {"query_name": "p99_latency",
                                                 "current_value": None}}, TypeError),
    ({"evidence_type": "metric_signal", "data": {"query_name": "memory", "is_anomalous": True,
                                                 "current_value": "high"}}, TypeError),
    ({"evidence_type": "kubernetes_node", "data": {"name": ["n"]}}, TypeError),
    ({"evidence_type": "kubernetes_node", "data": {"conditions": None}}, AttributeError),
    ({"evidence_type": "kubernetes_node", "data": {"conditions": {"Ready": None}}},
     AttributeError),
    ({"evidence_type": ["kubernetes_pod"]}, TypeError),
    ("not a dict", AttributeError),
]


@pytest.mark.parametrize("row,exc", BAD_ROWS)
def test_parallel_row_pass_raises_what_python_raises(row, exc):
    good = {"id": "ok", "evidence_type": "deploy_change", "data": {"is_recent_change": True}}
    lists = [[good] * 10 for _ in range(500)] + [[good, row, good]]
    with pytest.raises(exc):
        _encode_threads(lists, 4)


@pytest.mark.parametrize("row,exc", BAD_ROWS)
def test_native_encoder_raises_what_python_raises(row, exc):
    from egraph import catalog
    from egraph.encode import encode_batch, encode_batch_py
    cat = catalog.default()
    good = {"id": "ok", "evidence_type": "deploy_change", "data": {"is_recent_change": True}}
    for enc in (encode_batch_py, encode_batch):
        with pytest.raises(exc):
            enc([[good], [good, row, good]], cat)


def test_native_encoder_raises_like_the_reference_goldens():
    from egraph import catalog
    from egraph.encode import encode_batch
    cases = json.loads((REPO / "tests" / "golden" / "rules_errors.json").read_text())
    cat = catalog.default()
    for c in cases:
        with pytest.raises(Exception) as ei:
            encode_batch([c["evidence"]], cat)
        assert type(ei.value).__name__ == c["raises"], c["name"]


def test_node_keys_are_first_seen_order_across_fast_and_handed_over_rows():
    rows = [
        {"evidence_type": "kubernetes_pod", "data": {"restart_count": 1, "node_name": "n1"}},
        {"evidence_type": "kubernetes_pod", "data": _Dict(restart_count=1, node_name="n2")},
        {"evidence_type": "kubernetes_pod", "data": {"restart_count": 1, "node_name": "n3"}},
        {"evidence_type": "kubernetes_pod", "data": {"restart_count": 1, "node_name": "n2"}},
        {"evidence_type": "kubernetes_pod", "data": {"restart_count": 1, "node_name": 1}},
        {"evidence_type": "kubernetes_pod", "data": {"restart_count": 1, "node_name": True}},
    ]
    a, b = _encode_both([rows[:3], rows[3:]])
    _same(a, b)
    assert list(a.node) == [0, 1, 2, 1, 3, 3]


def _oracle_result(enc):
    import oracle
    from egraph import catalog
    from egraph.rca import RulesResult
    cat = catalog.default()
    o = oracle.rules_eval(cat.table, enc.flags, enc.vocab, enc.node, enc.err, enc.seg_off)
    return RulesResult(o["mask"], o["n_hyp"], o["order_conf"], o["order_rank"], o["confidence"],
                       o["final_score"], o["strength"])


@pytest.mark.parametrize("ranked", [False, True])
def test_native_assembly_matches_python_dicts(ranked):
    from egraph import catalog
    from egraph.encode import encode_batch
    from egraph.rca import hypothesis_dicts, hypothesis_lists
    cat = catalog.default()
    rng = random.Random(4)
    lists = [evidence_fuzz.random_evidence(rng) for _ in range(300)] + [[]]
    lists += [ev for _, ev in evidence_fuzz.scenario_cases()]
    enc = encode_batch(lists, cat)
    res = _oracle_result(enc)
    iids = [f"inc-{i}" for i in range(len(lists))]
    got = hypothesis_lists(cat, res, iids, enc.evidence_ids, ranked)
    assert len(got) == len(lists)
    ids = set()
    for i, hyps in enumerate(got):
        want = hypothesis_dicts(cat, res, i, iids[i], enc.evidence_ids[i], ranked)
        assert len(hyps) == len(want) >= 1
        for h, w in zip(hyps, want):
            assert list(h) == list(w)                        # same keys, same order
            u = uuid.UUID(h["id"])
            assert u.version == 4 and u.variant == uuid.RFC_4122 and str(u) == h["id"]
            ids.add(h["id"])
            h2, w2 = dict(h), dict(w)
            del h2["id"], w2["id"]
            assert h2 == w2
            assert all(type(h2[k]) is type(w2[k]) for k in h2)
            # fresh lists per dict: mutating one must not touch the catalog or a sibling
            assert h["recommended_actions"] is not w["recommended_actions"]
    assert len(ids) == sum(len(h) for h in got)


@pytest.mark.parametrize("odd", ["none", "int_name", "dict_subclass"])
def test_parallel_node_numbering_matches_python(odd):
    """The parallel pass numbers node names in its own map while every name is a str; an int
    name or a row the serial encoder takes hands the numbering to node_keys mid-batch -- the
    numbering stays the Python encoder's first-seen order either way."""
    from egraph import catalog
    from egraph.encode import encode_batch_py
    rng = random.Random(31)
    pod = lambda name: {"evidence_type": "kubernetes_pod",                     # noqa: E731
                        "data": {"restart_count": 1, "node_name": name}}
    lists = [[pod(f"node-{rng.randrange(300)}") for _ in range(12)] for _ in range(500)]
    if odd == "int_name":
        lists[250][3] = pod(7)
        lists[251][0] = pod(7.0)                     # == 7: the same dict key
    elif odd == "dict_subclass":
        lists[250][3] = {"evidence_type": "kubernetes_pod",
                         "data": _Dict(restart_count=1, node_name="node-new")}
    a = _encode_threads(lists, 4)
    assert a.n_rows > 4096
    _same(a, encode_batch_py(lists, catalog.default()))
