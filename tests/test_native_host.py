"""Host-side checks of libegraph.so that need no GPU: symbols, exact rounding, MERGE
semantics and the CSR the snapshot uploads (against the pure-Python restatement)."""
from __future__ import annotations

import random
import re

import numpy as np
import pytest

from conftest import REPO


def _header_functions() -> list[str]:
    text = (REPO / "include" / "egraph.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(egr_[a-z0-9_]+)\s*\(", text)))


def test_library_loads_and_exports_every_declared_symbol():
    from egraph import _lib as L
    names = _header_functions()
    assert len(names) >= 30
    for name in names:
        assert hasattr(L.lib, name), name
        assert name in L.SIGNATURES, f"{name} declared in egraph.h but not bound"
    assert L.lib.egr_version() == 1


def test_device_count_is_safe_without_gpu():
    from egraph import _lib as L
    assert L.lib.egr_device_count() >= 0


def test_exact_python_round_host():
    from egraph import _lib as L
    rng = random.Random(3)
    for _ in range(100000):
        x = rng.choice([rng.random() * 3, rng.uniform(-5, 5), round(rng.random(), 5),
                        rng.random() * 1e13, rng.random() * 1e17, rng.random() * 1e-7,
                        rng.randint(0, 10**6) / 2e4, rng.randint(0, 10**6) / 2e3])
        nd = rng.choice([0, 1, 2, 3, 4, 6, 9])
        assert L.lib.egr_py_round(x, nd) == round(x, nd), (x, nd)
    for x in (float("inf"), -float("inf"), 0.0, -0.0, 2.675, 0.00005, -0.00005, 1e300, 5e-324):
        r = L.lib.egr_py_round(x, 4)
        assert r == round(x, 4) and np.signbit(r) == np.signbit(round(x, 4))
    assert np.isnan(L.lib.egr_py_round(float("nan"), 4))


def _random_graph(rng: random.Random, n_ids=30, n_ent=60, n_rel=120):
    labels = ["Pod", "Node", "Deployment", "Incident", "Service"]
    types = ["AFFECTS", "SCHEDULED_ON", "OWNS", "CALLS"]
    ents = [{"id": f"id{rng.randrange(n_ids)}", "type": rng.choice(labels), "properties": {"k": i}}
            for i in range(n_ent)]
    rels = [{"source_id": f"id{rng.randrange(n_ids + 5)}", "target_id": f"id{rng.randrange(n_ids + 5)}",
             "relation_type": rng.choice(types), "properties": {}} for _ in range(n_rel)]
    return ents, rels


@pytest.mark.parametrize("seed", range(12))
def test_merge_semantics_and_csr_match_restatement(seed):
    import oracle
    from egraph.graph import EvidenceGraph
    rng = random.Random(seed)
    ents, rels = _random_graph(rng)
    g = EvidenceGraph()
    # feed in two batches to exercise incremental MERGE
    g.create_entities_batch(ents[:30])
    g.create_relations_batch(rels[:50])
    g.create_entities_batch(ents[30:])
    g.create_relations_batch(rels[50:])
    # reference order: node merges then edge merges interleaved the same way
    verts, _ = oracle.graph_reference(ents, [])
    _, e1 = oracle.graph_reference(ents[:30], rels[:50])
    vert_all, _ = oracle.graph_reference(ents, [])
    vid = {k: i for i, k in enumerate(vert_all)}
    # edges of batch 1 were matched against the first 30 entities only
    v30, _ = oracle.graph_reference(ents[:30], [])
    e_ref = [(vid[v30[s]], vid[v30[d]], t) for s, d, t in e1]
    _, e_all = oracle.graph_reference(ents, rels[50:])
    seen = set(e_ref)
    for s, d, t in e_all:
        if (s, d, t) not in seen:
            seen.add((s, d, t))
            e_ref.append((s, d, t))
    assert g.num_vertices == len(verts)
    labels = g.labels()
    vl, es, ed, et = g.export()
    assert [(labels[vl[v]], g.vertex_id(v)) for v in range(g.num_vertices)] == verts
    types = g.rel_types()
    assert list(zip(es.tolist(), ed.tolist(), [types[t] for t in et])) == e_ref
    # CSR
    w = g.weight_array({"AFFECTS": (1.0, 0.5), "OWNS": (0.25, 2.0)})
    csr = g.csr({"AFFECTS": (1.0, 0.5), "OWNS": (0.25, 2.0)})
    rp, col, meta, val = oracle.csr_reference(len(verts), e_ref, {t: i for i, t in enumerate(types)}, w)
    np.testing.assert_array_equal(csr["row_ptr"], rp)
    np.testing.assert_array_equal(csr["col"], col)
    np.testing.assert_array_equal(csr["meta"], meta)
    np.testing.assert_array_equal(csr["val"], val)


def test_dangling_edges_dropped_and_counts_are_attempts():
    from egraph.graph import EvidenceGraph
    g = EvidenceGraph()
    assert g.create_entities_batch([{"id": "pod:a", "type": "Pod"}, {"id": "pod:a", "type": "Pod"},
                                    {"id": "incident:1", "type": "Incident"}]) == 3
    assert g.num_vertices == 2
    rels = [{"source_id": "incident:1", "target_id": "pod:a", "relation_type": "AFFECTS"},
            {"source_id": "incident:1", "target_id": "pod:a", "relation_type": "AFFECTS"},
            {"source_id": "pod:a", "target_id": "node:healthy", "relation_type": "SCHEDULED_ON"}]
    assert g.create_relations_batch(rels) == 3          # attempted, like neo4j.py:166
    assert g.num_edges == 1                              # dedup + dangling SCHEDULED_ON dropped
    assert g.node_props[("Pod", "pod:a")]["id"] == "pod:a"


def test_custom_ops_registered():
    """lib/_egraph_ops.so registers torch.ops.egraph.* (CPU: schemas only, no CPU kernels)."""
    import torch
    from egraph import ops
    for name in ops.OPS:
        assert hasattr(torch.ops.egraph, name), name
    assert "Tensor rule_table" in str(torch.ops.egraph.rules_eval.default._schema)
    with pytest.raises(NotImplementedError):       # device kernels only: no CPU fallback
        torch.ops.egraph.reach(1, torch.zeros(4, dtype=torch.int32), 10, 3)


def test_entity_rows_match_python_assembly():
    """pyhost.entity_rows (GraphService.rank_root_causes' result dicts) equals the Python loop it
    replaces: per incident, {"id", "labels", "score", "rank"} for each ranked vertex up to the
    first EGR_NO_NODE, scores as the f32 values' Python floats."""
    import numpy as np
    from egraph import _lib
    rng = np.random.default_rng(3)
    B, k, V = 37, 10, 500
    ids = rng.integers(0, V, (B, k)).astype(np.uint32)
    for b in range(B):                      # ragged lists: EGR_NO_NODE past a random length
        ids[b, rng.integers(0, k + 1):] = 0xFFFFFFFF
    ids[3, :] = 0xFFFFFFFF
    scores = rng.random((B, k), dtype=np.float32) * 3
    scores[5, 0] = np.float32("inf")
    vlabel = rng.integers(0, 4, V).astype(np.uint8)
    names = ["Pod", "Node", "Service", "Deployment"]
    vids = [f"v:{i}" for i in range(V)]
    lab = np.zeros(ids.shape, np.uint8)
    ok = ids != 0xFFFFFFFF
    lab[ok] = vlabel[ids[ok]]
    got = _lib.pyhost.entity_rows(ids, scores, lab, k, vids, names)
    want = []
    for irow, srow in zip(ids.tolist(), scores.tolist()):
        row = []
        for r, (v, sc) in enumerate(zip(irow, srow)):
            if v == 0xFFFFFFFF:
                break
            row.append({"id": vids[v], "labels": [names[vlabel[v]]], "score": sc, "rank": r + 1})
        want.append(row)
    assert got == want
    assert [list(d) for d in got[0]] == [list(d) for d in want[0]]      # key order too
    import pytest
    with pytest.raises(ValueError):
        _lib.pyhost.entity_rows(ids, scores[:-1], lab, k, vids, names)
    with pytest.raises(IndexError):
        _lib.pyhost.entity_rows(ids, scores, lab, k, vids[:10], names)


def test_str_blob_native_matches_python():
    """egraph.graph.str_blob's native path (csrc/pyhost.c str_blob) gives the Python path's blob
    and offsets, UTF-8 included; non-str items and non-lists fall back to Python."""
    from egraph import _lib as L
    from egraph.graph import str_blob
    for strs in (["pod:ns:a", "node:n1", "", "café:é", "x" * 300], [], ["only"]):
        r = L.pyhost.str_blob(strs)
        enc = [s.encode() for s in strs]
        assert r[0] == b"".join(enc)
        assert np.frombuffer(r[1], np.int64).tolist() == np.concatenate([[0], np.cumsum([len(b) for b in enc])]).astype(np.int64).tolist()
        b, o = str_blob(strs)
        assert b == r[0] and o.tolist() == np.frombuffer(r[1], np.int64).tolist()
    assert L.pyhost.str_blob(["a", 3]) is None and L.pyhost.str_blob(("a",)) is None
    b, o = str_blob(("a", "bc"))
    assert b == b"abc" and o.tolist() == [0, 1, 3]


@pytest.mark.parametrize("seed", range(4))
def test_locality_order_native_matches_python(seed):
    """egr_locality_order (csrc/layout.hip, the frontier layout's vertex order) equals the
    Python statement egraph.graph.locality_order, and is a permutation."""
    from egraph import _lib as L
    from egraph import synth
    from egraph.graph import locality_order
    cfg = synth.ClusterConfig(pods=800 + 300 * seed, namespaces=5, nodes=20 + seed, deployments=80,
                              services=40, attach_fraction=0.3, seed=100 + seed)
    c = synth.build_cluster(cfg)
    synth.add_incidents(c, synth.make_incidents(c, 30, seed=seed))
    g = synth.build_graph(c)
    csr = g.csr()
    V = g.num_vertices
    out = np.empty(V, np.uint32)
    L.check(L.lib.egr_locality_order(csr["row_ptr"].ctypes.data, csr["col"].ctypes.data, V,
                                     out.ctypes.data), "egr_locality_order")
    want = locality_order(csr["row_ptr"], csr["col"])
    assert np.array_equal(out.astype(np.int64), want)
    assert np.array_equal(np.sort(out), np.arange(V))
    # a Node hub is followed by vertices hanging under it (its pods)
    labels = g.labels()
    vl, _, _, _ = g.export()
    pos = np.empty(V, np.int64)
    pos[out] = np.arange(V)
    first_node = out[np.flatnonzero(vl[out] == labels.index("Node"))[0]]
    assert vl[out[pos[first_node] + 1]] == labels.index("Pod")


@pytest.mark.parametrize("seed", range(4))
def test_labelled_lookup_vertex_of_and_id_list(seed):
    """egr_graph_lookup_labeled (MATCH (n:label {id})) and the VertexOf view against a Python
    model of MERGE, with ids carried by several labels, duplicates inside one batch and more
    ids than one pipelined lookup group (32); the id list merge_nodes keeps equals the native
    graph's; lookup() of present and absent ids equals egr_graph_find one at a time."""
    from egraph import _lib as L
    from egraph.graph import EvidenceGraph
    rng = random.Random(seed)
    g = EvidenceGraph()
    model: dict = {}
    order: list = []
    for _ in range(5):
        ids = [f"v{rng.randrange(150)}" for _ in range(rng.randrange(1, 90))]
        labels = [rng.choice(["Pod", "Node", "Incident"]) for _ in ids]
        out = g.merge_nodes(ids, labels)
        for i, lab, v in zip(ids, labels, out.tolist()):
            if (lab, i) not in model:
                model[(lab, i)] = len(order)
                order.append(i)
            assert model[(lab, i)] == v
    assert g._ids == order and g.vertex_ids() == [g.vertex_id(v) for v in range(g.num_vertices)]
    probe = [f"v{k}" for k in range(160)]
    for lab in ("Pod", "Node", "Incident", "Service"):
        got = g.lookup_labeled(probe, lab).tolist()
        assert got == [model.get((lab, i), -1) for i in probe]
    mixed = [rng.choice(["Pod", "Node", "Incident"]) for _ in probe]
    assert g.lookup_labeled(probe, mixed).tolist() == [model.get(k, -1) for k in zip(mixed, probe)]
    vo = g.vertex_of
    assert len(vo) == len(order) and dict(vo.items()) == model
    assert all(vo[k] == v for k, v in model.items()) and ("Service", "v1") not in vo
    with pytest.raises(KeyError):
        vo[("Service", "v1")]
    first = g.lookup(probe).tolist()
    assert first == [int(L.lib.egr_graph_find(g._h, i.encode(), len(i))) for i in probe]


def test_attach_idx_matches_numpy():
    """pyhost.attach_idx (first present candidate per row, the ids ranked before it) against the
    numpy statement it replaced."""
    from egraph import _lib
    rng = np.random.default_rng(3)
    count = rng.integers(1, 5, 400).astype(np.int64)
    n = int(count.sum())
    found = np.where(rng.random(n) < 0.4, rng.integers(0, 1000, n), -1).astype(np.int64)
    sv, ok, before, brow = _lib.pyhost.attach_idx(found, count)
    starts = np.concatenate([[0], np.cumsum(count)[:-1]])
    pos = np.where(found >= 0, np.arange(n), n)
    first = np.minimum.reduceat(pos, starts)
    e_ok = first < n
    e_before = np.flatnonzero(np.arange(n) < np.repeat(np.where(e_ok, first, n), count))
    e_row = np.repeat(np.arange(len(count)), count)[e_before]
    np.testing.assert_array_equal(np.frombuffer(ok, np.bool_), e_ok)
    np.testing.assert_array_equal(np.frombuffer(sv, np.uint32), found[first[e_ok]].astype(np.uint32))
    np.testing.assert_array_equal(np.frombuffer(before, np.int64), e_before)
    np.testing.assert_array_equal(np.frombuffer(brow, np.int64), e_row)
    with pytest.raises(ValueError):
        _lib.pyhost.attach_idx(found[:3], count)
