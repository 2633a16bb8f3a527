"""Snapshot file format (egraph/snapfile.py) on CPU: save -> load restores
the host graph exactly (vertex / edge order, label and type tables, properties, hence the same
CSR), the stored CSR equals the host build, and damaged / foreign files are rejected."""
from __future__ import annotations

import numpy as np
import pytest


def _graph():
    from egraph import synth
    from egraph.graph import EvidenceGraph
    c = synth.build_cluster(synth.ClusterConfig(pods=400, namespaces=4, nodes=12, deployments=40,
                                                services=20, attach_fraction=0.3, seed=13))
    cases = synth.make_incidents(c, 5, seed=14)
    synth.add_incidents(c, cases)
    g = EvidenceGraph()
    g.create_entities_batch([{"id": i, "type": t, "properties": {"k": n}}
                             for n, (i, t) in enumerate(zip(c.ids, c.labels))])
    g.create_relations_batch([{"source_id": s, "target_id": d, "relation_type": t}
                              for s, d, t in zip(c.src, c.dst, c.types)])
    # an id carried by two labels: a label-less MATCH fans out, the file must not
    g.merge_nodes(["shared"], ["Pod"])
    g.merge_nodes(["shared"], ["Service"])
    g.merge_edges(["shared"], [c.ids[0]], ["CALLS"])
    return g


def test_roundtrip_restores_the_graph_exactly(tmp_path):
    from egraph import snapfile
    g = _graph()
    p = tmp_path / "g.egrsnap"
    hdr = snapfile.save(p, g)
    assert hdr["vertices"] == g.num_vertices and hdr["edges"] == g.num_edges
    r = snapfile.load_graph(p)
    assert r.vertex_ids() == g.vertex_ids()
    assert r.labels() == g.labels() and r.rel_types() == g.rel_types()
    for a, b in zip(r.export(), g.export()):
        np.testing.assert_array_equal(a, b)
    c1, c2 = r.csr(), g.csr()
    for k in c1:
        assert c1[k].tobytes() == c2[k].tobytes()
    assert r.node_props == {k: dict(v) for k, v in g.node_props.items()}
    # the stored CSR is the host build
    _, sec = snapfile.read(p)
    for k in ("row_ptr", "col", "meta", "val"):
        assert sec["csr_" + k].tobytes() == c2[k].tobytes()
    # the restored graph keeps MERGE semantics for later writes
    assert r.merge_edges(["shared"], [g.vertex_ids()[0]], ["CALLS"]) == 0


def test_damaged_and_foreign_files_are_rejected(tmp_path):
    from egraph import snapfile
    g = _graph()
    p = tmp_path / "g.egrsnap"
    snapfile.save(p, g, include_props=False)
    raw = bytearray(p.read_bytes())
    hdr, _ = snapfile.read(p)
    off = hdr["sections"]["edge_dst"]["offset"]
    bad = bytearray(raw)
    bad[off + 5] ^= 0x40
    (tmp_path / "bad").write_bytes(bytes(bad))
    with pytest.raises(ValueError, match="checksum"):
        snapfile.read(tmp_path / "bad")
    (tmp_path / "short").write_bytes(bytes(raw[: off + 3]))
    with pytest.raises(ValueError, match="truncated"):
        snapfile.read(tmp_path / "short")
    v2 = bytearray(raw)
    v2[8] = 2
    (tmp_path / "v2").write_bytes(bytes(v2))
    with pytest.raises(ValueError, match="format 2"):
        snapfile.read(tmp_path / "v2")
    (tmp_path / "junk").write_bytes(b"PK\x03\x04" + bytes(100))
    with pytest.raises(ValueError, match="not an evidence-graph"):
        snapfile.read(tmp_path / "junk")
