"""Versioned on-disk / wire format of an evidence graph and its device snapshot (SURVEY.md §8f
rank 2: checkpoint / resume and shipping graphs to a GPU host; replaces the persistence the
reference gets from Neo4j, src/database/neo4j.py:95-167).

Layout (little-endian):
    b"EGRSNAP\\0"  u32 format (=1)  u32 header_bytes  header (UTF-8 JSON)  pad to 64
    sections, each 64-byte aligned, described by header["sections"][name] =
        {"offset", "nbytes", "dtype", "count", "crc32"}
Sections:
    vertex_id_off  int64 [V+1]   vertex_id_blob  uint8   vertex ids (UTF-8), creation order
    vertex_label   uint8 [V]     index into header["labels"]
    edge_src / edge_dst int32 [E], edge_type uint8 [E]   (index into header["rel_types"]),
                                 creation order -- replaying them reproduces the graph exactly
    csr_row_ptr uint32 [V+1], csr_col uint32 [2E], csr_meta uint8 [2E], csr_val float32 [2E]
                                 (optional) the symmetric typed CSR for header["weights"], so a
                                 GPU host uploads it without rebuilding (egr_snapshot_from_csr)
    props          uint8         (optional) JSON of node / edge properties
Every section carries a CRC-32; readers reject unknown formats, truncated files and checksum
mismatches.  Nothing is unpickled: the header is JSON, the sections are raw arrays.
"""
from __future__ import annotations

import json
import zlib
from pathlib import Path

import numpy as np

from egraph.graph import EvidenceGraph, Snapshot

MAGIC = b"EGRSNAP\0"
FORMAT = 1
ALIGN = 64


def _pad(n: int) -> int:
    return (-n) % ALIGN


def save(path, graph: EvidenceGraph, snapshot: Snapshot | None = None, weights=None,
         include_csr: bool = True, include_props: bool = True) -> dict:
    """Write `graph` (and its CSR: downloaded from `snapshot` if given, else built on the host
    with `weights`).  Returns the header."""
    V, E = graph.num_vertices, graph.num_edges
    ids = graph.vertex_ids()
    enc = [s.encode() for s in ids]
    off = np.zeros(V + 1, np.int64)
    if V:
        np.cumsum([len(b) for b in enc], out=off[1:])
    vl, es, ed, et = graph.export()
    sections: dict[str, np.ndarray] = {
        "vertex_id_off": off,
        "vertex_id_blob": np.frombuffer(b"".join(enc), np.uint8) if off[-1] else np.zeros(0, np.uint8),
        "vertex_label": vl, "edge_src": es, "edge_dst": ed, "edge_type": et,
    }
    w = graph.weight_array(weights if snapshot is None else snapshot.weights)
    if include_csr:
        if snapshot is not None:
            if snapshot.n_vertices != V or snapshot.n_entries != 2 * E:
                raise ValueError("snapshot is not in sync with the graph (Snapshot.sync first)")
            d = snapshot.download()
            csr = {k: d[k] for k in ("row_ptr", "col", "meta", "val")}
        else:
            csr = graph.csr(weights)
        for k, a in csr.items():
            sections["csr_" + k] = a
    if include_props:
        props = {"nodes": [[lab, i, p] for (lab, i), p in graph.node_props.items()],
                 "edges": [[s, t, d, p] for (s, t, d), p in graph.edge_props.items()]}
        sections["props"] = np.frombuffer(json.dumps(props, default=str).encode(), np.uint8)
    header = {"format": FORMAT, "vertices": V, "edges": E, "labels": graph.labels(),
              "rel_types": graph.rel_types(), "weights": [float(x) for x in w], "sections": {}}
    # reserve the header's size with worst-case offsets, then pad the real header to it
    big = 10 ** 15
    for name, a in sections.items():
        a = np.ascontiguousarray(a)
        header["sections"][name] = {"offset": big, "nbytes": a.nbytes, "dtype": a.dtype.str,
                                    "count": int(a.size), "crc32": 0xFFFFFFFF}
    reserve = len(json.dumps(header).encode())
    pos = len(MAGIC) + 8 + reserve
    pos += _pad(pos)
    for name, a in sections.items():
        a = np.ascontiguousarray(a)
        header["sections"][name].update(offset=pos, crc32=zlib.crc32(a.tobytes()))
        pos += a.nbytes + _pad(a.nbytes)
    hb = json.dumps(header).encode()
    hb += b" " * (reserve - len(hb))
    with open(path, "wb") as f:
        f.write(MAGIC)
        f.write(np.array([FORMAT, len(hb)], "<u4").tobytes())
        f.write(hb)
        f.write(b"\0" * _pad(f.tell()))
        for name, a in sections.items():
            assert f.tell() == header["sections"][name]["offset"]
            b = np.ascontiguousarray(a).tobytes()
            f.write(b)
            f.write(b"\0" * _pad(len(b)))
    return header


def read(path) -> tuple[dict, dict[str, np.ndarray]]:
    """(header, sections) with every section checked against its CRC-32."""
    raw = Path(path).read_bytes()
    if len(raw) < len(MAGIC) + 8 or raw[: len(MAGIC)] != MAGIC:
        raise ValueError(f"{path}: not an evidence-graph snapshot file")
    fmt, hlen = np.frombuffer(raw[len(MAGIC): len(MAGIC) + 8], "<u4")
    if fmt != FORMAT:
        raise ValueError(f"{path}: snapshot format {fmt}, this reader handles {FORMAT}")
    header = json.loads(raw[len(MAGIC) + 8: len(MAGIC) + 8 + int(hlen)].decode())
    out = {}
    for name, s in header["sections"].items():
        lo, hi = s["offset"], s["offset"] + s["nbytes"]
        if hi > len(raw):
            raise ValueError(f"{path}: section {name} truncated")
        b = raw[lo:hi]
        if zlib.crc32(b) != s["crc32"]:
            raise ValueError(f"{path}: section {name} fails its checksum")
        out[name] = np.frombuffer(b, np.dtype(s["dtype"])).copy()
    return header, out


def load_graph(path) -> EvidenceGraph:
    """The host graph, exactly: same vertex order, edge order, label / type tables, properties."""
    header, s = read(path)
    off, blob = s["vertex_id_off"], s["vertex_id_blob"].tobytes()
    ids = [blob[off[i]:off[i + 1]].decode() for i in range(header["vertices"])]
    labels = header["labels"]
    g = EvidenceGraph()
    g.merge_nodes(ids, [labels[x] for x in s["vertex_label"]])
    g.add_edges_indexed(s["edge_src"], s["edge_dst"], s["edge_type"].astype(np.int32),
                        header["rel_types"])
    if g.num_vertices != header["vertices"] or g.num_edges != header["edges"]:
        raise ValueError(f"{path}: restored {g.num_vertices} vertices / {g.num_edges} edges, "
                         f"header says {header['vertices']} / {header['edges']}")
    if "props" in s:
        props = json.loads(s["props"].tobytes().decode())
        for lab, i, p in props["nodes"]:
            g.node_props[(lab, i)] = p
        for src, t, d, p in props["edges"]:
            g.edge_props[(src, t, d)] = p
    return g


def load_snapshot(path, device=None) -> Snapshot:
    """Upload the stored CSR straight to the device (no host graph, no CSR rebuild)."""
    header, s = read(path)
    if "csr_row_ptr" not in s:
        raise ValueError(f"{path}: saved without its CSR (include_csr=False)")
    return Snapshot.from_csr(s["csr_row_ptr"], s["csr_col"], s["csr_meta"], s["csr_val"],
                             s["vertex_label"], header["labels"], device)
