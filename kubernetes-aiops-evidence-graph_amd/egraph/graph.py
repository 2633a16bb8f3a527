"""Evidence graph (host MERGE semantics), device snapshot and per-batch propagation plans.

  EvidenceGraph  <- GraphService.create_entities_batch / create_relations_batch
                    (src/database/neo4j.py:95-113, :145-167); vertex/edge structure lives in
                    libegraph (C++), properties stay here (SET n += props, last write wins).
  Snapshot       <- the Neo4j store: symmetric typed CSR resident in HBM.
  Plan           <- apoc.path.subgraphAll(maxLevel=k) candidate sets (neo4j.py:169-202) plus
                    the build-defined typed propagation / top-k.
"""
from __future__ import annotations

import ctypes as C
import os
from collections.abc import Iterable, Sequence

import numpy as np
import torch

from . import _lib as L
from .device import require_device, to_device

# Per relationship type (forward, reverse) propagation weights -- DESIGN.md §A9.
DEFAULT_WEIGHTS: dict[str, tuple[float, float]] = {
    "AFFECTS": (1.0, 1.0),
    "CORRELATES_WITH": (1.0, 1.0),
    "HAS_RECENT_CHANGE": (0.9, 0.9),
    "SCHEDULED_ON": (0.6, 0.6),
    "OWNS": (0.8, 0.8),
    "SELECTS": (0.7, 0.7),
    "CALLS": (0.5, 0.5),
    "HAS_EVENT": (0.9, 0.9),
    "HAS_LOG_PATTERN": (0.9, 0.9),
    "HAS_METRIC_ANOMALY": (0.9, 0.9),
    "OBSERVED_ON": (0.6, 0.6),
    "AGGREGATES": (0.8, 0.8),
}
DEFAULT_OTHER_WEIGHT = (0.5, 0.5)


def str_blob(strs: Sequence[str]) -> tuple[bytes, np.ndarray]:
    """UTF-8 blob + int64 offsets [n+1] for the C-ABI string arrays (native for a list of strs:
    csrc/pyhost.c str_blob)."""
    if type(strs) is list:
        r = L.pyhost.str_blob(strs)
        if r is not None:
            return r[0], np.frombuffer(r[1], np.int64)
    if isinstance(strs, list) and strs and all(type(s) is str for s in strs):
        joined = "".join(strs)
        if joined.isascii():                  # one encode; byte lengths = character lengths
            off = np.zeros(len(strs) + 1, np.int64)
            np.cumsum(np.fromiter(map(len, strs), np.int64, len(strs)), out=off[1:])
            return joined.encode("ascii"), off
    enc = [s.encode() for s in strs]
    off = np.zeros(len(enc) + 1, np.int64)
    if enc:
        np.cumsum([len(b) for b in enc], out=off[1:])
    return b"".join(enc), off


def _addr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


def _field(x, name, default=KeyError):
    if isinstance(x, dict):
        return x[name] if default is KeyError else x.get(name, default)
    return getattr(x, name) if default is KeyError else getattr(x, name, default)


def locality_order(row_ptr: np.ndarray, col: np.ndarray) -> np.ndarray:
    """A vertex order that keeps the rows a 3-hop frontier walks close together: every vertex
    hangs under its highest-degree neighbour when that one has a higher degree (ties: the lower
    id), and the resulting forest is laid out root by root, each root followed by its subtrees
    (children by id).  On a Kubernetes evidence graph the roots are the Node hubs, deployments and
    services, a Node's pods follow it and each pod's attachments follow the pod -- the pods a
    Node hub expands to (most of a frontier's last-hop rows) become contiguous.  Returns the new
    order as a list of old vertex ids (order[i] = the vertex placed at i)."""
    rp = np.asarray(row_ptr, np.int64)
    col = np.asarray(col, np.int64)
    V = len(rp) - 1
    deg = np.diff(rp)
    parent = np.full(V, -1, np.int64)
    if len(col):
        src = np.repeat(np.arange(V), deg)
        o = np.lexsort((col, -deg[col], src))          # per row: highest degree, then lowest id
        first = np.ones(len(o), bool)
        first[1:] = src[o][1:] != src[o][:-1]
        sel = o[first]
        best = np.full(V, -1, np.int64)
        best[src[sel]] = col[sel]
        ok = best >= 0
        parent[ok] = np.where(deg[best[ok]] > deg[ok], best[ok], -1)
    # depth and root of every vertex (degrees strictly grow towards a root: no cycles)
    root = np.arange(V)
    top = np.arange(V)          # the vertex right under the root (itself for roots / children)
    depth = np.zeros(V, np.int64)
    cur = parent.copy()
    while True:
        m = cur >= 0
        if not m.any():
            break
        top = np.where(m & (parent[np.maximum(cur, 0)] >= 0), cur, top)
        root = np.where(m, cur, root)
        depth += m
        cur = np.where(m, parent[np.maximum(cur, 0)], -1)
    return np.lexsort((np.arange(V), depth, top, root))


class VertexOf:
    """EvidenceGraph.vertex_of: a read-only (label, id) -> vertex mapping over the native graph
    (egr_graph_lookup_labeled).  It replaces a Python dict mirror of every MERGEd (label, id)
    pair, whose upkeep cost about a microsecond per merged node on a 250k-vertex graph."""
    __slots__ = ("_g",)

    def __init__(self, g: "EvidenceGraph"):
        self._g = g

    def get(self, key, default=None):
        lab, i = key
        v = int(self._g.lookup_labeled([str(i)], [str(lab)])[0])
        return default if v < 0 else v

    def __getitem__(self, key) -> int:
        v = self.get(key)
        if v is None:
            raise KeyError(key)
        return v

    def __contains__(self, key) -> bool:
        return self.get(key) is not None

    def __len__(self) -> int:
        return self._g.num_vertices

    def items(self):
        g = self._g
        labels, vl, ids = g.labels(), g.vertex_labels(), g._vertex_ids()
        return (((labels[int(vl[v])], ids[v]), v) for v in range(len(ids)))

    def __iter__(self):
        return (k for k, _ in self.items())


class EvidenceGraph:
    """The evidence graph with the reference's MERGE semantics (host side, C++)."""

    def __init__(self):
        h = C.c_void_p()
        L.check(L.lib.egr_graph_create(C.byref(h)), "egr_graph_create")
        self._h = h
        self._label_names: list[str] = []
        self._type_names: list[str] = []
        self.node_props: dict[tuple[str, str], dict] = {}
        self._ids: list[str] = []                           # vertex -> id (creation order)
        self.edge_props: dict[tuple[str, str, str], dict] = {}

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and getattr(L, "lib", None) is not None:
            L.lib.egr_graph_free(h)
            self._h = None

    @property
    def handle(self):
        return self._h

    # ---- writes ---------------------------------------------------------------------------
    def merge_nodes(self, ids: Sequence[str], labels: Sequence[str]) -> np.ndarray:
        """MERGE (n:label {id}) for each pair; returns the vertex index of each item."""
        if len(ids) != len(labels):
            raise ValueError("ids and labels differ in length")
        ib, io = str_blob(ids)
        lb, lo = str_blob(labels)
        out = np.empty(len(ids), np.int32)
        n0 = int(L.lib.egr_graph_num_vertices(self._h))
        L.check(L.lib.egr_graph_merge_nodes(self._h, ib, _addr(io), lb, _addr(lo), len(ids),
                                            _addr(out)), "egr_graph_merge_nodes")
        new = out >= n0
        if len(self._ids) == n0 and new.any():
            # the new vertices are numbered n0.. in creation order: each one's first item
            _, first = np.unique(out[new], return_index=True)
            self._ids.extend(ids[j] for j in np.flatnonzero(new)[first].tolist())
        return out

    @property
    def vertex_of(self) -> "VertexOf":
        """(label, id) -> vertex, read from the native graph (a mapping view)."""
        return VertexOf(self)

    def lookup_labeled(self, ids: Sequence[str], labels: Sequence[str] | str) -> np.ndarray:
        """MATCH (n:label {id}) per id: its vertex or -1 (egr_graph_lookup_labeled).  `labels`:
        one label per id, or one label for all of them."""
        if isinstance(labels, str):
            labels = [labels] * len(ids)
        if len(ids) != len(labels):
            raise ValueError("ids and labels differ in length")
        ib, io = str_blob(list(ids))
        lb, lo = str_blob(list(labels))
        out = np.empty(len(ids), np.int32)
        L.check(L.lib.egr_graph_lookup_labeled(self._h, ib, _addr(io), len(out), lb, _addr(lo),
                                               _addr(out)), "egr_graph_lookup_labeled")
        return out

    def merge_edges(self, src: Sequence[str], dst: Sequence[str], types: Sequence[str]) -> int:
        """MATCH/MATCH/MERGE per relation; returns the number of edges actually created."""
        if not (len(src) == len(dst) == len(types)):
            raise ValueError("src, dst and types differ in length")
        sb, so = str_blob(src)
        db, do = str_blob(dst)
        tb, to = str_blob(types)
        created = C.c_int64(0)
        L.check(L.lib.egr_graph_merge_edges(self._h, sb, _addr(so), db, _addr(do), tb, _addr(to),
                                            len(src), C.byref(created)), "egr_graph_merge_edges")
        return created.value

    def add_edges_indexed(self, src: np.ndarray, dst: np.ndarray, type_idx: np.ndarray,
                          type_names: Sequence[str]) -> int:
        """MERGE edges by vertex index (exact restore; egr_graph_add_edges_indexed)."""
        src = np.ascontiguousarray(src, np.int32)
        dst = np.ascontiguousarray(dst, np.int32)
        ti = np.ascontiguousarray(type_idx, np.int32)
        if not (len(src) == len(dst) == len(ti)):
            raise ValueError("edge arrays differ in length")
        tb, to = str_blob(type_names)
        created = C.c_int64(0)
        L.check(L.lib.egr_graph_add_edges_indexed(self._h, _addr(src), _addr(dst), tb, _addr(to),
                                                  len(type_names), _addr(ti), len(src),
                                                  C.byref(created)), "egr_graph_add_edges_indexed")
        return created.value

    def create_entities_batch(self, entities: Iterable) -> int:
        """GraphService.create_entities_batch: returns the number of items attempted (:112)."""
        entities = list(entities)
        ids = [str(_field(e, "id")) for e in entities]
        labels = [str(_field(e, "type")) for e in entities]
        self.merge_nodes(ids, labels)
        for e, i, lab in zip(entities, ids, labels):
            props = dict(_field(e, "properties", None) or {})
            props["id"] = i                                    # neo4j.py:101-102
            self.node_props.setdefault((lab, i), {}).update(props)
        return len(entities)

    def create_relations_batch(self, relations: Iterable) -> int:
        """GraphService.create_relations_batch: returns the number of items attempted (:166)."""
        relations = list(relations)
        src = [str(_field(r, "source_id")) for r in relations]
        dst = [str(_field(r, "target_id")) for r in relations]
        typ = [str(_field(r, "relation_type")) for r in relations]
        self.merge_edges(src, dst, typ)
        known = set(self.vertex_ids_set())
        for r, s, d, t in zip(relations, src, dst, typ):
            if s in known and d in known:
                self.edge_props.setdefault((s, t, d), {}).update(dict(_field(r, "properties", None) or {}))
        return len(relations)

    # ---- reads ----------------------------------------------------------------------------
    @property
    def num_vertices(self) -> int:
        return int(L.lib.egr_graph_num_vertices(self._h))

    @property
    def num_edges(self) -> int:
        return int(L.lib.egr_graph_num_edges(self._h))

    def _names(self, cache: list, count_fn, name_fn) -> list[str]:
        # label / type numbers are interned in creation order and never renumbered: only the
        # names added since the last call are fetched
        for i in range(len(cache), count_fn(self._h)):
            n = name_fn(self._h, i, None, 0)
            buf = C.create_string_buffer(max(int(n), 1))
            name_fn(self._h, i, buf, n)
            cache.append(buf.raw[:n].decode())
        return list(cache)

    def labels(self) -> list[str]:
        return self._names(self._label_names, L.lib.egr_graph_num_labels, L.lib.egr_graph_label_name)

    def rel_types(self) -> list[str]:
        return self._names(self._type_names, L.lib.egr_graph_num_rel_types,
                           L.lib.egr_graph_rel_type_name)

    def vertex_id(self, v: int) -> str:
        if 0 <= v < len(self._ids):
            return self._ids[v]
        n = L.lib.egr_graph_vertex_id(self._h, v, None, 0)
        if n < 0:
            raise IndexError(v)
        buf = C.create_string_buffer(max(int(n), 1))
        L.lib.egr_graph_vertex_id(self._h, v, buf, n)
        return buf.raw[:n].decode()

    def vertex_ids(self) -> list[str]:
        """The id of every vertex, by vertex index (a copy: callers may edit it)."""
        return list(self._vertex_ids())

    def _vertex_ids(self) -> list[str]:
        """The graph's own id list (kept by merge_nodes; rebuilt from the native graph if it
        ever disagrees with it).  Read-only for callers inside the package."""
        V = self.num_vertices
        if len(self._ids) != V:
            self._ids = []
            self._ids = [self.vertex_id(v) for v in range(V)]
        return self._ids

    def vertex_ids_set(self) -> set[str]:
        return set(self._vertex_ids())

    def lookup(self, ids: Sequence[str]) -> np.ndarray:
        """First vertex carrying each id (-1 if none)."""
        return self.lookup_blob(*str_blob(ids))

    def lookup_blob(self, blob: bytes, off: np.ndarray) -> np.ndarray:
        """lookup() of ids given as a utf-8 blob + int64 offsets [n+1] (str_blob's form)."""
        off = np.ascontiguousarray(off, np.int64)
        out = np.empty(len(off) - 1, np.int32)
        L.check(L.lib.egr_graph_lookup(self._h, blob, _addr(off), len(out), _addr(out)),
                "egr_graph_lookup")
        return out

    def export(self) -> tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
        """(vertex_label u8[V], edge_src i32[E], edge_dst i32[E], edge_type u8[E])."""
        V, E = self.num_vertices, self.num_edges
        vl = np.empty(V, np.uint8)
        es, ed = np.empty(E, np.int32), np.empty(E, np.int32)
        et = np.empty(E, np.uint8)
        L.check(L.lib.egr_graph_export(self._h, _addr(vl), _addr(es), _addr(ed), _addr(et)),
                "egr_graph_export")
        return vl, es, ed, et

    def vertex_labels(self, first: int = 0) -> np.ndarray:
        """u8 labels of vertices [first, V) (no edge copy)."""
        vl = np.empty(max(self.num_vertices, 1), np.uint8)
        L.check(L.lib.egr_graph_export(self._h, _addr(vl), None, None, None), "egr_graph_export")
        return vl[first:self.num_vertices]

    def export_edges(self, first: int, n: int | None = None) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Edges [first, first + n) in creation order (what MERGE batches appended since)."""
        if n is None:
            n = self.num_edges - first
        es, ed = np.empty(max(n, 1), np.int32), np.empty(max(n, 1), np.int32)
        et = np.empty(max(n, 1), np.uint8)
        L.check(L.lib.egr_graph_export_edges(self._h, first, n, _addr(es), _addr(ed), _addr(et)),
                "egr_graph_export_edges")
        return es[:n], ed[:n], et[:n]

    def weight_array(self, weights: dict[str, tuple[float, float]] | None = None) -> np.ndarray:
        """[n_types*2] fp32 (fwd, rev) weights in this graph's type order."""
        weights = DEFAULT_WEIGHTS if weights is None else weights
        names = self.rel_types()
        w = np.empty(max(2 * len(names), 2), np.float32)
        for t, name in enumerate(names):
            w[2 * t: 2 * t + 2] = weights.get(name, DEFAULT_OTHER_WEIGHT)
        return w

    def csr(self, weights=None) -> dict[str, np.ndarray]:
        """Host copy of the symmetric typed CSR (exactly what the snapshot uploads)."""
        V, E = self.num_vertices, self.num_edges
        w = self.weight_array(weights)
        row_ptr = np.empty(V + 1, np.uint32)
        col = np.empty(max(2 * E, 1), np.uint32)
        meta = np.empty(max(2 * E, 1), np.uint8)
        val = np.empty(max(2 * E, 1), np.float32)
        L.check(L.lib.egr_graph_csr(self._h, _addr(w), len(self.rel_types()), _addr(row_ptr),
                                    _addr(col), _addr(meta), _addr(val)), "egr_graph_csr")
        return {"row_ptr": row_ptr, "col": col[:2 * E], "meta": meta[:2 * E], "val": val[:2 * E]}

    def snapshot(self, weights=None, device=None) -> "Snapshot":
        return Snapshot(self, weights, device)

    def within_hops(self, v: int, hops: int) -> np.ndarray:
        """bool[V]: the vertices within `hops` undirected hops of vertex v, v included (the node
        set of apoc.path.subgraphAll(maxLevel=hops), host side)."""
        csr = self.csr()
        rp, col = csr["row_ptr"].astype(np.int64), csr["col"]
        seen = np.zeros(self.num_vertices, bool)
        seen[v] = True
        fr = np.array([v], np.int64)
        for _ in range(hops):
            if not len(fr):
                break
            lens = rp[fr + 1] - rp[fr]
            idx = np.repeat(rp[fr] - np.concatenate(([0], np.cumsum(lens)[:-1])), lens) + np.arange(lens.sum())
            nb = np.unique(col[idx])
            fr = nb[~seen[nb]].astype(np.int64)
            seen[fr] = True
        return seen

    def subgraph(self, keep: np.ndarray) -> "EvidenceGraph":
        """A new graph of the vertices with keep[v] (ids, labels, properties, relative order)
        and the edges between them (creation order, types, properties): what DETACH DELETE of
        the other vertices leaves."""
        keep = np.asarray(keep, bool)
        vl, es, ed, et = self.export()
        labels, types, ids = self.labels(), self.rel_types(), self._vertex_ids()
        kept = np.nonzero(keep)[0]
        out = EvidenceGraph()
        if len(kept):
            out.merge_nodes([ids[v] for v in kept], [labels[vl[v]] for v in kept])
        remap = np.full(len(vl), -1, np.int64)
        remap[kept] = np.arange(len(kept))
        ok = keep[es] & keep[ed] if len(es) else np.zeros(0, bool)
        if ok.any():
            out.add_edges_indexed(remap[es[ok]], remap[ed[ok]], et[ok].astype(np.int32), types)
        if self.node_props:
            keys = list(self.node_props)
            vs = self.lookup_labeled([i for _, i in keys], [lab for lab, _ in keys])
            out.node_props = {k: dict(self.node_props[k]) for k, v in zip(keys, vs.tolist())
                              if v >= 0 and keep[v]}
        alive = out.vertex_ids_set()
        out.edge_props = {k: dict(p) for k, p in self.edge_props.items()
                          if k[0] in alive and k[2] in alive}
        return out


class Snapshot:
    """Typed CSR + vertex labels resident in HBM on one device."""

    def __init__(self, graph: EvidenceGraph | None, weights=None, device=None, _handle=None,
                 _labels=None):
        self.dev = require_device(device)
        if _handle is None:
            w = graph.weight_array(weights)
            h = C.c_void_p()
            L.check(L.lib.egr_snapshot_create(graph.handle, _addr(w), len(graph.rel_types()),
                                              self.dev.index, C.byref(h)), "egr_snapshot_create")
        else:
            h = _handle
        self._h = h
        self.weights = weights
        self._refresh_info()
        self.labels = graph.labels() if graph is not None else list(_labels or [])
        # the host graph's edge count this snapshot reflects (for incremental sync)
        self.synced_edges = graph.num_edges if graph is not None else None

    def _refresh_info(self):
        nv, ne = C.c_int64(), C.c_int64()
        L.check(L.lib.egr_snapshot_info(self._h, C.byref(nv), C.byref(ne)), "egr_snapshot_info")
        self.n_vertices, self.n_entries = nv.value, ne.value

    @property
    def version(self) -> int:
        return int(L.lib.egr_snapshot_version(self._h))

    def update(self, new_vlabel: torch.Tensor, edge_src: torch.Tensor, edge_dst: torch.Tensor,
               edge_type: torch.Tensor, weight_array: np.ndarray, stream=None) -> None:
        """egr_snapshot_update with device tensors (u8 labels, i32 ids, u8 types): append
        vertices and NEW edges, rebuilding the affected rows and values on the device."""
        n, m = new_vlabel.numel(), edge_src.numel()
        if not (edge_dst.numel() == m == edge_type.numel()):
            raise ValueError("edge arrays differ in length")
        w = np.ascontiguousarray(weight_array, np.float32)
        st = L.stream_handle(self.dev) if stream is None else stream
        L.check(L.lib.egr_snapshot_update(self._h, L.ptr(new_vlabel), n, L.ptr(edge_src),
                                          L.ptr(edge_dst), L.ptr(edge_type), m, _addr(w),
                                          len(w) // 2, st), "egr_snapshot_update")
        self._refresh_info()

    def sync(self, graph: EvidenceGraph, stream=None) -> tuple[int, int]:
        """Bring the snapshot up to `graph` (the one it was built from, grown by MERGE batches
        since) with one incremental update.  Returns (new vertices, new edges)."""
        if self.synced_edges is None:
            raise ValueError("snapshot was not built from an EvidenceGraph")
        V0, E0 = self.n_vertices, self.synced_edges
        V, E = graph.num_vertices, graph.num_edges
        if V == V0 and E == E0:
            return 0, 0
        vl = graph.vertex_labels(V0)
        es, ed, et = graph.export_edges(E0, E - E0)
        with torch.cuda.device(self.dev):
            self.update(to_device(np.ascontiguousarray(vl), self.dev),
                        to_device(es.view(np.uint32), self.dev), to_device(ed.view(np.uint32), self.dev),
                        to_device(et, self.dev), graph.weight_array(self.weights), stream)
        self.synced_edges = E
        self.labels = graph.labels()
        return V - V0, E - E0

    def within(self, sources: torch.Tensor, hops: int, stream=None) -> torch.Tensor:
        """uint8 [V] device tensor: undirected hops from the nearest source vertex (i32 device
        tensor), 255 beyond `hops` (egr_snapshot_within)."""
        out = torch.empty(max(self.n_vertices, 1), dtype=torch.uint8, device=self.dev)[: self.n_vertices]
        st = L.stream_handle(self.dev) if stream is None else stream
        L.check(L.lib.egr_snapshot_within(self._h, L.ptr(sources), sources.numel(), hops, L.ptr(out), st),
                "egr_snapshot_within")
        return out

    OUT, IN = 1, 0      # typed_neighbors directions: (v)-[:T]->(u) / (v)<-[:T]-(u)

    def typed_neighbors(self, vertices, rel_type: int, direction: int, label: int = -1,
                        stream=None) -> list[np.ndarray]:
        """One typed hop of a Cypher path pattern, per query vertex (egr_snapshot_typed_neighbors):
        the neighbours u with (v)-[:rel_type]->(u) (direction OUT) or (v)<-[:rel_type]-(u) (IN)
        and label index `label` (-1: any), in CSR order (u ascending), as int64 arrays.  Two
        launches: the counts, then the matches into their segments."""
        q = np.ascontiguousarray(vertices, np.int64)
        n = len(q)
        if n == 0:
            return []
        if rel_type < 0:                   # a relationship type the graph has never seen
            return [np.empty(0, np.int64) for _ in range(n)]
        st = L.stream_handle(self.dev) if stream is None else stream
        dq = to_device(np.where(q >= 0, q, 0xFFFFFFFF).astype(np.uint32), self.dev)
        cnt = torch.empty(n, dtype=torch.int32, device=self.dev)
        L.check(L.lib.egr_snapshot_typed_neighbors(self._h, L.ptr(dq), n, int(rel_type), int(direction),
                                                   int(label), None, None, L.ptr(cnt), st),
                "egr_snapshot_typed_neighbors")
        counts = cnt.cpu().numpy().astype(np.int64)
        off = np.concatenate([[0], np.cumsum(counts)])
        out = torch.empty(max(int(off[-1]), 1), dtype=torch.int32, device=self.dev)
        doff = to_device(off[:-1], self.dev)
        L.check(L.lib.egr_snapshot_typed_neighbors(self._h, L.ptr(dq), n, int(rel_type), int(direction),
                                                   int(label), L.ptr(doff), L.ptr(out), L.ptr(cnt), st),
                "egr_snapshot_typed_neighbors")
        flat = out.cpu().numpy().view(np.uint32).astype(np.int64)
        return [flat[off[i]:off[i + 1]] for i in range(n)]

    def download(self) -> dict[str, np.ndarray]:
        """Host copy of the device CSR (the layout of EvidenceGraph.csr()) and labels."""
        V, NE = self.n_vertices, self.n_entries
        rp = np.empty(V + 1, np.uint32)
        col, meta = np.empty(max(NE, 1), np.uint32), np.empty(max(NE, 1), np.uint8)
        val, vl = np.empty(max(NE, 1), np.float32), np.empty(max(V, 1), np.uint8)
        L.check(L.lib.egr_snapshot_download(self._h, _addr(rp), _addr(col), _addr(meta), _addr(val),
                                            _addr(vl)), "egr_snapshot_download")
        return {"row_ptr": rp, "col": col[:NE], "meta": meta[:NE], "val": val[:NE], "vlabel": vl[:V]}

    @classmethod
    def from_csr(cls, row_ptr, col, meta, val, vlabel, labels=None, device=None) -> "Snapshot":
        """A snapshot of raw CSR arrays (host numpy), e.g. a partition's local graph
        (egraph.shard.LocalGraph): egr_snapshot_from_csr."""
        dev = require_device(device)
        arrs = [np.ascontiguousarray(row_ptr, np.uint32), np.ascontiguousarray(col, np.uint32),
                np.ascontiguousarray(meta, np.uint8), np.ascontiguousarray(val, np.float32),
                np.ascontiguousarray(vlabel, np.uint8)]
        h = C.c_void_p()
        L.check(L.lib.egr_snapshot_from_csr(*[_addr(a) for a in arrs], len(arrs[0]) - 1,
                                            dev.index, C.byref(h)), "egr_snapshot_from_csr")
        return cls(None, device=dev, _handle=h, _labels=labels)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and getattr(L, "lib", None) is not None:
            L.lib.egr_snapshot_free(h)
            self._h = None

    @property
    def handle(self):
        return self._h

    def plan(self, n_cols: int, max_seeds: int, k: int = 10) -> "Plan":
        return Plan(self, n_cols, max_seeds, k)

    def frontier(self, n_cols: int, max_seeds: int, k: int = 10, pool_entries: int = 0) -> "Frontier":
        return Frontier(self, n_cols, max_seeds, k, pool_entries)


class Plan:
    """Per-batch device workspace: B incident columns over one snapshot."""

    def __init__(self, snap: Snapshot, n_cols: int, max_seeds: int, k: int = 10):
        self.snap = snap
        self.dev = snap.dev
        self.B, self.k = n_cols, k
        h = C.c_void_p()
        L.check(L.lib.egr_plan_create(snap.handle, n_cols, max_seeds, k, C.byref(h)), "egr_plan_create")
        self._h = h
        self.tile_width = L.lib.egr_plan_tile_width(h)
        self.out_ids = torch.empty(n_cols * k, dtype=torch.int32, device=self.dev)
        self.out_scores = torch.empty(n_cols * k, dtype=torch.float32, device=self.dev)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and getattr(L, "lib", None) is not None:
            L.lib.egr_plan_free(h)
            self._h = None

    def _st(self, stream):
        return L.stream_handle(self.dev) if stream is None else stream

    @property
    def padded_cols(self) -> int:
        """Columns padded to the tile width (row length of the pack/unpack buffers)."""
        return (self.B + self.tile_width - 1) // self.tile_width * self.tile_width

    def set_owned(self, n_owned: int):
        """Rows [0, n_owned) are the only top-k candidates (a partition's owned vertices)."""
        L.check(L.lib.egr_plan_set_owned(self._h, n_owned), "egr_plan_set_owned")

    def pack_scores(self, rows: torch.Tensor, out: torch.Tensor, stream=None):
        L.check(L.lib.egr_plan_pack_scores(self._h, L.ptr(rows), rows.numel(), L.ptr(out),
                                           self._st(stream)), "egr_plan_pack_scores")

    def unpack_scores(self, rows: torch.Tensor, src: torch.Tensor, inp: torch.Tensor, stream=None):
        L.check(L.lib.egr_plan_unpack_scores(self._h, L.ptr(rows), L.ptr(src), rows.numel(),
                                             L.ptr(inp), self._st(stream)), "egr_plan_unpack_scores")

    def pack_reach(self, rows: torch.Tensor, out: torch.Tensor, stream=None):
        L.check(L.lib.egr_plan_pack_reach(self._h, L.ptr(rows), rows.numel(), L.ptr(out),
                                          self._st(stream)), "egr_plan_pack_reach")

    def unpack_reach(self, rows: torch.Tensor, src: torch.Tensor, inp: torch.Tensor, stream=None):
        L.check(L.lib.egr_plan_unpack_reach(self._h, L.ptr(rows), L.ptr(src), rows.numel(),
                                            L.ptr(inp), self._st(stream)), "egr_plan_unpack_reach")

    def pack_sparse(self, what: str, rows: torch.Tensor, seg: np.ndarray, out: torch.Tensor,
                    stream=None) -> list[int]:
        """Non-zero entries of the send rows (egr_plan_pack_sparse) into `out` (int64, device);
        returns the entry count per peer (synchronises the stream)."""
        P = len(seg) - 1
        seg = np.ascontiguousarray(seg, dtype=np.int64)
        counts = np.zeros(P, np.int64)
        L.check(L.lib.egr_plan_pack_sparse(self._h, 1 if what == "reach" else 0, L.ptr(rows),
                                           rows.numel(), _addr(seg), P, L.ptr(out), out.numel(),
                                           _addr(counts), self._st(stream)), "egr_plan_pack_sparse")
        return counts.tolist()

    def unpack_sparse(self, what: str, recv_vertex: torch.Tensor, entries: torch.Tensor,
                      eseg: torch.Tensor, rbase: torch.Tensor, stream=None) -> None:
        n = entries.numel() // (2 if what == "reach" else 1)
        L.check(L.lib.egr_plan_unpack_sparse(self._h, 1 if what == "reach" else 0,
                                             L.ptr(recv_vertex), recv_vertex.numel(), L.ptr(entries),
                                             n, L.ptr(eseg), L.ptr(rbase), rbase.numel(),
                                             self._st(stream)), "egr_plan_unpack_sparse")

    @staticmethod
    def slot_words(what: str, peer_cap: int) -> int:
        """int64 words of one peer slot of the fixed-capacity exchange: the header (the
        sender's entry count for that peer), then peer_cap entries of 1 (scores) / 2 (reach)."""
        return 1 + peer_cap * (2 if what == "reach" else 1)

    def pack_sparse_cap(self, what: str, rows: torch.Tensor, seg_dev: torch.Tensor, out: torch.Tensor,
                        peer_cap: int, overflow: torch.Tensor, counts: torch.Tensor | None = None,
                        stream=None) -> None:
        """egr_plan_pack_sparse_cap: the non-zero entries into fixed slots, one per peer
        (out: int64 [P * slot_words]), each slot headed by its entry count; past peer_cap the
        entries are dropped and `overflow` (device int32 [1]) is set.  `counts` (device int64
        [P]), when given, gets the counts too.  One launch chain, no synchronisation."""
        P = seg_dev.numel() - 1
        if out.numel() < P * self.slot_words(what, peer_cap) or (counts is not None and counts.numel() < P):
            raise ValueError("pack_sparse_cap: output slots or counts too small")
        L.check(L.lib.egr_plan_pack_sparse_cap(self._h, 1 if what == "reach" else 0, L.ptr(rows),
                                               rows.numel(), L.ptr(seg_dev), P, L.ptr(out), int(peer_cap),
                                               L.ptr(counts), L.ptr(overflow), self._st(stream)),
                "egr_plan_pack_sparse_cap")

    def unpack_sparse_cap(self, what: str, recv_vertex: torch.Tensor, entries: torch.Tensor,
                          peer_cap: int, rbase: torch.Tensor, overflow: torch.Tensor | None = None,
                          stream=None) -> None:
        """egr_plan_unpack_sparse_cap: zero the received halo rows and scatter every sender's
        slot (its header's count of entries, at most peer_cap); a header past peer_cap sets
        `overflow` when given."""
        L.check(L.lib.egr_plan_unpack_sparse_cap(self._h, 1 if what == "reach" else 0,
                                                 L.ptr(recv_vertex), recv_vertex.numel(), L.ptr(entries),
                                                 int(peer_cap), L.ptr(overflow), L.ptr(rbase),
                                                 rbase.numel(), self._st(stream)),
                "egr_plan_unpack_sparse_cap")

    def halo_exchange_rccl(self, what: str, rows: torch.Tensor, seg_dev: torch.Tensor,
                           peer_cap: int, send_slots: torch.Tensor, recv_slots: torch.Tensor,
                           recv_vertex: torch.Tensor, rbase: torch.Tensor, overflow: torch.Tensor,
                           rccl_comm: int, stream=None) -> None:
        """egr_plan_halo_exchange: pack_sparse_cap, ONE ncclAllToAll of the slots over the RCCL
        communicator `rccl_comm` (an ncclComm_t address of P ranks), unpack_sparse_cap -- the
        C-ABI path for callers without torch.distributed (egraph/shard.py's TorchComm issues
        the same steps through torch)."""
        P = seg_dev.numel() - 1
        if min(send_slots.numel(), recv_slots.numel()) < P * self.slot_words(what, peer_cap):
            raise ValueError("halo_exchange_rccl: slot buffers too small")
        L.check(L.lib.egr_plan_halo_exchange(self._h, 1 if what == "reach" else 0, L.ptr(rows),
                                             rows.numel(), L.ptr(seg_dev), P, int(peer_cap),
                                             L.ptr(send_slots), L.ptr(recv_slots), L.ptr(recv_vertex),
                                             recv_vertex.numel(), L.ptr(rbase), L.ptr(overflow),
                                             rccl_comm, self._st(stream)), "egr_plan_halo_exchange")

    def set_seeds(self, vertex: torch.Tensor, col: torch.Tensor, val: torch.Tensor, stream=None):
        n = vertex.numel()
        if not (col.numel() == n == val.numel()):
            raise ValueError("seed arrays differ in length")
        L.check(L.lib.egr_plan_set_seeds(self._h, L.ptr(vertex), L.ptr(col), L.ptr(val), n,
                                         self._st(stream)), "egr_plan_set_seeds")

    def set_sources(self, source_vertex: torch.Tensor, stream=None):
        if source_vertex.numel() != self.B:
            raise ValueError(f"need one source vertex per column ({self.B})")
        L.check(L.lib.egr_plan_set_sources(self._h, L.ptr(source_vertex), self._st(stream)),
                "egr_plan_set_sources")

    def hop(self, stream=None):
        L.check(L.lib.egr_plan_hop(self._h, self._st(stream)), "egr_plan_hop")

    def step(self, stream=None):
        """One hop of propagation and one of reachability (egr_plan_step)."""
        L.check(L.lib.egr_plan_step(self._h, self._st(stream)), "egr_plan_step")

    def final_step(self, exclude_label: int = -1, stream=None):
        """The last hop: step() plus the top-k candidate lists for topk(exclude_label)."""
        L.check(L.lib.egr_plan_final_step(self._h, exclude_label, self._st(stream)),
                "egr_plan_final_step")

    def candidates(self, exclude_label: int = -1, stream=None):
        """Top-k candidate lists from the current reach sets (no hop)."""
        L.check(L.lib.egr_plan_candidates(self._h, exclude_label, self._st(stream)),
                "egr_plan_candidates")

    def reach_hop(self, stream=None):
        L.check(L.lib.egr_plan_reach_hop(self._h, self._st(stream)), "egr_plan_reach_hop")

    def topk(self, exclude_label: int = -1, stream=None) -> tuple[torch.Tensor, torch.Tensor]:
        L.check(L.lib.egr_plan_topk(self._h, exclude_label, L.ptr(self.out_ids),
                                    L.ptr(self.out_scores), self._st(stream)), "egr_plan_topk")
        return self.out_ids.view(self.B, self.k), self.out_scores.view(self.B, self.k)

    def run(self, hops: int = 3, exclude_label: int = -1, stream=None):
        L.check(L.lib.egr_plan_run(self._h, hops, exclude_label, L.ptr(self.out_ids),
                                   L.ptr(self.out_scores), self._st(stream)), "egr_plan_run")
        return self.out_ids.view(self.B, self.k), self.out_scores.view(self.B, self.k)

    def read_scores(self, stream=None) -> torch.Tensor:
        out = torch.empty(self.snap.n_vertices * self.B, dtype=torch.float32, device=self.dev)
        L.check(L.lib.egr_plan_read_scores(self._h, L.ptr(out), self._st(stream)), "egr_plan_read_scores")
        return out.view(self.snap.n_vertices, self.B)

    def read_reach(self, stream=None) -> torch.Tensor:
        W = (self.B + 63) // 64
        out = torch.empty(W * self.snap.n_vertices, dtype=torch.int64, device=self.dev)
        L.check(L.lib.egr_plan_read_reach(self._h, L.ptr(out), self._st(stream)), "egr_plan_read_reach")
        return out.view(W, self.snap.n_vertices)

    def induced_edges(self, col: int, stream=None) -> np.ndarray:
        """(src, dst, type) rows of the induced subgraph of column `col`'s reach set."""
        n = C.c_int64(0)
        L.check(L.lib.egr_plan_induced_edges(self._h, col, None, None, None, 0, C.byref(n),
                                             self._st(stream)), "egr_plan_induced_edges")
        cap = n.value
        src = torch.empty(max(cap, 1), dtype=torch.int32, device=self.dev)
        dst = torch.empty(max(cap, 1), dtype=torch.int32, device=self.dev)
        typ = torch.empty(max(cap, 1), dtype=torch.uint8, device=self.dev)
        L.check(L.lib.egr_plan_induced_edges(self._h, col, L.ptr(src), L.ptr(dst), L.ptr(typ), cap,
                                             C.byref(n), self._st(stream)), "egr_plan_induced_edges")
        out = np.stack([src[:cap].cpu().numpy(), dst[:cap].cpu().numpy(),
                        typ[:cap].cpu().numpy().astype(np.int32)], axis=1)
        return out[np.lexsort((out[:, 2], out[:, 0], out[:, 1]))] if cap else out.reshape(0, 3)


def group_seeds(vertex: np.ndarray, col: np.ndarray, val: np.ndarray, n_cols: int):
    """(seed_ptr u32 [n_cols+1], vertex u32, val f32) of seed triples grouped by column (stable;
    triples whose column is >= n_cols are dropped): the input of Frontier.run_grouped."""
    col = np.asarray(col, np.int64)
    keep = (col >= 0) & (col < n_cols)
    order = np.argsort(col[keep], kind="stable")
    c = col[keep][order]
    ptr = np.searchsorted(c, np.arange(n_cols + 1)).astype(np.uint32)
    return (ptr, np.ascontiguousarray(np.asarray(vertex, np.uint32)[keep][order]),
            np.ascontiguousarray(np.asarray(val, np.float32)[keep][order]))


def launch_order(seed_ptr: np.ndarray, vertex: np.ndarray, row_ptr: np.ndarray) -> np.ndarray:
    """u32 [n_cols]: the columns costliest first (cost = sum over the column's seeds of
    1 + the seed vertex's degree, the predictor egr_frontier_set_seeds sorts by), ties in column
    order -- the longest-processing-time-first launch order for Frontier.run_grouped."""
    ptr = np.asarray(seed_ptr, np.int64)
    v = np.asarray(vertex, np.int64)
    rp = np.asarray(row_ptr, np.int64)
    ok = v < len(rp) - 1
    deg = np.zeros(len(v), np.int64)
    deg[ok] = rp[v[ok] + 1] - rp[v[ok]] + 1
    csum = np.concatenate([[0], np.cumsum(deg)])
    cost = csum[ptr[1:]] - csum[ptr[:-1]]
    return np.argsort(-cost, kind="stable").astype(np.uint32)


class Frontier:
    """Per-batch frontier engine (egr_frontier_*): the same seeds / sources / top-k contract as
    Plan.run, computed per incident column over only the vertices that column touches."""

    def __init__(self, snap: Snapshot, n_cols: int, max_seeds: int, k: int = 10,
                 pool_entries: int = 0):
        self.snap = snap
        self.dev = snap.dev
        self.B, self.k, self.max_seeds = n_cols, k, max_seeds
        self.pool_entries = pool_entries
        h = C.c_void_p()
        L.check(L.lib.egr_frontier_create(snap.handle, n_cols, max_seeds, k, pool_entries,
                                          C.byref(h)), "egr_frontier_create")
        self._h = h
        self.max_vertices = int(L.lib.egr_frontier_max_vertices(h))
        self.out_ids = torch.empty(n_cols * k, dtype=torch.int32, device=self.dev)
        self.out_scores = torch.empty(n_cols * k, dtype=torch.float32, device=self.dev)
        self.retry_blocks = 0
        self.continuation_regions = 0
        self.wide_first = self.FIRST_NARROW
        self._mid_checked = False
        self._adapt_calls = 0

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and getattr(L, "lib", None) is not None:
            L.lib.egr_frontier_free(h)
            self._h = None

    def _st(self, stream):
        return L.stream_handle(self.dev) if stream is None else stream

    def halo_exchange_rccl(self, what: str, rows: torch.Tensor, seg_dev: torch.Tensor,
                           peer_cap: int, send_slots: torch.Tensor, recv_slots: torch.Tensor,
                           recv_vertex: torch.Tensor, rbase: torch.Tensor, overflow: torch.Tensor,
                           rccl_comm: int, stream=None) -> None:
        """egr_plan_halo_exchange: pack_sparse_cap, ONE ncclAllToAll of the slots over the RCCL
        communicator `rccl_comm` (an ncclComm_t address of P ranks), unpack_sparse_cap -- the
        C-ABI path for callers without torch.distributed (egraph/shard.py's TorchComm issues
        the same steps through torch)."""
        P = seg_dev.numel() - 1
        if min(send_slots.numel(), recv_slots.numel()) < P * self.slot_words(what, peer_cap):
            raise ValueError("halo_exchange_rccl: slot buffers too small")
        L.check(L.lib.egr_plan_halo_exchange(self._h, 1 if what == "reach" else 0, L.ptr(rows),
                                             rows.numel(), L.ptr(seg_dev), P, int(peer_cap),
                                             L.ptr(send_slots), L.ptr(recv_slots), L.ptr(recv_vertex),
                                             recv_vertex.numel(), L.ptr(rbase), L.ptr(overflow),
                                             rccl_comm, self._st(stream)), "egr_plan_halo_exchange")

    def set_seeds(self, vertex: torch.Tensor, col: torch.Tensor, val: torch.Tensor, stream=None):
        n = vertex.numel()
        if not (col.numel() == n == val.numel()):
            raise ValueError("seed arrays differ in length")
        L.check(L.lib.egr_frontier_set_seeds(self._h, L.ptr(vertex), L.ptr(col), L.ptr(val), n,
                                             self._st(stream)), "egr_frontier_set_seeds")

    def run(self, sources: torch.Tensor, hops: int = 3, exclude_label: int = -1, stream=None):
        if sources.numel() != self.B:
            raise ValueError(f"need one source vertex per column ({self.B})")
        L.check(L.lib.egr_frontier_run(self._h, L.ptr(sources), hops, exclude_label,
                                       L.ptr(self.out_ids), L.ptr(self.out_scores),
                                       self._st(stream)), "egr_frontier_run")
        return self.out_ids.view(self.B, self.k), self.out_scores.view(self.B, self.k)

    def run_grouped(self, seed_ptr: torch.Tensor, vertex: torch.Tensor, val: torch.Tensor,
                    sources: torch.Tensor, hops: int = 3, exclude_label: int = -1, stream=None,
                    order: torch.Tensor | None = None):
        """One pass over seeds grouped by column (egr_frontier_run_grouped): column b's seeds are
        entries [seed_ptr[b], seed_ptr[b+1]) of vertex / val (device tensors; group_seeds()
        builds them from triples).  No set_seeds, no sort on the device.  `order`: the columns'
        launch order (device u32); None = costliest first, computed on the device."""
        if sources.numel() != self.B or seed_ptr.numel() != self.B + 1:
            raise ValueError(f"need one source vertex per column ({self.B}) and {self.B + 1} seed offsets")
        if vertex.numel() != val.numel():
            raise ValueError("seed arrays differ in length")
        if order is not None and order.numel() != self.B:
            raise ValueError(f"order needs {self.B} entries")
        L.check(L.lib.egr_frontier_run_grouped(self._h, L.ptr(seed_ptr), L.ptr(vertex), L.ptr(val),
                                               vertex.numel(),
                                               L.ptr(order) if order is not None else None,
                                               L.ptr(sources), hops, exclude_label,
                                               L.ptr(self.out_ids), L.ptr(self.out_scores),
                                               self._st(stream)), "egr_frontier_run_grouped")
        return self.out_ids.view(self.B, self.k), self.out_scores.view(self.B, self.k)

    STATS = ("pull_entries", "expand_entries", "rows", "members", "overflowed", "pool_used",
             "seed_entries", "continued", "global_columns")

    RETRY_BLOCKS = 512          # two wide workgroups per CU
    # global-memory regions in which a narrow-table overflow continues inside the grid
    # (egr_frontier_set_continuation), switched on with the retry; $EGRAPH_FRONTIER_CONTINUATION
    # overrides (0 = off: the wide retry grid after the narrow one)
    CONTINUATION_REGIONS = int(os.environ.get("EGRAPH_FRONTIER_CONTINUATION", "128"))
    MAX_CONTINUATION_REGIONS = 4096     # (egr_frontier_set_continuation's bound; 128 KB each)
    MID_CONTINUATION = os.environ.get("EGRAPH_FRONTIER_MID_CONT") is not None

    def set_retry(self, blocks: int) -> None:
        """Wide-table second chance for the columns that overflow the narrow table (see
        egr_frontier_set_retry); 0 turns it off."""
        L.check(L.lib.egr_frontier_set_retry(self._h, int(blocks)), "egr_frontier_set_retry")
        self.retry_blocks = int(blocks)

    def set_continuation(self, regions: int) -> None:
        """Finish the narrow table's overflowing columns inside the grid, each in a global-memory
        region of its own (egr_frontier_set_continuation); 0 = off."""
        L.check(L.lib.egr_frontier_set_continuation(self._h, int(regions)),
                "egr_frontier_set_continuation")
        self.continuation_regions = int(regions)

    # the first table a column tries (egr_frontier_set_wide_first): narrow, the wide grid, or the
    # 2.8k-slot mid table (then the wide grid for what overflows it)
    FIRST_NARROW, FIRST_WIDE, FIRST_MID = 0, 1, 2

    def set_wide_first(self, mode: int) -> None:
        """With the retry on: the table every column tries first -- FIRST_NARROW (0 / False),
        FIRST_WIDE (1 / True: every column straight to the wide table) or FIRST_MID (2)."""
        mode = int(mode)
        L.check(L.lib.egr_frontier_set_wide_first(self._h, mode), "egr_frontier_set_wide_first")
        self.wide_first = mode

    # a run in which more than this fraction of the columns overflowed the narrow table starts
    # every column in the mid table (the narrow attempt of such columns is wasted work); if the
    # first checked mid-first run overflows that table for as many, wide-first
    WIDE_FIRST_FRACTION = 0.5

    def adapt(self, stats: dict | None = None) -> bool:
        """After a run: turn the wide retry on if that run had overflowing columns (graphs with
        large 3-hop neighbourhoods, e.g. the dense C4), and start every column in the mid table
        if most of them overflowed (then in the wide table if most overflow the mid one too).
        Returns True if it changed."""
        if self.pool_entries >= 0:
            return False
        if self.retry_blocks != 0 and (self.wide_first != self.FIRST_MID or self._mid_checked):
            return False
        self._adapt_calls += 1
        if stats is None and self._adapt_calls % 16 != 1:      # a stats read synchronises
            return False
        st = self.stats() if stats is None else stats
        over = st["overflowed"] > self.WIDE_FIRST_FRACTION * self.B
        if self.retry_blocks == 0:
            if st["overflowed"] > 0:
                self.set_retry(min(self.RETRY_BLOCKS, self.B))
                if self.CONTINUATION_REGIONS > 0:
                    self.set_continuation(self.CONTINUATION_REGIONS)
                if over:
                    self.set_wide_first(self.FIRST_MID)
                return True
            return False
        self._mid_checked = True        # (one check of a mid-first run)
        if over:
            self.set_wide_first(self.FIRST_WIDE)
            return True
        # ($EGRAPH_FRONTIER_MID_CONT: the mid table's overflowing columns continue in regions
        # too -- enough for all of them, with headroom -- instead of the serial wide retry; off
        # by default: 30 % slower at C4, profiles/r06_ab_c4_mid_continuation.txt)
        want = min(self.MAX_CONTINUATION_REGIONS, (st["overflowed"] * 5 + 3) // 4)
        if self.MID_CONTINUATION and self.CONTINUATION_REGIONS > 0 and want > self.continuation_regions:
            self.set_continuation(want)
            return True
        return False

    def stats(self, stream=None) -> dict:
        """Work counters of the last run (synchronous)."""
        out = np.zeros(9, np.int64)
        L.check(L.lib.egr_frontier_stats(self._h, _addr(out), self._st(stream)),
                "egr_frontier_stats")
        return dict(zip(self.STATS, out.tolist()))

    def phase_times(self, stream=None) -> np.ndarray | None:
        """[B, 40, 1 + waves] s_memrealtime stamps (100 MHz): per phase boundary the stamp
        after the barrier, then each wave's stamp before it (slot 20: the column's member
        count; slots 24-35: per-wave sub-step sums of the last pull); None when the frontier
        was created without $EGRAPH_FRONTIER_PROFILE."""
        cap = self.B * 40 * 64
        out = np.zeros(cap, np.int64)
        slots = L.lib.egr_frontier_phase_times(self._h, _addr(out), cap, self._st(stream))
        if slots < 0:
            L.check(slots, "egr_frontier_phase_times")
        return out[: self.B * slots].reshape(self.B, 40, -1) if slots > 0 else None

    def read_scores(self, stream=None) -> torch.Tensor:
        out = torch.empty(self.snap.n_vertices * self.B, dtype=torch.float32, device=self.dev)
        L.check(L.lib.egr_frontier_read_scores(self._h, L.ptr(out), self._st(stream)),
                "egr_frontier_read_scores")
        return out.view(self.snap.n_vertices, self.B)

    def read_reach(self, stream=None) -> torch.Tensor:
        W = (self.B + 63) // 64
        out = torch.empty(W * self.snap.n_vertices, dtype=torch.int64, device=self.dev)
        L.check(L.lib.egr_frontier_read_reach(self._h, L.ptr(out), self._st(stream)),
                "egr_frontier_read_reach")
        return out.view(W, self.snap.n_vertices)

    def members(self, col: int, stream=None) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
        """(vertex, score, depth+1) of one column's members, sorted by vertex."""
        n = C.c_int64(0)
        L.check(L.lib.egr_frontier_members(self._h, col, None, None, None, 0, C.byref(n),
                                           self._st(stream)), "egr_frontier_members")
        v = np.empty(n.value, np.uint32)
        s = np.empty(n.value, np.float32)
        d = np.empty(n.value, np.uint8)
        L.check(L.lib.egr_frontier_members(self._h, col, _addr(v), _addr(s), _addr(d), n.value,
                                           C.byref(n), self._st(stream)), "egr_frontier_members")
        o = np.argsort(v, kind="stable")
        return v[o], s[o], d[o]
