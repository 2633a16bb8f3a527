"""ORACLE (test infrastructure only) -- ctypes access to liboracle.so + a pure-Python restatement
of the GraphService write semantics.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
It is the checker, never the thing measured or shipped.

  graph_reference   neo4j.py:95-167 MERGE semantics, restated with Python dicts
  csr_reference     the symmetric typed CSR of DESIGN.md §A7 built from that edge list
  rules_eval / rank / reach / propagate / topk   -> oracle/egraph_oracle.c
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"


def _load() -> C.CDLL:
    if not LIB.is_file():
        subprocess.run(["make", "-C", str(HERE)], check=True, capture_output=True)
    lib = C.CDLL(str(LIB))
    lib.orc_round.restype = C.c_double
    lib.orc_round.argtypes = [C.c_double, C.c_int]
    for name in ("orc_rules_eval", "orc_rank", "orc_reach", "orc_propagate", "orc_topk",
                 "orc_hop_step", "orc_frontier"):
        getattr(lib, name).restype = C.c_int
    return lib


lib = _load()


def _p(a: np.ndarray):
    return C.c_void_p(a.ctypes.data if a.size else 0)


def rules_eval(table, flags, vocab, node, err, seg_off):
    """Host restatement of egr_rules_eval over the same encoded columns."""
    B = len(seg_off) - 1
    S = table.n_rules + 1
    out = {
        "mask": np.zeros(B, np.uint32), "n_hyp": np.zeros(B, np.uint8),
        "order_conf": np.zeros(B * S, np.uint8), "order_rank": np.zeros(B * S, np.uint8),
        "confidence": np.zeros(B * S), "final_score": np.zeros(B * S), "strength": np.zeros(B * S),
    }
    lib.orc_rules_eval(C.byref(table), _p(flags), _p(vocab), _p(node), _p(err), _p(seg_off),
                       C.c_int32(B), _p(out["mask"]), _p(out["n_hyp"]), _p(out["order_conf"]),
                       _p(out["order_rank"]), _p(out["confidence"]), _p(out["final_score"]),
                       _p(out["strength"]))
    for k in ("order_conf", "order_rank", "confidence", "final_score", "strength"):
        out[k] = out[k].reshape(B, S)
    return out


def rank(conf, w, sup, strength, off):
    n = int(off[-1])
    final = np.zeros(n)
    order = np.zeros(n, np.int32)
    lib.orc_rank(_p(conf), _p(w), _p(sup), _p(strength), _p(off), C.c_int32(len(off) - 1),
                 _p(final), _p(order))
    return final, order


def reach(row_ptr, col, src, hops, threads=0):
    V = len(row_ptr) - 1
    B = len(src)
    out = np.zeros(((B + 63) // 64, V), np.uint64)
    lib.orc_reach(_p(row_ptr), _p(col), C.c_int64(V), _p(src), C.c_int32(B), C.c_int32(hops),
                  _p(out), C.c_int(threads))
    return out


def propagate(row_ptr, col, val, seed_v, seed_c, seed_s, B, hops, threads=0):
    V = len(row_ptr) - 1
    out = np.zeros((V, B), np.float32)
    rc = lib.orc_propagate(_p(row_ptr), _p(col), _p(val), C.c_int64(V), _p(seed_v), _p(seed_c),
                           _p(seed_s), C.c_int64(len(seed_v)), C.c_int32(B), C.c_int32(hops),
                           _p(out), C.c_int(threads))
    if rc != 0:
        raise MemoryError("orc_propagate")
    return out


def topk(scores, reach_bits, vlabel, exclude_label, k):
    V, B = scores.shape
    ids = np.zeros(B * k, np.uint32)
    sc = np.zeros(B * k, np.float32)
    lib.orc_topk(_p(np.ascontiguousarray(scores)), C.c_int64(V), C.c_int32(B),
                 _p(np.ascontiguousarray(reach_bits)), _p(vlabel), C.c_int32(exclude_label),
                 C.c_int32(k), _p(ids), _p(sc))
    return ids.reshape(B, k), sc.reshape(B, k)


def frontier(row_ptr, col, val, vlabel, seed_v, seed_c, seed_s, src, hops, exclude_label, k,
             threads=0, prune=True):
    """orc_frontier: top-k ids / scores [B, k] equal to propagate + reach + topk, computed per
    column over the touched vertices only; also (CSR entries read, rows walked)."""
    V = len(row_ptr) - 1
    B = len(src)
    ids = np.zeros(B * k, np.uint32)
    sc = np.zeros(B * k, np.float32)
    work = np.zeros(2, np.int64)
    rc = lib.orc_frontier(_p(row_ptr), _p(col), _p(val), _p(vlabel), C.c_int64(V), _p(seed_v),
                          _p(seed_c), _p(seed_s), C.c_int64(len(seed_v)), _p(src), C.c_int32(B),
                          C.c_int32(hops), C.c_int32(exclude_label), C.c_int32(k),
                          C.c_int(1 if prune else 0), _p(ids),
                          _p(sc), _p(work), C.c_int(threads))
    if rc != 0:
        raise MemoryError("orc_frontier")
    return ids.reshape(B, k), sc.reshape(B, k), (int(work[0]), int(work[1]))


# ---- pure-Python graph write semantics (neo4j.py:95-167) ---------------------------------------
def graph_reference(entities, relations):
    """Returns (vertices [(label, id)] in creation order, edges [(s, d, type)] in creation order)."""
    vertices, key = [], {}
    by_id: dict[str, list[int]] = {}
    for e in entities:
        k = (e["type"], e["id"])
        if k not in key:
            key[k] = len(vertices)
            vertices.append(k)
            by_id.setdefault(e["id"], []).append(key[k])
    edges, seen = [], set()
    for r in relations:
        for s in by_id.get(r["source_id"], []):
            for d in by_id.get(r["target_id"], []):
                k = (s, d, r["relation_type"])
                if k not in seen:
                    seen.add(k)
                    edges.append(k)
    return vertices, edges


def csr_reference(n_vertices, edges, type_index, weights):
    """Rows sorted by (neighbour, type, dir); val = w[type][dir] / deg(neighbour), fp32."""
    rows = [[] for _ in range(n_vertices)]
    for s, d, t in edges:
        ti = type_index[t]
        rows[d].append((s, ti, 0))
        rows[s].append((d, ti, 1))
    deg = [len(r) for r in rows]
    row_ptr, col, meta, val = [0], [], [], []
    for r in rows:
        for u, ti, di in sorted(r):
            col.append(u)
            meta.append(ti << 1 | di)
            w = weights[2 * ti + di] if 2 * ti + di < len(weights) else np.float32(1.0)
            val.append(np.float32(w) / np.float32(deg[u]))
        row_ptr.append(len(col))
    return (np.array(row_ptr, np.uint32), np.array(col, np.uint32), np.array(meta, np.uint8),
            np.array(val, np.float32))


def hop_step(row_ptr, col, val, xin, s0):
    """One hop of the A9 recurrence on given scores (partitioned-protocol tests)."""
    V, B = xin.shape
    out = np.zeros((V, B), np.float32)
    lib.orc_hop_step(_p(row_ptr), _p(col), _p(val), C.c_int64(V), C.c_int32(B),
                     _p(np.ascontiguousarray(xin, np.float32)),
                     _p(np.ascontiguousarray(s0, np.float32)), _p(out))
    return out
