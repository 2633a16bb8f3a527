"""ctypes binding of libegraph.so (the C-ABI declared in include/egraph.h).

There is no fallback: if the library is missing or fails to load, importing this module
raises ImportError naming the build command.  torch is imported first so that the HIP
runtime torch already mapped (soname libamdhip64.so.7) is the one libegraph resolves to.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import torch  # noqa: F401  (must precede the CDLL load: shared HIP runtime)

PKG_ROOT = Path(__file__).resolve().parents[1]
LIB_PATH = Path(os.environ.get("EGRAPH_LIB", PKG_ROOT / "lib" / "libegraph.so"))

EGR_OK, EGR_EINVAL, EGR_EDEVICE, EGR_ENOMEM, EGR_ESTATE = 0, -1, -2, -3, -4
EGR_MAX_RULES = 32
EGR_MAX_CONDS = 4
EGR_NO_NODE = 0xFFFFFFFF

# per-row flag bits (include/egraph.h EGR_F_*)
F_RECENT_DEPLOY = 1 << 0
F_IMAGE_CHANGED = 1 << 1
F_MEMORY_HIGH = 1 << 2
F_HPA_AT_MAX = 1 << 3
F_LATENCY_HIGH = 1 << 4
F_NODE_ISSUE = 1 << 5
F_NOT_READY = 1 << 6
F_READINESS_FAIL = 1 << 7
F_ERR_FLOAT = 1 << 8


class EgrRule(C.Structure):
    _fields_ = [
        ("n_conds", C.c_int32),
        ("cond_type", C.c_int32 * EGR_MAX_CONDS),
        ("cond_mask", C.c_uint32 * EGR_MAX_CONDS),
        ("cond_param", C.c_double * EGR_MAX_CONDS),
        ("cond_strength", C.c_double * EGR_MAX_CONDS),
        ("confidence_base", C.c_double),
        ("category_weight", C.c_double),
    ]


class EgrRuleTable(C.Structure):
    _fields_ = [
        ("n_rules", C.c_int32),
        ("network_vocab_bit", C.c_uint32),
        ("unknown_confidence", C.c_double),
        ("unknown_category_weight", C.c_double),
        ("rules", EgrRule * EGR_MAX_RULES),
    ]


class EgrRulesOut(C.Structure):
    _fields_ = [
        ("mask", C.c_void_p),
        ("n_hyp", C.c_void_p),
        ("order_conf", C.c_void_p),
        ("order_rank", C.c_void_p),
        ("confidence", C.c_void_p),
        ("final_score", C.c_void_p),
        ("strength", C.c_void_p),
    ]


P = C.c_void_p
I32, I64, U32, F64 = C.c_int32, C.c_int64, C.c_uint32, C.c_double
PI32, PI64 = C.POINTER(C.c_int32), C.POINTER(C.c_int64)

# name -> (restype, argtypes); every symbol include/egraph.h declares
SIGNATURES: dict[str, tuple] = {
    "egr_last_error": (C.c_char_p, []),
    "egr_version": (C.c_int, []),
    "egr_device_count": (C.c_int, []),
    "egr_rules_eval": (C.c_int, [C.POINTER(EgrRuleTable), P, P, P, P, P, I32,
                                 C.POINTER(EgrRulesOut), P]),
    "egr_rank": (C.c_int, [P, P, P, P, P, I32, P, P, P]),
    "egr_py_round": (F64, [F64, I32]),
    "egr_graph_create": (C.c_int, [C.POINTER(P)]),
    "egr_graph_free": (None, [P]),
    "egr_graph_merge_nodes": (C.c_int, [P, C.c_char_p, P, C.c_char_p, P, I64, P]),
    "egr_graph_merge_edges": (C.c_int, [P, C.c_char_p, P, C.c_char_p, P, C.c_char_p, P, I64, PI64]),
    "egr_graph_num_vertices": (I64, [P]),
    "egr_graph_num_edges": (I64, [P]),
    "egr_graph_num_labels": (I32, [P]),
    "egr_graph_num_rel_types": (I32, [P]),
    "egr_graph_label_name": (I64, [P, I32, C.c_char_p, I64]),
    "egr_graph_rel_type_name": (I64, [P, I32, C.c_char_p, I64]),
    "egr_graph_vertex_id": (I64, [P, I64, C.c_char_p, I64]),
    "egr_graph_lookup": (C.c_int, [P, C.c_char_p, P, I64, P]),
    "egr_graph_lookup_labeled": (C.c_int, [P, C.c_char_p, P, I64, C.c_char_p, P, P]),
    "egr_graph_find": (I32, [P, C.c_char_p, I64]),
    "egr_graph_export": (C.c_int, [P, P, P, P, P]),
    "egr_graph_csr": (C.c_int, [P, P, I32, P, P, P, P]),
    "egr_snapshot_create": (C.c_int, [P, P, I32, I32, C.POINTER(P)]),
    "egr_snapshot_free": (None, [P]),
    "egr_snapshot_info": (C.c_int, [P, PI64, PI64]),
    "egr_plan_create": (C.c_int, [P, I32, I64, I32, C.POINTER(P)]),
    "egr_plan_free": (None, [P]),
    "egr_plan_tile_width": (C.c_int, [P]),
    "egr_plan_shape": (C.c_int, [P, P, P]),
    "egr_plan_set_seeds": (C.c_int, [P, P, P, P, I64, P]),
    "egr_plan_set_sources": (C.c_int, [P, P, P]),
    "egr_plan_hop": (C.c_int, [P, P]),
    "egr_plan_reach_hop": (C.c_int, [P, P]),
    "egr_plan_step": (C.c_int, [P, P]),
    "egr_plan_final_step": (C.c_int, [P, I32, P]),
    "egr_plan_candidates": (C.c_int, [P, I32, P]),
    "egr_plan_topk": (C.c_int, [P, I32, P, P, P]),
    "egr_plan_run": (C.c_int, [P, I32, I32, P, P, P]),
    "egr_plan_read_scores": (C.c_int, [P, P, P]),
    "egr_plan_read_reach": (C.c_int, [P, P, P]),
    "egr_plan_induced_edges": (C.c_int, [P, I32, P, P, P, I64, PI64, P]),
    "egr_snapshot_from_csr": (C.c_int, [P, P, P, P, P, I64, I32, C.POINTER(P)]),
    "egr_plan_set_owned": (C.c_int, [P, I64]),
    "egr_plan_pack_scores": (C.c_int, [P, P, I64, P, P]),
    "egr_plan_unpack_scores": (C.c_int, [P, P, P, I64, P, P]),
    "egr_plan_pack_reach": (C.c_int, [P, P, I64, P, P]),
    "egr_plan_unpack_reach": (C.c_int, [P, P, P, I64, P, P]),
    "egr_plan_pack_sparse": (C.c_int, [P, I32, P, I64, P, I32, P, I64, P, P]),
    "egr_plan_unpack_sparse": (C.c_int, [P, I32, P, I64, P, I64, P, P, I32, P]),
    "egr_plan_pack_sparse_cap": (C.c_int, [P, I32, P, I64, P, I32, P, I64, P, P, P]),
    "egr_plan_unpack_sparse_cap": (C.c_int, [P, I32, P, I64, P, I64, P, P, I32, P]),
    "egr_plan_halo_exchange": (C.c_int, [P, I32, P, I64, P, I32, I64, P, P, P, I64, P, P, P, P]),
    "egr_frontier_create": (C.c_int, [P, I32, I64, I32, I64, C.POINTER(P)]),
    "egr_frontier_free": (None, [P]),
    "egr_frontier_set_seeds": (C.c_int, [P, P, P, P, I64, P]),
    "egr_frontier_run": (C.c_int, [P, P, I32, I32, P, P, P]),
    "egr_frontier_run_grouped": (C.c_int, [P, P, P, P, I64, P, P, I32, I32, P, P, P]),
    "egr_frontier_shape": (C.c_int, [P, P, P]),
    "egr_frontier_stats": (C.c_int, [P, P, P]),
    "egr_frontier_set_retry": (C.c_int, [P, I32]),
    "egr_frontier_set_continuation": (C.c_int, [P, I32]),
    "egr_frontier_set_wide_first": (C.c_int, [P, I32]),
    "egr_frontier_read_scores": (C.c_int, [P, P, P]),
    "egr_frontier_phase_times": (C.c_int, [P, P, I64, P]),
    "egr_frontier_read_reach": (C.c_int, [P, P, P]),
    "egr_frontier_members": (C.c_int, [P, I32, P, P, P, I64, PI64, P]),
    "egr_snapshot_update": (C.c_int, [P, P, I64, P, P, P, I64, P, I32, P]),
    "egr_snapshot_download": (C.c_int, [P, P, P, P, P, P]),
    "egr_snapshot_version": (I64, [P]),
    "egr_locality_order": (C.c_int, [P, P, I64, P]),
    "egr_snapshot_within": (C.c_int, [P, P, I64, I32, P, P]),
    "egr_snapshot_typed_neighbors": (C.c_int, [P, P, I64, I32, I32, I32, P, P, P, P]),
    "egr_frontier_max_vertices": (I64, [P]),
    "egr_graph_export_edges": (C.c_int, [P, I64, I64, P, P, P]),
    "egr_graph_add_edges_indexed": (C.c_int, [P, P, P, C.c_char_p, P, I32, P, I64, PI64]),
    "egr_fingerprint": (C.c_int, [P, P, I64, P, P, P]),
    "egr_dedup_create": (C.c_int, [I32, I64, C.POINTER(P)]),
    "egr_dedup_free": (None, [P]),
    "egr_dedup_ingest": (C.c_int, [P, P, I64, I64, I64, U32, P, P, P, P]),
    "egr_dedup_lookup": (C.c_int, [P, P, I64, I64, P, P, P]),
    "egr_dedup_register": (C.c_int, [P, P, I64, I64, I64, P, P, P]),
    "egr_dedup_remove": (C.c_int, [P, P, I64, P]),
    "egr_dedup_extend": (C.c_int, [P, P, I64, I64, I64, P, P]),
    "egr_dedup_stats": (C.c_int, [P, I64, PI64]),
    "egr_dedup_compact": (C.c_int, [P, I64, I64]),
    "egr_topk": (C.c_int, [P, P, P, I32, I32, I32, P, P, P]),
    "egr_host_alloc": (C.c_int, [I64, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]),
    "egr_host_free": (C.c_int, [P]),
    "egr_rules_eval_small": (C.c_int, [C.POINTER(EgrRuleTable), P, P, P, P, I32, C.POINTER(EgrRulesOut), P]),
    "egr_rules_eval_staged": (C.c_int, [C.POINTER(EgrRuleTable), P, P, P, P, I64, I64, I64, I32, P]),
    "egr_rules_server_create": (C.c_int, [C.POINTER(EgrRuleTable), I32, C.POINTER(P)]),
    "egr_rules_server_post": (C.c_int, [P, P, P, P, P, I32]),
    "egr_rules_server_poll": (C.c_int, [P, P, P, P, P, P, P, P]),
    "egr_rules_server_free": (None, [P]),
}


def _load() -> C.CDLL:
    if not LIB_PATH.is_file():
        raise ImportError(
            f"libegraph.so not found at {LIB_PATH}; build it with "
            f"`make -C {PKG_ROOT}` (or python -c 'import __graft_entry__ as g; g.build()')")
    lib = C.CDLL(str(LIB_PATH))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def build_hash(path: Path | None = None) -> str:
    """SHA-256 (first 16 hex digits) of the loaded libegraph.so: stamps counter summaries in
    profiles/ so that a figure taken on another build is never read as this build's."""
    import hashlib
    return hashlib.sha256(Path(path or LIB_PATH).read_bytes()).hexdigest()[:16]


def _load_pyhost():
    """The CPython extension with the host side of the rules boundary (csrc/pyhost.c)."""
    import importlib.machinery
    import importlib.util
    import sysconfig
    name = "_egr_pyhost" + sysconfig.get_config_var("EXT_SUFFIX")
    # $EGRAPH_PYHOST_DIR: an A/B build of the extension (scripts/, never set in production)
    path = Path(os.environ.get("EGRAPH_PYHOST_DIR", PKG_ROOT / "lib")) / name
    if not path.is_file():
        raise ImportError(f"{path.name} not found in {path.parent}; build it with "
                          f"`make -C {PKG_ROOT}`")
    loader = importlib.machinery.ExtensionFileLoader("_egr_pyhost", str(path))
    spec = importlib.util.spec_from_file_location("_egr_pyhost", str(path), loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    return mod


pyhost = _load_pyhost()


class EgraphError(RuntimeError):
    """Device-side failure reported by libegraph (retryable in the workflow's terms)."""


def check(rc: int, what: str = "") -> None:
    """Map a C status to the reference's error classes (incident_workflow.py:60-65):
    bad input -> ValueError (non-retryable), device / memory -> RuntimeError."""
    if rc == EGR_OK:
        return
    msg = (lib.egr_last_error() or b"").decode(errors="replace")
    where = f"{what}: " if what else ""
    if rc == EGR_EINVAL:
        raise ValueError(where + msg)
    if rc == EGR_ENOMEM:
        raise MemoryError(where + msg)
    raise EgraphError(where + (msg or f"status {rc}"))


def ptr(t) -> int:
    """Raw address of a torch tensor (or None -> 0)."""
    return 0 if t is None else t.data_ptr()


def stream_handle(device: torch.device | None = None) -> int:
    """hipStream_t of torch's current stream on `device`."""
    return torch.cuda.current_stream(device).cuda_stream
