"""torch.ops.egraph.* -- the hot path registered as PyTorch-ROCm custom ops.

The ops are registered in C++ (csrc/torch_ops.cpp, TORCH_LIBRARY(egraph)) by lib/_egraph_ops.so
and call the same C-ABI as the rest of the package (libegraph.so, include/egraph.h) on torch's
current HIP stream.  They have only device (HIP) kernels: CPU tensors fail in the dispatcher.
Importing this module loads the library or raises ImportError -- there is no fallback.

  torch.ops.egraph.rules_eval(row_flags, row_vocab, row_node, row_err, seg_off, rule_table)
      -> (mask, n_hyp, order_conf, order_rank, confidence, final_score, strength)
  torch.ops.egraph.frontier_run(frontier, seed_vertex, seed_col, seed_val, sources, n_cols, k,
                                hops, exclude_label) -> (ids [B, k] i32, scores [B, k] f32)
  torch.ops.egraph.propagate(plan, seed_vertex, seed_col, seed_val, V, B, hops) -> [V, B] f32
  torch.ops.egraph.reach(plan, sources, V, hops) -> [ceil(B/64), V] i64 bits
  torch.ops.egraph.topk(snapshot, scores [V, B], reach_bits, k, exclude_label) -> (ids, scores)

Engine state lives in libegraph objects whose handles the wrappers below pass as int64.
Callers in this package: the drop-in RulesEngine (rules_eval) and GraphService.rank_root_causes
(frontier_run) -- the reference's activities (src/services/workflow/activities.py:124-170) reach
the GPU through these ops.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib as L

OPS_PATH = L.PKG_ROOT / "lib" / "_egraph_ops.so"
if not OPS_PATH.is_file():
    raise ImportError(f"{OPS_PATH.name} not found in {OPS_PATH.parent}; build it with "
                      f"`make -C {L.PKG_ROOT}`")
torch.ops.load_library(str(OPS_PATH))
OPS = ("rules_eval", "frontier_run", "propagate", "reach", "topk")


def _h(obj) -> int:
    """int64 value of a libegraph handle (ctypes c_void_p)."""
    return int(obj._h.value if isinstance(obj._h, C.c_void_p) else obj._h)


def rule_table_tensor(cat) -> torch.Tensor:
    """The catalog's egr_rule_table as a CPU uint8 tensor (the rules_eval argument)."""
    return torch.frombuffer(bytearray(bytes(cat.table)), dtype=torch.uint8)


def rules_eval(flags, vocab, node, err, seg_off, table: torch.Tensor):
    return torch.ops.egraph.rules_eval(flags, vocab, node, err, seg_off, table)


def frontier_run(fr, seed_vertex, seed_col, seed_val, sources, hops: int = 3,
                 exclude_label: int = -1):
    """set_seeds + run of an egraph.graph.Frontier through the custom op."""
    return torch.ops.egraph.frontier_run(_h(fr), seed_vertex.view(torch.int32),
                                         seed_col.view(torch.int32), seed_val,
                                         sources.view(torch.int32), fr.B, fr.k, hops,
                                         exclude_label)


def propagate(plan, seed_vertex, seed_col, seed_val, hops: int = 3) -> torch.Tensor:
    return torch.ops.egraph.propagate(_h(plan), seed_vertex.view(torch.int32),
                                      seed_col.view(torch.int32), seed_val,
                                      plan.snap.n_vertices, plan.B, hops)


def reach(plan, sources, hops: int = 3) -> torch.Tensor:
    return torch.ops.egraph.reach(_h(plan), sources.view(torch.int32), plan.snap.n_vertices, hops)


def topk(snap, scores, reach_bits, k: int = 10, exclude_label: int = -1):
    return torch.ops.egraph.topk(_h(snap), scores, reach_bits, k, exclude_label)
