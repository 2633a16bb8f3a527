"""Batched RCA on the GPU: encoded evidence rows -> ranked hypotheses (A1-A6).

One egr_rules_eval launch evaluates every incident of a batch (one wavefront each); the host
turns the per-incident slot orders back into the reference's hypothesis dicts
(src/services/rca/rules_engine.py:235-262, :457-478; hypothesis_ranker.py:63-71).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from uuid import uuid4

import numpy as np
import torch

from . import _lib as L
from .catalog import Catalog, default
from .device import require_device, to_device
from .encode import EncodedBatch, encode_batch


@dataclass
class RulesResult:
    """Host copy of the kernel outputs for a batch (S = n_rules + 1 slots per incident)."""
    mask: np.ndarray          # u32 [B]
    n_hyp: np.ndarray         # u8  [B]
    order_conf: np.ndarray    # u8  [B, S]
    order_rank: np.ndarray    # u8  [B, S]
    confidence: np.ndarray    # f64 [B, S]
    final_score: np.ndarray   # f64 [B, S]
    strength: np.ndarray      # f64 [B, S]


class RulesDeviceBatch:
    """Device-resident inputs + outputs of one rules launch (reusable for repeated runs)."""

    def __init__(self, enc: EncodedBatch, cat: Catalog, device=None):
        self.dev = require_device(device)
        self.cat = cat
        self.B = enc.n_incidents
        S = cat.n_rules + 1
        d = self.dev
        self.flags = to_device(enc.flags, d)
        self.vocab = to_device(enc.vocab, d)
        self.node = to_device(enc.node, d)
        self.err = to_device(enc.err, d)
        self.seg = to_device(enc.seg_off, d)
        B = max(self.B, 1)
        self.mask = torch.empty(B, dtype=torch.int32, device=d)
        self.n_hyp = torch.empty(B, dtype=torch.uint8, device=d)
        self.order_conf = torch.empty(B * S, dtype=torch.uint8, device=d)
        self.order_rank = torch.empty(B * S, dtype=torch.uint8, device=d)
        self.confidence = torch.zeros(B * S, dtype=torch.float64, device=d)
        self.final_score = torch.zeros(B * S, dtype=torch.float64, device=d)
        self.strength = torch.zeros(B * S, dtype=torch.float64, device=d)
        self._out = L.EgrRulesOut(
            L.ptr(self.mask), L.ptr(self.n_hyp), L.ptr(self.order_conf), L.ptr(self.order_rank),
            L.ptr(self.confidence), L.ptr(self.final_score), L.ptr(self.strength))

    def launch(self, stream: int | None = None) -> None:
        """Enqueue egr_rules_eval on `stream` (default: torch's current stream)."""
        st = L.stream_handle(self.dev) if stream is None else stream
        L.check(L.lib.egr_rules_eval(
            self.cat.table, L.ptr(self.flags), L.ptr(self.vocab), L.ptr(self.node),
            L.ptr(self.err), L.ptr(self.seg), self.B, self._out, st), "egr_rules_eval")

    def evaluate_op(self) -> RulesResult:
        """One evaluation through the registered custom op (torch.ops.egraph.rules_eval, the
        same egr_rules_eval on the current stream, fresh output tensors) -> host results."""
        from . import ops
        outs = ops.rules_eval(self.flags, self.vocab, self.node, self.err, self.seg,
                              self._table_tensor())
        B = self.B
        h = [t.cpu().numpy() for t in outs]
        return RulesResult(h[0][:B].view(np.uint32), h[1][:B], h[2], h[3], h[4], h[5], h[6])

    def _table_tensor(self) -> torch.Tensor:
        t = getattr(self.cat, "_table_tensor", None)
        if t is None:
            from . import ops
            t = self.cat._table_tensor = ops.rule_table_tensor(self.cat)
        return t

    def fetch(self) -> RulesResult:
        """Copy the outputs to the host (synchronises with the current stream)."""
        S = self.cat.n_rules + 1
        B = self.B
        host = [t.cpu().numpy() for t in (self.mask, self.n_hyp, self.order_conf, self.order_rank,
                                           self.confidence, self.final_score, self.strength)]
        return RulesResult(host[0][:B].view(np.uint32), host[1][:B],
                           host[2][:B * S].reshape(B, S), host[3][:B * S].reshape(B, S),
                           host[4][:B * S].reshape(B, S), host[5][:B * S].reshape(B, S),
                           host[6][:B * S].reshape(B, S))


def evaluate(evidence_lists: list[list[dict]], cat: Catalog | None = None,
             device=None) -> tuple[EncodedBatch, RulesResult]:
    """Encode and evaluate a batch; returns the encoded batch and the host results."""
    cat = cat or default()
    enc = encode_batch(evidence_lists, cat)
    with torch.cuda.device(require_device(device)):
        batch = RulesDeviceBatch(enc, cat, device)
        batch.launch()
        res = batch.fetch()
    return enc, res


def hypothesis_dicts(cat: Catalog, res: RulesResult, i: int, incident_id: str,
                     evidence_ids: list, ranked: bool) -> list[dict]:
    """Assemble incident i's hypotheses exactly as the reference emits them.

    ranked=False: RulesEngine.generate_hypotheses output (confidence order, rank 0 / unknown 1).
    ranked=True : the same dicts after HypothesisRanker.rank (final_score, rank = position).
    """
    R = cat.n_rules
    order = res.order_rank[i] if ranked else res.order_conf[i]
    out = []
    for p in range(int(res.n_hyp[i])):
        slot = int(order[p])
        if slot == R:
            u = cat.unknown
            h = {
                "id": str(uuid4()), "incident_id": incident_id, "category": u["category"],
                "title": u["title"], "description": u["description"],
                "confidence": u["confidence"], "rank": u["rank"],
                "supporting_evidence_ids": list(evidence_ids),
                "recommended_actions": list(u["recommended_actions"]),
                "generated_by": u["generated_by"], "rule_id": u["rule_id"],
                "support_count": u["support_count"], "signal_strength": u["signal_strength"],
            }
        else:
            rule = cat.rules[slot]
            h = {
                "id": str(uuid4()), "incident_id": incident_id, "category": rule["category"],
                "title": rule["name"], "description": rule["description"],
                "confidence": float(res.confidence[i, slot]), "rank": 0,
                "supporting_evidence_ids": list(evidence_ids),
                "recommended_actions": list(rule["actions"]),
                "generated_by": "rules_engine", "rule_id": rule["id"],
                "support_count": len(rule["conditions"]),
                "signal_strength": float(res.strength[i, slot]),
            }
        if ranked:
            h["final_score"] = float(res.final_score[i, slot])
            h["rank"] = p + 1
        out.append(h)
    return out


def _templates(cat: Catalog) -> tuple:
    """Per-rule (category, title, description, actions, rule_id, support_count) and the
    unknown hypothesis's fields, in the order csrc/pyhost.c assemble() reads them."""
    t = getattr(cat, "_hyp_templates", None)
    if t is None:
        rules = tuple((r["category"], r["name"], r["description"], list(r["actions"]), r["id"],
                       len(r["conditions"])) for r in cat.rules)
        u = cat.unknown
        unknown = (u["category"], u["title"], u["description"], u["confidence"], u["rank"],
                   list(u["recommended_actions"]), u["generated_by"], u["rule_id"],
                   u["support_count"], u["signal_strength"])
        t = (rules, unknown)
        cat._hyp_templates = t
    return t


def hypothesis_lists(cat: Catalog, res: RulesResult, incident_ids: list, evidence_ids: list,
                     ranked: bool) -> list[list[dict]]:
    """hypothesis_dicts for every incident of a batch, assembled natively (csrc/pyhost.c).

    Same dicts, keys in the same order; `id` is a fresh uuid4 string per hypothesis drawn from
    os.urandom, as uuid.uuid4() draws it."""
    rules, unknown = _templates(cat)
    order = res.order_rank if ranked else res.order_conf
    n = int(res.n_hyp.sum(dtype=np.int64))
    return L.pyhost.assemble(
        rules, unknown, np.ascontiguousarray(res.n_hyp), np.ascontiguousarray(order),
        np.ascontiguousarray(res.confidence), np.ascontiguousarray(res.final_score),
        np.ascontiguousarray(res.strength), [str(i) for i in incident_ids],
        list(evidence_ids), bool(ranked), os.urandom(16 * n))
