"""Drop-in RulesEngine (reference src/services/rca/rules_engine.py:193-478) running on the GPU.

Same public surface: `RulesEngine().generate_hypotheses(incident, evidence)` is a coroutine
function (tests/unit/test_async_contracts.py:18-19 of the reference) returning the same dicts
in the same order (confidence descending, rank 0; the single "unknown" hypothesis when nothing
matches).  Additive batch entry points put many incidents into one kernel launch:
`generate_hypotheses_batch` (unranked, = N x generate_hypotheses) and `rank_incidents_batch`
(generate + HypothesisRanker.rank fused, as the workflow runs them back to back).

All signal extraction, rule matching, confidence, ranking and ordering run in
egr_rules_eval (csrc/rules.hip), called as the custom op torch.ops.egraph.rules_eval
(egraph/ops.py); the host encodes rows and assembles dicts in native code
(csrc/pyhost.c: encode_rows, assemble).  There is no CPU
fallback: without a ROCm GPU the call raises RuntimeError.
"""
from __future__ import annotations

import asyncio

from egraph import catalog as _catalog
from egraph.encode import encode_batch
from egraph.rca import RulesDeviceBatch, hypothesis_lists
from src.models import HypothesisCategory

# The reference's rule table, with categories as enums as in rules_engine.py:15-190.
DIAGNOSIS_RULES = [
    {**{k: v for k, v in r.items() if k != "category"},
     "category": HypothesisCategory(r["category"])}
    for r in _catalog.default().rules
]


class RulesEngine:
    """Deterministic rules engine; evaluation is batched on the GPU."""

    def __init__(self, catalog: _catalog.Catalog | None = None, device=None):
        self.catalog = catalog or _catalog.default()
        self.rules = DIAGNOSIS_RULES if catalog is None else [
            {**r, "category": HypothesisCategory(r["category"])} for r in catalog.rules]
        self.device = device

    async def _run(self, incidents, evidence_lists, ranked: bool) -> list[list[dict]]:
        if len(incidents) != len(evidence_lists):
            raise ValueError("incidents and evidence_lists differ in length")
        enc = encode_batch(evidence_lists, self.catalog)   # raises like the reference
        res = await asyncio.to_thread(self._launch_fetch, enc)
        return hypothesis_lists(self.catalog, res, [inc.id for inc in incidents],
                                enc.evidence_ids, ranked)

    def _launch_fetch(self, enc):
        # torch.ops.egraph.rules_eval: the registered custom op over egr_rules_eval
        return RulesDeviceBatch(enc, self.catalog, self.device).evaluate_op()

    async def generate_hypotheses(self, incident, evidence: list[dict]) -> list[dict]:
        """Generate hypotheses by matching evidence against rules (rules_engine.py:199-233)."""
        return (await self._run([incident], [evidence], ranked=False))[0]

    async def generate_hypotheses_batch(self, incidents: list, evidence_lists: list[list[dict]]
                                        ) -> list[list[dict]]:
        """generate_hypotheses for many incidents in one launch."""
        return await self._run(list(incidents), list(evidence_lists), ranked=False)

    async def rank_incidents_batch(self, incidents: list, evidence_lists: list[list[dict]]
                                   ) -> list[list[dict]]:
        """generate_hypotheses followed by HypothesisRanker.rank, fused in one launch."""
        return await self._run(list(incidents), list(evidence_lists), ranked=True)
