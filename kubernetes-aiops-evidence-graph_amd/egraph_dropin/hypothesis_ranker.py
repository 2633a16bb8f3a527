"""Drop-in HypothesisRanker (reference src/services/rca/hypothesis_ranker.py:10-80) on the GPU.

`rank(hypotheses)` keeps the reference contract: synchronous, mutates the dicts (adds
`final_score`, sets `rank`) and returns them in stable descending final_score order; `[]`
returns `[]`.  The score and Python-exact round(score, 4) run in egr_rank (csrc/rules.hip).
"""
from __future__ import annotations

from egraph.ranker import FUSED, rank_lists


class HypothesisRanker:
    """Ranks and prioritizes RCA hypotheses."""

    def __init__(self, device=None):
        self.device = device

    def rank(self, hypotheses: list[dict]) -> list[dict]:
        if not hypotheses:
            return []
        # a list the rules kernel generated and ranked: its fused ranking, verified field by
        # field (egraph/ranker.py FusedRanks); anything else goes through egr_rank
        r = FUSED.apply(hypotheses)
        return r if r is not None else rank_lists([hypotheses], self.device, fused=False)[0]

    def rank_many(self, lists: list[list[dict]]) -> list[list[dict]]:
        """Rank many independent hypothesis lists in one launch."""
        return rank_lists(lists, self.device)
