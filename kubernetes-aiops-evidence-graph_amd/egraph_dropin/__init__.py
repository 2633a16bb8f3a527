"""The drop-in service classes of the evidence-graph correlation path, under a top-level name
that cannot collide with the reference's own `src` package.

The reference's callers import through its regular package `src` (activities.py:12, :100,
:131, :165; worker.py:12-26; ingestion/main.py:16-17).  Once that package is loaded, nothing on
sys.path can redirect `src.*`, so the GPU classes live here and a maintainer imports them by
this name:

    from egraph_dropin import GraphService, HypothesisRanker, RulesEngine
    from egraph_dropin import AlertDeduplicator, AlertNormalizer, RateLimiter
    from egraph_dropin import activities      # generate_and_rank_batch, rank_root_causes, ...

Nothing in this package imports `src.*` except the optional LLM step of
activities.generate_hypotheses, which reaches for the deployed reference's own `src.config` and
`src.services.rca.llm_summarizer`.  The repository's `src/` tree is a mirror of these modules
under the reference's module paths (each leaf module IS the module here), for tests written
like the reference's.
"""
from egraph_dropin.deduplicator import AlertDeduplicator, RateLimiter
from egraph_dropin.graph_service import GraphConnection, GraphService, Neo4jConnection
from egraph_dropin.hypothesis_ranker import HypothesisRanker
from egraph_dropin.normalizer import AlertNormalizer
from egraph_dropin.rules_engine import DIAGNOSIS_RULES, RulesEngine

__all__ = ["AlertDeduplicator", "AlertNormalizer", "DIAGNOSIS_RULES", "GraphConnection",
           "GraphService", "HypothesisRanker", "Neo4jConnection", "RateLimiter", "RulesEngine"]
