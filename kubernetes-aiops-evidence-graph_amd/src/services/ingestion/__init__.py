"""Mirror of the alert ingestion front end (reference src/services/ingestion/__init__.py):
egraph_dropin.normalizer / egraph_dropin.deduplicator."""
from egraph_dropin.deduplicator import AlertDeduplicator, RateLimiter
from egraph_dropin.normalizer import AlertNormalizer

__all__ = ["AlertNormalizer", "AlertDeduplicator", "RateLimiter"]
