"""Alert ingestion front end (reference src/services/ingestion/__init__.py): normalizer with GPU
fingerprints, deduplicator backed by the GPU TTL table."""
from src.services.ingestion.deduplicator import AlertDeduplicator, RateLimiter
from src.services.ingestion.normalizer import AlertNormalizer

__all__ = ["AlertNormalizer", "AlertDeduplicator", "RateLimiter"]
