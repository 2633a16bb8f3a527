"""Graph store of the hot path (reference src/database/__init__.py exports GraphService)."""
from src.database.graph import GraphService

__all__ = ["GraphService"]
