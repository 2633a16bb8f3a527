"""Mirror of the graph store (reference src/database/__init__.py exports GraphService and
Neo4jConnection): egraph_dropin.graph_service."""
from egraph_dropin.graph_service import GraphService, Neo4jConnection

__all__ = ["GraphService", "Neo4jConnection"]
