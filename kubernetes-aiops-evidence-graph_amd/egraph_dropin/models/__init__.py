"""Models on the evidence-graph hot path (reference src/models/__init__.py)."""
from .evidence import (
    CollectorResult,
    Evidence,
    EvidenceSource,
    EvidenceType,
    GraphEntity,
    GraphRelation,
)
from .hypothesis import (
    DiagnosisRule,
    Hypothesis,
    HypothesisCategory,
    HypothesisSource,
    RCAResult,
)
from .incident import (
    Incident,
    IncidentCreate,
    IncidentSeverity,
    IncidentSource,
    IncidentStatus,
)

__all__ = [
    "CollectorResult", "DiagnosisRule", "Evidence", "EvidenceSource", "EvidenceType",
    "GraphEntity", "GraphRelation", "Hypothesis", "HypothesisCategory", "HypothesisSource",
    "Incident", "IncidentCreate", "IncidentSeverity", "IncidentSource", "IncidentStatus", "RCAResult",
]
