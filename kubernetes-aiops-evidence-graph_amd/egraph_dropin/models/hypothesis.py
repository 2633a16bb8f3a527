"""Hypothesis / ranking output models (reference src/models/hypothesis.py:12-153).
The hot path itself emits plain dicts (rules_engine.py:248-262); these models validate them."""
from __future__ import annotations

from datetime import datetime
from enum import Enum
from uuid import UUID, uuid4

from pydantic import BaseModel, Field


class HypothesisCategory(str, Enum):
    RESOURCE_EXHAUSTION = "resource_exhaustion"
    BAD_DEPLOYMENT = "bad_deployment"
    CONFIGURATION_ERROR = "configuration_error"
    DEPENDENCY_FAILURE = "dependency_failure"
    INFRASTRUCTURE_ISSUE = "infrastructure_issue"
    NETWORK_ISSUE = "network_issue"
    SCALING_ISSUE = "scaling_issue"
    SECURITY_ISSUE = "security_issue"
    EXTERNAL_DEPENDENCY = "external_dependency"
    DATA_ISSUE = "data_issue"
    UNKNOWN = "unknown"


class HypothesisSource(str, Enum):
    RULES_ENGINE = "rules_engine"
    LLM = "llm"
    HYBRID = "hybrid"
    MANUAL = "manual"


class Hypothesis(BaseModel):
    id: UUID = Field(default_factory=uuid4)
    incident_id: UUID
    category: HypothesisCategory
    title: str = Field(..., max_length=500)
    description: str
    confidence: float = Field(..., ge=0.0, le=1.0)
    rank: int = Field(..., ge=1)
    supporting_evidence_ids: list[UUID] = Field(default_factory=list)
    contradicting_evidence_ids: list[UUID] = Field(default_factory=list)
    support_count: int = 0
    recency_weight: float = 0.0
    scope_weight: float = 0.0
    signal_strength: float = 0.0
    recommended_actions: list[str] = Field(default_factory=list)
    why_not_notes: str | None = None
    reasoning: str | None = None
    generated_at: datetime = Field(default_factory=datetime.utcnow)
    generated_by: HypothesisSource


class DiagnosisRule(BaseModel):
    id: str
    name: str
    description: str | None = None
    conditions: list[dict]
    hypothesis_template: str
    category: HypothesisCategory
    confidence_base: float = Field(..., ge=0.0, le=1.0)
    recommended_actions: list[str] = Field(default_factory=list)
    priority: int = 50
    enabled: bool = True


class RCAResult(BaseModel):
    incident_id: UUID
    hypotheses: list[Hypothesis] = Field(default_factory=list)
    top_hypothesis: Hypothesis | None = None
    evidence_summary: str = ""
    analysis_duration_seconds: float = 0.0
    rules_matched: list[str] = Field(default_factory=list)
    llm_used: bool = False
    generated_at: datetime = Field(default_factory=datetime.utcnow)
