"""Incident model -- input type of the hot path (reference src/models/incident.py:11-91).
Only `id` is read on the path (rules_engine.py:250); the schema is kept for drop-in use."""
from __future__ import annotations

from datetime import datetime
from enum import Enum
from uuid import UUID, uuid4

from pydantic import BaseModel, Field


class IncidentSeverity(str, Enum):
    CRITICAL = "critical"
    HIGH = "high"
    MEDIUM = "medium"
    LOW = "low"
    INFO = "info"


class IncidentStatus(str, Enum):
    OPEN = "open"
    INVESTIGATING = "investigating"
    IDENTIFIED = "identified"
    REMEDIATING = "remediating"
    RESOLVED = "resolved"
    CLOSED = "closed"


class IncidentSource(str, Enum):
    ALERTMANAGER = "alertmanager"
    GRAFANA = "grafana"
    PROMETHEUS = "prometheus"
    MANUAL = "manual"
    SYNTHETIC = "synthetic"


class Incident(BaseModel):
    id: UUID = Field(default_factory=uuid4)
    fingerprint: str
    title: str = Field(..., max_length=500)
    description: str | None = None
    severity: IncidentSeverity
    status: IncidentStatus = IncidentStatus.OPEN
    source: IncidentSource
    cluster: str
    namespace: str
    service: str | None = None
    labels: dict[str, str] = Field(default_factory=dict)
    annotations: dict[str, str] = Field(default_factory=dict)
    started_at: datetime
    acknowledged_at: datetime | None = None
    resolved_at: datetime | None = None
    created_at: datetime = Field(default_factory=datetime.utcnow)
    updated_at: datetime = Field(default_factory=datetime.utcnow)


class IncidentCreate(BaseModel):
    """Schema for creating a new incident (reference src/models/incident.py:92-104); the output of
    AlertNormalizer."""
    fingerprint: str
    title: str
    description: str | None = None
    severity: IncidentSeverity
    source: IncidentSource
    cluster: str
    namespace: str
    service: str | None = None
    labels: dict[str, str] = Field(default_factory=dict)
    annotations: dict[str, str] = Field(default_factory=dict)
    started_at: datetime
