"""Evidence-side schema of the hot path (reference src/models/evidence.py:13-161):
the evidence rows the rules read and the graph items the builder merges."""
from __future__ import annotations

from datetime import datetime
from enum import Enum
from typing import Any
from uuid import UUID, uuid4

from pydantic import BaseModel, Field


class EvidenceType(str, Enum):
    KUBERNETES_POD = "kubernetes_pod"
    KUBERNETES_DEPLOYMENT = "kubernetes_deployment"
    KUBERNETES_REPLICASET = "kubernetes_replicaset"
    KUBERNETES_EVENT = "kubernetes_event"
    KUBERNETES_NODE = "kubernetes_node"
    KUBERNETES_SERVICE = "kubernetes_service"
    KUBERNETES_CONFIGMAP = "kubernetes_configmap"
    KUBERNETES_HPA = "kubernetes_hpa"
    KUBERNETES_PVC = "kubernetes_pvc"
    LOG_SIGNAL = "log_signal"
    METRIC_SIGNAL = "metric_signal"
    DEPLOY_CHANGE = "deploy_change"
    CONFIG_CHANGE = "config_change"
    IMAGE_CHANGE = "image_change"
    DEPENDENCY_STATE = "dependency_state"
    NETWORK_TOPOLOGY = "network_topology"


class EvidenceSource(str, Enum):
    KUBERNETES_API = "kubernetes_api"
    PROMETHEUS = "prometheus"
    LOKI = "loki"
    ARGOCD = "argocd"
    HELM = "helm"
    GIT = "git"
    KUBE_STATE_METRICS = "kube_state_metrics"


class Evidence(BaseModel):
    id: UUID = Field(default_factory=uuid4)
    incident_id: UUID
    evidence_type: EvidenceType
    source: EvidenceSource
    entity_name: str
    entity_namespace: str
    entity_uid: str | None = None
    data: dict[str, Any]
    summary: str | None = None
    signal_strength: float = Field(default=0.5, ge=0.0, le=1.0)
    is_anomaly: bool = False
    collected_at: datetime = Field(default_factory=datetime.utcnow)
    time_window_start: datetime | None = None
    time_window_end: datetime | None = None


class GraphEntity(BaseModel):
    """A vertex: MERGEd by (type, id)."""
    id: str
    type: str
    properties: dict[str, Any] = Field(default_factory=dict)


class GraphRelation(BaseModel):
    """An edge: MERGEd by (source vertex, relation_type, target vertex)."""
    source_id: str
    target_id: str
    relation_type: str
    properties: dict[str, Any] = Field(default_factory=dict)


class CollectorResult(BaseModel):
    collector_name: str
    success: bool
    evidence: list[Evidence] = Field(default_factory=list)
    entities: list[GraphEntity] = Field(default_factory=list)
    relations: list[GraphRelation] = Field(default_factory=list)
    errors: list[str] = Field(default_factory=list)
    duration_seconds: float = 0.0
