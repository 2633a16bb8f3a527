"""Drop-in AlertNormalizer (reference src/services/ingestion/normalizer.py:15-218) whose
fingerprints are computed on the GPU (egr_fingerprint, csrc/alerts.hip).

Field mapping follows the reference per source:
  alertmanager (:32-102), grafana (:104-168, commonLabels/commonAnnotations merged under the
  alert's own), prometheus (:170-206); fingerprint = sha256(f"{source}:{alertname}:{namespace}:
  {service}").hexdigest()[:32] (:208-218).
The per-alert classmethods keep the reference's signatures; the *_batch variants normalise a
whole payload with ONE fingerprint launch (the alert-storm path).  Timestamps are parsed with the
running interpreter's datetime.fromisoformat after the reference's "Z" -> "+00:00" rewrite.
"""
from __future__ import annotations

from datetime import datetime, timezone
from typing import Any

from egraph import alerts as _alerts
from egraph_dropin.models import IncidentCreate, IncidentSeverity, IncidentSource

UTC = timezone.utc


def _started_at(alert: dict[str, Any]) -> datetime:
    s = alert.get("startsAt")
    if not s:
        return datetime.now(UTC)
    try:
        return datetime.fromisoformat(s.replace("Z", "+00:00"))
    except ValueError:
        return datetime.now(UTC)


class AlertNormalizer:
    """Normalizes alerts from different sources to IncidentCreate."""

    SEVERITY_MAP = {
        "critical": IncidentSeverity.CRITICAL,
        "high": IncidentSeverity.HIGH,
        "warning": IncidentSeverity.MEDIUM,
        "info": IncidentSeverity.INFO,
        "low": IncidentSeverity.LOW,
        "alerting": IncidentSeverity.HIGH,
        "error": IncidentSeverity.HIGH,
        "warn": IncidentSeverity.MEDIUM,
    }

    # ---- per-source field extraction: (IncidentCreate kwargs without fingerprint, key) ------
    @classmethod
    def _severity(cls, labels: dict) -> IncidentSeverity:
        return cls.SEVERITY_MAP.get(labels.get("severity", "warning").lower(), IncidentSeverity.MEDIUM)

    @classmethod
    def _fields_alertmanager(cls, alert: dict, payload: dict) -> tuple[dict, str]:
        labels = alert.get("labels", {})
        annotations = alert.get("annotations", {})
        alertname = labels.get("alertname", "Unknown Alert")
        namespace = labels.get("namespace", "default")
        cluster = labels.get("cluster") or labels.get("kubernetes_cluster") or "default-cluster"
        service = labels.get("service") or labels.get("job") or labels.get("deployment")
        pod = labels.get("pod")
        target = pod or service
        title = f"{alertname}: {target}" if target else alertname
        kw = dict(title=title,
                  description=annotations.get("description") or annotations.get("summary") or "",
                  severity=cls._severity(labels), source=IncidentSource.ALERTMANAGER,
                  cluster=cluster, namespace=namespace, service=service, labels=labels,
                  annotations=annotations, started_at=_started_at(alert))
        return kw, _alerts.fingerprint_key("alertmanager", alertname, namespace, service or pod or "")

    @classmethod
    def _fields_grafana(cls, alert: dict, payload: dict) -> tuple[dict, str]:
        labels = {**payload.get("commonLabels", {}), **alert.get("labels", {})}
        annotations = {**payload.get("commonAnnotations", {}), **alert.get("annotations", {})}
        alertname = labels.get("alertname") or alert.get("alertname", "Grafana Alert")
        namespace = labels.get("namespace", "default")
        service = labels.get("service") or labels.get("grafana_folder")
        kw = dict(title=annotations.get("summary") or alertname,
                  description=annotations.get("description", ""),
                  severity=cls._severity(labels), source=IncidentSource.GRAFANA,
                  cluster=labels.get("cluster", "default-cluster"), namespace=namespace,
                  service=service, labels=labels, annotations=annotations,
                  started_at=_started_at(alert))
        return kw, _alerts.fingerprint_key("grafana", alertname, namespace, service or "")

    @classmethod
    def _fields_prometheus(cls, alert: dict, payload: dict | None = None) -> tuple[dict, str]:
        labels = alert.get("labels", {})
        annotations = alert.get("annotations", {})
        alertname = labels.get("alertname", "Prometheus Alert")
        namespace = labels.get("namespace", "default")
        service = labels.get("service") or labels.get("instance")
        kw = dict(title=alertname, description=annotations.get("description", ""),
                  severity=cls._severity(labels), source=IncidentSource.PROMETHEUS,
                  cluster=labels.get("cluster", "default-cluster"), namespace=namespace,
                  service=service, labels=labels, annotations=annotations,
                  started_at=datetime.now(UTC))
        return kw, _alerts.fingerprint_key("prometheus", alertname, namespace, service or "")

    @classmethod
    def _batch(cls, fields: list[tuple[dict, str]], device=None) -> list[IncidentCreate]:
        if not fields:
            return []
        _, hexes = _alerts.fingerprints([k for _, k in fields], device=device, hex=True)
        return [IncidentCreate(fingerprint=h, **kw) for (kw, _), h in zip(fields, hexes)]

    # ---- the reference's API ----------------------------------------------------------------
    @classmethod
    def normalize_alertmanager(cls, alert: dict[str, Any], payload: dict[str, Any]) -> IncidentCreate:
        return cls._batch([cls._fields_alertmanager(alert, payload)])[0]

    @classmethod
    def normalize_grafana(cls, alert: dict[str, Any], payload: dict[str, Any]) -> IncidentCreate:
        return cls._batch([cls._fields_grafana(alert, payload)])[0]

    @classmethod
    def normalize_prometheus(cls, alert: dict[str, Any]) -> IncidentCreate:
        return cls._batch([cls._fields_prometheus(alert)])[0]

    @classmethod
    def _generate_fingerprint(cls, source: str, alertname: str, namespace: str, service: str) -> str:
        _, hexes = _alerts.fingerprints([_alerts.fingerprint_key(source, alertname, namespace, service)],
                                        hex=True)
        return hexes[0]

    # ---- batch entry points (one fingerprint launch per payload) ----------------------------
    @classmethod
    def normalize_alertmanager_batch(cls, alerts: list[dict], payload: dict, device=None) -> list[IncidentCreate]:
        return cls._batch([cls._fields_alertmanager(a, payload) for a in alerts], device)

    @classmethod
    def normalize_grafana_batch(cls, alerts: list[dict], payload: dict, device=None) -> list[IncidentCreate]:
        return cls._batch([cls._fields_grafana(a, payload) for a in alerts], device)

    @classmethod
    def normalize_prometheus_batch(cls, alerts: list[dict], device=None) -> list[IncidentCreate]:
        return cls._batch([cls._fields_prometheus(a) for a in alerts], device)
