"""Seeded random evidence-list generator used to build parity cases.

Test infrastructure only.  Produces evidence dicts in the shape the reference
collectors emit (and the minimal shape of the reference's own test builders,
``tests/conftest.py:25-78`` of the reference), deliberately covering every
predicate edge case that ``RulesEngine._process_*_evidence``
(``src/services/rca/rules_engine.py:294-376``) distinguishes: falsy strings,
missing keys, bool-as-int, float restart counts, multiple Ready conditions,
unknown evidence types, ``==1`` comparisons with ``True``/``1.0`` and so on.

Cases built here never raise in the reference; ``raising_cases`` builds the
inputs on which the reference raises (TypeError / AttributeError), used to pin
the product encoder's error behaviour.
"""
from __future__ import annotations

import random

WAITING = [None, "", "CrashLoopBackOff", "ImagePullBackOff", "ErrImagePull",
           "ImageInspectError", "ContainerCreating", "OOMKilled", "PodInitializing"]
TERMINATED = [None, "", "OOMKilled", "ContainerCannotRun", "CreateContainerConfigError",
              "Error", "Completed", "CrashLoopBackOff"]
PATTERNS = ["network", "connection", "error", "critical", "oom", "auth", "missing",
            "null_pointer", "disk", "tls", "Network"]
QUERY_NAMES = ["memory_usage_percentage", "memory_working_set", "oom_killed_total",
               "hpa_at_max", "hpa_max_replicas", "hpa_current_replicas", "p99_latency",
               "p95_latency", "latency_by_endpoint", "http_5xx_rate", "cpu_throttling",
               "restart_count", "memory_hpa_max_latency", "", "MEMORY_usage", "hpamax"]
NODES = ["node-1", "node-2", "node-3", "node-4", None, ""]


def _pick(rng: random.Random, seq):
    return seq[rng.randrange(len(seq))]


def _maybe(rng: random.Random, d: dict, key: str, value, p_missing: float = 0.15):
    if rng.random() >= p_missing:
        d[key] = value


def pod_row(rng: random.Random, ev_id) -> dict:
    data: dict = {}
    _maybe(rng, data, "waiting_reason", _pick(rng, WAITING))
    _maybe(rng, data, "terminated_reason", _pick(rng, TERMINATED))
    _maybe(rng, data, "restart_count", _pick(rng, [0, 0, 0, 1, 3, 5, 2.5, -1, True, False, 0.0]))
    _maybe(rng, data, "node_name", _pick(rng, NODES))
    _maybe(rng, data, "phase", _pick(rng, ["Running", "Running", "Pending", "Failed", ""]))
    conds = []
    for _ in range(rng.randrange(0, 4)):
        c = {}
        _maybe(rng, c, "type", _pick(rng, ["Ready", "Ready", "PodScheduled", "ContainersReady"]), 0.1)
        _maybe(rng, c, "status", _pick(rng, ["True", "False", "Unknown", True]), 0.1)
        _maybe(rng, c, "reason", _pick(rng, ["ContainersNotReady", None, "PodCompleted", ""]), 0.2)
        conds.append(c)
    _maybe(rng, data, "conditions", conds, 0.2)
    data["name"] = f"pod-{rng.randrange(1000)}"
    return {"id": ev_id, "evidence_type": "kubernetes_pod", "data": data}


def deploy_row(rng: random.Random, ev_id) -> dict:
    data: dict = {}
    _maybe(rng, data, "is_recent_change", _pick(rng, [True, False, 1, 0, "yes", "", None]))
    return {"id": ev_id, "evidence_type": "deploy_change", "data": data}


def image_row(rng: random.Random, ev_id) -> dict:
    data: dict = {}
    _maybe(rng, data, "image_changed", _pick(rng, [True, False, None]))
    return {"id": ev_id, "evidence_type": "image_change", "data": data}


def log_row(rng: random.Random, ev_id) -> dict:
    data: dict = {}
    k = rng.randrange(0, 4)
    _maybe(rng, data, "patterns_found", rng.sample(PATTERNS, k))
    _maybe(rng, data, "error_count", _pick(rng, [0, 1, 3, 5, 9, 10, 15, 2.5, 7.25, True, -4]))
    return {"id": ev_id, "evidence_type": "log_signal", "data": data}


def metric_row(rng: random.Random, ev_id) -> dict:
    data: dict = {}
    qn = _pick(rng, QUERY_NAMES)
    _maybe(rng, data, "query_name", qn, 0.05)
    _maybe(rng, data, "is_anomalous", _pick(rng, [True, False, 1, 0, None]))
    # current_value None only where the reference tolerates it (no "latency" in name)
    choices = [95, 90, 90.5, 1, 1.0, True, 0.5, 2, 0, 99.9, 1.0000001, False]
    if "latency" not in (data.get("query_name") or ""):
        choices = choices + [None]
    _maybe(rng, data, "current_value", _pick(rng, choices))
    return {"id": ev_id, "evidence_type": "metric_signal", "data": data}


def node_row(rng: random.Random, ev_id) -> dict:
    data: dict = {}
    _maybe(rng, data, "name", _pick(rng, NODES))
    conds: dict = {}
    r = rng.random()
    if r < 0.7:
        ready: dict = {}
        _maybe(rng, ready, "status", _pick(rng, ["True", "False", "Unknown", True]), 0.1)
        conds["Ready"] = ready
    if rng.random() < 0.3:
        conds["DiskPressure"] = {"status": "True"}
    _maybe(rng, data, "conditions", conds, 0.1)
    return {"id": ev_id, "evidence_type": "kubernetes_node", "data": data}


def other_row(rng: random.Random, ev_id) -> dict:
    t = _pick(rng, ["kubernetes_event", "kubernetes_deployment", "kubernetes_hpa",
                    "config_change", "KUBERNETES_POD", None, "dependency_state"])
    row = {"id": ev_id, "data": {"reason": "BackOff", "waiting_reason": "CrashLoopBackOff"}}
    if t is not None:
        row["evidence_type"] = t
    return row


MAKERS = [pod_row] * 6 + [deploy_row, image_row, log_row, metric_row, metric_row, node_row, other_row]


def random_evidence(rng: random.Random, n_rows: int | None = None) -> list[dict]:
    n = rng.randrange(0, 24) if n_rows is None else n_rows
    # each case draws from its own random mix of row kinds so that rule-match masks vary
    makers = rng.sample(MAKERS, rng.randrange(1, len(MAKERS) + 1))
    rows = []
    for i in range(n):
        ev_id = _pick(rng, [f"ev-{i}", f"ev-{i}", i, None]) if rng.random() < 0.1 else f"ev-{i}"
        row = _pick(rng, makers)(rng, ev_id)
        if rng.random() < 0.03:
            row.pop("data", None)  # missing data -> {} in the reference
        if rng.random() < 0.02:
            row.pop("id", None)
        rows.append(row)
    return rows


def raising_cases() -> list[tuple[str, list[dict]]]:
    """Inputs on which the reference raises, with a short label each."""
    ok_pod = {"id": "a", "evidence_type": "kubernetes_pod", "data": {"restart_count": 1, "node_name": "n"}}
    return [
        ("pod_restart_none", [ok_pod, {"id": "b", "evidence_type": "kubernetes_pod", "data": {"restart_count": None}}]),
        ("pod_restart_str", [{"id": "b", "evidence_type": "kubernetes_pod", "data": {"restart_count": "3"}}]),
        ("pod_data_none", [{"id": "b", "evidence_type": "kubernetes_pod", "data": None}]),
        ("pod_conditions_none", [{"id": "b", "evidence_type": "kubernetes_pod", "data": {"conditions": None}}]),
        ("pod_condition_not_dict", [{"id": "b", "evidence_type": "kubernetes_pod", "data": {"conditions": ["Ready"]}}]),
        ("metric_latency_none", [{"id": "b", "evidence_type": "metric_signal",
                                  "data": {"query_name": "p99_latency", "current_value": None}}]),
        ("metric_query_none", [{"id": "b", "evidence_type": "metric_signal", "data": {"query_name": None}}]),
        ("log_error_count_none", [{"id": "b", "evidence_type": "log_signal", "data": {"error_count": None}}]),
        ("log_patterns_none", [{"id": "b", "evidence_type": "log_signal", "data": {"patterns_found": None}}]),
        ("node_conditions_none", [{"id": "b", "evidence_type": "kubernetes_node", "data": {"conditions": None}}]),
        ("deploy_data_none", [{"id": "b", "evidence_type": "deploy_change", "data": None}]),
        ("row_not_dict", [["kubernetes_pod"]]),
    ]


def scenario_cases() -> list[tuple[str, list[dict]]]:
    """The reference's seven rules-engine scenarios (tests/unit/test_rules_engine.py:24-102),
    restated with the builders' default shapes (tests/conftest.py:25-78)."""

    def pod(evidence_id="ev-1", waiting_reason=None, terminated_reason=None, restart_count=0,
            node_name="node-1", phase="Running", conditions=None):
        return {"id": evidence_id, "evidence_type": "kubernetes_pod",
                "data": {"name": "api-server-abc123", "namespace": "default", "phase": phase,
                         "node_name": node_name, "restart_count": restart_count,
                         "waiting_reason": waiting_reason, "terminated_reason": terminated_reason,
                         "conditions": conditions or []}}

    def deploy(evidence_id="ev-deploy", is_recent_change=True):
        return {"id": evidence_id, "evidence_type": "deploy_change", "data": {"is_recent_change": is_recent_change}}

    def node(evidence_id="ev-node", node_name="node-1", ready=False):
        return {"id": evidence_id, "evidence_type": "kubernetes_node",
                "data": {"name": node_name, "conditions": {"Ready": {"status": "True" if ready else "False"}}}}

    def log(evidence_id="ev-log", patterns_found=None, error_count=0):
        return {"id": evidence_id, "evidence_type": "log_signal",
                "data": {"patterns_found": patterns_found or [], "error_count": error_count}}

    return [
        ("crashloop_recent_deploy", [pod(waiting_reason="CrashLoopBackOff", restart_count=5), deploy(is_recent_change=True)]),
        ("oom_killed", [pod(terminated_reason="OOMKilled")]),
        ("empty", []),
        ("node_failure", [pod(evidence_id="ev-1", waiting_reason="CrashLoopBackOff", node_name="node-1"),
                          pod(evidence_id="ev-2", restart_count=3, node_name="node-1"),
                          node(node_name="node-1", ready=False)]),
        ("readiness", [pod(phase="Running", conditions=[{"type": "Ready", "status": "False", "reason": "ContainersNotReady"}])]),
        ("network", [log(patterns_found=["network"], error_count=15)]),
        ("sorted", [pod(terminated_reason="OOMKilled"), log(patterns_found=["network"], error_count=15)]),
    ]
