"""Helpers shared by the parity tests."""
from __future__ import annotations


def unhex(x):
    return float.fromhex(x) if isinstance(x, str) and x.startswith(("0x", "-0x")) else x


def record(hyps: list[dict]) -> list[dict]:
    """The golden-fixture view of a hypothesis list (floats exact, random ids dropped)."""
    out = []
    for h in hyps:
        out.append({
            "rule_id": h["rule_id"], "category": h["category"], "title": h["title"],
            "confidence": float(h["confidence"]).hex(),
            "final_score": float(h["final_score"]).hex(), "rank": h["rank"],
            "support_count": h["support_count"],
            "signal_strength": float(h["signal_strength"]).hex(),
            "supporting_evidence_ids": h["supporting_evidence_ids"],
        })
    return out


def golden_record(expected: list[dict]) -> list[dict]:
    out = []
    for h in expected:
        h = dict(h)
        for k in ("confidence", "final_score", "signal_strength"):
            h[k] = float(unhex(h[k])).hex()
        out.append(h)
    return out


# rows that switch on exactly one rule each (rule order of the catalog), used to build an
# evidence list for any reachable 10-bit mask (rules 0 and 1 are mutually exclusive)
def mask_evidence(mask: int) -> list[dict]:
    ev = []
    k = 0

    def pod(**d):
        nonlocal k
        k += 1
        data = {"node_name": f"solo-{k}", "phase": "Pending", "restart_count": 0}
        data.update(d)
        ev.append({"id": f"m{k}", "evidence_type": "kubernetes_pod", "data": data})

    if mask & 0b11:
        pod(waiting_reason="CrashLoopBackOff")
        if mask & 0b01:
            ev.append({"id": "dep", "evidence_type": "deploy_change", "data": {"is_recent_change": True}})
    if mask >> 2 & 1:
        pod(terminated_reason="OOMKilled")
    if mask >> 3 & 1:
        ev.append({"id": "mem", "evidence_type": "metric_signal",
                   "data": {"query_name": "memory_usage_percentage", "is_anomalous": True, "current_value": 97}})
    if mask >> 4 & 1:
        pod(waiting_reason="ErrImagePull")
    if mask >> 5 & 1:
        pod(restart_count=2, node_name="hot-node")
        pod(restart_count=4, node_name="hot-node")
        ev.append({"id": "nd", "evidence_type": "kubernetes_node",
                   "data": {"name": "hot-node", "conditions": {"Ready": {"status": "False"}}}})
    if mask >> 6 & 1:
        ev.append({"id": "hpa", "evidence_type": "metric_signal", "data": {"query_name": "hpa_at_max", "current_value": 1}})
        ev.append({"id": "lat", "evidence_type": "metric_signal", "data": {"query_name": "p99_latency", "current_value": 3.5}})
    if mask >> 7 & 1:
        pod(conditions=[{"type": "Ready", "status": "False", "reason": "ContainersNotReady"}], phase="Running")
    if mask >> 8 & 1:
        pod(terminated_reason="CreateContainerConfigError")
    if mask >> 9 & 1:
        ev.append({"id": "log", "evidence_type": "log_signal", "data": {"patterns_found": ["network"], "error_count": 12}})
    return ev


def reachable_masks() -> list[int]:
    return [m for m in range(1024) if (m & 0b11) != 0b11]
