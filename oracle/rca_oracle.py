"""ORACLE (test infrastructure only) -- CPU restatement of the reference RCA path.

Never imported by the product package; only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg use it, and only as the checker.  Pinned against the golden fixtures that
oracle/gen_golden.py records by running the reference itself (tests/test_oracle_golden.py).

Restates, function by function (reference paths):
  extract_signals   src/services/rca/rules_engine.py:264-376
  condition_holds   src/services/rca/rules_engine.py:399-441
  match_rule        src/services/rca/rules_engine.py:378-397
  confidence        src/services/rca/rules_engine.py:443-455
  generate          src/services/rca/rules_engine.py:199-262, :457-478
  rank              src/services/rca/hypothesis_ranker.py:13-80
"""
from __future__ import annotations

import json
from pathlib import Path

CATALOG = (Path(__file__).resolve().parents[1] / "kubernetes-aiops-evidence-graph_amd"
           / "egraph" / "rules_catalog.json")

STRENGTH = {
    "waiting_reason": 0.9, "terminated_reason": 0.9, "recent_deploy": 0.8,
    "no_recent_deploy": 0.6, "memory_usage_high": 0.85, "hpa_at_max": 0.75,
    "latency_high": 0.7, "log_pattern": 0.65, "node_unhealthy": 0.8,
    "multiple_pods_same_node": 0.75, "pod_not_ready": 0.6, "readiness_probe_failing": 0.75,
    "network_errors_high": 0.7,
}
WEIGHTS = {
    "resource_exhaustion": 1.2, "bad_deployment": 1.15, "configuration_error": 1.1,
    "infrastructure_issue": 1.05, "dependency_failure": 1.0, "network_issue": 0.95,
    "scaling_issue": 0.9, "security_issue": 0.85, "external_dependency": 0.8,
    "data_issue": 0.75, "unknown": 0.5,
}


def load_catalog(path: Path = CATALOG) -> dict:
    return json.loads(Path(path).read_text())


def extract_signals(evidence: list[dict]) -> dict:
    sig = {"waiting": set(), "terminated": set(), "patterns": set(), "recent_deploy": False,
           "image_change": False, "memory_high": False, "hpa_max": False, "latency_high": False,
           "node_issues": {}, "restarts": 0, "errors": 0, "ids": [], "per_node": {},
           "not_ready": 0, "readiness": 0}
    for ev in evidence:
        ev_id, ev_type, data = ev.get("id"), ev.get("evidence_type"), ev.get("data", {})
        sig["ids"].append(ev_id)
        kind = {"kubernetes_pod": 1, "deploy_change": 2, "image_change": 3, "log_signal": 4,
                "metric_signal": 5, "kubernetes_node": 6}.get(ev_type)
        if kind == 1:
            if data.get("waiting_reason"):
                sig["waiting"].add(data["waiting_reason"])
            if data.get("terminated_reason"):
                sig["terminated"].add(data["terminated_reason"])
            sig["restarts"] = max(sig["restarts"], data.get("restart_count", 0))
            issue = bool(data.get("waiting_reason") or data.get("terminated_reason")
                         or data.get("restart_count", 0) > 0)
            node = data.get("node_name")
            if node and issue:
                sig["per_node"][node] = sig["per_node"].get(node, 0) + 1
            ready = None
            for c in data.get("conditions", []):
                if c.get("type") == "Ready":
                    ready = c
                    break
            if ready and ready.get("status") != "True" and data.get("phase") == "Running":
                sig["not_ready"] += 1
                if ready.get("reason") == "ContainersNotReady":
                    sig["readiness"] += 1
        elif kind == 2:
            if data.get("is_recent_change"):
                sig["recent_deploy"] = True
        elif kind == 3:
            if data.get("image_changed"):
                sig["image_change"] = True
        elif kind == 4:
            for p in data.get("patterns_found", []):
                sig["patterns"].add(p)
            sig["errors"] += data.get("error_count", 0)
        elif kind == 5:
            q = data.get("query_name", "")
            if "memory" in q and data.get("is_anomalous"):
                cur = data.get("current_value")
                if cur and cur > 90:
                    sig["memory_high"] = True
            if "hpa" in q and "max" in q and data.get("current_value") == 1:
                sig["hpa_max"] = True
            if "latency" in q and data.get("current_value", 0) > 1:
                sig["latency_high"] = True
        elif kind == 6:
            status = data.get("conditions", {}).get("Ready", {}).get("status")
            if status != "True":
                sig["node_issues"][data.get("name")] = data.get("conditions", {})
    return sig


def condition_holds(cond: dict, sig: dict) -> bool:
    t = cond["type"]
    if t == "waiting_reason":
        return bool(sig["waiting"] & set(cond.get("values", [])))
    if t == "terminated_reason":
        return bool(sig["terminated"] & set(cond.get("values", [])))
    if t == "recent_deploy":
        return sig["recent_deploy"]
    if t == "no_recent_deploy":
        return not sig["recent_deploy"]
    if t == "memory_usage_high":
        return sig["memory_high"]
    if t == "hpa_at_max":
        return sig["hpa_max"]
    if t == "latency_high":
        return sig["latency_high"]
    if t == "log_pattern":
        return bool(sig["patterns"] & set(cond.get("patterns", [])))
    if t == "node_unhealthy":
        return bool(sig["node_issues"])
    if t == "multiple_pods_same_node":
        return bool(sig["per_node"]) and max(sig["per_node"].values()) >= cond.get("threshold", 2)
    if t == "pod_not_ready":
        return sig["not_ready"] > 0
    if t == "readiness_probe_failing":
        return sig["readiness"] > 0
    if t == "network_errors_high":
        return sig["errors"] >= cond.get("threshold", 10) and "network" in sig["patterns"]
    return False


def match_rule(rule: dict, sig: dict) -> tuple[bool, int, float]:
    n, hit, strength = len(rule["conditions"]), 0, 0.0
    for cond in rule["conditions"]:
        if condition_holds(cond, sig):
            hit += 1
            strength += STRENGTH.get(cond["type"], 0.0)
    return (hit == n and n > 0), hit, strength / max(n, 1)


def confidence(base: float, hits: int, strength: float) -> float:
    c = base * 0.6 + strength * 0.4
    if hits > 2:
        c = min(c * 1.1, 0.99)
    return round(c, 3)


def generate(incident_id: str, evidence: list[dict], catalog: dict | None = None) -> list[dict]:
    """RulesEngine.generate_hypotheses minus the random `id` field."""
    catalog = catalog or load_catalog()
    sig = extract_signals(evidence)
    out = []
    for rule in catalog["rules"]:
        ok, hits, strength = match_rule(rule, sig)
        if ok:
            out.append({"incident_id": incident_id, "category": rule["category"],
                        "title": rule["name"], "description": rule["description"],
                        "confidence": confidence(rule["confidence_base"], hits, strength),
                        "rank": 0, "supporting_evidence_ids": sig["ids"][:5],
                        "recommended_actions": list(rule["actions"]),
                        "generated_by": "rules_engine", "rule_id": rule["id"],
                        "support_count": hits, "signal_strength": strength})
    out.sort(key=lambda h: h["confidence"], reverse=True)
    if not out:
        u = catalog["unknown"]
        out.append({"incident_id": incident_id, "category": u["category"], "title": u["title"],
                    "description": u["description"], "confidence": u["confidence"],
                    "rank": u["rank"], "supporting_evidence_ids": sig["ids"][:5],
                    "recommended_actions": list(u["recommended_actions"]),
                    "generated_by": u["generated_by"], "rule_id": u["rule_id"],
                    "support_count": u["support_count"], "signal_strength": u["signal_strength"]})
    return out


def rank(hyps: list[dict]) -> list[dict]:
    """HypothesisRanker.rank: mutates and returns the dicts."""
    if not hyps:
        return []
    for h in hyps:
        score = h.get("confidence", 0.5)
        score *= WEIGHTS.get(h.get("category", "unknown"), 1.0)
        sc = h.get("support_count", 0)
        if sc > 0:
            score *= 1 + (min(sc, 5) * 0.05)
        score *= 1 + (h.get("signal_strength", 0) * 0.2)
        h["final_score"] = round(score, 4)
    ranked = sorted(hyps, key=lambda h: h["final_score"], reverse=True)
    for i, h in enumerate(ranked):
        h["rank"] = i + 1
    return ranked


def rca(incident_id: str, evidence: list[dict], catalog: dict | None = None) -> list[dict]:
    """generate + rank, the workflow's two activities back to back."""
    return rank(generate(incident_id, evidence, catalog))
