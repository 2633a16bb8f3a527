"""Generate the committed golden fixtures under tests/golden/ by RUNNING THE REFERENCE.

Test infrastructure only: this script imports the reference implementation from
/root/reference (read-only, this container only) and records its outputs as
small JSON fixtures.  Nothing under oracle/ ships in the product path; the
reference never travels to the GPU box -- only the JSON it produced does.

Reference modules executed (by file path, see SURVEY.md §8c for the shims):
  * src/services/rca/rules_engine.py      RulesEngine.generate_hypotheses (:199-233)
  * src/services/rca/hypothesis_ranker.py HypothesisRanker.rank          (:13-80)
  * src/services/ingestion/normalizer.py  AlertNormalizer._generate_fingerprint (:208-218)

Shims (none touches arithmetic): a no-op ``structlog`` module (not installed);
``datetime.UTC`` for Python 3.10; modules loaded by path so that
``src/services/rca/__init__.py`` does not pull in ``pydantic_settings``.
``sys.dont_write_bytecode`` keeps __pycache__ out of /root/reference.

Usage:  python oracle/gen_golden.py [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import asyncio
import datetime as _dt
import importlib.util
import json
import random
import sys
import types
from pathlib import Path

sys.dont_write_bytecode = True
REPO = Path(__file__).resolve().parents[1]
GOLDEN = REPO / "tests" / "golden"
CATALOG = REPO / "kubernetes-aiops-evidence-graph_amd" / "egraph" / "rules_catalog.json"
sys.path.insert(0, str(REPO / "tests"))

import evidence_fuzz  # noqa: E402

N_RANDOM_CASES = 1000
SEED = 20260821


def _install_shims() -> None:
    class _NoLog:
        def __getattr__(self, _name):
            return lambda *a, **k: None

    stub = types.ModuleType("structlog")
    stub.get_logger = lambda *a, **k: _NoLog()
    sys.modules["structlog"] = stub
    if not hasattr(_dt, "UTC"):
        _dt.UTC = _dt.timezone.utc


def _load(path: Path, name: str):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _hex(x):
    return float(x).hex() if isinstance(x, float) else x


def _record(hyps: list[dict]) -> list[dict]:
    out = []
    for h in hyps:
        out.append({
            "rule_id": h["rule_id"],
            "category": h["category"],
            "title": h["title"],
            "confidence": _hex(h["confidence"]),
            "final_score": _hex(h["final_score"]),
            "rank": h["rank"],
            "support_count": h["support_count"],
            "signal_strength": _hex(h["signal_strength"]),
            "supporting_evidence_ids": h["supporting_evidence_ids"],
        })
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    ref = Path(args.ref)
    _install_shims()
    sys.path.insert(0, str(ref))

    from src.models import Incident, IncidentSeverity, IncidentSource  # reference models

    re_mod = _load(ref / "src/services/rca/rules_engine.py", "ref_rules_engine")
    rk_mod = _load(ref / "src/services/rca/hypothesis_ranker.py", "ref_hypothesis_ranker")
    nm_mod = _load(ref / "src/services/ingestion/normalizer.py", "ref_normalizer")
    engine = re_mod.RulesEngine()
    ranker = rk_mod.HypothesisRanker()

    incident = Incident(
        id="00000000-0000-4000-8000-000000000001", fingerprint="golden", title="golden",
        severity=IncidentSeverity.CRITICAL, source=IncidentSource.ALERTMANAGER,
        cluster="c", namespace="default", service="api-server",
        started_at=_dt.datetime(2026, 1, 5, 5, 0, tzinfo=_dt.timezone.utc))

    def run(evidence):
        hyps = asyncio.run(engine.generate_hypotheses(incident, evidence))
        return ranker.rank(hyps)

    GOLDEN.mkdir(parents=True, exist_ok=True)

    # --- rule catalog (data the product needs to emit identical dicts) -------------
    catalog = {"rules": [], "unknown": None}
    for r in re_mod.DIAGNOSIS_RULES:
        catalog["rules"].append({
            "id": r["id"], "name": r["name"], "category": r["category"].value,
            "hypothesis": r["hypothesis"], "description": r["description"],
            "confidence_base": r["confidence_base"], "actions": list(r["actions"]),
            "conditions": [dict(c) for c in r["conditions"]],
        })
    unk = engine._create_unknown_hypothesis(incident, engine._init_signals())
    catalog["unknown"] = {k: unk[k] for k in ("category", "title", "description", "confidence",
                                                "rank", "recommended_actions", "generated_by",
                                                "rule_id", "support_count", "signal_strength")}
    CATALOG.write_text(json.dumps(catalog, indent=1) + "\n")

    # --- scenarios + random cases ------------------------------------------------------
    cases = []
    for name, ev in evidence_fuzz.scenario_cases():
        cases.append({"name": name, "evidence": ev, "expected": _record(run(ev))})
    rng = random.Random(SEED)
    for i in range(N_RANDOM_CASES):
        ev = evidence_fuzz.random_evidence(rng)
        cases.append({"name": f"random_{i}", "evidence": ev, "expected": _record(run(ev))})
    # a few long incidents (collector-sized: ~100 rows)
    for i in range(16):
        ev = evidence_fuzz.random_evidence(rng, n_rows=rng.randrange(90, 200))
        cases.append({"name": f"long_{i}", "evidence": ev, "expected": _record(run(ev))})
    (GOLDEN / "rules_cases.json").write_text(json.dumps({"incident_id": str(incident.id),
                                                          "cases": cases}) + "\n")

    errors = []
    for name, ev in evidence_fuzz.raising_cases():
        try:
            run(ev)
            exc = None
        except Exception as e:  # noqa: BLE001 - we record the type the reference raises
            exc = type(e).__name__
        errors.append({"name": name, "evidence": ev, "raises": exc})
    (GOLDEN / "rules_errors.json").write_text(json.dumps(errors, indent=1) + "\n")

    # --- 1024-entry mask LUT via the reference's own per-rule machinery -----------------
    per_rule = []
    for rule in re_mod.DIAGNOSIS_RULES:
        # craft a signals dict that satisfies every condition of this rule
        sig = engine._init_signals()
        for c in rule["conditions"]:
            t = c["type"]
            if t == "waiting_reason":
                sig["waiting_reasons"].add(c["values"][0])
            elif t == "terminated_reason":
                sig["terminated_reasons"].add(c["values"][0])
            elif t == "recent_deploy":
                sig["has_recent_deploy"] = True
            elif t == "memory_usage_high":
                sig["memory_usage_high"] = True
            elif t == "hpa_at_max":
                sig["hpa_at_max"] = True
            elif t == "latency_high":
                sig["latency_high"] = True
            elif t == "log_pattern":
                sig["log_patterns"].add(c["patterns"][0])
            elif t == "node_unhealthy":
                sig["node_issues"]["n"] = {}
            elif t == "multiple_pods_same_node":
                sig["pods_by_node"]["n"] = 2
            elif t == "pod_not_ready":
                sig["not_ready_pods"] = 1
            elif t == "readiness_probe_failing":
                sig["readiness_probe_failures"] = 1
            elif t == "network_errors_high":
                sig["error_count"] = 10
                sig["log_patterns"].add("network")
        m = engine._match_rule(rule, sig)
        assert m["matched"], rule["id"]
        per_rule.append(engine._create_hypothesis(incident, rule, m))
    lut = []
    for mask in range(1 << len(per_rule)):
        hyps = [dict(per_rule[i]) for i in range(len(per_rule)) if mask >> i & 1]
        hyps.sort(key=lambda x: x["confidence"], reverse=True)  # rules_engine.py:228
        if not hyps:
            hyps.append(engine._create_unknown_hypothesis(incident, engine._init_signals()))
        ranked = ranker.rank(hyps)
        lut.append({"mask": mask, "rule_ids": [h["rule_id"] for h in ranked],
                    "confidence": [_hex(h["confidence"]) for h in ranked],
                    "final_score": [_hex(h["final_score"]) for h in ranked]})
    (GOLDEN / "mask_lut.json").write_text(json.dumps(lut) + "\n")

    # --- ranker cases (reference tests/unit/test_hypothesis_ranker.py:14-49 + random) ----
    rcases = []

    def mk(category, confidence, support_count=0, signal_strength=0.0):
        return {"category": category, "confidence": confidence,
                "support_count": support_count, "signal_strength": signal_strength}

    fixed = [
        [],
        [mk("unknown", 0.3), mk("resource_exhaustion", 0.9)],
        [mk("external_dependency", 0.75), mk("resource_exhaustion", 0.70)],
        [mk("unknown", 0.5, support_count=0), mk("unknown", 0.5, support_count=5)],
    ]
    cats = ["resource_exhaustion", "bad_deployment", "configuration_error", "infrastructure_issue",
            "dependency_failure", "network_issue", "scaling_issue", "security_issue",
            "external_dependency", "data_issue", "unknown", "not_a_category"]
    for _ in range(600):
        n = rng.randrange(0, 14)
        hs = []
        for _ in range(n):
            h = {}
            if rng.random() > 0.05:
                h["category"] = rng.choice(cats)
            if rng.random() > 0.05:
                h["confidence"] = rng.choice([rng.random(), round(rng.random(), 3), 0.3, 0.93, 1, 0, 0.5])
            if rng.random() > 0.1:
                h["support_count"] = rng.choice([0, 1, 2, 3, 5, 7, -1, 2.5, True])
            if rng.random() > 0.1:
                h["signal_strength"] = rng.choice([rng.random(), 0.85, 0.0, 0, 0.775, 1])
            hs.append(h)
        fixed.append(hs)
    # ties on purpose: identical hypotheses must keep input order (stable sort)
    fixed.append([mk("unknown", 0.5), mk("unknown", 0.5), mk("network_issue", 0.5 * 0.5 / 0.95)])
    for hs in fixed:
        inp = json.loads(json.dumps(hs))
        for i, h in enumerate(inp):
            h["_i"] = i
        out = ranker.rank([dict(h) for h in inp])
        rcases.append({"input": [{k: v for k, v in h.items() if k != "_i"} for h in inp],
                       "order": [h["_i"] for h in out],
                       "final_score": [_hex(h["final_score"]) for h in out]})
    (GOLDEN / "ranker_cases.json").write_text(json.dumps(rcases) + "\n")

    # --- normalizer fingerprints (next row: alert storm) ----------------------------------
    fps = []
    for i in range(64):
        key = ("alertmanager" if i % 3 else "grafana", f"Alert{i % 7}", f"ns{i % 5}", f"svc{i % 11}")
        fps.append({"key": list(key), "fingerprint": nm_mod.AlertNormalizer._generate_fingerprint(*key)})
    (GOLDEN / "fingerprints.json").write_text(json.dumps(fps, indent=0) + "\n")

    print(f"wrote {len(cases)} rule cases, {len(errors)} error cases, {len(lut)} LUT rows, "
          f"{len(rcases)} ranker cases, {len(fps)} fingerprints -> {GOLDEN}")


if __name__ == "__main__":
    main()
