"""Diagnosis-rule catalog -> device rule table + string vocabularies.

The catalog (rules_catalog.json) is the data of the reference's DIAGNOSIS_RULES
(src/services/rca/rules_engine.py:15-190), exported from the reference by
oracle/gen_golden.py so that titles, descriptions and actions are byte-identical.
The evaluation semantics live in the kernel (csrc/rules.hip); this module only lowers
each condition to (type code, vocabulary mask, parameter, strength):

  * strengths per condition type: rules_engine.py:404-433
  * default thresholds: multiple_pods_same_node 2 (:424), network_errors_high 10 (:430)
  * category weights of the ranker: hypothesis_ranker.py:28-40 (1.0 for unknown names, :50)
  * parameters the reference ignores (within_minutes, threshold of memory_usage_high,
    threshold_ms, duration_seconds, value, node_unhealthy's conditions) are ignored here too.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from pathlib import Path

from . import _lib as L

CATALOG_PATH = Path(__file__).with_name("rules_catalog.json")

COND_CODES = {
    "waiting_reason": 0, "terminated_reason": 1, "recent_deploy": 2, "no_recent_deploy": 3,
    "memory_usage_high": 4, "hpa_at_max": 5, "latency_high": 6, "log_pattern": 7,
    "node_unhealthy": 8, "multiple_pods_same_node": 9, "pod_not_ready": 10,
    "readiness_probe_failing": 11, "network_errors_high": 12,
}
COND_STRENGTH = {
    "waiting_reason": 0.9, "terminated_reason": 0.9, "recent_deploy": 0.8,
    "no_recent_deploy": 0.6, "memory_usage_high": 0.85, "hpa_at_max": 0.75,
    "latency_high": 0.7, "log_pattern": 0.65, "node_unhealthy": 0.8,
    "multiple_pods_same_node": 0.75, "pod_not_ready": 0.6, "readiness_probe_failing": 0.75,
    "network_errors_high": 0.7,
}
CATEGORY_WEIGHTS = {
    "resource_exhaustion": 1.2, "bad_deployment": 1.15, "configuration_error": 1.1,
    "infrastructure_issue": 1.05, "dependency_failure": 1.0, "network_issue": 0.95,
    "scaling_issue": 0.9, "security_issue": 0.85, "external_dependency": 0.8,
    "data_issue": 0.75, "unknown": 0.5,
}
UNSUPPORTED = -1

# vocabulary bit ranges inside row_vocab
WAITING_BITS = range(0, 8)
TERMINATED_BITS = range(8, 16)
PATTERN_BITS = range(16, 32)


@dataclass
class Catalog:
    rules: list[dict]
    unknown: dict
    waiting_vocab: dict = field(default_factory=dict)     # reason -> bit mask
    terminated_vocab: dict = field(default_factory=dict)
    pattern_vocab: dict = field(default_factory=dict)
    table: L.EgrRuleTable | None = None

    @property
    def n_rules(self) -> int:
        return len(self.rules)


def _vocab_add(vocab: dict, bits: range, value, what: str) -> int:
    if value not in vocab:
        if len(vocab) >= len(bits):
            raise ValueError(f"rule catalog uses more than {len(bits)} distinct {what}")
        vocab[value] = 1 << bits[len(vocab)]
    return vocab[value]


def build(rules: list[dict], unknown: dict) -> Catalog:
    """Lower a rule list (reference DIAGNOSIS_RULES shape) to the device table."""
    if len(rules) > L.EGR_MAX_RULES:
        raise ValueError(f"at most {L.EGR_MAX_RULES} rules are supported")
    cat = Catalog(rules=rules, unknown=unknown)
    _vocab_add(cat.pattern_vocab, PATTERN_BITS, "network", "log patterns")  # :431 literal
    t = L.EgrRuleTable()
    t.n_rules = len(rules)
    t.unknown_confidence = float(unknown["confidence"])
    t.unknown_category_weight = CATEGORY_WEIGHTS.get(unknown["category"], 1.0)
    for r, rule in enumerate(rules):
        conds = rule["conditions"]
        if len(conds) > L.EGR_MAX_CONDS:
            raise ValueError(f"rule {rule['id']}: at most {L.EGR_MAX_CONDS} conditions")
        tr = t.rules[r]
        tr.n_conds = len(conds)
        tr.confidence_base = float(rule["confidence_base"])
        tr.category_weight = CATEGORY_WEIGHTS.get(rule["category"], 1.0)
        for c, cond in enumerate(conds):
            ctype = cond["type"]
            code = COND_CODES.get(ctype, UNSUPPORTED)
            tr.cond_type[c] = code
            tr.cond_strength[c] = COND_STRENGTH.get(ctype, 0.0)
            mask = 0
            if ctype == "waiting_reason":
                for v in cond.get("values", []):
                    mask |= _vocab_add(cat.waiting_vocab, WAITING_BITS, v, "waiting reasons")
            elif ctype == "terminated_reason":
                for v in cond.get("values", []):
                    mask |= _vocab_add(cat.terminated_vocab, TERMINATED_BITS, v, "terminated reasons")
            elif ctype == "log_pattern":
                for v in cond.get("patterns", []):
                    mask |= _vocab_add(cat.pattern_vocab, PATTERN_BITS, v, "log patterns")
            elif ctype == "multiple_pods_same_node":
                tr.cond_param[c] = float(cond.get("threshold", 2))
            elif ctype == "network_errors_high":
                tr.cond_param[c] = float(cond.get("threshold", 10))
            tr.cond_mask[c] = mask
    t.network_vocab_bit = (cat.pattern_vocab["network"]).bit_length() - 1
    cat.table = t
    return cat


def load(path: Path = CATALOG_PATH) -> Catalog:
    data = json.loads(Path(path).read_text())
    return build(data["rules"], data["unknown"])


_DEFAULT: Catalog | None = None


def default() -> Catalog:
    global _DEFAULT
    if _DEFAULT is None:
        _DEFAULT = load()
    return _DEFAULT
