"""Pin the oracle (CPU restatement) against fixtures recorded from the reference itself.

tests/golden/*.json were produced by oracle/gen_golden.py running the reference's
RulesEngine / HypothesisRanker / AlertNormalizer.  If these pass, the oracle
is a faithful stand-in for the reference on every recorded input.
"""
from __future__ import annotations

import hashlib

import numpy as np
import pytest

import rca_oracle
from helpers import golden_record, mask_evidence, reachable_masks, record, unhex


def test_python_oracle_matches_every_golden_case(golden):
    iid = golden["rules"]["incident_id"]
    for case in golden["rules"]["cases"]:
        got = record(rca_oracle.rca(iid, case["evidence"]))
        assert got == golden_record(case["expected"]), case["name"]


def test_python_oracle_raises_like_the_reference(golden):
    for case in golden["errors"]:
        if case["raises"] is None:
            rca_oracle.rca("x", case["evidence"])
            continue
        with pytest.raises(Exception) as ei:
            rca_oracle.rca("x", case["evidence"])
        assert type(ei.value).__name__ == case["raises"], case["name"]


def test_mask_lut_reproduced_by_oracle_formulas(golden):
    cat = rca_oracle.load_catalog()
    per_rule = []
    for rule in cat["rules"]:
        strength = sum(rca_oracle.STRENGTH[c["type"]] for c in rule["conditions"]) / len(rule["conditions"])
        per_rule.append({"rule_id": rule["id"], "category": rule["category"],
                         "confidence": rca_oracle.confidence(rule["confidence_base"],
                                                             len(rule["conditions"]), strength),
                         "support_count": len(rule["conditions"]), "signal_strength": strength})
    for row in golden["lut"]:
        hyps = [dict(per_rule[i]) for i in range(len(per_rule)) if row["mask"] >> i & 1]
        hyps.sort(key=lambda h: h["confidence"], reverse=True)
        if not hyps:
            hyps = [{"rule_id": "unknown", "category": "unknown", "confidence": 0.3,
                     "support_count": 0, "signal_strength": 0.0}]
        ranked = rca_oracle.rank(hyps)
        assert [h["rule_id"] for h in ranked] == row["rule_ids"], row["mask"]
        assert [h["confidence"] for h in ranked] == [unhex(x) for x in row["confidence"]]
        assert [h["final_score"] for h in ranked] == [unhex(x) for x in row["final_score"]]


def test_mask_evidence_builder_hits_every_reachable_mask(golden):
    lut = {row["mask"]: row["rule_ids"] for row in golden["lut"]}
    for m in reachable_masks():
        got = [h["rule_id"] for h in rca_oracle.rca("x", mask_evidence(m))]
        assert got == lut[m], m


def test_python_oracle_ranker_matches_golden(golden):
    for case in golden["ranker"]:
        hyps = [dict(h, _i=i) for i, h in enumerate(case["input"])]
        out = rca_oracle.rank(hyps)
        assert [h["_i"] for h in out] == case["order"]
        assert [h["final_score"] for h in out] == [unhex(x) for x in case["final_score"]]


def test_c_oracle_round_matches_python():
    import oracle
    rng = np.random.default_rng(7)
    xs = np.concatenate([rng.random(20000) * 3, rng.uniform(-5, 5, 5000),
                         np.round(rng.random(5000), 5), rng.integers(0, 100000, 5000) / 2e4])
    for x in xs:
        for nd in (3, 4):
            assert oracle.lib.orc_round(float(x), nd) == round(float(x), nd)


def test_fingerprint_vectors(golden):
    # normalizer.py:208-218 restated; pins the next-row (alert storm) front end
    for fp in golden["fingerprints"]:
        key = ":".join(fp["key"])
        assert hashlib.sha256(key.encode()).hexdigest()[:32] == fp["fingerprint"]
