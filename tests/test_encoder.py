"""Host encoder (product) + C oracle over the encoded columns, against the golden fixtures.

The encoder is the host half of the rules path; this pins it on CPU: golden inputs ->
egraph.encode.encode_batch -> oracle/egraph_oracle.c orc_rules_eval -> dicts, compared with
what the reference produced.  The GPU tests run the same columns through egr_rules_eval.
"""
from __future__ import annotations

import random

import numpy as np
import pytest

import oracle
from helpers import golden_record, record


def _to_dicts(cat, out, i, ids, incident_id):
    """Assemble fused generate+rank dicts from oracle outputs (same layout as the kernel)."""
    from egraph.rca import RulesResult, hypothesis_dicts
    res = RulesResult(out["mask"], out["n_hyp"], out["order_conf"], out["order_rank"],
                      out["confidence"], out["final_score"], out["strength"])
    return hypothesis_dicts(cat, res, i, incident_id, ids, ranked=True)


def test_encoder_plus_c_oracle_match_goldens(golden):
    from egraph import catalog
    from egraph.encode import encode_batch
    cat = catalog.default()
    cases = golden["rules"]["cases"]
    enc = encode_batch([c["evidence"] for c in cases], cat)
    out = oracle.rules_eval(cat.table, enc.flags, enc.vocab, enc.node, enc.err, enc.seg_off)
    for i, case in enumerate(cases):
        got = record(_to_dicts(cat, out, i, enc.evidence_ids[i], golden["rules"]["incident_id"]))
        assert got == golden_record(case["expected"]), case["name"]


def test_encoder_raises_like_the_reference(golden):
    from egraph import catalog
    from egraph.encode import encode_batch
    for case in golden["errors"]:
        if case["raises"] is None:
            encode_batch([case["evidence"]], catalog.default())
            continue
        with pytest.raises(Exception) as ei:
            encode_batch([case["evidence"]], catalog.default())
        assert type(ei.value).__name__ == case["raises"], case["name"]


def test_encoder_matches_python_oracle_on_fresh_random_cases():
    import evidence_fuzz
    import rca_oracle
    from egraph import catalog
    from egraph.encode import encode_batch
    cat = catalog.default()
    rng = random.Random(99)
    lists = [evidence_fuzz.random_evidence(rng) for _ in range(400)]
    enc = encode_batch(lists, cat)
    out = oracle.rules_eval(cat.table, enc.flags, enc.vocab, enc.node, enc.err, enc.seg_off)
    for i, ev in enumerate(lists):
        assert record(_to_dicts(cat, out, i, enc.evidence_ids[i], "x")) == \
            record(rca_oracle.rca("x", ev)), i


def test_float_error_counts_sum_in_row_order():
    from egraph import _lib as L
    from egraph import catalog
    from egraph.encode import encode_batch
    rows = [{"id": i, "evidence_type": "log_signal",
             "data": {"patterns_found": ["network"], "error_count": c}}
            for i, c in enumerate([0.1, 0.2, 0.3, 9.4])]     # 0.1+0.2+0.3+9.4 = 10.000000000000002
    enc = encode_batch([rows], catalog.default())
    assert enc.flags[0] & L.F_ERR_FLOAT
    out = oracle.rules_eval(catalog.default().table, enc.flags, enc.vocab, enc.node, enc.err, enc.seg_off)
    assert out["mask"][0] >> 9 & 1 == (0.1 + 0.2 + 0.3 + 9.4 >= 10)


def test_row_width_is_twenty_bytes():
    from egraph import catalog
    from egraph.encode import encode_batch
    enc = encode_batch([[{"id": 1, "evidence_type": "kubernetes_pod", "data": {}}]], catalog.default())
    assert sum(a.itemsize for a in (enc.flags, enc.vocab, enc.node, enc.err)) == 20
    assert enc.seg_off.dtype == np.int64
