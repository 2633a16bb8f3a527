"""GPU parity of the rules path (egr_rules_eval / egr_rank through the drop-in API).

Bar: bit-exact -- rule order, confidence / final_score / signal_strength as float64 bit
patterns, ranks and evidence ids -- against the fixtures recorded from the reference and
against the C oracle over the same encoded columns.
"""
from __future__ import annotations

import asyncio
import random

import numpy as np
import pytest

import oracle
from helpers import golden_record, mask_evidence, reachable_masks, record, unhex

pytestmark = pytest.mark.gpu


class _Inc:
    def __init__(self, iid):
        self.id = iid


def _engine():
    from src.services.rca.rules_engine import RulesEngine
    return RulesEngine()


def test_dropin_generate_then_rank_matches_golden(golden):
    from src.services.rca.hypothesis_ranker import HypothesisRanker
    eng, rk = _engine(), HypothesisRanker()
    inc = _Inc(golden["rules"]["incident_id"])
    for case in golden["rules"]["cases"][:120]:
        hyps = asyncio.run(eng.generate_hypotheses(inc, case["evidence"]))
        assert all("final_score" not in h for h in hyps)
        assert all(h["incident_id"] == inc.id for h in hyps)
        ranked = rk.rank(hyps)
        assert record(ranked) == golden_record(case["expected"]), case["name"]


def test_batched_fused_path_matches_every_golden_case(golden):
    cases = golden["rules"]["cases"]
    incs = [_Inc(golden["rules"]["incident_id"])] * len(cases)
    out = asyncio.run(_engine().rank_incidents_batch(incs, [c["evidence"] for c in cases]))
    for case, hyps in zip(cases, out):
        assert record(hyps) == golden_record(case["expected"]), case["name"]


def test_unranked_batch_equals_python_oracle_generate(golden):
    import rca_oracle
    cases = golden["rules"]["cases"]
    incs = [_Inc("i")] * len(cases)
    out = asyncio.run(_engine().generate_hypotheses_batch(incs, [c["evidence"] for c in cases]))
    for case, hyps in zip(cases, out):
        exp = rca_oracle.generate("i", case["evidence"])
        strip = lambda hs: [{k: v for k, v in h.items() if k != "id"} for h in hs]  # noqa: E731
        assert strip(hyps) == exp, case["name"]


def test_every_reachable_mask_matches_lut(golden):
    lut = {row["mask"]: row for row in golden["lut"]}
    masks = reachable_masks()
    out = asyncio.run(_engine().rank_incidents_batch([_Inc("m")] * len(masks),
                                                     [mask_evidence(m) for m in masks]))
    for m, hyps in zip(masks, out):
        row = lut[m]
        assert [h["rule_id"] for h in hyps] == row["rule_ids"], m
        assert [h["confidence"] for h in hyps] == [unhex(x) for x in row["confidence"]], m
        assert [h["final_score"] for h in hyps] == [unhex(x) for x in row["final_score"]], m


def test_errors_raise_like_reference(golden):
    eng = _engine()
    for case in golden["errors"]:
        if case["raises"] is None:
            continue
        with pytest.raises(Exception) as ei:
            asyncio.run(eng.generate_hypotheses(_Inc("e"), case["evidence"]))
        assert type(ei.value).__name__ == case["raises"], case["name"]


def test_generate_is_still_a_coroutine_function():
    import inspect
    from src.services.rca.rules_engine import RulesEngine
    assert inspect.iscoroutinefunction(RulesEngine.generate_hypotheses)


@pytest.mark.parametrize("seed,n,long_rows", [(1, 4096, 0), (2, 257, 700), (3, 1, 3000)])
def test_kernel_outputs_equal_c_oracle(seed, n, long_rows):
    import evidence_fuzz
    from egraph import catalog
    from egraph.encode import encode_batch
    from egraph.rca import RulesDeviceBatch
    rng = random.Random(seed)
    lists = [evidence_fuzz.random_evidence(rng, n_rows=(rng.randrange(long_rows) if long_rows else None))
             for _ in range(n)]
    lists.append([])                                   # empty incident -> unknown
    cat = catalog.default()
    enc = encode_batch(lists, cat)
    b = RulesDeviceBatch(enc, cat)
    b.launch()
    got = b.fetch()
    exp = oracle.rules_eval(cat.table, enc.flags, enc.vocab, enc.node, enc.err, enc.seg_off)
    np.testing.assert_array_equal(got.mask, exp["mask"])
    np.testing.assert_array_equal(got.n_hyp, exp["n_hyp"])
    for i in range(enc.n_incidents):
        nh = int(exp["n_hyp"][i])
        for key in ("order_conf", "order_rank"):
            np.testing.assert_array_equal(getattr(got, key)[i, :nh], exp[key][i, :nh])
        slots = exp["order_conf"][i, :nh]
        for key in ("confidence", "final_score", "strength"):
            assert getattr(got, key)[i, slots].tobytes() == exp[key][i, slots].tobytes(), (i, key)


def test_ranker_matches_golden(golden):
    from src.services.rca.hypothesis_ranker import HypothesisRanker
    rk = HypothesisRanker()
    lists = []
    for case in golden["ranker"]:
        hyps = [dict(h, _i=i) for i, h in enumerate(case["input"])]
        out = rk.rank(hyps)
        assert [h["_i"] for h in out] == case["order"]
        assert [h["final_score"] for h in out] == [unhex(x) for x in case["final_score"]]
        assert [h["rank"] for h in out] == list(range(1, len(out) + 1))
        lists.append([dict(h, _i=i) for i, h in enumerate(case["input"])])
    for case, out in zip(golden["ranker"], rk.rank_many(lists)):      # one launch for all
        assert [h["_i"] for h in out] == case["order"]


def test_ranker_long_lists_equal_c_oracle():
    from egraph.ranker import rank_lists
    rng = random.Random(5)
    lists = [[{"category": rng.choice(["unknown", "network_issue", "bad_deployment"]),
               "confidence": rng.choice([0.5, 0.3, rng.random()]),
               "support_count": rng.choice([0, 1, 2]), "signal_strength": rng.choice([0.0, 0.5])}
              for _ in range(rng.randrange(0, 300))] for _ in range(40)]
    ranked = rank_lists([[dict(h, _i=i) for i, h in enumerate(hs)] for hs in lists])
    from egraph.catalog import CATEGORY_WEIGHTS
    conf = np.array([h["confidence"] for hs in lists for h in hs], np.float64)
    w = np.array([CATEGORY_WEIGHTS[h["category"]] for hs in lists for h in hs], np.float64)
    sup = np.array([h["support_count"] for hs in lists for h in hs], np.float64)
    st = np.array([h["signal_strength"] for hs in lists for h in hs], np.float64)
    off = np.cumsum([0] + [len(hs) for hs in lists]).astype(np.int64)
    final, order = oracle.rank(conf, w, sup, st, off)
    for j, out in enumerate(ranked):
        assert [h["_i"] for h in out] == order[off[j]:off[j + 1]].tolist()
        assert [h["final_score"] for h in out] == final[off[j] + order[off[j]:off[j + 1]]].tolist()
