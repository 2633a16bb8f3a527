"""egraph.ranker.FusedRanks on the CPU: the rules kernel's fused ranking reused by
HypothesisRanker.rank (hypothesis_ranker.py:13-80) only for lists it generated, unchanged.

The kernel's outputs come from the C oracle here (oracle/egraph_oracle.c orc_rules_eval, the
checker the GPU tests compare the kernel with bit for bit); the dicts are assembled by the
native host code exactly as the drop-in assembles them.  Every reuse must equal the reference
ranker (oracle/rca_oracle.py rank) on copies of the same dicts, and any edit to a field the
ranker reads, a reordering or a foreign list must miss.
"""
from __future__ import annotations

import copy
import json
import random

import numpy as np

import evidence_fuzz
import oracle
import rca_oracle
from helpers import record


def _generated(lists):
    from egraph import catalog
    from egraph.encode import encode_batch
    from egraph.rca import RulesResult, hypothesis_lists
    cat = catalog.default()
    enc = encode_batch(lists, cat)
    x = oracle.rules_eval(cat.table, enc.flags, enc.vocab, enc.node, enc.err, enc.seg_off)
    B, S = enc.n_incidents, cat.n_rules + 1
    res = RulesResult(x["mask"].view(np.uint32), x["n_hyp"], *(x[k].reshape(B, S) for k in (
        "order_conf", "order_rank", "confidence", "final_score", "strength")))
    hyps = hypothesis_lists(cat, res, [f"inc-{i}" for i in range(B)], enc.evidence_ids, False)
    return cat, res, hyps


def test_reuse_equals_the_reference_ranker():
    from egraph.ranker import FusedRanks
    rng = random.Random(5)
    lists = [evidence_fuzz.random_evidence(rng) for _ in range(300)]
    lists += [ev for _, ev in evidence_fuzz.scenario_cases()] + [[]]
    cat, res, hyps = _generated(lists)
    fr = FusedRanks()
    fr.register(cat, res, hyps, range(len(hyps)))
    for h in hyps:
        want = rca_oracle.rank(copy.deepcopy(h))
        # the list as the next activity receives it: a JSON round trip (new dicts, same values)
        got = fr.apply(json.loads(json.dumps(h)))
        assert got is not None
        assert record(got) == record(want)
        assert [x["id"] for x in got] == [x["id"] for x in want]
        mine = fr.apply(h)                       # and in place, as HypothesisRanker.rank mutates
        assert mine is not None and record(mine) == record(want)
        assert all(a is b for a, b in zip(sorted(mine, key=id), sorted(h, key=id)))
    assert fr.misses == 0 and fr.hits == 2 * len(hyps)


def test_edited_reordered_or_foreign_lists_miss():
    from egraph.ranker import FusedRanks
    rng = random.Random(9)
    lists = [ev for _, ev in evidence_fuzz.scenario_cases()]
    lists += [evidence_fuzz.random_evidence(rng) for _ in range(50)]
    cat, res, hyps = _generated(lists)
    fr = FusedRanks()
    fr.register(cat, res, hyps, range(len(hyps)))
    multi = [h for h in hyps if len(h) >= 2]
    assert multi
    h = copy.deepcopy(multi[0])
    h[0]["confidence"] = 0.5
    assert fr.apply(h) is None
    for key, val in (("category", "network"), ("support_count", 5), ("signal_strength", 0.1)):
        h = copy.deepcopy(multi[0])
        h[-1][key] = val
        assert fr.apply(h) is None, key
    h = copy.deepcopy(multi[0])
    h.reverse()
    assert fr.apply(h) is None
    h = copy.deepcopy(multi[0])
    h.pop()
    assert fr.apply(h) is None
    h = copy.deepcopy(multi[0])
    del h[0]["confidence"]                       # the reference would use its 0.5 default
    assert fr.apply(h) is None
    assert fr.apply([{"confidence": 0.9, "category": "deployment"}]) is None
    assert fr.apply([]) is None


def test_capacity_evicts_oldest():
    from egraph.ranker import FusedRanks
    rng = random.Random(2)
    cat, res, hyps = _generated([evidence_fuzz.random_evidence(rng) for _ in range(40)])
    fr = FusedRanks(capacity=10)
    fr.register(cat, res, hyps, range(len(hyps)))
    assert len(fr.recs) == 10
    assert fr.apply(copy.deepcopy(hyps[0])) is None
    assert fr.apply(copy.deepcopy(hyps[-1])) is not None


def test_python_path_equals_the_native_one():
    """A list subclass skips the native check (pyhost.fused_apply): FusedRanks.apply's own
    statements read the same packed row and must give the same ranking, and miss the same edits."""
    from egraph.ranker import FusedRanks

    class Hyps(list):
        pass
    rng = random.Random(11)
    lists = [evidence_fuzz.random_evidence(rng) for _ in range(120)]
    cat, res, hyps = _generated(lists)
    fr = FusedRanks()
    fr.register(cat, res, hyps, range(len(hyps)))
    for h in hyps:
        want = rca_oracle.rank(copy.deepcopy(h))
        got = fr.apply(Hyps(copy.deepcopy(h)))
        assert got is not None and record(got) == record(want)
        assert record(fr.apply(copy.deepcopy(h))) == record(want)
    multi = [h for h in hyps if len(h) >= 2]
    h = Hyps(copy.deepcopy(multi[0]))
    h[-1]["signal_strength"] = 0.123
    assert fr.apply(h) is None
