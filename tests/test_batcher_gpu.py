"""The drop-in rules path under concurrency (egraph/batcher.py): concurrent RulesEngine calls
coalesce into fewer launches and every call still gets exactly the reference's dicts; a call
whose evidence makes the reference raise raises alone; RulesRunner's packed launch equals the
C oracle bit for bit."""
from __future__ import annotations

import asyncio
import random

import numpy as np
import pytest

import oracle
from helpers import golden_record, record

pytestmark = pytest.mark.gpu


class _Inc:
    def __init__(self, iid):
        self.id = iid


def test_runner_matches_oracle():
    import evidence_fuzz
    from egraph import catalog
    from egraph.batcher import RulesRunner
    from egraph.encode import encode_batch
    rng = random.Random(17)
    cat = catalog.default()
    runner = RulesRunner(cat)
    # zero-copy (mapped host memory) for small batches, the staged device buffer above
    # ZERO_COPY_ROWS; grows, then reuses the buffers with a smaller batch
    # and a single incident of <= 128 rows in the kernel arguments (egr_rules_eval_small)
    seen = set()
    for n, big in ((1, False), (3, False), (700, False), (40, False), (2000, False), (0, False),
                   (5, False), (1, True), (1, False)):
        lists = [evidence_fuzz.random_evidence(rng) for _ in range(n)]
        if big:
            lists = [(lists[0] or [{"id": "x"}]) * 200]   # one incident of > 128 rows
        enc = encode_batch(lists, cat)
        res = runner.run_sync(enc)
        want = ("small" if n == 1 and enc.n_rows <= runner.SMALL_ROWS else
                "zero_copy" if enc.n_rows <= runner.ZERO_COPY_ROWS else "staged")
        assert runner.mode == want
        seen.add(want)
        exp = oracle.rules_eval(cat.table, enc.flags, enc.vocab, enc.node, enc.err, enc.seg_off)
        np.testing.assert_array_equal(res.mask, exp["mask"])
        np.testing.assert_array_equal(res.order_rank, exp["order_rank"])
        np.testing.assert_array_equal(res.order_conf, exp["order_conf"])
        assert res.final_score.tobytes() == exp["final_score"].tobytes()
        assert res.confidence.tobytes() == exp["confidence"].tobytes()
        assert res.strength.tobytes() == exp["strength"].tobytes()
    assert seen == {"small", "zero_copy", "staged"}


def test_concurrent_calls_coalesce_and_match_golden(golden):
    """All golden cases as concurrent single calls (half generate -> rank, half the fused
    batch API with one incident): fewer launches than calls, every result as recorded from
    the reference."""
    from src.services.rca.hypothesis_ranker import HypothesisRanker
    from src.services.rca import rules_engine as RE
    eng = RE.RulesEngine()
    cases = golden["rules"]["cases"]
    inc = _Inc(golden["rules"]["incident_id"])
    rk = HypothesisRanker()

    async def one(i, case):
        if i % 2:
            return rk.rank(await eng.generate_hypotheses(inc, case["evidence"]))
        return (await eng.rank_incidents_batch([inc], [case["evidence"]]))[0]

    from egraph.ranker import FUSED
    h0 = FUSED.hits

    async def go():
        b = RE._batcher(eng.catalog, eng.device)          # (one batcher per event loop)
        return b, await asyncio.gather(*[one(i, c) for i, c in enumerate(cases)])

    b, out = asyncio.run(go())
    l0, c0 = 0, 0
    assert b.calls - c0 == len(cases)
    assert b.launches - l0 < len(cases) // 4            # coalesced
    assert FUSED.hits - h0 == len(cases) // 2           # rank() reused the kernel's ranking
    for case, hyps in zip(cases, out):
        assert record(hyps) == golden_record(case["expected"]), case["name"]


def test_error_raises_in_its_own_call_only(golden):
    from src.services.rca import rules_engine as RE
    eng = RE.RulesEngine()
    good = golden["rules"]["cases"][:20]
    bad = [c for c in golden["errors"] if c["raises"] is not None]

    async def go():
        calls = [eng.generate_hypotheses(_Inc("g"), c["evidence"]) for c in good]
        calls += [eng.generate_hypotheses(_Inc("b"), c["evidence"]) for c in bad]
        return await asyncio.gather(*calls, return_exceptions=True)

    out = asyncio.run(go())
    import rca_oracle
    for c, r in zip(good, out[:len(good)]):
        assert not isinstance(r, BaseException)
        strip = [{k: v for k, v in h.items() if k != "id"} for h in r]
        assert strip == rca_oracle.generate("g", c["evidence"])
    for c, r in zip(bad, out[len(good):]):
        assert isinstance(r, BaseException) and type(r).__name__ == c["raises"], c["name"]


def test_cancelled_launcher_leaves_the_batch_intact(golden):
    """The call that launched a batch is cancelled (an activity timeout) while its kernel runs:
    the calls coalesced behind it still get the reference's dicts, and the next launch, which
    reuses the same buffers, is correct too."""
    import rca_oracle
    from src.services.rca import rules_engine as RE
    eng = RE.RulesEngine()
    cases = golden["rules"]["cases"][:48]

    def strip(hs):
        return [{k: v for k, v in h.items() if k != "id"} for h in hs]

    async def go():
        first = asyncio.ensure_future(eng.generate_hypotheses(_Inc("c"), cases[0]["evidence"]))
        rest = [asyncio.ensure_future(eng.generate_hypotheses(_Inc("c"), c["evidence"]))
                for c in cases[1:]]
        await asyncio.sleep(0)            # `first` has launched and yields while its kernel runs
        first.cancel()
        got = await asyncio.gather(*rest)
        after = await eng.rank_incidents_batch([_Inc("c")] * 8, [c["evidence"] for c in cases[:8]])
        try:
            await first
        except asyncio.CancelledError:
            pass
        return first, got, after

    first, got, after = asyncio.run(go())
    assert first.cancelled()
    for c, r in zip(cases[1:], got):
        assert strip(r) == rca_oracle.generate("c", c["evidence"]), c["name"]
    for c, r in zip(cases[:8], after):
        assert strip(r) == strip(rca_oracle.rca("c", c["evidence"])), c["name"]


def test_batchers_follow_catalog_and_loop():
    """A batcher belongs to one catalog object and one event loop: a new loop gets a fresh,
    idle batcher, and a catalog's batcher is never handed to another catalog."""
    from egraph import catalog
    from src.services.rca import rules_engine as RE

    async def get(cat):
        return RE._batcher(cat, None)

    c1 = catalog.default()
    b1 = asyncio.run(get(c1))
    b2 = asyncio.run(get(c1))
    assert b1 is not b2 and not b2.busy

    async def same_loop():
        return RE._batcher(c1, None) is RE._batcher(c1, None)
    assert asyncio.run(same_loop())
    c2 = catalog.Catalog(**{f: getattr(c1, f) for f in c1.__dataclass_fields__})
    assert asyncio.run(get(c2)).cat is c2
