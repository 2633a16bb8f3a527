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
    # ZERO_COPY_ROWS; grows, then reuses the buffers with a smaller batch; a single incident
    # of <= 1024 rows through the resident rules server (egr_rules_server_*)
    seen = set()
    # (rep: one incident of its first list repeated -- 30x: 129..1024 rows, still the server's;
    # 600x: past its mailbox, zero-copy)
    for n, rep in ((1, 0), (3, 0), (700, 0), (40, 0), (2000, 0), (0, 0), (5, 0), (1, 600),
                   (1, 30), (1, 0)):
        lists = [evidence_fuzz.random_evidence(rng) for _ in range(n)]
        if rep:
            lists = [(lists[0] or [{"id": "x"}]) * rep]
        enc = encode_batch(lists, cat)
        res = runner.run_sync(enc)
        want = ("server" if n == 1 and enc.n_rows <= runner.SERVER_ROWS else
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
    assert seen == {"server", "zero_copy", "staged"}


def _check_one(res, enc, cat):
    exp = oracle.rules_eval(cat.table, enc.flags, enc.vocab, enc.node, enc.err, enc.seg_off)
    np.testing.assert_array_equal(res.mask, exp["mask"])
    np.testing.assert_array_equal(res.n_hyp, exp["n_hyp"])
    np.testing.assert_array_equal(res.order_rank, exp["order_rank"])
    np.testing.assert_array_equal(res.order_conf, exp["order_conf"])
    assert res.final_score.tobytes() == exp["final_score"].tobytes()
    assert res.confidence.tobytes() == exp["confidence"].tobytes()
    assert res.strength.tobytes() == exp["strength"].tobytes()


def test_rules_server_sequence_idle_exit_and_small_kernel(golden):
    """The resident rules server (egr_rules_server_*): every golden case posted one after
    another through the same mailbox -- each result equals the C oracle and the one-launch
    small kernel's, so no request reads a previous one's rows or outputs; the server wave leaves
    after ~2 ms idle and the next call starts it again; a pending post is refused."""
    import time
    from egraph import catalog
    from egraph.batcher import RulesRunner
    from egraph.encode import encode_batch
    from egraph import _lib as L
    cat = catalog.default()
    srv, small = RulesRunner(cat), RulesRunner(cat)
    small.USE_SERVER = False
    cases = golden["rules"]["cases"]
    n_small = 0
    for i, case in enumerate(cases):
        enc = encode_batch([case["evidence"]], cat)
        if enc.n_rows > RulesRunner.SMALL_ROWS:
            continue
        a = srv.run_sync(enc)
        assert srv.mode == "server"
        _check_one(a, enc, cat)
        if i % 7 == 0:
            b = small.run_sync(enc)
            assert small.mode == "small"
            for x, y in zip(a.__dict__.values(), b.__dict__.values()):
                assert x.tobytes() == y.tobytes()
            n_small += 1
        if i in (100, 500):
            time.sleep(0.05)                   # idle past the wave's ~2 ms: it leaves, and
            e0 = encode_batch([[]], cat)       # the next post starts it again
            _check_one(srv.run_sync(e0), e0, cat)
            h = srv._srv                       # one incident in flight: a second post is refused
            assert L.lib.egr_rules_server_post(h, None, None, None, None, 0) == L.EGR_OK
            # (unless the wave has already answered the first: a PCIe round trip or two)
            assert L.lib.egr_rules_server_post(h, None, None, None, None, 0) in (L.EGR_ESTATE, L.EGR_OK)
            srv._srv_wait.arm().synchronize()
    assert n_small > 100


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


def test_coalesced_batch_calls_of_mixed_sizes(golden):
    """Batch calls coalesced into one launch -- an empty one, two-incident ones, single
    incidents -- each get their own lists: the one-incident-per-call delivery is taken only when
    every call holds one incident (an empty call beside a two-incident call also sums to one
    incident per call)."""
    import rca_oracle
    from src.services.rca import rules_engine as RE
    eng = RE.RulesEngine()
    cases = golden["rules"]["cases"][:9]

    def strip(hs):
        return [{k: v for k, v in h.items() if k != "id"} for h in hs]

    async def go():
        b = RE._batcher(eng.catalog, eng.device)
        first = asyncio.ensure_future(eng.generate_hypotheses(_Inc("a"), cases[0]["evidence"]))
        await asyncio.sleep(0)            # `first` has launched: the next calls coalesce
        assert b.busy
        calls = [eng.generate_hypotheses_batch([], []),
                 eng.generate_hypotheses_batch([_Inc("a")] * 2, [cases[1]["evidence"], cases[2]["evidence"]]),
                 eng.generate_hypotheses(_Inc("a"), cases[3]["evidence"]),
                 eng.generate_hypotheses_batch([], []),
                 eng.generate_hypotheses_batch([_Inc("a")] * 2, [cases[4]["evidence"], cases[5]["evidence"]]),
                 eng.generate_hypotheses_batch([_Inc("a")], [cases[6]["evidence"]])]
        return await first, await asyncio.gather(*calls)

    first, (e0, two1, one, e1, two2, one1) = asyncio.run(go())
    exp = [rca_oracle.generate("a", c["evidence"]) for c in cases]
    assert strip(first) == exp[0]
    assert e0 == [] and e1 == []
    assert [strip(x) for x in two1] == exp[1:3]
    assert strip(one) == exp[3]
    assert [strip(x) for x in two2] == exp[4:6]
    assert len(one1) == 1 and strip(one1[0]) == exp[6]


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
