"""Drop-in RulesEngine (reference src/services/rca/rules_engine.py:193-478) running on the GPU.

Same public surface: `RulesEngine().generate_hypotheses(incident, evidence)` is a coroutine
function (tests/unit/test_async_contracts.py:18-19 of the reference) returning the same dicts
in the same order (confidence descending, rank 0; the single "unknown" hypothesis when nothing
matches).  Additive batch entry points put many incidents into one kernel launch:
`generate_hypotheses_batch` (unranked, = N x generate_hypotheses) and `rank_incidents_batch`
(generate + HypothesisRanker.rank fused, as the workflow runs them back to back).

All signal extraction, rule matching, confidence, ranking and ordering run in
egr_rules_eval (csrc/rules.hip), launched by egraph/batcher.py's RulesRunner (the same
entry point is registered as torch.ops.egraph.rules_eval, egraph/ops.py); the host encodes
rows and assembles dicts in native code
(csrc/pyhost.c: encode_rows, assemble).  There is no CPU
fallback: without a ROCm GPU the call raises RuntimeError.
"""
from __future__ import annotations

import asyncio
import weakref

from egraph import catalog as _catalog
from egraph.batcher import RulesBatcher
from egraph_dropin.models import HypothesisCategory

# The reference's rule table, with categories as enums as in rules_engine.py:15-190.
DIAGNOSIS_RULES = [
    {**{k: v for k, v in r.items() if k != "category"},
     "category": HypothesisCategory(r["category"])}
    for r in _catalog.default().rules
]


# id(catalog) -> (weak ref to the catalog, {event loop (weak) -> {device: batcher}}).  A batcher
# lives as long as its catalog and its loop: a new catalog that reuses a dead one's id() gets a
# batcher of its own (never the old rule table), and a loop that closed mid-launch (asyncio.run
# in tests, a worker restart) leaves no busy batcher behind for the next loop to wait on.
_BATCHERS: dict = {}


# The last hit, as ONE immutable tuple (weak catalog, weak loop, device, weak batcher) that a
# caller reads once: several threads, each with its own event loop, may call concurrently, and a
# tuple read once cannot mix one thread's loop with another's batcher.  The batcher is held
# weakly (it is owned by _BATCHERS), so the cache keeps no catalog alive.
_LAST: tuple | None = None


def _batcher(catalog: _catalog.Catalog, device) -> RulesBatcher:
    """The batcher of a (catalog, running event loop, device): concurrent activities of one
    worker loop share it, so calls that overlap in time go out in one launch."""
    global _LAST
    loop = asyncio.get_running_loop()
    last = _LAST
    if last is not None and last[0]() is catalog and last[1]() is loop and last[2] == device:
        b = last[3]()
        if b is not None:
            return b                   # (one call per incident: the common case is a repeat)
    b = _batcher_slow(catalog, device, loop)
    _LAST = (weakref.ref(catalog), weakref.ref(loop), device, weakref.ref(b))
    return b


def _batcher_slow(catalog: _catalog.Catalog, device, loop) -> RulesBatcher:
    key = id(catalog)
    ent = _BATCHERS.get(key)
    if ent is None or ent[0]() is not catalog:
        ent = _BATCHERS[key] = (weakref.ref(catalog, lambda _r, k=key: _BATCHERS.pop(k, None)),
                                weakref.WeakKeyDictionary())
    per_dev = ent[1].get(loop)
    if per_dev is None:
        per_dev = ent[1][loop] = {}
    b = per_dev.get(str(device))
    if b is None:
        b = per_dev[str(device)] = RulesBatcher(catalog, device)
    return b


class RulesEngine:
    """Deterministic rules engine; evaluation is batched on the GPU.

    Every call goes through a process-wide RulesBatcher (egraph/batcher.py): an idle engine
    launches a single call at once (one packed upload, one kernel, one packed download, the
    completion polled from the event loop); calls that arrive while a launch is in flight --
    concurrent Temporal activities -- are coalesced into the next launch."""

    def __init__(self, catalog: _catalog.Catalog | None = None, device=None):
        self.catalog = catalog or _catalog.default()
        self.rules = DIAGNOSIS_RULES if catalog is None else [
            {**r, "category": HypothesisCategory(r["category"])} for r in catalog.rules]
        self.device = device
        self._last = None              # (event loop, its batcher): the previous call's, read once

    def _batcher(self) -> RulesBatcher:
        # one call per incident: the common case is the previous call's loop (the engine holds
        # its catalog, so the catalog cannot change under it)
        loop = asyncio.get_running_loop()
        last = self._last
        if last is not None and last[0] is loop:
            return last[1]
        b = _batcher(self.catalog, self.device)
        self._last = (loop, b)
        return b

    async def _run(self, incidents, evidence_lists, ranked: bool) -> list[list[dict]]:
        if len(incidents) != len(evidence_lists):
            raise ValueError("incidents and evidence_lists differ in length")
        return await self._batcher().submit_many(
            [inc.id for inc in incidents], evidence_lists, ranked)

    async def generate_hypotheses(self, incident, evidence: list[dict]) -> list[dict]:
        """Generate hypotheses by matching evidence against rules (rules_engine.py:199-233)."""
        b = self._batcher()
        # (a launch in flight: the call joins the next one through its future directly)
        return await (b.queued(incident.id, evidence, False) if b.busy
                      else b.submit(incident.id, evidence, False))

    async def generate_hypotheses_batch(self, incidents: list, evidence_lists: list[list[dict]]
                                        ) -> list[list[dict]]:
        """generate_hypotheses for many incidents in one launch."""
        return await self._run(list(incidents), list(evidence_lists), ranked=False)

    async def rank_incidents_batch(self, incidents: list, evidence_lists: list[list[dict]]
                                   ) -> list[list[dict]]:
        """generate_hypotheses followed by HypothesisRanker.rank, fused in one launch."""
        return await self._run(list(incidents), list(evidence_lists), ranked=True)
