"""The three workflow activities on the hot path (reference
src/services/workflow/activities.py:94-170), same names, argument shapes and results, plus
additive batch / root-cause activities.

They stay drop-in sockets for IncidentWorkflow (incident_workflow.py:96-139): JSON-shaped
dicts in and out.  When temporalio is installed they are registered with @activity.defn,
otherwise they are plain coroutines.  The optional LLM enhancement of generate_hypotheses
(:141-151) is not rebuilt (network-bound), but its step is kept: when the deployment provides
the reference's `src.config.settings` and `src.services.rca.llm_summarizer` (the reference's
own `src` package beside this one) and `settings.llm_provider` is set, the rules' hypotheses go through
`LLMSummarizer.enhance_hypotheses` with the reference's fallback to rules-only on any error.
"""
from __future__ import annotations

import logging

from egraph_dropin.graph_service import GraphService
from egraph_dropin.hypothesis_ranker import HypothesisRanker
from egraph_dropin.models import GraphEntity, GraphRelation, Incident
from egraph_dropin.rules_engine import RulesEngine

try:  # pragma: no cover - temporalio is not part of this image
    from temporalio import activity as _activity

    _defn = _activity.defn
except ImportError:  # plain coroutines
    def _defn(fn):
        return fn

logger = logging.getLogger(__name__)


@_defn
async def build_evidence_graph(data: dict) -> dict:
    """Merge the collected entities / relations into the evidence graph (:94-121)."""
    evidence_data = data["evidence"]
    entities = [GraphEntity(**e) for e in evidence_data.get("entities", [])]
    relations = [GraphRelation(**r) for r in evidence_data.get("relations", [])]
    node_count = await GraphService.create_entities_batch(entities)
    edge_count = await GraphService.create_relations_batch(relations)
    logger.info("evidence graph built: incident=%s nodes=%d edges=%d",
                data["incident"].get("id"), node_count, edge_count)
    return {"node_count": node_count, "edge_count": edge_count}


_REFERENCE_LLM = None   # (settings, LLMSummarizer) of the deployed reference, or False: resolved once


def _reference_llm():
    """The reference's settings module and LLMSummarizer class, imported on first use only (a
    failed import is not cached by Python: probing it on every activity call would walk the
    finders each time)."""
    global _REFERENCE_LLM
    if _REFERENCE_LLM is None:
        try:
            from src.config import settings  # the reference's settings module, when deployed with it
            from src.services.rca.llm_summarizer import LLMSummarizer
            _REFERENCE_LLM = (settings, LLMSummarizer)
        except ImportError:
            _REFERENCE_LLM = False
    return _REFERENCE_LLM


def _llm_enhancer():
    """The reference's LLM step (activities.py:142-151) when the deployment has it configured:
    an `async (hypotheses, evidence) -> hypotheses` callable, or None.  HYPOTHESIS_ENHANCER, if
    set, takes precedence (tests, or a deployment wiring its own summarizer); `llm_provider` is
    read on every call, as the reference does (:143)."""
    if HYPOTHESIS_ENHANCER is not None:
        return HYPOTHESIS_ENHANCER
    ref = _reference_llm()
    if not ref or not getattr(ref[0], "llm_provider", None):
        return None
    summarizer = ref[1]

    async def enhance(hypotheses, evidence):
        return await summarizer().enhance_hypotheses(hypotheses=hypotheses, evidence=evidence)
    return enhance


HYPOTHESIS_ENHANCER = None


@_defn
async def generate_hypotheses(data: dict) -> list[dict]:
    """Rules-engine hypotheses for one incident (:124-159), then the optional LLM enhancement
    (:142-151): skipped without hypotheses, rules-only on any error."""
    incident = Incident(**data["incident"])
    evidence = data["evidence"].get("evidence", [])
    hypotheses = await RulesEngine().generate_hypotheses(incident=incident, evidence=evidence)
    enhance = _llm_enhancer() if hypotheses else None
    if enhance is not None:
        try:
            hypotheses = await enhance(hypotheses, evidence)
        except Exception as e:  # noqa: BLE001 -- the reference's fallback (:150-151)
            logger.warning("LLM enhancement failed, using rules-only: %s", e)
    return hypotheses


@_defn
async def rank_hypotheses(hypotheses: list[dict]) -> list[dict]:
    """Rank hypotheses (:162-170)."""
    return HypothesisRanker().rank(hypotheses)


@_defn
async def generate_and_rank_batch(data: list[dict]) -> list[list[dict]]:
    """Additive: generate + rank for many incidents in one GPU launch."""
    incidents = [Incident(**d["incident"]) for d in data]
    evidence = [d["evidence"].get("evidence", []) for d in data]
    return await RulesEngine().rank_incidents_batch(incidents, evidence)


@_defn
async def rank_root_causes(data: dict) -> list[dict]:
    """Additive (build-defined): the incident's top-k root-cause graph entities
    by 3-hop evidence propagation, same input dict as generate_hypotheses (+ optional "k")."""
    inc = data["incident"]
    ev = data["evidence"].get("evidence", [])
    out = await GraphService.rank_root_causes([str(inc["id"])], [ev], k=int(data.get("k", 10)))
    return out[0]


@_defn
async def rank_root_causes_batch(data: list[dict]) -> list[list[dict]]:
    """Additive: rank_root_causes for many incidents in one frontier launch."""
    ids = [str(d["incident"]["id"]) for d in data]
    ev = [d["evidence"].get("evidence", []) for d in data]
    k = int(data[0].get("k", 10)) if data else 10
    return await GraphService.rank_root_causes(ids, ev, k=k)
