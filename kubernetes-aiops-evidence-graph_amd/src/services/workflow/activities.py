"""The three workflow activities on the hot path (reference
src/services/workflow/activities.py:94-170), same names, argument shapes and results, plus
additive batch / root-cause activities.

They stay drop-in sockets for IncidentWorkflow (incident_workflow.py:96-139): JSON-shaped
dicts in and out.  When temporalio is installed they are registered with @activity.defn,
otherwise they are plain coroutines.  The optional LLM enhancement of generate_hypotheses
(:141-151) is out of scope (network-bound; a no-op without an API key in the reference).
"""
from __future__ import annotations

import logging

from src.database import GraphService
from src.models import GraphEntity, GraphRelation, Incident
from src.services.rca.hypothesis_ranker import HypothesisRanker
from src.services.rca.rules_engine import RulesEngine

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


@_defn
async def generate_hypotheses(data: dict) -> list[dict]:
    """Rules-engine hypotheses for one incident (:124-159)."""
    incident = Incident(**data["incident"])
    return await RulesEngine().generate_hypotheses(
        incident=incident, evidence=data["evidence"].get("evidence", []))


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
