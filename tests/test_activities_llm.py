"""generate_hypotheses keeps the reference's optional LLM step (reference
src/services/workflow/activities.py:142-151): enhancement runs only with hypotheses present,
and any error falls back to the rules-only list.  Host logic only: the rules engine is stubbed
(its GPU parity is tests/test_rules_gpu.py)."""
from __future__ import annotations

import asyncio
import uuid

import pytest


def _data():
    return {"incident": {"id": str(uuid.uuid4()), "fingerprint": "f", "title": "t",
                         "severity": "high", "source": "alertmanager", "cluster": "c",
                         "namespace": "default", "started_at": "2026-01-01T00:00:00Z"},
            "evidence": {"evidence": [{"kind": "log"}]}}


@pytest.fixture
def acts(monkeypatch):
    from src.services.workflow import activities

    produced = {"hyps": [{"title": "OOM", "confidence": 0.9}]}

    class _Rules:
        async def generate_hypotheses(self, incident, evidence):
            return [dict(h) for h in produced["hyps"]]

    monkeypatch.setattr(activities, "RulesEngine", _Rules)
    monkeypatch.setattr(activities, "HYPOTHESIS_ENHANCER", None)
    return activities, produced


def test_no_enhancer_configured_is_rules_only(acts):
    act, _ = acts
    assert act._llm_enhancer() is None       # no reference settings module in this package
    out = asyncio.run(act.generate_hypotheses(_data()))
    assert out == [{"title": "OOM", "confidence": 0.9}]


def test_enhancer_applied(acts, monkeypatch):
    act, _ = acts
    seen = []

    async def enhance(hyps, evidence):
        seen.append(evidence)
        return [dict(h, summary="llm") for h in hyps]

    monkeypatch.setattr(act, "HYPOTHESIS_ENHANCER", enhance)
    out = asyncio.run(act.generate_hypotheses(_data()))
    assert out == [{"title": "OOM", "confidence": 0.9, "summary": "llm"}]
    assert seen == [[{"kind": "log"}]]


def test_enhancer_error_falls_back(acts, monkeypatch):
    act, _ = acts

    async def boom(hyps, evidence):
        raise RuntimeError("provider down")

    monkeypatch.setattr(act, "HYPOTHESIS_ENHANCER", boom)
    out = asyncio.run(act.generate_hypotheses(_data()))
    assert out == [{"title": "OOM", "confidence": 0.9}]


def test_enhancer_skipped_without_hypotheses(acts, monkeypatch):
    act, produced = acts
    produced["hyps"] = []
    called = []

    async def enhance(hyps, evidence):
        called.append(1)
        return hyps

    monkeypatch.setattr(act, "HYPOTHESIS_ENHANCER", enhance)
    assert asyncio.run(act.generate_hypotheses(_data())) == []
    assert called == []
