"""The drop-in binding of INTEGRATION.md §1, applied from inside a reference-shaped tree.

The reference's callers import through its own regular package `src`
(src/services/workflow/activities.py:11-13, :100, :130-131, :165; worker.py:12-26;
ingestion/main.py:15-23).  This test writes a stand-in of that tree -- the same module paths,
the reference's import lines and call sites, CPU stand-in classes where the reference has its
Neo4j / Python services -- applies INTEGRATION.md's patch block VERBATIM, and imports the
reference-shaped `src` FIRST in a fresh interpreter with this package at the end of the path (as
INTEGRATION.md installs it).  Then:
  * activities.GraphService and the RulesEngine / HypothesisRanker the activities import at
    their call sites are egraph_dropin's GPU classes (the activities are run; the GPU calls are
    recorded, not launched -- there is no GPU here);
  * build_evidence_graph writes the reference's models into egraph_dropin.GraphService's host
    graph (no GPU needed for MERGE);
  * the worker registers the additive activities; the ingestion service resolves GraphService,
    Neo4jConnection, AlertDeduplicator and AlertNormalizer to egraph_dropin and its startup's
    init_constraints() runs;
  * every module the patch does not touch is still the reference's own (src.services.rca.*).
The patch also applies to the real reference files when /root/reference is present (this
container; the GPU box has no copy)."""
from __future__ import annotations

import os
import re
import subprocess
import sys
import textwrap
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
PKG = REPO / "kubernetes-aiops-evidence-graph_amd"
REF = Path("/root/reference")

# the stand-in reference tree: module paths, import lines and call sites of the reference
STANDIN = {
    "src/__init__.py": "",
    "src/config/__init__.py": "from src.config.settings import settings\n",
    "src/config/settings.py": textwrap.dedent("""\
        class Settings:
            llm_provider = None
        settings = Settings()
        """),
    "src/models/__init__.py": textwrap.dedent("""\
        class _Model:
            def __init__(self, **kw):
                self.__dict__.update(kw)
        class Incident(_Model): pass
        class IncidentCreate(_Model): pass
        class GraphEntity(_Model): pass
        class GraphRelation(_Model): pass
        """),
    "src/database/__init__.py": textwrap.dedent("""\
        from src.database.neo4j import GraphService, Neo4jConnection, get_neo4j_session
        from src.database.postgres import (check_database_connection, close_database, get_session,
                                           init_database)
        """),
    "src/database/neo4j.py": textwrap.dedent("""\
        REFERENCE = True
        class Neo4jConnection:
            REFERENCE = True
        class GraphService:
            REFERENCE = True
        def get_neo4j_session():
            raise RuntimeError("no Neo4j here")
        """),
    "src/database/postgres.py": textwrap.dedent("""\
        async def check_database_connection(): return True
        async def close_database(): return None
        async def init_database(): return None
        def get_session(): raise RuntimeError("no Postgres here")
        """),
    "src/services/__init__.py": "",
    "src/services/rca/__init__.py": textwrap.dedent("""\
        from src.services.rca.hypothesis_ranker import HypothesisRanker
        from src.services.rca.llm_summarizer import LLMSummarizer
        from src.services.rca.rules_engine import RulesEngine
        """),
    "src/services/rca/rules_engine.py": "class RulesEngine:\n    REFERENCE = True\n",
    "src/services/rca/hypothesis_ranker.py": "class HypothesisRanker:\n    REFERENCE = True\n",
    "src/services/rca/llm_summarizer.py": "class LLMSummarizer:\n    REFERENCE = True\n",
    "src/services/ingestion/__init__.py": textwrap.dedent("""\
        from src.services.ingestion.deduplicator import AlertDeduplicator, RateLimiter
        from src.services.ingestion.normalizer import AlertNormalizer
        """),
    "src/services/ingestion/deduplicator.py": textwrap.dedent("""\
        class AlertDeduplicator:
            REFERENCE = True
        class RateLimiter:
            REFERENCE = True
        """),
    "src/services/ingestion/normalizer.py": "class AlertNormalizer:\n    REFERENCE = True\n",
    # ingestion/main.py:15-23 import lines and the lifespan's startup call (:55)
    "src/services/ingestion/main.py": textwrap.dedent("""\
        from src.config import settings
        from src.database import check_database_connection, close_database, init_database
        from src.database.neo4j import GraphService, Neo4jConnection
        from src.models import (
            Incident,
            IncidentCreate,
        )
        from src.services.ingestion.deduplicator import AlertDeduplicator
        from src.services.ingestion.normalizer import AlertNormalizer


        async def startup():
            await init_database()
            await GraphService.init_constraints()
        """),
    "src/services/workflow/__init__.py": "",
    "src/services/workflow/incident_workflow.py": "class IncidentWorkflow:\n    pass\n",
    # activities.py: the module imports (:11-13) and the three hot-path activities (:94-170)
    "src/services/workflow/activities.py": textwrap.dedent("""\
        from src.config import settings
        from src.database import GraphService, get_session
        from src.models import Incident


        async def build_evidence_graph(data: dict) -> dict:
            incident_data = data["incident"]
            evidence_data = data["evidence"]

            from src.models import GraphEntity, GraphRelation

            entities = [GraphEntity(**e) for e in evidence_data.get("entities", [])]
            relations = [GraphRelation(**r) for r in evidence_data.get("relations", [])]
            entity_count = await GraphService.create_entities_batch(entities)
            relation_count = await GraphService.create_relations_batch(relations)
            return {"node_count": entity_count, "edge_count": relation_count}


        async def generate_hypotheses(data: dict) -> list[dict]:
            incident_data = data["incident"]
            evidence_data = data["evidence"]

            from src.services.rca.llm_summarizer import LLMSummarizer
            from src.services.rca.rules_engine import RulesEngine

            incident = Incident(**incident_data)
            rules_engine = RulesEngine()
            hypotheses = await rules_engine.generate_hypotheses(
                incident=incident,
                evidence=evidence_data.get("evidence", []),
            )
            if settings.llm_provider and hypotheses:
                hypotheses = await LLMSummarizer().enhance_hypotheses(hypotheses=hypotheses,
                                                                      evidence=[])
            return hypotheses


        async def rank_hypotheses(hypotheses: list[dict]) -> list[dict]:
            from src.services.rca.hypothesis_ranker import HypothesisRanker

            ranker = HypothesisRanker()
            ranked = ranker.rank(hypotheses)

            return ranked
        """),
    # worker.py:12-26 imports and the activity list of Worker(...) (:46-59)
    "src/services/workflow/worker.py": (
        "from src.services.workflow.activities import (\n"
        "    build_evidence_graph,\n"
        "    generate_hypotheses,\n"
        "    rank_hypotheses,\n"
        ")\n"
        "from src.services.workflow.incident_workflow import IncidentWorkflow\n"
        "\n"
        "def create_ticket(): pass\n"
        "def close_incident(): pass\n"
        "def Worker(client, **kw): return kw\n"
        "\n"
        "def make_worker(client):\n"
        "    worker = Worker(\n"
        "        client,\n"
        "        workflows=[IncidentWorkflow],\n"
        "        activities=[\n"
        "            build_evidence_graph,\n"
        "            generate_hypotheses,\n"
        "            rank_hypotheses,\n"
        "            create_ticket,\n"
        "            close_incident,\n"
        "        ],\n"
        "    )\n"
        "    return worker\n"
        "\n"
        "ACTIVITIES = make_worker(None)['activities']\n"),
}


def parse_patch(md: str) -> dict[str, list[tuple[str, str]]]:
    """INTEGRATION.md's binding patch -> {path: [(old text, new text), ...]} per hunk: context
    (' ') and removed ('-') lines make the old text, context and added ('+') lines the new."""
    m = re.search(r"<!-- dropin-binding-patch[^>]*-->\s*```diff\n(.*?)```", md, re.S)
    assert m, "INTEGRATION.md has no dropin-binding-patch block"
    out: dict[str, list] = {}
    path, old, new = None, None, None

    def flush():
        if path is not None and old is not None:
            out.setdefault(path, []).append(("".join(old), "".join(new)))
    for line in m.group(1).splitlines(keepends=True):
        if line.startswith("--- a/"):
            flush()
            path, old, new = line[6:].strip(), None, None
        elif line.startswith("+++ "):
            continue
        elif line.startswith("@@"):
            flush()
            old, new = [], []
        elif line[:1] == " ":
            old.append(line[1:])
            new.append(line[1:])
        elif line[:1] == "-":
            old.append(line[1:])
        elif line[:1] == "+":
            new.append(line[1:])
    flush()
    return out


def apply_patch(root: Path, patch: dict) -> None:
    for path, hunks in patch.items():
        f = root / path
        text = f.read_text()
        for old, new in hunks:
            assert text.count(old) == 1, f"{path}: hunk does not apply exactly once:\n{old}"
            text = text.replace(old, new)
        f.write_text(text)


PATCH = parse_patch((REPO / "INTEGRATION.md").read_text())

CHECK = textwrap.dedent("""\
    import asyncio, sys
    root = sys.argv[1]
    import src                                    # the reference's own package, first
    assert src.__file__.startswith(root), src.__file__
    import src.services.workflow.worker as worker
    import src.services.workflow.activities as acts
    import src.services.ingestion.main as ingest
    import egraph_dropin
    from egraph_dropin import activities as gpu_acts
    assert acts.__file__.startswith(root)
    assert acts.GraphService is egraph_dropin.GraphService
    # every module the patch does not touch is still the reference's
    import src.services.rca.rules_engine as ref_rules, src.database as ref_db
    assert ref_rules.RulesEngine.REFERENCE and ref_db.GraphService.REFERENCE
    import src.services.rca as ref_rca
    assert ref_rca.HypothesisRanker.REFERENCE
    # the activities' call sites reach the GPU classes (recorded, not launched: no GPU here)
    seen = []
    async def gen(self, incident, evidence):
        seen.append((type(self), incident.id, len(evidence)))
        return [{"id": "h1", "confidence": 0.9}]
    def rank(self, hyps):
        seen.append((type(self), len(hyps)))
        return hyps
    egraph_dropin.RulesEngine.generate_hypotheses = gen
    egraph_dropin.HypothesisRanker.rank = rank
    data = {"incident": {"id": "inc-1"}, "evidence": {
        "evidence": [{"id": "e1"}],
        "entities": [{"id": "incident:inc-1", "type": "Incident", "properties": {}},
                     {"id": "pod:ns:a", "type": "Pod", "properties": {"name": "a"}}],
        "relations": [{"source_id": "incident:inc-1", "target_id": "pod:ns:a",
                       "relation_type": "AFFECTS", "properties": {}},
                      {"source_id": "incident:inc-1", "target_id": "pod:ns:missing",
                       "relation_type": "AFFECTS", "properties": {}}]}}
    hyps = asyncio.run(acts.generate_hypotheses(data))
    ranked = asyncio.run(acts.rank_hypotheses(hyps))
    assert seen == [(egraph_dropin.RulesEngine, "inc-1", 1), (egraph_dropin.HypothesisRanker, 1)], seen
    assert ranked == [{"id": "h1", "confidence": 0.9}]
    # build_evidence_graph: the reference's own models into the GPU service's host graph
    out = asyncio.run(acts.build_evidence_graph(data))
    assert out == {"node_count": 2, "edge_count": 2}, out        # attempted counts (neo4j.py:112, :166)
    g = egraph_dropin.GraphService.graph()
    assert g.num_vertices == 2 and g.num_edges == 1              # dangling AFFECTS dropped
    # the worker registers the additive activities next to the reference's
    names = [f.__name__ for f in worker.ACTIVITIES]
    assert names[:5] == ["build_evidence_graph", "generate_hypotheses", "rank_hypotheses",
                         "create_ticket", "close_incident"]
    assert worker.ACTIVITIES[5:] == [gpu_acts.generate_and_rank_batch, gpu_acts.rank_root_causes,
                                     gpu_acts.rank_root_causes_batch]
    # the ingestion service
    assert ingest.GraphService is egraph_dropin.GraphService
    assert ingest.Neo4jConnection is egraph_dropin.Neo4jConnection
    assert ingest.AlertDeduplicator is egraph_dropin.AlertDeduplicator
    assert ingest.AlertNormalizer is egraph_dropin.AlertNormalizer
    asyncio.run(ingest.startup())
    asyncio.run(ingest.Neo4jConnection.close())
    # nothing of this repository's src mirror was loaded
    assert all(not getattr(m, "__file__", None) or m.__file__.startswith(root) or "egraph" in m.__file__
               for n, m in sys.modules.items() if n == "src" or n.startswith("src.")), \\
        [m.__file__ for n, m in sys.modules.items() if n.startswith("src")]
    print("BINDING-OK")
    """)


def _write_standin(root: Path) -> None:
    for path, text in STANDIN.items():
        f = root / path
        f.parent.mkdir(parents=True, exist_ok=True)
        f.write_text(text)


def test_patch_block_parses():
    assert set(PATCH) == {"src/services/workflow/activities.py", "src/services/workflow/worker.py",
                          "src/services/ingestion/main.py"}
    assert len(PATCH["src/services/workflow/activities.py"]) == 3


def test_binding_resolves_gpu_classes_inside_reference_tree(tmp_path):
    _write_standin(tmp_path)
    apply_patch(tmp_path, PATCH)
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1",
               # the package directory at the END of the module path
               PYTHONPATH=os.pathsep.join(filter(None, [os.environ.get("PYTHONPATH", ""), str(PKG)])))
    r = subprocess.run([sys.executable, "-c", CHECK, str(tmp_path)], cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "BINDING-OK" in r.stdout, r.stdout + r.stderr


def test_unpatched_tree_keeps_reference_classes(tmp_path):
    """Control: without the patch the same tree resolves to the reference's classes, i.e. the
    package on the path alone cannot redirect `src.*` (what the patch is for)."""
    _write_standin(tmp_path)
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", PYTHONPATH=str(PKG))
    code = ("import src.services.workflow.activities as a, src.database.neo4j as n;"
            "assert a.GraphService is n.GraphService and n.GraphService.REFERENCE; print('REF-OK')")
    r = subprocess.run([sys.executable, "-c", code], cwd=tmp_path, env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0 and "REF-OK" in r.stdout, r.stdout + r.stderr


@pytest.mark.skipif(not REF.is_dir(), reason="the reference checkout is only in the build container")
def test_patch_applies_to_the_real_reference_files(tmp_path):
    """Every hunk applies exactly once to the reference's own files (read as text, patched in a
    scratch copy; nothing is imported or run)."""
    for path in PATCH:
        dst = tmp_path / path
        dst.parent.mkdir(parents=True, exist_ok=True)
        dst.write_text((REF / path).read_text())
    apply_patch(tmp_path, PATCH)
    text = (tmp_path / "src/services/workflow/activities.py").read_text()
    assert "from egraph_dropin import RulesEngine" in text
    assert "from src.services.rca.rules_engine import RulesEngine" not in text
