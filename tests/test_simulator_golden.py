"""The reference simulator's scenarios (src/simulator/incident_simulator.py: crashloop, oom,
imagepull, slowapp) and BASELINE config C1, rendered by the collector-shaped generator
(egraph/synth.py) and judged by the REFERENCE (tests/golden/simulator_cases.json, recorded by
oracle/gen_golden_simulator.py): the oracle restatement reproduces every recorded ranking, the
generator reproduces every recorded evidence list, and the generator's log analysis (the logs
collector's first-match pattern semantics, logs_collector.py:193-208) reproduces the
reference's own counts, categories and strengths.  CPU only."""
from __future__ import annotations

import json

import numpy as np
import pytest

from conftest import REPO
from helpers import golden_record, record


@pytest.fixture(scope="module")
def sim():
    return json.loads((REPO / "tests" / "golden" / "simulator_cases.json").read_text())


def test_every_scenario_is_covered(sim):
    from egraph import synth
    seen = {c["scenario"] for c in sim["cases"]}
    assert set(synth.SIMULATOR_SCENARIOS) <= seen
    assert any(c["name"] == "C1" for c in sim["cases"])


def test_oracle_matches_reference_on_simulator_cases(sim):
    import rca_oracle
    for c in sim["cases"]:
        assert record(rca_oracle.rca(c["incident_id"], c["evidence"])) == golden_record(c["expected"]), c["name"]


def test_generator_reproduces_the_recorded_evidence(sim):
    from egraph import synth
    cl = synth.build_cluster(synth.ClusterConfig(pods=400, namespaces=4, nodes=12, deployments=40,
                                                 services=30, seed=97))
    for c in sim["cases"]:
        if c["seed"] is None:
            continue
        case = synth.incident_case(cl, c["deployment"], c["scenario"], c["incident_id"],
                                   np.random.default_rng(c["seed"]))
        assert json.loads(json.dumps(case.evidence)) == c["evidence"], c["name"]
    _, c1 = synth.c1_world()
    want = next(c for c in sim["cases"] if c["name"] == "C1")
    assert json.loads(json.dumps(c1.evidence)) == want["evidence"]


def test_log_analysis_matches_reference_collector(sim):
    from egraph import synth
    for lc in sim["log_cases"]:
        got = synth.log_analysis(lc["lines"])
        assert {k: got[k] for k in lc["expected"]} == lc["expected"], lc["scenario"]
    # first match decides: a line matching both "error" and "network" counts as an error only
    got = synth.log_analysis(["connection timed out: error", "request timed out"])
    assert got["error_count"] == 1 and got["warning_count"] == 1
    assert got["patterns_found"] == ["error", "network"]


def test_c1_shape():
    """C1: one CrashLoop incident, ~100 evidence rows, ~100 graph vertices."""
    from egraph import synth
    cl, case = synth.c1_world()
    assert case.scenario == "crashloop_deploy"
    assert 90 <= len(case.evidence) <= 110
    assert 90 <= len(cl.ids) <= 110
    kinds = [e["evidence_type"] for e in case.evidence]
    assert kinds.count("kubernetes_pod") == 10 and kinds.count("kubernetes_event") == 60
    assert kinds.count("log_signal") == 1 and kinds.count("metric_signal") == 15
    assert sum(1 for lab in cl.labels if lab == "Node") == 3 and cl.unhealthy_nodes
