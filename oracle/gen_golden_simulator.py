"""Generate tests/golden/simulator_cases.json (and the collector's log-pattern table) by
RUNNING THE REFERENCE -- test infrastructure only, this container only.

SURVEY.md §8c(4): the reference simulator's four scenarios (src/simulator/incident_simulator.py
:13-160 crashloop / oom / imagepull / slowapp) cannot run offline (they kubectl-apply manifests
to a live cluster), so their evidence is rendered by the build's collector-shaped generator
(egraph/synth.py) and the REFERENCE judges it:
  * the logs collector's pattern table (logs_collector.py:19-38) is exported to
    kubernetes-aiops-evidence-graph_amd/egraph/log_patterns.json (data the generator needs);
  * every generated log row's lines go through the reference's own
    LogsCollector._extract_log_patterns + _calculate_log_signal_strength (:166-244): the
    expected counts / categories / strength are recorded beside the lines;
  * every incident's evidence goes through the reference RulesEngine.generate_hypotheses +
    HypothesisRanker.rank: the ranked hypotheses are recorded (as tests/golden/rules_cases.json).
Cases: each simulator scenario under several seeds, plus the C1 incident (synth.c1_world).

Shims (arithmetic untouched): the structlog stub of gen_golden.py, a stub `src.config` module
whose `settings` carries the two values LogsCollector.__init__ would read (the collector class
is used without its network I/O), and a bare `src.services.collectors` package module (its
__init__ imports the absent Kubernetes client).

Usage:  python oracle/gen_golden_simulator.py [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import asyncio
import datetime as _dt
import json
import sys
import types
from pathlib import Path

sys.dont_write_bytecode = True
REPO = Path(__file__).resolve().parents[1]
PKG = REPO / "kubernetes-aiops-evidence-graph_amd"
sys.path.insert(0, str(REPO / "oracle"))

from gen_golden import _install_shims, _load, _record  # noqa: E402

SEEDS_PER_SCENARIO = 12


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    ref = Path(args.ref)
    _install_shims()
    cfg = types.ModuleType("src.config")
    cfg.settings = types.SimpleNamespace(loki_url="http://loki.invalid", max_log_lines=1000)
    sys.path.insert(0, str(ref))
    import src  # noqa: F401  (the reference package, for src.models)
    sys.modules["src.config"] = cfg
    # the collectors package __init__ imports the Kubernetes client (absent): a bare package
    # module pointing at the same directory lets base.py / logs_collector.py load alone
    coll = types.ModuleType("src.services.collectors")
    coll.__path__ = [str(ref / "src/services/collectors")]
    sys.modules["src.services.collectors"] = coll
    logs_mod = _load(ref / "src/services/collectors/logs_collector.py", "ref_logs_collector")
    (PKG / "egraph" / "log_patterns.json").write_text(json.dumps({
        "source": "src/services/collectors/logs_collector.py:19-38 (exported by "
                  "oracle/gen_golden_simulator.py)",
        "error_patterns": [list(x) for x in logs_mod.ERROR_PATTERNS],
        "stack_trace_patterns": list(logs_mod.STACK_TRACE_PATTERNS)}, indent=1) + "\n")

    from src.models import Incident, IncidentSeverity, IncidentSource  # reference models
    re_mod = _load(ref / "src/services/rca/rules_engine.py", "ref_rules_engine")
    rk_mod = _load(ref / "src/services/rca/hypothesis_ranker.py", "ref_hypothesis_ranker")
    engine, ranker = re_mod.RulesEngine(), rk_mod.HypothesisRanker()
    collector = object.__new__(logs_mod.LogsCollector)      # pattern methods only, no I/O

    # the build's generator (imports after log_patterns.json exists)
    for p in (PKG,):
        sys.path.insert(0, str(p))
    import numpy as np

    from egraph import synth

    def judge(iid, evidence):
        inc = Incident(id=iid, fingerprint="sim", title="sim", severity=IncidentSeverity.CRITICAL,
                       source=IncidentSource.ALERTMANAGER, cluster="c", namespace="default",
                       service="svc", started_at=_dt.datetime(2026, 1, 5, tzinfo=_dt.timezone.utc))
        return _record(ranker.rank(asyncio.run(engine.generate_hypotheses(inc, evidence))))

    def ref_logs(lines):
        a = collector._extract_log_patterns([{"line": ln} for ln in lines])
        return {"error_count": a["error_count"], "warning_count": a["warning_count"],
                "patterns_found": sorted(a["patterns_found"]),
                "signal_strength": collector._calculate_log_signal_strength(a)}

    cl = synth.build_cluster(synth.ClusterConfig(pods=400, namespaces=4, nodes=12, deployments=40,
                                                 services=30, seed=97))
    cases, logs = [], []
    for sc in synth.SIMULATOR_SCENARIOS:
        for k in range(SEEDS_PER_SCENARIO):
            seed = 5000 + 100 * synth.SIMULATOR_SCENARIOS.index(sc) + k
            rng = np.random.default_rng(seed)
            iid = f"00000000-0000-4000-a000-{seed:012x}"
            case = synth.incident_case(cl, k % len(cl.deploy_name), sc, iid, rng)
            cases.append({"name": f"{sc}-{k}", "scenario": sc, "seed": seed, "deployment": k % len(cl.deploy_name),
                          "incident_id": iid, "evidence": case.evidence,
                          "expected": judge(iid, case.evidence)})
            lines = synth.scenario_log_lines(sc, np.random.default_rng(seed + 7))
            logs.append({"scenario": sc, "lines": lines, "expected": ref_logs(lines)})
    c1, c1case = synth.c1_world()
    cases.append({"name": "C1", "scenario": "crashloop_deploy (C1)", "seed": None, "deployment": 0,
                  "incident_id": c1case.incident["id"], "evidence": c1case.evidence,
                  "expected": judge(c1case.incident["id"], c1case.evidence)})
    out = {"generator": "egraph/synth.py incident_case / c1_world; cluster ClusterConfig(pods=400, "
                        "namespaces=4, nodes=12, deployments=40, services=30, seed=97)",
           "cases": cases, "log_cases": logs}
    (REPO / "tests" / "golden" / "simulator_cases.json").write_text(json.dumps(out) + "\n")
    print(f"wrote {len(cases)} simulator cases, {len(logs)} log cases")


if __name__ == "__main__":
    main()
