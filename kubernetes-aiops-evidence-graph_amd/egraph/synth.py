"""Synthetic cluster graphs and collector-shaped incident evidence (BASELINE configs C1-C4).

The reference's simulator applies faulty manifests to a live cluster
(src/simulator/incident_simulator.py:13-269) and the collectors turn what they observe into
Evidence / GraphEntity / GraphRelation items.  Offline, this module generates the same shapes:

  * vertices / edges with the collectors' id scheme (kubernetes_collector.py:93-314,
    deploy_diff_collector.py:246-269) plus the build-side superset Service / Event /
    LogPattern / MetricAnomaly, laid out namespace by namespace so that
    neighbouring vertices get neighbouring indices;
  * per incident ~100 evidence rows whose `data` payloads follow the collectors
    (kubernetes_collector.py:136-195, :386-485, :512-626; deploy_diff_collector.py:127-183;
    logs_collector.py:133-164; metrics_collector.py:100-145) and whose signal_strength seeds
    follow their scoring functions.

All draws come from numpy Generators seeded per config (default 20260821 + config index).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

PROMQL = {  # query names of src/config/promql_queries.yaml used by the metric rows
    "crashloop": ["restart_count", "container_exit_code"],
    "oom": ["memory_usage_percentage", "oom_killed_total", "memory_working_set"],
    "latency": ["p99_latency", "p95_latency"],
    "hpa": ["hpa_at_max", "hpa_current_replicas", "hpa_max_replicas"],
    "resource": ["cpu_usage_percentage", "cpu_throttling", "disk_usage"],
    "deployment": ["deployment_replicas_unavailable", "deployment_generation_mismatch"],
    "error_rate": ["http_5xx_rate", "grpc_error_rate", "error_rate_increase"],
}


@dataclass
class ClusterConfig:
    pods: int = 10_000
    namespaces: int = 20
    nodes: int = 200
    deployments: int = 1_000
    services: int = 1_000
    calls_per_service: int = 3
    attach_fraction: float = 0.2      # pods with an Event / LogPattern / MetricAnomaly vertex
    unhealthy_node_fraction: float = 0.05
    seed: int = 20260821
    # denser telemetry links (C4's ~10M CSR entries): every Event /
    # LogPattern / MetricAnomaly vertex is also OBSERVED_ON its pod's Node and AGGREGATED by its
    # pod's Deployment, a Service SELECTS each pod of its deployments, and the sibling pods of a
    # deployment share its LogPattern vertices (HAS_LOG_PATTERN)
    dense_links: bool = False


CONFIGS = {
    "C2": ClusterConfig(),
    "C3": ClusterConfig(pods=100_000, namespaces=100, nodes=2_000, deployments=10_000,
                        services=10_000, attach_fraction=0.35, seed=20260823),
    "C4": ClusterConfig(pods=400_000, namespaces=400, nodes=8_000, deployments=40_000,
                        services=40_000, attach_fraction=0.5, seed=20260824, dense_links=True),
}


@dataclass
class Cluster:
    cfg: ClusterConfig
    ids: list = field(default_factory=list)
    labels: list = field(default_factory=list)
    src: list = field(default_factory=list)
    dst: list = field(default_factory=list)
    types: list = field(default_factory=list)
    ns_names: list = field(default_factory=list)
    deploy_ns: np.ndarray | None = None        # deployment -> namespace index
    deploy_name: list = field(default_factory=list)
    deploy_pods: list = field(default_factory=list)   # deployment -> list of pod names
    pod_node: dict = field(default_factory=dict)       # pod name -> node name
    unhealthy_nodes: set = field(default_factory=set)
    attachments: dict = field(default_factory=dict)    # pod name -> [(label, vertex id)]
    # dense_links: extra edges by vertex position in `ids` (EvidenceGraph.add_edges_indexed)
    extra_src: np.ndarray | None = None
    extra_dst: np.ndarray | None = None
    extra_type: np.ndarray | None = None
    EXTRA_TYPES = ("OBSERVED_ON", "AGGREGATES", "SELECTS", "HAS_LOG_PATTERN")

    def add_vertex(self, vid: str, label: str) -> None:
        self.ids.append(vid)
        self.labels.append(label)

    def add_edge(self, s: str, d: str, t: str) -> None:
        self.src.append(s)
        self.dst.append(d)
        self.types.append(t)


def build_cluster(cfg: ClusterConfig) -> Cluster:
    rng = np.random.default_rng(cfg.seed)
    c = Cluster(cfg)
    c.ns_names = [f"ns-{i:03d}" for i in range(cfg.namespaces)]
    node_names = [f"node-{i:05d}" for i in range(cfg.nodes)]
    bad = rng.random(cfg.nodes) < cfg.unhealthy_node_fraction
    c.unhealthy_nodes = {n for n, b in zip(node_names, bad) if b}
    for n in node_names:
        c.add_vertex(f"node:{n}", "Node")
    dense = cfg.dense_links
    att_rows: list = []        # dense_links: (attachment, pod, node, deployment, kind) positions
    pod_rows: list = []        # dense_links: (pod, service, deployment) positions
    c.deploy_ns = np.sort(rng.integers(0, cfg.namespaces, cfg.deployments))
    svc_ns = np.sort(rng.integers(0, cfg.namespaces, cfg.services))
    pods_per = np.full(cfg.deployments, cfg.pods // cfg.deployments)
    pods_per[: cfg.pods % cfg.deployments] += 1
    pod_nodes = rng.integers(0, cfg.nodes, cfg.pods)
    attach = rng.random((cfg.pods, 3)) < cfg.attach_fraction
    svc_of_deploy = np.minimum((np.arange(cfg.deployments) * cfg.services) // cfg.deployments,
                               cfg.services - 1)
    p = 0
    d = 0
    s = 0
    for ns_i, ns in enumerate(c.ns_names):
        while s < cfg.services and svc_ns[s] == ns_i:
            c.add_vertex(f"service:{ns}:svc-{s}", "Service")
            s += 1
        while d < cfg.deployments and c.deploy_ns[d] == ns_i:
            dname = f"app-{d}"
            c.deploy_name.append(dname)
            did = f"deployment:{ns}:{dname}"
            d_pos = len(c.ids)
            c.add_vertex(did, "Deployment")
            sv = int(svc_of_deploy[d])
            c.add_edge(f"service:{c.ns_names[svc_ns[sv]]}:svc-{sv}", did, "SELECTS")
            pods = []
            for j in range(int(pods_per[d])):
                pname = f"{dname}-{j:02d}-{p:06x}"
                pid = f"pod:{ns}:{pname}"
                node = node_names[pod_nodes[p]]
                p_pos = len(c.ids)
                c.add_vertex(pid, "Pod")
                c.add_edge(did, pid, "OWNS")
                if dense:
                    pod_rows.append((p_pos, int(svc_of_deploy[d]), d_pos))
                c.add_edge(pid, f"node:{node}", "SCHEDULED_ON")
                c.pod_node[pname] = node
                att = []
                for k, (lab, et, pre) in enumerate((("Event", "HAS_EVENT", "event"),
                                                     ("LogPattern", "HAS_LOG_PATTERN", "logpattern"),
                                                     ("MetricAnomaly", "HAS_METRIC_ANOMALY", "metric"))):
                    if attach[p, k]:
                        vid = f"{pre}:{ns}:{pname}"
                        if dense:
                            att_rows.append((len(c.ids), p_pos, int(pod_nodes[p]), d_pos, k))
                        c.add_vertex(vid, lab)
                        c.add_edge(pid, vid, et)
                        att.append((lab, vid))
                if att:
                    c.attachments[pname] = att
                pods.append(pname)
                p += 1
            c.deploy_pods.append(pods)
            d += 1
    if dense:
        _dense_links(c, np.array(att_rows, np.int64).reshape(-1, 5),
                     np.array(pod_rows, np.int64).reshape(-1, 3), svc_ns, cfg)
    # service call graph: mostly within the namespace
    for sv in range(cfg.services):
        for _ in range(cfg.calls_per_service):
            if rng.random() < 0.9:
                lo = np.searchsorted(svc_ns, svc_ns[sv])
                hi = np.searchsorted(svc_ns, svc_ns[sv], side="right")
                t = int(rng.integers(lo, hi))
            else:
                t = int(rng.integers(0, cfg.services))
            if t != sv:
                c.add_edge(f"service:{c.ns_names[svc_ns[sv]]}:svc-{sv}",
                           f"service:{c.ns_names[svc_ns[t]]}:svc-{t}", "CALLS")
    return c


def _dense_links(c: Cluster, att: np.ndarray, pods: np.ndarray, svc_ns: np.ndarray,
                 cfg: ClusterConfig) -> None:
    """The dense_links edges as position arrays (vectorised: C4 adds ~3.4M of them)."""
    pos = {v: i for i, v in enumerate(c.ids) if v.startswith("service:")}
    svc_pos = np.array([pos[f"service:{c.ns_names[svc_ns[s]]}:svc-{s}"] for s in range(cfg.services)],
                       np.int64)
    src, dst, typ = [], [], []
    # attachment -> its pod's Node (node vertices are the first cfg.nodes positions)
    src.append(att[:, 2]), dst.append(att[:, 0]), typ.append(np.full(len(att), 0))
    # deployment AGGREGATES the attachment
    src.append(att[:, 3]), dst.append(att[:, 0]), typ.append(np.full(len(att), 1))
    # service SELECTS each pod of its deployments
    src.append(svc_pos[pods[:, 1]]), dst.append(pods[:, 0]), typ.append(np.full(len(pods), 2))
    # sibling pods of a deployment share its LogPattern vertices
    lp = att[att[:, 4] == 1]
    dep_of_pod = pods[:, 2]
    order = np.argsort(dep_of_pod, kind="stable")
    d_sorted = dep_of_pod[order]
    lo = np.searchsorted(d_sorted, lp[:, 3], side="left")
    hi = np.searchsorted(d_sorted, lp[:, 3], side="right")
    n = hi - lo
    rep = np.repeat(np.arange(len(lp)), n)
    off = np.arange(int(n.sum())) - np.repeat(np.cumsum(n) - n, n)
    sib = pods[order[lo[rep] + off], 0]
    keep = sib != lp[rep, 1]                      # the owning pod already has its edge
    src.append(sib[keep]), dst.append(lp[rep, 0][keep]), typ.append(np.full(int(keep.sum()), 3))
    c.extra_src = np.concatenate(src).astype(np.int32)
    c.extra_dst = np.concatenate(dst).astype(np.int32)
    c.extra_type = np.concatenate(typ).astype(np.int32)


def build_graph(c: Cluster):
    """The EvidenceGraph of a cluster (+ its incidents): MERGE of every vertex and edge, the
    dense_links edges by vertex position."""
    from .graph import EvidenceGraph
    g = EvidenceGraph()
    g.merge_nodes(c.ids, c.labels)
    g.merge_edges(c.src, c.dst, c.types)
    if c.extra_src is not None and len(c.extra_src):
        g.add_edges_indexed(c.extra_src, c.extra_dst, c.extra_type, list(c.EXTRA_TYPES))
    return g


# ---------------------------------------------------------------------------------------------
# incidents
SCENARIOS = ("crashloop_deploy", "crashloop", "oom", "imagepull")
SCENARIO_P = (0.2, 0.2, 0.3, 0.3)   # BASELINE C2 mix: 40 % CrashLoop (half with deploy), 30/30
# the reference simulator's four scenarios (src/simulator/incident_simulator.py:13-160, :164-169)
SIMULATOR_SCENARIOS = ("crashloop", "oom", "imagepull", "slowapp")

# ---- log lines and the logs collector's analysis (logs_collector.py:166-244) ----------------
# The (regex, category) table and the stack-trace regexes are the collector's own, exported from
# the reference by oracle/gen_golden_simulator.py (data, like rules_catalog.json).
_LOG_PATTERNS = None


def _log_patterns():
    global _LOG_PATTERNS
    if _LOG_PATTERNS is None:
        import json
        import re
        from pathlib import Path
        d = json.loads((Path(__file__).with_name("log_patterns.json")).read_text())
        _LOG_PATTERNS = ([(re.compile(p), c) for p, c in d["error_patterns"]],
                         [re.compile(p) for p in d["stack_trace_patterns"]])
    return _LOG_PATTERNS


def log_analysis(lines: list[str]) -> dict:
    """_extract_log_patterns + _calculate_log_signal_strength over log lines: per line the FIRST
    matching error pattern decides (:193-208): its category joins patterns_found, and the line
    counts as an error if the category names "error" or "critical", else as a warning."""
    errs, stacks = _log_patterns()
    error_count = warning_count = 0
    found: set = set()
    sample_errors: list = []
    stack_traces: list = []
    for line in lines:
        for rx, cat in errs:
            if rx.search(line):
                found.add(cat)
                if "error" in cat or "critical" in cat:
                    if len(sample_errors) < 10:
                        sample_errors.append(line[:500])
                    error_count += 1
                else:
                    warning_count += 1
                break
        if len(stack_traces) < 5:
            for rx in stacks:
                if rx.search(line):
                    stack_traces.append(line[:1000])
                    break
    strength = 0.3
    if error_count > 10:
        strength = 0.9
    elif error_count > 5:
        strength = 0.8
    elif error_count > 0:
        strength = 0.6
    elif warning_count > 10:
        strength = 0.5
    if "oom" in found or "critical" in found:
        strength = max(strength, 0.95)
    return {"error_count": error_count, "warning_count": warning_count,
            "patterns_found": sorted(found), "sample_errors": sample_errors,
            "stack_traces": stack_traces, "signal_strength": strength}


# log lines a pod of each scenario writes (what Loki would return for the incident window)
_LOG_LINES = {
    "crashloop": ["Starting", "exit status 1", "Error: container exited with code 1",
                  "Back-off restarting failed container", "panic: runtime error: invalid memory address",
                  "goroutine 1 [running]:", "failed to load config: no such file or directory"],
    "oom": ["Killed process 4242 (python) total-vm:2097152kB", "MemoryError: out of memory",
            "container terminated: OOMKilled", "java.lang.OutOfMemoryError: Java heap space",
            "allocating 10000000 bytes", "GC overhead limit exceeded"],
    "imagepull": [],          # the container never starts: no application log lines
    "slowapp": ["GET / HTTP/1.1 200 OK", "GET / HTTP/1.1 500 Internal Server Error",
                "upstream request timed out after 5.0s", "connection reset by peer",
                "GET /health HTTP/1.1 200 OK", "slow request: 4.2s",
                '  File "/app/server.py", line 12, in do_GET'],
}


def scenario_log_lines(sc: str, rng: np.random.Generator, n: int | None = None) -> list[str]:
    base = "crashloop" if sc.startswith("crashloop") else sc
    pool = _LOG_LINES.get(base, [])
    if not pool:
        return []
    n = int(rng.integers(0, 60)) if n is None else n
    return [pool[int(i)] for i in rng.integers(0, len(pool), n)]


@dataclass
class IncidentCase:
    incident: dict            # Incident model fields
    scenario: str
    evidence: list            # evidence dicts (Evidence.model_dump(mode="json") shape)
    entities: list            # GraphEntity dicts added by this incident
    relations: list           # GraphRelation dicts added by this incident


def _pod_strength(wr, tr, restarts, phase):   # kubernetes_collector.py:255-270
    if wr in ("CrashLoopBackOff", "ImagePullBackOff", "ErrImagePull"):
        return 0.95
    if tr == "OOMKilled":
        return 0.95
    if restarts > 3:
        return 0.8
    if phase != "Running":
        return 0.7
    return 0.3


def _metric_strength(name, v):   # metrics_collector.py:246-328
    if "restart" in name:
        return 0.9 if v > 5 else 0.7 if v > 2 else 0.5 if v > 0 else 0.3
    if "error" in name or "5xx" in name:
        return 0.9 if v > 0.1 else 0.8 if v > 0.05 else 0.6 if v > 0.01 else 0.3
    if "memory" in name or "usage" in name:
        return 0.9 if v > 90 else 0.7 if v > 80 else 0.5 if v > 70 else 0.3
    if "latency" in name:
        return 0.9 if v > 5 else 0.7 if v > 2 else 0.5 if v > 1 else 0.3
    if "throttl" in name:
        return 0.8 if v > 0.5 else 0.6 if v > 0.1 else 0.3
    if "oom" in name:
        return 0.95 if v > 0 else 0.3
    if "hpa" in name:
        return 0.8 if ("max" in name and v == 1) else 0.3
    return 0.3


def make_incidents(c: Cluster, n: int, seed: int = 7, events_per_incident: int = 60,
                   scenario: str | None = None) -> list[IncidentCase]:
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        sc = scenario or SCENARIOS[int(rng.choice(len(SCENARIOS), p=SCENARIO_P))]
        d = int(rng.integers(0, len(c.deploy_name)))
        iid = f"00000000-0000-4000-8000-{seed:04x}{i:08x}"
        out.append(incident_case(c, d, sc, iid, rng, events_per_incident, fingerprint=f"fp-{i}"))
    return out


def incident_case(c: Cluster, d: int, sc: str, iid: str, rng: np.random.Generator,
                  events_per_incident: int = 60, fingerprint: str | None = None) -> IncidentCase:
    """One incident on deployment `d` with scenario `sc`: the Incident vertex, its AFFECTS /
    CORRELATES_WITH relations and collector-shaped evidence rows."""
    ns = c.ns_names[int(c.deploy_ns[d])]
    dname = c.deploy_name[d]
    inc = {"id": iid, "fingerprint": fingerprint or f"fp-{iid}", "title": f"{sc}: {dname}",
           "severity": "critical", "source": "synthetic", "cluster": "synthetic",
           "namespace": ns, "service": dname, "started_at": "2026-08-21T00:00:00Z"}
    ev, ents, rels = [], [], []
    k = 0

    def row(etype, entity, data, strength, source="kubernetes_api"):
        nonlocal k
        k += 1
        ev.append({"id": f"{iid[-12:]}-{k:04d}", "incident_id": iid, "evidence_type": etype,
                   "source": source, "entity_name": entity, "entity_namespace": ns,
                   "data": data, "signal_strength": strength})

    ents.append({"id": f"incident:{iid}", "type": "Incident",
                 "properties": {"id": iid, "title": inc["title"], "namespace": ns}})
    pods = c.deploy_pods[d]
    for pname in pods:
        restarts = int(rng.geometric(0.3)) - 1
        wr = tr = None
        phase = "Running"
        if sc.startswith("crashloop"):
            wr = "CrashLoopBackOff" if rng.random() < 0.8 else None
            tr = "Error" if rng.random() < 0.5 else None
        elif sc == "oom":
            tr = "OOMKilled" if rng.random() < 0.7 else None
        elif sc == "imagepull":
            wr = ("ImagePullBackOff", "ErrImagePull")[int(rng.integers(0, 2))]
            phase, restarts = "Pending", 0
        elif sc == "slowapp":
            restarts = 0               # serves, slowly: 500s on 30 % of requests, 1-5 s latency
        ready = "True" if (wr is None and tr is None and rng.random() < 0.7) else "False"
        conds = [{"type": "Ready", "status": ready,
                  "reason": None if ready == "True" else "ContainersNotReady"}]
        row("kubernetes_pod", pname,
            {"name": pname, "namespace": ns, "phase": phase, "node_name": c.pod_node[pname],
             "restart_count": restarts, "waiting_reason": wr, "terminated_reason": tr,
             "conditions": conds}, _pod_strength(wr, tr, restarts, phase))
        rels.append({"source_id": f"incident:{iid}", "target_id": f"pod:{ns}:{pname}",
                     "relation_type": "AFFECTS"})
    row("kubernetes_deployment", dname,
        {"name": dname, "namespace": ns, "replicas": len(pods), "ready_replicas": 0,
         "unavailable_replicas": len(pods)}, 0.8)
    for j in range(events_per_incident):
        pname = pods[j % len(pods)]
        reason = ("BackOff", "Unhealthy", "Failed", "Pulled", "Created")[int(rng.integers(0, 5))]
        warn = reason in ("BackOff", "Unhealthy", "Failed")
        row("kubernetes_event", pname,
            {"type": "Warning" if warn else "Normal", "reason": reason, "message": reason,
             "involved_object": {"kind": "Pod", "name": pname, "namespace": ns}, "count": 1},
            0.9 if warn else 0.4)
    lines = scenario_log_lines(sc, rng)
    la = log_analysis(lines)
    row("log_signal", dname, {"total_lines": len(lines), "error_count": la["error_count"],
                              "warning_count": la["warning_count"],
                              "patterns_found": la["patterns_found"],
                              "sample_errors": la["sample_errors"],
                              "stack_traces": la["stack_traces"]},
        la["signal_strength"], "loki")
    if sc == "slowapp":
        cats = ["deployment", "resource", "latency", "error_rate"]
    else:
        cats = ["crashloop", "resource", "deployment"] + (["oom"] if sc == "oom" else ["latency", "hpa"])
    names = [q for cat in cats for q in PROMQL[cat]]
    for j in range(15):
        qn = names[j % len(names)]
        if "memory" in qn:
            v = float(rng.uniform(0, 100))
        elif "latency" in qn:
            v = float(rng.uniform(1, 5) if sc == "slowapp" else rng.uniform(0, 5))
        elif "5xx" in qn or "error" in qn:
            v = float(rng.uniform(0.2, 0.4) if sc == "slowapp" else rng.uniform(0, 0.05))
        elif "hpa" in qn:
            v = float(rng.integers(0, 2))
        else:
            v = float(rng.uniform(0, 10))
        st = _metric_strength(qn, v)
        row("metric_signal", qn, {"query_name": qn, "current_value": v, "is_anomalous": st > 0.7},
            st, "prometheus")
    for node in sorted({c.pod_node[p] for p in pods} & c.unhealthy_nodes):
        row("kubernetes_node", node,
            {"name": node, "conditions": {"Ready": {"status": "False"},
                                          "MemoryPressure": {"status": "True"}}}, 0.9)
    recent = sc in ("crashloop_deploy", "imagepull")
    row("deploy_change", dname, {"deployment_name": dname, "namespace": ns,
                                 "is_recent_change": recent, "current_revision": "7"},
        0.95 if recent else 0.3)
    if recent:
        cid = f"change:deployment:{ns}:{dname}:7"
        ents.append({"id": cid, "type": "ChangeEvent",
                     "properties": {"deployment": dname, "namespace": ns, "revision": "7"}})
        rels.append({"source_id": f"deployment:{ns}:{dname}", "target_id": cid,
                     "relation_type": "HAS_RECENT_CHANGE"})
        rels.append({"source_id": f"incident:{iid}", "target_id": cid,
                     "relation_type": "CORRELATES_WITH"})
        row("image_change", dname, {"deployment": dname, "image_changed": True}, 0.85)
    return IncidentCase(inc, sc, ev, ents, rels)


def c1_world(seed: int = 20260820) -> tuple[Cluster, IncidentCase]:
    """BASELINE config C1: ONE CrashLoopBackOff incident after a recent deploy
    on a small cluster -- 1 Deployment with 10 Pods on 3 Nodes (one NotReady), its Service, the
    recent ChangeEvent, 60 Kubernetes Event rows (each its own Event vertex), 1 log row and 15
    metric rows: ~100 evidence rows and ~100 graph vertices.  Returns the cluster with the
    incident added and the incident case."""
    cfg = ClusterConfig(pods=10, namespaces=1, nodes=3, deployments=1, services=1,
                        calls_per_service=0, attach_fraction=1.0, unhealthy_node_fraction=0.0,
                        seed=seed)
    c = build_cluster(cfg)
    c.unhealthy_nodes = {"node-00001"}            # one of the three Nodes is NotReady
    rng = np.random.default_rng(seed + 1)
    case = incident_case(c, 0, "crashloop_deploy", f"00000000-0000-4000-8000-{seed:012x}", rng,
                         events_per_incident=60, fingerprint="c1")
    # each event row is its own Event vertex (event:<ns>:<event name>) attached to its pod
    ns = c.ns_names[0]
    for j, ev in enumerate(x for x in case.evidence if x["evidence_type"] == "kubernetes_event"):
        pod = ev["entity_name"]
        ev["entity_name"] = f"{pod}.{j:04x}"
        case.entities.append({"id": f"event:{ns}:{ev['entity_name']}", "type": "Event",
                              "properties": {"reason": ev["data"]["reason"]}})
        case.relations.append({"source_id": f"pod:{ns}:{pod}", "target_id": f"event:{ns}:{ev['entity_name']}",
                               "relation_type": "HAS_EVENT"})
    add_incidents(c, [case])
    return c, case


def add_incidents(c: Cluster, cases: list[IncidentCase]) -> None:
    for case in cases:
        for e in case.entities:
            c.add_vertex(e["id"], e["type"])
        for r in case.relations:
            c.add_edge(r["source_id"], r["target_id"], r["relation_type"])


# seeds: evidence row -> graph vertex (the product rule, DESIGN.md §5, lives in egraph.seeds)
from .seeds import attach_ids, seeds_for_batch  # noqa: E402,F401  (re-exported for callers)


# ---------------------------------------------------------------------------------------------
# alert storm (BASELINE config C5): 100k alerts/min, Zipf(1.1) over 10k (alertname, namespace,
# service) keys, incremental topology deltas every tick
STORM_ALERTS = ("KubePodCrashLooping", "KubePodNotReady", "OOMKilled", "ImagePullBackOff")
STORM_SCENARIO = {"KubePodCrashLooping": "crashloop", "KubePodNotReady": "crashloop_deploy",
                  "OOMKilled": "oom", "ImagePullBackOff": "imagepull"}


class StormWorkload:
    """Seeded alert stream over a cluster: alert i of a tick draws key r ~ Zipf(s) over
    `n_keys` keys; key r = (alertname, namespace, service) of deployment r % n_deployments.
    make_case builds the incident the first alert of a fingerprint opens; topology(tick) adds
    Event vertices to pods that had none (rows of open incidents may re-attach to them)."""

    def __init__(self, c: Cluster, n_keys: int = 10_000, zipf_s: float = 1.1, seed: int = 20260825,
                 events_per_incident: int = 20):
        self.c = c
        self.rng = np.random.default_rng(seed)
        nd = len(c.deploy_name)
        self.key_deploy = np.arange(n_keys) % nd
        self.key_alert = (np.arange(n_keys) // nd) % len(STORM_ALERTS)
        w = 1.0 / np.arange(1, n_keys + 1) ** zipf_s
        self.p = w / w.sum()
        self.n_keys = n_keys
        self.events_per_incident = events_per_incident
        self.keys = [f"alertmanager:{STORM_ALERTS[self.key_alert[r]]}:"
                     f"{c.ns_names[int(c.deploy_ns[self.key_deploy[r]])]}:"
                     f"{c.deploy_name[self.key_deploy[r]]}" for r in range(n_keys)]
        self._tick_keys = None
        self._events_added: set = set()

    def alerts(self, n: int) -> list[str]:
        """The next n alert keys (the normalizer.py:217 strings); remembers their key ranks."""
        self._tick_keys = self.rng.choice(self.n_keys, size=n, p=self.p)
        return [self.keys[r] for r in self._tick_keys]

    def make_case(self, handle: int, alert_index: int):
        from egraph.storm import StormCase
        r = int(self._tick_keys[alert_index])
        iid = f"00000000-0000-4000-9000-{handle:012x}"
        case = incident_case(self.c, int(self.key_deploy[r]),
                             STORM_SCENARIO[STORM_ALERTS[self.key_alert[r]]], iid, self.rng,
                             self.events_per_incident)
        return StormCase(iid, [(e["id"], e["type"]) for e in case.entities],
                         [(x["source_id"], x["target_id"], x["relation_type"]) for x in case.relations],
                         case.evidence)

    def topology(self, n_events: int):
        """n_events new Event vertices (+ HAS_EVENT edges) on random pods without one."""
        ids, labels, src, dst, types = [], [], [], [], []
        for _ in range(n_events):
            d = int(self.rng.integers(0, len(self.c.deploy_name)))
            pods = self.c.deploy_pods[d]
            pname = pods[int(self.rng.integers(0, len(pods)))]
            ns = self.c.ns_names[int(self.c.deploy_ns[d])]
            vid = f"event:{ns}:{pname}"
            if vid in self._events_added or any(v == vid for _, v in self.c.attachments.get(pname, ())):
                continue
            self._events_added.add(vid)
            ids.append(vid)
            labels.append("Event")
            src.append(f"pod:{ns}:{pname}")
            dst.append(vid)
            types.append("HAS_EVENT")
        return ids, labels, src, dst, types
