"""GPU: the drop-in GraphService's typed path queries (find_related_changes,
find_affected_by_node, get_service_dependencies -- reference neo4j.py:205-279), each a chain of
typed hops on the device snapshot (egr_snapshot_typed_neighbors), against the CPU oracle
(oracle/graph_queries.py) on the known-answer graph, on C1 and on a C3 slice -- parity
unpinned (no Neo4j here; the reference holds no fixture for these queries)."""
from __future__ import annotations

import asyncio
import datetime as dt

import numpy as np
import pytest

import graph_queries as gq
from graph_query_cases import NOW, affected_key, deps_key, known_answer_world

pytestmark = pytest.mark.gpu


def _oracle_world(g):
    vl, es, ed, et = g.export()
    labels, types, ids = g.labels(), g.rel_types(), g.vertex_ids()
    lab = [labels[x] for x in vl]
    edges = [(int(s), int(d), types[int(t)]) for s, d, t in zip(es, ed, et)]
    return lab, ids, edges, g.node_props


def _load(entities, relations):
    from src.database import GraphService
    from src.models.evidence import GraphEntity, GraphRelation
    GraphService.reset()
    asyncio.run(GraphService.create_entities_batch(
        [GraphEntity(id=i, type=lab, properties=p) for i, lab, p in entities]))
    asyncio.run(GraphService.create_relations_batch(
        [GraphRelation(source_id=s, target_id=d, relation_type=t) for s, d, t in relations]))
    return GraphService


def _check_all(GS, incidents, nodes, services, now=NOW):
    lab, ids, edges, props = _oracle_world(GS.graph())
    def by_time(rows):       # ORDER BY changed_at DESC leaves ties in an unspecified order
        return sorted(rows, key=lambda p: (p["changed_at"], p["id"]))
    for inc in incidents:
        for w in (30, 90):
            got = GS.find_related_changes_sync(inc, w, now=now)
            assert [p["changed_at"] for p in got] == sorted((p["changed_at"] for p in got), reverse=True)
            assert by_time(got) == by_time(gq.related_changes(lab, ids, edges, props, inc, w, now=now)), (inc, w)
    for n in nodes:
        got = asyncio.run(GS.find_affected_by_node(n))
        assert affected_key(got) == affected_key(gq.affected_by_node(lab, ids, edges, props, n)), n
    for name, ns in services:
        got = asyncio.run(GS.get_service_dependencies(name, ns))
        want = gq.service_dependencies(lab, ids, edges, props, name, ns)
        # collect(DISTINCT): each service once (list order unspecified), the same property dicts
        assert deps_key(got) == deps_key(want) and got["service"] == want["service"], (name, ns)
        for side in ("downstream", "upstream"):
            assert sorted(got[side], key=lambda p: p["id"]) == sorted(want[side], key=lambda p: p["id"])


def test_typed_queries_known_answer():
    E, R, exp = known_answer_world()
    GS = _load(E, R)
    try:
        got = GS.find_related_changes_sync("incident:i1", 30, now=NOW)
        assert got == exp["related_changes"]
        assert affected_key(asyncio.run(GS.find_affected_by_node("node-a"))) == exp["affected_by_node"]
        assert deps_key(asyncio.run(GS.get_service_dependencies("api", "ns"))) == exp["service_dependencies"]
        _check_all(GS, ["incident:i1", "incident:i2", "incident:none"], ["node-a", "node-b", "node-z"],
                   [("api", "ns"), ("api", "other"), ("web", "ns"), ("x", "ns")])
        # a write after a read: the next query sees it through the snapshot's incremental update
        from src.models.evidence import GraphEntity, GraphRelation
        asyncio.run(GS.create_entities_batch([GraphEntity(id="change:c9", type="ChangeEvent",
                                                          properties={"changed_at": NOW})]))
        asyncio.run(GS.create_relations_batch([GraphRelation(source_id="change:c9", target_id="pod:ns:p2",
                                                             relation_type="APPLIES_TO")]))
        assert [c["id"] for c in GS.find_related_changes_sync("incident:i1", 30, now=NOW)][:1] == ["change:c9"]
        _check_all(GS, ["incident:i1"], ["node-a"], [("api", "ns")])
    finally:
        GS.reset()


def test_owner_chain_depth_and_cycle():
    """(p)<-[:OWNS*]-(d:Deployment) has no depth bound: an owner chain 24 levels deep (past the
    old bound of 16) reaches its Deployment, and an OWNS cycle ends by relationship uniqueness."""
    E = [("node:n", "Node", {"name": "n"}), ("pod:ns:p", "Pod", {"name": "p"}),
         ("pod:ns:q", "Pod", {"name": "q"}), ("deployment:ns:deep", "Deployment", {"name": "deep"}),
         ("deployment:ns:c1", "Deployment", {"name": "c1"}), ("replicaset:ns:c2", "ReplicaSet", {})]
    R = [("pod:ns:p", "node:n", "SCHEDULED_ON"), ("pod:ns:q", "node:n", "SCHEDULED_ON")]
    prev = "pod:ns:p"
    for j in range(23):
        E.append((f"owner:ns:o{j}", "ReplicaSet", {}))
        R.append((f"owner:ns:o{j}", prev, "OWNS"))
        prev = f"owner:ns:o{j}"
    R.append(("deployment:ns:deep", prev, "OWNS"))
    # q <- c2 <- c1 <- c2 (a cycle through c1, a Deployment)
    R += [("replicaset:ns:c2", "pod:ns:q", "OWNS"), ("deployment:ns:c1", "replicaset:ns:c2", "OWNS"),
          ("replicaset:ns:c2", "deployment:ns:c1", "OWNS")]
    GS = _load(E, R)
    try:
        got = asyncio.run(GS.find_affected_by_node("n"))
        assert {(r["pod"]["name"], r["deployment"]["name"]) for r in got} == {("p", "deep"), ("q", "c1")}
        _check_all(GS, [], ["n"], [])
    finally:
        GS.reset()


def test_typed_query_leaves_the_event_loop_free():
    """A typed query waits for the service lock (held here by another thread, as a ranking call
    holds it for its whole run) in a worker thread: the event loop keeps running other tasks."""
    import threading
    import time
    E, R, _ = known_answer_world()
    GS = _load(E, R)
    try:
        GS.find_affected_by_node_sync("node-a")          # (snapshot built outside the timing)
        held = threading.Event()

        def holder():
            with GS._lock:
                held.set()
                time.sleep(0.4)
        th = threading.Thread(target=holder)
        th.start()
        held.wait()

        async def go():
            ticks = 0

            async def ticker():
                nonlocal ticks
                while True:
                    await asyncio.sleep(0.01)
                    ticks += 1
            t = asyncio.ensure_future(ticker())
            rows = await GS.find_affected_by_node("node-a")
            t.cancel()
            return rows, ticks
        rows, ticks = asyncio.run(go())
        th.join()
        assert rows and ticks >= 10
    finally:
        GS.reset()


def _with_props(cl, rng, n_changes: int, incidents: list[str]):
    """A synthetic cluster's vertices as the collectors would write them: Nodes with `name`,
    Services / Pods / Deployments with `name` + `namespace` (parsed from the id scheme), plus
    ChangeEvents with tz-aware `changed_at` APPLIES_TO the incidents' affected targets."""
    ents = []
    for i, lab in zip(cl.ids, cl.labels):
        p = {}
        parts = i.split(":")
        if lab == "Node":
            p = {"name": parts[-1]}
        elif lab in ("Service", "Pod", "Deployment") and len(parts) == 3:
            p = {"namespace": parts[1], "name": parts[2]}
        ents.append((i, lab, p))
    rels = list(zip(cl.src, cl.dst, cl.types))
    affects = {}
    for s, d, t in rels:
        if t == "AFFECTS":
            affects.setdefault(s, []).append(d)
    for j in range(n_changes):
        inc = incidents[j % len(incidents)]
        tg = affects.get(inc, [])
        if not tg:
            continue
        cid = f"change:syn:{j}"
        ents.append((cid, "ChangeEvent", {"changed_at": NOW - dt.timedelta(minutes=float(rng.integers(0, 120)))}))
        for d in rng.choice(tg, size=min(2, len(tg)), replace=False):
            rels.append((cid, str(d), "APPLIES_TO"))
    return ents, rels


def test_typed_queries_c1():
    from egraph import synth
    cl, case = synth.c1_world()
    inc = f"incident:{case.incident['id']}"
    ents, rels = _with_props(cl, np.random.default_rng(1), 12, [inc])
    GS = _load(ents, rels)
    try:
        nodes = [i.split(":", 1)[1] for i, lab in zip(cl.ids, cl.labels) if lab == "Node"]
        svcs = [tuple(i.split(":")[1:][::-1]) for i, lab in zip(cl.ids, cl.labels) if lab == "Service"]
        assert len(nodes) == 3 and svcs
        assert len(GS.find_related_changes_sync(inc, 120, now=NOW)) > 0
        assert sum(len(asyncio.run(GS.find_affected_by_node(n))) for n in nodes) >= 10
        _check_all(GS, [inc], nodes, svcs)
    finally:
        GS.reset()


def test_typed_queries_c3_slice():
    """The 100k-pod C3 cluster with 64 incidents; a slice of its Nodes (hubs of ~50 pods each),
    Services (CALLS both ways) and incidents checked against the oracle on the whole graph."""
    from egraph import synth
    cl = synth.build_cluster(synth.CONFIGS["C3"])
    cases = synth.make_incidents(cl, 64, seed=4242)
    synth.add_incidents(cl, cases)
    rng = np.random.default_rng(7)
    incs = [f"incident:{x.incident['id']}" for x in cases]
    ents, rels = _with_props(cl, rng, 200, incs)
    GS = _load(ents, rels)
    try:
        nodes = [i.split(":", 1)[1] for i, lab in zip(cl.ids, cl.labels) if lab == "Node"]
        svcs = [tuple(i.split(":")[1:][::-1]) for i, lab in zip(cl.ids, cl.labels) if lab == "Service"]
        pick = lambda xs, n: [xs[j] for j in rng.choice(len(xs), size=min(n, len(xs)), replace=False)]
        sn, ss, si = pick(nodes, 12), pick(svcs, 40), pick(incs, 16)
        assert sum(len(asyncio.run(GS.find_affected_by_node(n))) for n in sn) > 100
        assert any(asyncio.run(GS.get_service_dependencies(n, s))["upstream"] for n, s in ss)
        _check_all(GS, si, sn, ss)
    finally:
        GS.reset()
