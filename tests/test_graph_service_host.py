"""GraphService's host-side administration calls (no GPU needed): init_constraints
(reference src/database/neo4j.py:299-321), cleanup_incident_graph (:282-297: DETACH DELETE of
every node within 10 undirected hops of the incident, RETURN count(*) -- one row per matched
incident), save / load through the snapshot file, and the Neo4jConnection stand-in."""
from __future__ import annotations

import asyncio

import numpy as np


def _ents(ids):
    return [{"id": i, "type": t, "properties": {"name": i.split(":")[-1]}} for i, t in ids]


def _rels(pairs, t="AFFECTS"):
    return [{"source_id": s, "target_id": d, "relation_type": t, "properties": {"w": 1}} for s, d in pairs]


def _service():
    from egraph_dropin import GraphService
    GraphService.reset()
    # incident A -> a0 -> a1 -> ... -> a11 (a chain of 12 pods), incident B -> b0, and a
    # Node that both a0 and b0 are scheduled on (so B is within 3 hops of A)
    chain = [f"pod:ns:a{i}" for i in range(12)]
    ents = [("incident:A", "Incident"), ("incident:B", "Incident"), ("node:n1", "Node"),
            ("pod:ns:b0", "Pod"), ("pod:ns:lonely", "Pod")] + [(c, "Pod") for c in chain]
    asyncio.run(GraphService.create_entities_batch(_ents(ents)))
    rels = _rels([("incident:A", chain[0]), ("incident:B", "pod:ns:b0")])
    rels += _rels(list(zip(chain[:-1], chain[1:])), "CALLS")
    rels += _rels([(chain[0], "node:n1"), ("pod:ns:b0", "node:n1")], "SCHEDULED_ON")
    asyncio.run(GraphService.create_relations_batch(rels))
    return GraphService


def test_init_constraints_creates_the_graph():
    from egraph_dropin import GraphService
    GraphService.reset()
    assert asyncio.run(GraphService.init_constraints()) is None
    assert GraphService._graph is not None and GraphService.graph().num_vertices == 0


def test_cleanup_incident_graph_deletes_ten_hops():
    GS = _service()
    g = GS.graph()
    assert g.num_vertices == 17
    # A reaches: A(0) a0(1) a1..a10 (2..11: a10 is 11 hops) -- so a0..a9 are within 10 hops,
    # n1 (2), b0 (3), B (4); a10 (11 hops) and a11 (12) and the lonely pod survive
    assert asyncio.run(GS.cleanup_incident_graph("incident:A")) == 1
    g = GS.graph()
    assert sorted(g.vertex_ids()) == ["pod:ns:a10", "pod:ns:a11", "pod:ns:lonely"]
    assert g.num_edges == 1                                  # a10 -CALLS-> a11
    assert g.node_props[("Pod", "pod:ns:a10")] == {"name": "a10", "id": "pod:ns:a10"}
    assert list(g.edge_props) == [("pod:ns:a10", "CALLS", "pod:ns:a11")]
    # the graph keeps working: new writes MERGE into the rebuilt graph
    asyncio.run(GS.create_entities_batch(_ents([("incident:C", "Incident")])))
    asyncio.run(GS.create_relations_batch(_rels([("incident:C", "pod:ns:lonely")])))
    assert GS.graph().num_vertices == 4 and GS.graph().num_edges == 2
    GS.reset()


def test_cleanup_unknown_incident_returns_zero():
    GS = _service()
    assert asyncio.run(GS.cleanup_incident_graph("incident:nope")) == 0
    assert asyncio.run(GS.cleanup_incident_graph("A")) == 0     # {id: $incident_id} is literal
    assert GS.graph().num_vertices == 17
    GS.reset()


def test_within_hops_matches_bfs():
    GS = _service()
    g = GS.graph()
    a = g.vertex_of[("Incident", "incident:A")]
    for h in range(0, 13):
        got = set(np.nonzero(g.within_hops(a, h))[0].tolist())
        vl, es, ed, _ = g.export()
        adj = {v: set() for v in range(g.num_vertices)}
        for s, d in zip(es.tolist(), ed.tolist()):
            adj[s].add(d)
            adj[d].add(s)
        seen, fr = {a}, {a}
        for _ in range(h):
            fr = {n for v in fr for n in adj[v]} - seen
            seen |= fr
        assert got == seen, h
    GS.reset()


def test_save_load_hands_the_graph_over(tmp_path):
    GS = _service()
    before = (GS.graph().vertex_ids(), GS.graph().export()[1].tolist(), dict(GS.graph().node_props))
    GS.save(tmp_path / "g.egr")
    GS.reset()
    GS.load(tmp_path / "g.egr")
    g = GS.graph()
    assert (g.vertex_ids(), g.export()[1].tolist(), dict(g.node_props)) == before
    GS.reset()


def test_vertex_ids_is_a_copy():
    GS = _service()
    g = GS.graph()
    ids = g.vertex_ids()
    ids.append("junk")
    assert len(g.vertex_ids()) == g.num_vertices
    GS.reset()


def test_connection_stand_in():
    from egraph_dropin import GraphConnection, Neo4jConnection
    assert Neo4jConnection is GraphConnection
    assert asyncio.run(Neo4jConnection.close()) is None
    assert asyncio.run(Neo4jConnection.verify_connectivity()) in (True, False)
