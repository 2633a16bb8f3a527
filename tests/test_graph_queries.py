"""CPU: the oracle of GraphService's typed path queries (oracle/graph_queries.py, restating
neo4j.py:205-279 on an edge list) against the known-answer graph of graph_query_cases -- parity
unpinned: there is no Neo4j here and the reference has no fixture for these queries."""
from __future__ import annotations

import graph_queries as gq
from graph_query_cases import NOW, affected_key, deps_key, known_answer_world


def _world():
    E, R, exp = known_answer_world()
    vid = {i: v for v, (i, _, _) in enumerate(E)}
    labels = [lab for _, lab, _ in E]
    ids = [i for i, _, _ in E]
    props = {(lab, i): dict(p, id=i) for i, lab, p in E}
    edges = [(vid[s], vid[d], t) for s, d, t in R]
    return labels, ids, edges, props, exp


def test_related_changes_known_answer():
    labels, ids, edges, props, exp = _world()
    got = gq.related_changes(labels, ids, edges, props, "incident:i1", 30, now=NOW)
    assert got == exp["related_changes"]
    assert [c["revision"] for c in got] == ["6", "1", "5", "5"]
    # window and incident edges: 90 minutes also takes c2; an unknown incident matches nothing
    assert [c["revision"] for c in gq.related_changes(labels, ids, edges, props, "incident:i1", 90,
                                                      now=NOW)] == ["6", "1", "5", "5", "2"]
    assert gq.related_changes(labels, ids, edges, props, "incident:nope", 30, now=NOW) == []
    assert [c["revision"] for c in gq.related_changes(labels, ids, edges, props, "incident:i2", 30,
                                                      now=NOW)] == ["7"]


def test_affected_by_node_known_answer():
    labels, ids, edges, props, exp = _world()
    got = gq.affected_by_node(labels, ids, edges, props, "node-a")
    assert affected_key(got) == exp["affected_by_node"]
    assert len(got) == 5
    assert affected_key(gq.affected_by_node(labels, ids, edges, props, "node-b")) == \
        [(("pod:ns:p4",), "deployment:ns:d2", None)]
    assert gq.affected_by_node(labels, ids, edges, props, "node-z") == []


def test_service_dependencies_known_answer():
    labels, ids, edges, props, exp = _world()
    got = gq.service_dependencies(labels, ids, edges, props, "api", "ns")
    assert deps_key(got) == exp["service_dependencies"]
    assert got["service"]["namespace"] == "ns"
    assert deps_key(gq.service_dependencies(labels, ids, edges, props, "api", "other")) == \
        {"service": "service:other:api", "downstream": ["service:ns:api"], "upstream": []}
    assert gq.service_dependencies(labels, ids, edges, props, "api", "missing") == \
        {"service": None, "downstream": [], "upstream": []}
