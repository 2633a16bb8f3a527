"""Alert-storm front end on CPU: the oracle pinned to the reference's outputs, and the host side
of the normalizer mirror (field extraction; the fingerprint itself is computed on the GPU and
checked in tests/test_alerts_gpu.py).

Fixtures (tests/golden/, produced by running the reference, oracle/gen_golden_alerts.py):
  normalizer_cases.json  300 alerts x {alertmanager, grafana, prometheus} with every label
                         fallback, severity spelling, startsAt form and commonLabels merge
  storm_cases.json       60 ticks of the webhook loop against a TTL-honouring Redis:
                         1149 alerts, Zipf keys, gaps past the 4 h TTL, remove / extend ops
"""
from __future__ import annotations

import pytest

import alerts_oracle as AO


def test_oracle_fingerprints_match_reference(golden):
    for fp in golden["fingerprints"]:
        assert AO.fingerprint(":".join(fp["key"])) == fp["fingerprint"]
    for c in golden["normalizer"]:
        assert len(c["expected"]["fingerprint"]) == 32


def _replay_oracle(storm):
    store = AO.TTLStore()
    ttl = storm["ttl_s"]
    n_created = 0
    for t in storm["ticks"]:
        now = t["now_ms"]
        for op in t["ops"]:
            if op["op"] == "remove":
                store.delete(op["fingerprint"])
            else:
                assert store.expire(op["fingerprint"], now, op["ttl_s"]) == op["ok"]
        firing = [e for e in t["expected"] if e is not None]
        dup, inc, n_new = AO.webhook_loop(store, [e["fingerprint"] for e in firing], now, ttl, n_created)
        for e, d, i in zip(firing, dup, inc):
            assert d == e["dup"]
            assert f"inc-{i}" == e["incident"]
        n_created += n_new
    return n_created


def test_oracle_webhook_loop_replays_reference_storm(golden):
    assert _replay_oracle(golden["storm"]) == 225


def test_normalizer_host_fields_match_reference(golden):
    from src.services.ingestion.normalizer import AlertNormalizer
    from src.models import IncidentCreate
    f = {"alertmanager": AlertNormalizer._fields_alertmanager,
         "grafana": AlertNormalizer._fields_grafana,
         "prometheus": AlertNormalizer._fields_prometheus}
    for c in golden["normalizer"]:
        kw, key = f[c["source"]](c["alert"], c["payload"])
        exp = c["expected"]
        assert AO.fingerprint(key) == exp["fingerprint"]
        got = IncidentCreate(fingerprint=AO.fingerprint(key), **kw).model_dump(mode="json")
        for k, v in exp.items():
            if k == "started_at" and v is None:
                continue
            assert got[k] == v, (c, k)


def test_rate_limiter_window():
    import asyncio
    from src.services.ingestion.deduplicator import RateLimiter
    RateLimiter._counters.clear()
    res = [asyncio.run(RateLimiter.check_rate_limit("k", 3)) for _ in range(5)]
    assert res == [(True, 2), (True, 1), (True, 0), (False, 0), (False, 0)]


@pytest.mark.parametrize("bad", [None, 5])
def test_normalizer_severity_requires_string(bad):
    from src.services.ingestion.normalizer import AlertNormalizer
    with pytest.raises(AttributeError):     # labels["severity"].lower(), as in the reference
        AlertNormalizer._fields_alertmanager({"labels": {"severity": bad}}, {})


def test_seed_pending_ids_name_the_vertices_that_would_reattach():
    from egraph.graph import EvidenceGraph
    from egraph.seeds import seeds_for_batch
    g = EvidenceGraph()
    g.merge_nodes(["pod:ns:p1", "deployment:ns:d"], ["Pod", "Deployment"])
    ev = [[{"evidence_type": "kubernetes_event", "entity_namespace": "ns", "entity_name": "p1",
            "data": {"involved_object": {"kind": "Pod", "name": "p1", "namespace": "ns"}},
            "signal_strength": 0.9},
           {"evidence_type": "log_signal", "entity_namespace": "ns", "entity_name": "d",
            "signal_strength": 0.6},
           {"evidence_type": "kubernetes_pod", "entity_namespace": "ns", "entity_name": "gone",
            "signal_strength": 0.9},
           {"evidence_type": "kubernetes_pod", "entity_namespace": "ns", "entity_name": "p1",
            "signal_strength": 0.0}]]
    pend: list = []
    sv, sc, ss = seeds_for_batch(g, ev, pending=pend)
    assert sv.tolist() == [0, 1] and sc.tolist() == [0, 0]
    assert pend == [{"event:ns:p1", "logpattern:ns:d", "service:ns:d", "pod:ns:gone"}]
