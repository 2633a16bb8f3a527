"""Alert-storm front end on the GPU (csrc/alerts.hip through the C-ABI): fingerprints bit-exact
against hashlib and the reference's vectors, the TTL table replaying the reference's webhook loop
(tests/golden/storm_cases.json), the drop-in AlertNormalizer / AlertDeduplicator, and large
batches against the oracle."""
from __future__ import annotations

import asyncio
from datetime import timedelta

import numpy as np
import pytest
import torch

import alerts_oracle as AO

pytestmark = pytest.mark.gpu


def _hex_of(fp16: torch.Tensor) -> list[str]:
    return [bytes(r).hex() for r in fp16.cpu().numpy()]


def test_fingerprint_kernel_matches_reference_vectors(golden):
    from egraph import alerts
    keys = [":".join(f["key"]) for f in golden["fingerprints"]]
    fp, hx = alerts.fingerprints(keys, hex=True)
    want = [f["fingerprint"] for f in golden["fingerprints"]]
    assert hx == want
    assert _hex_of(fp) == want


def test_fingerprint_kernel_lengths_and_bytes():
    """Every padding case (0..300 bytes: one, two and many 64-byte blocks, the 55/56 boundary),
    non-ASCII UTF-8 and arbitrary bytes."""
    from egraph import alerts
    rng = np.random.default_rng(3)
    keys: list = [bytes(rng.integers(0, 256, n, dtype=np.uint8)) for n in range(0, 301)]
    keys += ["é:ü:名前:" * k for k in range(1, 9)] + [""]
    fp, hx = alerts.fingerprints(keys, hex=True)
    assert hx == [AO.fingerprint(k) for k in keys]
    assert _hex_of(fp) == hx


def test_fingerprint_empty_batch():
    from egraph import alerts
    fp, hx = alerts.fingerprints([], hex=True)
    assert fp.shape == (0, 16) and hx == []


def test_normalizer_matches_reference_cases(golden):
    from src.services.ingestion.normalizer import AlertNormalizer
    for src in ("alertmanager", "grafana", "prometheus"):
        cases = [c for c in golden["normalizer"] if c["source"] == src]
        if src == "alertmanager":
            got = [AlertNormalizer.normalize_alertmanager_batch([c["alert"]], c["payload"])[0] for c in cases[:5]]
            got += [AlertNormalizer.normalize_alertmanager(c["alert"], c["payload"]) for c in cases[5:]]
        elif src == "grafana":
            got = [AlertNormalizer.normalize_grafana(c["alert"], c["payload"]) for c in cases]
        else:
            got = AlertNormalizer.normalize_prometheus_batch([c["alert"] for c in cases])
        for c, inc in zip(cases, got):
            d = inc.model_dump(mode="json")
            for k, v in c["expected"].items():
                if k == "started_at" and v is None:
                    continue
                assert d[k] == v, (c, k)


def test_reference_normalizer_unit_cases():
    """The reference's tests/unit/test_normalizer.py:6-77, through the drop-in."""
    from src.models import IncidentSeverity, IncidentSource
    from src.services.ingestion.normalizer import AlertNormalizer
    alert = {"status": "firing",
             "labels": {"alertname": "PodCrashLooping", "namespace": "prod", "cluster": "us-east-1",
                        "service": "api-server", "severity": "critical"},
             "annotations": {"summary": "Pod is crash looping"}, "startsAt": "2026-01-05T05:00:00Z"}
    inc = AlertNormalizer.normalize_alertmanager(alert, {"receiver": "aiops", "alerts": [alert]})
    assert inc.title == "PodCrashLooping: api-server"
    assert inc.severity == IncidentSeverity.CRITICAL and inc.source == IncidentSource.ALERTMANAGER
    assert inc.namespace == "prod" and inc.cluster == "us-east-1"
    a = {"labels": {"alertname": "PodCrashLooping", "namespace": "prod", "service": "api-server"},
         "annotations": {}}
    b = {"labels": {"alertname": "PodCrashLooping", "namespace": "prod", "service": "worker"},
         "annotations": {}}
    assert AlertNormalizer.normalize_alertmanager(a, {}).fingerprint == \
        AlertNormalizer.normalize_alertmanager(dict(a), {}).fingerprint
    assert AlertNormalizer.normalize_alertmanager(a, {}).fingerprint != \
        AlertNormalizer.normalize_alertmanager(b, {}).fingerprint
    g = AlertNormalizer.normalize_grafana(
        {"labels": {"severity": "alerting"}, "annotations": {}},
        {"commonLabels": {"alertname": "HighLatency", "namespace": "prod"},
         "commonAnnotations": {"summary": "Latency is high"}})
    assert g.title == "Latency is high" and g.namespace == "prod"
    assert g.severity == IncidentSeverity.HIGH
    d = AlertNormalizer.normalize_alertmanager({"labels": {}, "annotations": {}}, {})
    assert d.title == "Unknown Alert" and d.namespace == "default"
    assert d.severity == IncidentSeverity.MEDIUM
    assert AlertNormalizer._generate_fingerprint("grafana", "Alert0", "ns0", "svc0") == \
        "2b5f39954f21375be8484d70cf5205c2"


def test_dedup_table_replays_reference_storm(golden):
    """The webhook loop of the reference over 60 ticks (TTL expiry, DEL, EXPIRE), one ingest
    launch per tick."""
    from egraph import alerts
    storm = golden["storm"]
    t = alerts.DedupTable(capacity=4096)
    ttl_ms = storm["ttl_s"] * 1000
    names: dict[int, str] = {}
    n_created = 0
    for tick in storm["ticks"]:
        now = tick["now_ms"]
        for op in tick["ops"]:
            k = alerts.fingerprints_from_hex([op["fingerprint"]])
            if op["op"] == "remove":
                t.remove(k)
            else:
                assert bool(t.extend(k, now, op["ttl_s"] * 1000)[0]) == op["ok"]
        firing = [e for e in tick["expected"] if e is not None]
        keys = alerts.fingerprints_from_hex([e["fingerprint"] for e in firing])
        dup, inc, n_new = t.ingest(keys, now, ttl_ms)
        for h in range(n_created, n_created + n_new):
            names[h] = f"inc-{h}"
        n_created += n_new
        dup, inc = dup.cpu().tolist(), inc.cpu().tolist()
        for e, d, i in zip(firing, dup, inc):
            assert d == e["dup"]
            assert names[i] == e["incident"]
    assert n_created == 225


def test_dedup_large_batches_match_oracle():
    """200k alerts over Zipf(1.1) keys in batches of 50k, with clock jumps past the TTL."""
    from egraph import alerts
    rng = np.random.default_rng(11)
    n_keys = 20000
    ranks = np.arange(1, n_keys + 1)
    p = 1.0 / ranks ** 1.1
    p /= p.sum()
    keys = [f"alertmanager:A{i % 97}:ns{i % 31}:svc{i}" for i in range(n_keys)]
    fp_all, hx_all = alerts.fingerprints(keys, hex=True)
    t = alerts.DedupTable(capacity=n_keys)
    store = AO.TTLStore()
    ttl_s = 60
    now = 1_000_000
    nxt = 0
    for b in range(4):
        now += [1000, 30_000, 61_000, 5][b]
        pick = rng.choice(n_keys, size=50_000, p=p)
        dup, inc, n_new = t.ingest(fp_all[torch.from_numpy(pick).to(fp_all.device)], now, ttl_s * 1000)
        edup, einc, en = AO.webhook_loop(store, [hx_all[i] for i in pick], now, ttl_s, nxt)
        assert n_new == en
        np.testing.assert_array_equal(dup.cpu().numpy(), np.array(edup))
        np.testing.assert_array_equal(inc.cpu().numpy(), np.array(einc))
        nxt += en
    st = t.stats(now)
    assert st["live"] == sum(1 for v in store.kv.values() if now < v[1])
    t.compact(now)
    assert t.stats(now)["live"] == st["live"] == t.stats(now)["used_slots"]
    dup, inc = t.lookup(fp_all, now)
    for i in rng.choice(n_keys, 500):
        e = store.get(hx_all[i], now)
        assert bool(dup[i]) == (e is not None)
        if e is not None:
            assert int(inc[i]) == e


def test_dedup_table_full_fails_loudly():
    from egraph import alerts
    t = alerts.DedupTable(capacity=16, auto_compact=False)   # 64 slots
    fp, _ = alerts.fingerprints([f"k{i}" for i in range(100)])
    with pytest.raises(MemoryError):
        t.ingest(fp, 0, 1000)


def test_alert_deduplicator_reference_unit_cases(monkeypatch):
    """The reference's tests/unit/test_deduplicator.py:39-74 through the drop-in, plus the TTL
    behaviour its fake Redis does not model."""
    from src.services.ingestion.deduplicator import AlertDeduplicator as D
    D.reset()
    clock = [5_000_000]
    monkeypatch.setattr(D, "now_ms", staticmethod(lambda: clock[0]))
    run = asyncio.run
    assert run(D.check_duplicate("fp-1")) == (False, None)
    assert run(D.register_fingerprint("fp-1", "incident-123"))
    assert run(D.check_duplicate("fp-1")) == (True, "incident-123")
    assert run(D.remove_fingerprint("fp-1"))
    assert run(D.check_duplicate("fp-1"))[0] is False
    # default TTL 4 h = 14400 s
    fp = "0123456789abcdef0123456789abcdef"
    assert run(D.register_fingerprint(fp, "i-2"))
    clock[0] += 14400 * 1000 - 1
    assert run(D.check_duplicate(fp)) == (True, "i-2")
    clock[0] += 1
    assert run(D.check_duplicate(fp)) == (False, None)
    # extend only when live; EX <= 0 is rejected by SET; EXPIRE <= 0 deletes
    assert run(D.extend_fingerprint(fp)) is False
    assert run(D.register_fingerprint(fp, "i-3", ttl=timedelta(seconds=10)))
    assert run(D.extend_fingerprint(fp, timedelta(seconds=100)))
    clock[0] += 50_000
    assert run(D.check_duplicate(fp)) == (True, "i-3")
    assert run(D.register_fingerprint(fp, "i-4", ttl=timedelta(milliseconds=500))) is False
    assert run(D.extend_fingerprint(fp, timedelta(seconds=-1))) is True
    assert run(D.check_duplicate(fp)) == (False, None)
    # re-registering overwrites (SET)
    assert run(D.register_fingerprint("fp-1", "a")) and run(D.register_fingerprint("fp-1", "b"))
    assert run(D.check_duplicate("fp-1")) == (True, "b")
    # the batch webhook loop
    from egraph import alerts
    keys = D.keys(["x", "y", "x", "fp-1", "y"])
    dup, ids, created = D.ingest_batch(keys, new_id=iter(["n1", "n2"]).__next__)
    assert dup.tolist() == [False, False, True, True, True]
    assert ids == ["n1", "n2", "n1", "b", "n2"] and created == ["n1", "n2"]
    assert alerts.NO_INCIDENT == 0xFFFFFFFF
    # close() only disconnects, as the reference's Redis client close: keys survive
    run(D.close())
    assert run(D.check_duplicate("fp-1")) == (True, "b")
    D.reset()
    assert run(D.check_duplicate("fp-1")) == (False, None)


def test_dedup_auto_compaction_expiring_keys():
    """More distinct fingerprints than the capacity, through expiring TTLs: the table compacts
    itself (no MemoryError, no unbounded growth) and every decision still equals the oracle
    webhook loop (slots were never reclaimed)."""
    import alerts_oracle as AO
    from egraph import alerts
    t = alerts.DedupTable(capacity=64)           # 128 slots
    slots0 = t.stats(0)["slots"]
    store = AO.TTLStore()
    nxt = 0
    now = 1_000_000
    for tick in range(40):                       # 40 x 60 fresh keys, 10 s TTL, 4 s per tick
        now += 4000
        keys = [f"alertmanager:A:ns:{tick}-{i % 50}" for i in range(60)]
        fp, hx = alerts.fingerprints(keys, hex=True)
        t.next_id = nxt
        dup, inc, n_new = t.ingest(fp, now, 10_000)
        edup, einc, en = AO.webhook_loop(store, hx, now, 10, nxt)
        assert n_new == en
        np.testing.assert_array_equal(dup.cpu().numpy(), np.array(edup))
        np.testing.assert_array_equal(inc.cpu().numpy(), np.array(einc))
        nxt += en
    assert t.compactions > 0
    assert t.stats(now)["slots"] <= 4 * slots0   # live keys stay ~3 ticks' worth


def test_dedup_auto_compaction_grows_for_live_keys():
    """Live keys beyond the requested capacity: the table grows instead of filling up."""
    from egraph import alerts
    t = alerts.DedupTable(capacity=16)
    fp, _ = alerts.fingerprints([f"k{i}" for i in range(1000)])
    dup, inc, n_new = t.ingest(fp, 0, 10**9)
    assert n_new == 1000 and not dup.any()
    assert t.stats(1)["live"] == 1000
    dup, inc = t.lookup(fp, 1)
    assert dup.all() and sorted(inc.cpu().tolist()) == list(range(1000))
