"""Generate the alert-storm golden fixtures (tests/golden/normalizer_cases.json,
tests/golden/storm_cases.json) by RUNNING THE REFERENCE.

Test infrastructure only: imports the reference from /root/reference (read-only, this container
only) and records its outputs as JSON.  Nothing here ships; the reference never travels.

Reference code executed:
  * src/services/ingestion/normalizer.py    AlertNormalizer.normalize_{alertmanager,grafana,
                                            prometheus} (:32-206), _generate_fingerprint
  * src/services/ingestion/deduplicator.py  AlertDeduplicator.check_duplicate /
                                            register_fingerprint / remove_fingerprint /
                                            extend_fingerprint (:41-140)
Restated here (the module cannot be imported: FastAPI app, database and Temporal clients): the
webhook loop of src/services/ingestion/main.py:141-170 -- skip non-firing alerts, normalize,
check_duplicate, skip duplicates, create the incident, register_fingerprint (create_incident,
:392).

Shims (none touches the logic under test): a no-op ``structlog``; ``datetime.UTC`` for Python
3.10; a ``redis.asyncio`` module and ``src.config.settings`` so deduplicator.py imports (the
client is replaced, as the reference's own tests/unit/test_deduplicator.py:31-36 do, by a fake
Redis -- here one that honours SET EX / EXPIRE against a simulated millisecond clock, the Redis
semantics: a key exists while now < set time + EX seconds; EXPIRE with a TTL <= 0 deletes it;
SET with EX <= 0 is an error).

Usage:  python oracle/gen_golden_alerts.py [--ref /root/reference]
"""
from __future__ import annotations

import argparse
import asyncio
import datetime as _dt
import importlib.util
import json
import random
import sys
import types
from pathlib import Path

sys.dont_write_bytecode = True
REPO = Path(__file__).resolve().parents[1]
GOLDEN = REPO / "tests" / "golden"
SEED = 20260905


def _install_shims() -> None:
    class _NoLog:
        def __getattr__(self, _name):
            return lambda *a, **k: None

    stub = types.ModuleType("structlog")
    stub.get_logger = lambda *a, **k: _NoLog()
    sys.modules["structlog"] = stub
    if not hasattr(_dt, "UTC"):
        _dt.UTC = _dt.timezone.utc
    redis = types.ModuleType("redis")
    redis_async = types.ModuleType("redis.asyncio")
    redis_async.Redis = object
    redis_async.from_url = lambda *a, **k: None
    redis.asyncio = redis_async
    sys.modules["redis"], sys.modules["redis.asyncio"] = redis, redis_async
    cfg = types.ModuleType("src.config")
    cfg.settings = types.SimpleNamespace(redis_connection_url="redis://unused")
    sys.modules["src.config"] = cfg


def _load(path: Path, name: str):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class ClockRedis:
    """Fake redis.asyncio client with SET EX / EXPIRE honoured against `now_ms`."""

    def __init__(self):
        self.store: dict[str, tuple[str, int]] = {}
        self.now_ms = 0

    def _live(self, key):
        v = self.store.get(key)
        if v is not None and self.now_ms >= v[1]:
            del self.store[key]
            v = None
        return v

    async def get(self, key):
        v = self._live(key)
        return None if v is None else v[0]

    async def set(self, key, value, ex=None):
        if ex is not None and ex <= 0:
            raise ValueError("invalid expire time in 'set' command")
        self.store[key] = (value, self.now_ms + ex * 1000 if ex else 1 << 62)

    async def delete(self, key):
        self.store.pop(key, None)

    async def exists(self, key):
        return self._live(key) is not None

    async def expire(self, key, ttl):
        v = self._live(key)
        if v is None:
            return False
        if ttl <= 0:
            del self.store[key]
        else:
            self.store[key] = (v[0], self.now_ms + ttl * 1000)
        return True


def _labels(rng: random.Random, keys: list[tuple]) -> dict:
    lab = {}
    name, ns, svc = keys[rng.randrange(len(keys))]
    if rng.random() < 0.9:
        lab["alertname"] = name
    if rng.random() < 0.8:
        lab["namespace"] = ns
    r = rng.random()
    if r < 0.5:
        lab["service"] = svc
    elif r < 0.6:
        lab["job"] = svc + "-job"
    elif r < 0.7:
        lab["deployment"] = svc + "-deploy"
    elif r < 0.75:
        lab["instance"] = "10.0.0.%d:9100" % rng.randrange(255)
    elif r < 0.8:
        lab["grafana_folder"] = "folder-" + svc
    if rng.random() < 0.3:
        lab["pod"] = f"{svc}-{rng.randrange(1000):03d}"
    r = rng.random()
    if r < 0.5:
        lab["cluster"] = "c%d" % rng.randrange(3)
    elif r < 0.6:
        lab["kubernetes_cluster"] = "k%d" % rng.randrange(3)
    if rng.random() < 0.85:
        lab["severity"] = rng.choice(["critical", "HIGH", "warning", "info", "Low", "alerting",
                                      "error", "warn", "page", "Critical"])
    return lab


def _alert(rng: random.Random, keys) -> dict:
    a = {"labels": _labels(rng, keys), "annotations": {}}
    if rng.random() < 0.5:
        a["annotations"]["summary"] = "summary %d" % rng.randrange(100)
    if rng.random() < 0.5:
        a["annotations"]["description"] = "description %d" % rng.randrange(100)
    r = rng.random()
    if r < 0.5:
        a["startsAt"] = "2026-0%d-1%dT0%d:00:00Z" % (rng.randrange(1, 10), rng.randrange(10), rng.randrange(10))
    elif r < 0.6:
        a["startsAt"] = "2026-01-05T05:00:00.123+00:00"
    elif r < 0.7:
        a["startsAt"] = "not-a-time"
    if rng.random() < 0.1:
        a["alertname"] = "top-level-name"
    a["status"] = "firing" if rng.random() < 0.85 else "resolved"
    return a


def _record(inc) -> dict:
    d = inc.model_dump(mode="json")
    return {k: d[k] for k in ("fingerprint", "title", "description", "severity", "source", "cluster",
                              "namespace", "service", "labels", "annotations")} | {
        "started_at": d["started_at"]}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()
    ref = Path(args.ref)
    _install_shims()
    sys.path.insert(0, str(ref))
    nm = _load(ref / "src/services/ingestion/normalizer.py", "ref_normalizer").AlertNormalizer
    dd = _load(ref / "src/services/ingestion/deduplicator.py", "ref_deduplicator").AlertDeduplicator
    rng = random.Random(SEED)
    keys = [(f"Alert{i % 13}", f"ns{i % 7}", f"svc{i % 17}") for i in range(40)]

    # ---- normalizer cases --------------------------------------------------------------
    cases = []
    for i in range(300):
        src = ("alertmanager", "grafana", "prometheus")[i % 3]
        alert = _alert(rng, keys)
        payload = {}
        if src == "grafana" and rng.random() < 0.6:
            payload["commonLabels"] = _labels(rng, keys)
            if rng.random() < 0.5:
                payload["commonAnnotations"] = {"summary": "common summary"}
        if src == "alertmanager":
            out = nm.normalize_alertmanager(alert, payload)
        elif src == "grafana":
            out = nm.normalize_grafana(alert, payload)
        else:
            out = nm.normalize_prometheus(alert)
        rec = _record(out)
        # started_at is datetime.now() when missing / unparseable: not comparable
        parsed = src != "prometheus" and "startsAt" in alert and alert["startsAt"] != "not-a-time"
        if not parsed:
            rec["started_at"] = None
        cases.append({"source": src, "alert": alert, "payload": payload, "expected": rec})
    (GOLDEN / "normalizer_cases.json").write_text(json.dumps(cases) + "\n")

    # ---- storm: the webhook loop over ticks, TTL expiry, remove / extend ----------------
    fake = ClockRedis()
    dd._redis_client = fake
    ttl_s = int(dd.FINGERPRINT_TTL.total_seconds())
    zipf_w = [1.0 / (r + 1) ** 1.1 for r in range(len(keys))]
    created: list[str] = []
    ticks = []

    async def run():
        t_ms = 1_700_000_000_000
        for tick in range(60):
            # gaps of up to ~3 h, so 4 h TTLs expire inside the sequence
            t_ms += rng.choice([1000, 1000, 60_000, 3_600_000, 2 * 3_600_000 + 7])
            fake.now_ms = t_ms
            n = rng.randrange(0, 40)
            alerts = []
            for _ in range(n):
                a = _alert(rng, keys)
                name, ns, svc = rng.choices(keys, weights=zipf_w)[0]
                a["labels"].update(alertname=name, namespace=ns, service=svc)
                a["labels"].pop("pod", None)
                alerts.append(a)
            ops = []
            if created and rng.random() < 0.3:      # resolve: remove a fingerprint
                k = rng.choice(keys)
                fp = nm._generate_fingerprint("alertmanager", *k)
                await dd.remove_fingerprint(fp)
                ops.append({"op": "remove", "fingerprint": fp})
            if created and rng.random() < 0.3:      # extend
                k = rng.choice(keys)
                fp = nm._generate_fingerprint("alertmanager", *k)
                sec = rng.choice([60, 3600, 4 * 3600, 0])
                ok = await dd.extend_fingerprint(fp, _dt.timedelta(seconds=sec) if sec else None)
                ops.append({"op": "extend", "fingerprint": fp, "ttl_s": sec or ttl_s, "ok": ok})
            out = []
            for a in alerts:                          # main.py:141-170
                if a.get("status") != "firing":
                    out.append(None)
                    continue
                inc = nm.normalize_alertmanager(a, {"alerts": alerts})
                dup, existing = await dd.check_duplicate(inc.fingerprint)
                if dup:
                    out.append({"fingerprint": inc.fingerprint, "dup": True, "incident": existing})
                    continue
                iid = f"inc-{len(created)}"
                created.append(iid)
                await dd.register_fingerprint(inc.fingerprint, iid)
                out.append({"fingerprint": inc.fingerprint, "dup": False, "incident": iid})
            ticks.append({"now_ms": t_ms, "ops": ops, "alerts": alerts, "expected": out})

    asyncio.run(run())
    (GOLDEN / "storm_cases.json").write_text(json.dumps({"ttl_s": ttl_s, "ticks": ticks}) + "\n")
    print(f"wrote {len(cases)} normalizer cases, {len(ticks)} storm ticks "
          f"({sum(len(t['alerts']) for t in ticks)} alerts, {len(created)} incidents) -> {GOLDEN}")


if __name__ == "__main__":
    main()
