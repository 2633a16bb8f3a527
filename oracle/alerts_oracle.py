"""ORACLE (test infrastructure only) for the alert-storm front end: a CPU restatement of the
reference's fingerprint, Redis-TTL deduplication and webhook loop.  Only tests/ and bench.py's
cpu_baseline leg import it; the product path is csrc/alerts.hip.

  fingerprint     src/services/ingestion/normalizer.py:208-218 (hashlib SHA-256, 32 hex chars)
  TTLStore        the Redis commands AlertDeduplicator issues (deduplicator.py:41-140):
                  GET, SET EX (EX <= 0 is an error), DEL, EXISTS + EXPIRE (TTL <= 0 deletes);
                  a key exists while now_ms < set time + EX seconds
  webhook_loop    src/services/ingestion/main.py:141-170 + create_incident's registration
                  (:392): per alert in order, a live fingerprint is a duplicate of its
                  incident; otherwise a new incident is created and registered.
Pinned by tests/golden/fingerprints.json and tests/golden/storm_cases.json, which were produced by
running the reference (oracle/gen_golden.py, oracle/gen_golden_alerts.py).
"""
from __future__ import annotations

import hashlib


def fingerprint(key: str | bytes) -> str:
    b = key.encode() if isinstance(key, str) else key
    return hashlib.sha256(b).hexdigest()[:32]


class TTLStore:
    def __init__(self):
        self.kv: dict[str, tuple[object, int]] = {}

    def get(self, key, now_ms):
        v = self.kv.get(key)
        if v is None or now_ms >= v[1]:
            return None
        return v[0]

    def set(self, key, value, now_ms, ex_s):
        if ex_s <= 0:
            raise ValueError("invalid expire time")
        self.kv[key] = (value, now_ms + ex_s * 1000)

    def delete(self, key):
        self.kv.pop(key, None)

    def expire(self, key, now_ms, ttl_s) -> bool:
        if self.get(key, now_ms) is None:
            return False
        if ttl_s <= 0:
            del self.kv[key]
        else:
            self.kv[key] = (self.kv[key][0], now_ms + ttl_s * 1000)
        return True


def webhook_loop(store: TTLStore, fps: list, now_ms: int, ttl_s: int, first_id: int):
    """-> (dup flags, incident per alert, number of new incidents); new incidents are numbered
    first_id, first_id + 1, ... in creation order."""
    dup, inc = [], []
    nxt = first_id
    for fp in fps:
        e = store.get(fp, now_ms)
        if e is not None:
            dup.append(True)
            inc.append(e)
            continue
        store.set(fp, nxt, now_ms, ttl_s)
        dup.append(False)
        inc.append(nxt)
        nxt += 1
    return dup, inc, nxt - first_id
