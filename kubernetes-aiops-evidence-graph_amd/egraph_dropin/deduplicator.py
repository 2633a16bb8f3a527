"""Drop-in AlertDeduplicator (reference src/services/ingestion/deduplicator.py:15-140) backed by
the GPU TTL table (egraph.alerts.DedupTable, csrc/alerts.hip) instead of Redis.

Same coroutine API and results:
  check_duplicate(fp)            -> (is_duplicate, existing_incident_id | None)     (:41-71)
  register_fingerprint(fp, id, ttl=None) -> bool; SET EX int(ttl seconds), 4 h default (:73-104)
  remove_fingerprint(fp)         -> bool                                           (:106-118)
  extend_fingerprint(fp, ttl=None) -> bool, only when the key exists               (:120-140)
Redis details kept: EX is int(ttl.total_seconds()) seconds, and an EX <= 0 is an error the
reference catches (register returns False); EXPIRE with a non-positive TTL deletes the key
(extend returns True).  Any error inside a call fails open exactly as the reference's `except
Exception` does.

Table keys: a 32-character hex fingerprint (the normalizer's output) is its own 16 bytes; any
other string is keyed by the first 16 bytes of its SHA-256 (computed on the GPU).  Incident id
strings are interned into u32 handles here on the host.

Memory: the table compacts itself (expired keys drop out); the host keeps one interned id
string per incident ever registered (`_ids`, about 100 B each) until `reset()` -- a service that
opens 100k incidents a day holds ~10 MB after a day.  Recycling the handles of expired keys
needs a device-side remap of the table's incident column (not built).

Additive batch entry point: `ingest_batch` runs the webhook loop of
src/services/ingestion/main.py:141-170 (check -> create -> register, in payload order) for a
whole batch in three kernels (egr_dedup_ingest).
"""
from __future__ import annotations

import logging
import re
import time
import uuid
from datetime import timedelta

import torch

from egraph import alerts as _alerts

logger = logging.getLogger(__name__)
_HEX32 = re.compile(r"[0-9a-f]{32}")


def _redis_value(x) -> str:
    """The string a Redis SET stores for `x` and a decode_responses GET returns (redis-py's
    Encoder.encode): str as is, bytes decoded, int / float by repr; bool and any other type
    raise (DataError in redis-py), which the caller's fail-open turns into False."""
    if isinstance(x, str):
        return x
    if isinstance(x, (bytes, memoryview)):
        return bytes(x).decode()
    if isinstance(x, bool):
        raise TypeError("Invalid input of type: 'bool'. Convert to a bytes, string, int or float first.")
    if isinstance(x, (int, float)):
        return repr(x)
    raise TypeError(f"Invalid input of type: '{type(x).__name__}'. Convert to a bytes, string, "
                    "int or float first.")


class AlertDeduplicator:
    """Deduplicates alerts based on fingerprint (GPU TTL table)."""

    FINGERPRINT_TTL = timedelta(hours=4)
    CAPACITY = 1 << 20

    _table: _alerts.DedupTable | None = None
    _ids: list[str] = []
    _handles: dict[str, int] = {}

    @staticmethod
    def now_ms() -> int:
        """Wall clock in milliseconds (patch in tests)."""
        return int(time.time() * 1000)

    @classmethod
    def table(cls) -> _alerts.DedupTable:
        if cls._table is None:
            cls._table = _alerts.DedupTable(cls.CAPACITY)
        return cls._table

    @classmethod
    async def close(cls) -> None:
        """The reference's close() only disconnects from Redis (:33-39); its keys survive.  The
        table is this process's store, so close() releases nothing a later call would miss:
        registered fingerprints stay live across close / reuse.  reset() drops them."""

    @classmethod
    def reset(cls) -> None:
        """Drop every fingerprint and interned incident id (tests; FLUSHDB in Redis terms)."""
        cls._table = None
        cls._ids, cls._handles = [], {}

    @classmethod
    def keys(cls, fingerprints: list[str]) -> torch.Tensor:
        """[n, 16] uint8 table keys of fingerprint strings."""
        t = cls.table()
        if all(_HEX32.fullmatch(f) for f in fingerprints):
            return _alerts.fingerprints_from_hex(fingerprints, t.dev)
        other = [i for i, f in enumerate(fingerprints) if not _HEX32.fullmatch(f)]
        out = _alerts.fingerprints_from_hex(
            [f if _HEX32.fullmatch(f) else "0" * 32 for f in fingerprints], t.dev)
        hashed, _ = _alerts.fingerprints([fingerprints[i] for i in other], t.dev)
        out[torch.tensor(other, device=t.dev)] = hashed
        return out

    @classmethod
    def _intern(cls, incident_id: str) -> int:
        h = cls._handles.get(incident_id)
        if h is None:
            h = cls._handles[incident_id] = len(cls._ids)
            cls._ids.append(incident_id)
        return h

    # ---- the reference's API ----------------------------------------------------------------
    # Every method fails open exactly where the reference's does: any exception inside its try
    # (a device error, a key or TTL the store rejects, an incident id Redis cannot encode) is
    # logged and turned into the reference's failure result (deduplicator.py:68-71, :102-104,
    # :116-118, :138-140).  The fingerprint is formatted into the key as the reference's
    # f"aiops:fingerprint:{fingerprint}" does, so a non-str fingerprint is keyed by its str().
    @classmethod
    async def check_duplicate(cls, fingerprint: str) -> tuple[bool, str | None]:
        try:
            dup, inc = cls.table().lookup(cls.keys([f"{fingerprint}"]), cls.now_ms())
            if bool(dup[0]):
                existing = cls._ids[int(inc[0])]
                if existing:             # `if existing_id:` (:58): a stored "" is no duplicate
                    return True, existing
            return False, None
        except Exception as e:  # noqa: BLE001 -- fail open (:68-71)
            logger.error("dedup table error during deduplication: %s", e)
            return False, None

    @classmethod
    async def register_fingerprint(cls, fingerprint: str, incident_id: str,
                                   ttl: timedelta | None = None) -> bool:
        try:
            ttl = ttl or cls.FINGERPRINT_TTL
            ex = int(ttl.total_seconds())
            if ex <= 0:                  # Redis: "invalid expire time in 'set' command"
                raise ValueError("invalid expire time in 'set' command")
            h = cls._intern(_redis_value(incident_id))
            t = cls.table()
            t.register(cls.keys([f"{fingerprint}"]), cls.now_ms(), ex * 1000,
                       torch.tensor([h], dtype=torch.int64))
            return True
        except Exception as e:  # noqa: BLE001 -- (:102-104)
            logger.error("dedup table error during fingerprint registration: %s", e)
            return False

    @classmethod
    async def remove_fingerprint(cls, fingerprint: str) -> bool:
        try:
            cls.table().remove(cls.keys([f"{fingerprint}"]))
            return True
        except Exception as e:  # noqa: BLE001 -- (:116-118)
            logger.error("dedup table error during fingerprint removal: %s", e)
            return False

    @classmethod
    async def extend_fingerprint(cls, fingerprint: str, additional_ttl: timedelta | None = None) -> bool:
        try:
            ttl = additional_ttl or cls.FINGERPRINT_TTL
            ex = int(ttl.total_seconds())
            t, k, now = cls.table(), cls.keys([f"{fingerprint}"]), cls.now_ms()
            if ex <= 0:                  # EXPIRE with a non-positive TTL deletes the key
                dup, _ = t.lookup(k, now)
                if not bool(dup[0]):
                    return False
                t.remove(k)
                return True
            return bool(t.extend(k, now, ex * 1000)[0])
        except Exception as e:  # noqa: BLE001 -- (:138-140)
            logger.error("dedup table error during TTL extension: %s", e)
            return False

    # ---- batch: the webhook loop ------------------------------------------------------------
    @classmethod
    def ingest_batch(cls, keys: torch.Tensor, new_id=lambda: str(uuid.uuid4()),
                     ttl: timedelta | None = None, now_ms: int | None = None):
        """keys [n, 16] (from fingerprints / keys()) in payload order -> (is_duplicate bool [n],
        incident id per alert, list of the new incidents' ids in creation order).  New incident
        ids come from `new_id()` (uuid4 strings like create_incident)."""
        ex = int((ttl or cls.FINGERPRINT_TTL).total_seconds())
        if ex <= 0:
            raise ValueError("ttl must be at least one second")
        t = cls.table()
        t.next_id = len(cls._ids)
        dup, inc, n_new = t.ingest(keys, cls.now_ms() if now_ms is None else now_ms, ex * 1000)
        created = [new_id() for _ in range(n_new)]
        for s in created:
            cls._intern(s)
        ids = [cls._ids[h] for h in inc.cpu().tolist()]
        return dup.cpu(), ids, created


class RateLimiter:
    """Fixed-window rate limiter (reference deduplicator.py:143-176: INCR + EXPIRE per call).
    Host-side: one counter per key; the window restarts window_seconds after the last call,
    as the reference's EXPIRE on every call does."""

    _counters: dict[str, tuple[int, float]] = {}

    @classmethod
    async def check_rate_limit(cls, key: str, limit: int, window_seconds: int = 60) -> tuple[bool, int]:
        try:
            now = time.time()
            rk = f"aiops:ratelimit:{key}"
            count, until = cls._counters.get(rk, (0, 0.0))
            count = count + 1 if now < until else 1
            cls._counters[rk] = (count, now + window_seconds)
            return count <= limit, max(0, limit - count)
        except Exception as e:  # noqa: BLE001 -- fail open (:173-176)
            logger.error("rate limiter error: %s", e)
            return True, limit
