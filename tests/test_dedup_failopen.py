"""AlertDeduplicator / RateLimiter fail open exactly where the reference's do (reference
src/services/ingestion/deduplicator.py:52-71, :88-104, :106-118, :120-140, :159-176: every
method wraps its whole body in `except Exception` and returns (False, None) / False / (True,
limit)).  Host logic only: the TTL table is replaced by a stand-in (its GPU parity is
tests/test_alerts_gpu.py)."""
from __future__ import annotations

import asyncio
from datetime import timedelta

import pytest


class _Table:
    """Stand-in TTL table: a dict of key -> (incident handle, expiry ms)."""

    def __init__(self, fail=None):
        self.d, self.fail = {}, fail

    def _maybe_fail(self):
        if self.fail is not None:
            raise self.fail

    def lookup(self, keys, now):
        self._maybe_fail()
        v = self.d.get(keys[0])
        return ([v is not None and v[1] > now], [v[0] if v else 0])

    def register(self, keys, now, ttl_ms, handles):
        self._maybe_fail()
        self.d[keys[0]] = (int(handles[0]), now + ttl_ms)

    def remove(self, keys):
        self._maybe_fail()
        self.d.pop(keys[0], None)

    def extend(self, keys, now, ttl_ms):
        self._maybe_fail()
        v = self.d.get(keys[0])
        if v is None or v[1] <= now:
            return [False]
        self.d[keys[0]] = (v[0], now + ttl_ms)
        return [True]


@pytest.fixture
def D(monkeypatch):
    from src.services.ingestion.deduplicator import AlertDeduplicator as D
    D.reset()
    tab = _Table()
    monkeypatch.setattr(D, "table", classmethod(lambda cls: tab))
    monkeypatch.setattr(D, "keys", classmethod(lambda cls, fps: [str(f) for f in fps]))
    monkeypatch.setattr(D, "now_ms", staticmethod(lambda: 1_000_000))
    D._tab = tab
    yield D
    D.reset()


def run(c):
    return asyncio.run(c)


def test_round_trip_with_stand_in_table(D):
    assert run(D.check_duplicate("fp")) == (False, None)
    assert run(D.register_fingerprint("fp", "inc-1")) is True
    assert run(D.check_duplicate("fp")) == (True, "inc-1")
    assert run(D.extend_fingerprint("fp")) is True
    assert run(D.remove_fingerprint("fp")) is True
    assert run(D.check_duplicate("fp")) == (False, None)
    assert run(D.extend_fingerprint("fp")) is False


@pytest.mark.parametrize("exc", [RuntimeError("device"), ValueError("bad key"), KeyError("k"),
                                 TypeError("odd"), OSError("io")])
def test_table_errors_fail_open(D, exc):
    D._tab.fail = exc
    assert run(D.check_duplicate("fp")) == (False, None)
    assert run(D.register_fingerprint("fp", "inc-1")) is False
    assert run(D.remove_fingerprint("fp")) is False
    assert run(D.extend_fingerprint("fp")) is False


def test_key_errors_fail_open(D, monkeypatch):
    def bad_keys(cls, fps):
        raise ValueError("EGR_EINVAL: malformed key")
    monkeypatch.setattr(D, "keys", classmethod(bad_keys))
    assert run(D.check_duplicate("fp")) == (False, None)
    assert run(D.register_fingerprint("fp", "inc-1")) is False
    assert run(D.remove_fingerprint("fp")) is False
    assert run(D.extend_fingerprint("fp")) is False


def test_real_keys_on_odd_input_fail_open():
    """Without a GPU the real table cannot even be created: every call still fails open, as the
    reference's do when Redis is unreachable."""
    from src.services.ingestion.deduplicator import AlertDeduplicator as D
    D.reset()
    try:
        assert run(D.check_duplicate(object())) == (False, None)
        assert run(D.register_fingerprint(12345, "inc")) is False
        assert run(D.remove_fingerprint(None)) is False
        assert run(D.extend_fingerprint(b"\xff")) is False
    finally:
        D.reset()


def test_ttl_errors_fail_open(D):
    # a non-timedelta TTL raises inside the reference's try (ttl.total_seconds()): False
    assert run(D.register_fingerprint("fp", "inc-1", ttl=3600)) is False
    assert run(D.extend_fingerprint("fp", additional_ttl="4h")) is False
    # SET EX 0 / negative: Redis rejects it ("invalid expire time"), the reference returns False
    assert run(D.register_fingerprint("fp", "inc-1", ttl=timedelta(milliseconds=500))) is False
    assert run(D.register_fingerprint("fp", "inc-1", ttl=timedelta(seconds=-5))) is False
    # timedelta(0) is falsy: `ttl or FINGERPRINT_TTL` takes the 4 h default
    assert run(D.register_fingerprint("fp", "inc-1", ttl=timedelta(0))) is True
    assert D._tab.d["fp"][1] == 1_000_000 + 4 * 3600 * 1000


def test_incident_id_encoding_follows_redis(D):
    """redis-py stores str / bytes / int / float (int and float by repr) and refuses bool and
    other types with DataError, which the reference's except turns into False."""
    assert run(D.register_fingerprint("a", 17)) is True
    assert run(D.check_duplicate("a")) == (True, "17")
    assert run(D.register_fingerprint("b", 2.5)) is True
    assert run(D.check_duplicate("b")) == (True, "2.5")
    assert run(D.register_fingerprint("c", b"inc-c")) is True
    assert run(D.check_duplicate("c")) == (True, "inc-c")
    assert run(D.register_fingerprint("d", True)) is False
    assert run(D.register_fingerprint("e", ["x"])) is False
    assert run(D.check_duplicate("d")) == (False, None)


def test_empty_incident_id_is_not_a_duplicate(D):
    """`if existing_id:` (:58): a stored empty string reads as no duplicate."""
    assert run(D.register_fingerprint("fp", "")) is True
    assert run(D.check_duplicate("fp")) == (False, None)


def test_non_str_fingerprint_is_formatted_into_the_key(D):
    """f"aiops:fingerprint:{fingerprint}": 42 and "42" name the same key."""
    assert run(D.register_fingerprint(42, "inc-42")) is True
    assert run(D.check_duplicate("42")) == (True, "inc-42")


def test_rate_limiter_fails_open():
    from src.services.ingestion.deduplicator import RateLimiter
    RateLimiter._counters.clear()
    assert run(RateLimiter.check_rate_limit("k", 2)) == (True, 1)
    # limit - count raises TypeError inside the reference's try: (True, limit)
    assert run(RateLimiter.check_rate_limit("k2", "3")) == (True, "3")
    assert run(RateLimiter.check_rate_limit("k3", 5, window_seconds="60")) == (True, 5)
    RateLimiter._counters.clear()
