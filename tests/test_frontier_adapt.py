"""Frontier.adapt()'s table choice (host logic only, no GPU): the wide retry on after a run with
overflowing columns, the mid table first when most columns overflowed the narrow one, and one
second look that moves to wide-first only if most columns overflow the mid table too
(egraph/graph.py Frontier.adapt; the device side is tests/test_configs_gpu.py::test_c4_frontier_b256)."""
from __future__ import annotations

import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "kubernetes-aiops-evidence-graph_amd"))

from egraph.graph import Frontier  # noqa: E402


class _Probe(Frontier):
    """A Frontier without a device handle: the two setters record instead of calling the library."""

    def __init__(self, B: int, pool_entries: int = -1):
        self.B = B
        self.pool_entries = pool_entries
        self.retry_blocks = 0
        self.wide_first = self.FIRST_NARROW
        self._mid_checked = False
        self._adapt_calls = 0
        self.calls = []

    def __del__(self):
        pass

    def set_retry(self, blocks: int) -> None:
        self.calls.append(("retry", blocks))
        self.retry_blocks = blocks

    def set_wide_first(self, mode: int) -> None:
        self.calls.append(("first", int(mode)))
        self.wide_first = int(mode)

    def set_continuation(self, regions: int) -> None:
        self.calls.append(("continuation", regions))


def _st(overflowed: int) -> dict:
    return {"overflowed": overflowed}


def test_no_overflow_keeps_narrow():
    f = _Probe(1024)
    assert not f.adapt(_st(0))
    assert f.calls == [] and f.wide_first == f.FIRST_NARROW


def test_few_overflows_retry_only():
    f = _Probe(1024)
    assert f.adapt(_st(115))                         # C3: ~0.5 % of the columns
    # (overflowing columns continue in global-memory regions inside the grid, unless switched off)
    assert f.calls == [("retry", min(f.RETRY_BLOCKS, 1024))] + (
        [("continuation", f.CONTINUATION_REGIONS)] if f.CONTINUATION_REGIONS > 0 else [])
    assert f.wide_first == f.FIRST_NARROW
    n = len(f.calls)
    assert not f.adapt(_st(1000))                    # settled: no second look in narrow mode
    assert len(f.calls) == n


def test_most_overflow_mid_first_then_kept():
    f = _Probe(1024)
    assert f.adapt(_st(1018))                        # C4 in the narrow table
    assert f.wide_first == f.FIRST_MID and f.retry_blocks > 0
    assert not f.adapt(_st(78))                      # C4 in the mid table: 7.6 % overflow
    assert f.wide_first == f.FIRST_MID and f._mid_checked
    assert not f.adapt(_st(1024))                    # one look only
    assert f.wide_first == f.FIRST_MID


def test_mid_overflowing_moves_to_wide_first():
    f = _Probe(256)
    assert f.adapt(_st(250))
    assert f.adapt(_st(200))                         # most overflow the mid table too
    assert f.wide_first == f.FIRST_WIDE
    assert not f.adapt(_st(256))


def test_member_pool_frontiers_never_adapt():
    f = _Probe(1024, pool_entries=0)
    assert not f.adapt(_st(1024)) and f.calls == []


def test_periodic_stats_reads_only():
    # without explicit stats, adapt() reads the counters (a synchronising read) on calls 1, 17, ...
    f = _Probe(1024)
    reads = []
    f.stats = lambda stream=None: reads.append(1) or _st(0)
    for _ in range(20):
        f.adapt()
    assert len(reads) == 2
