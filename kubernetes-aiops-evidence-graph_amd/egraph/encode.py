"""Evidence dicts -> the 20-byte row columns consumed by egr_rules_eval.

Host side of the rules path: per row, the string / dict predicates of
RulesEngine._process_*_evidence (src/services/rca/rules_engine.py:294-376) are resolved to
bits; every per-incident reduction (set unions, counters, pods_by_node, the error sum), the
rule matching, confidences and both sorts run on the GPU.

Error behaviour follows the reference row by row: the same Python expressions are evaluated
in the same order, so a row that makes the reference raise (restart_count=None,
query_name=None, data=None on a known type, a latency metric whose current_value is None, ...)
raises the same exception type here, before anything reaches the device.

`encode_batch` runs the rows through the native encoder (csrc/pyhost.c, `encode_rows`): a row
whose values are all plain built-in types is encoded there; any other row is handed to
`_RowEncoder.row` below, the Python statement of the same predicates, which also raises what
the reference raises.  `encode_batch_py` is the all-Python encoder the tests check it against.
"""
from __future__ import annotations

import os

from dataclasses import dataclass

import numpy as np

from . import _lib as L
from .catalog import Catalog

_INT_LIMIT = 1 << 31   # |count| below this is summed exactly in any order on the device


@dataclass
class EncodedBatch:
    """Columns of a batch of incidents (host numpy arrays)."""
    flags: np.ndarray      # u32 [rows]
    vocab: np.ndarray      # u32 [rows]
    node: np.ndarray       # u32 [rows]
    err: np.ndarray        # f64 [rows]
    seg_off: np.ndarray    # i64 [incidents + 1]
    evidence_ids: list     # per incident: first five evidence ids (rules_engine.py:395)

    @property
    def n_incidents(self) -> int:
        return len(self.seg_off) - 1

    @property
    def n_rows(self) -> int:
        return int(self.seg_off[-1])


def _is_number(x) -> bool:
    return isinstance(x, (int, float))


class _RowEncoder:
    """Per-row predicate evaluation; one instance per batch (node keys are batch-global)."""

    def __init__(self, cat: Catalog):
        self.waiting = cat.waiting_vocab
        self.terminated = cat.terminated_vocab
        self.patterns = cat.pattern_vocab
        self.node_keys: dict = {}
        self._dispatch = None

    @property
    def dispatch(self) -> dict:
        """evidence_type -> processor (built on first use: the native encoder needs it only
        for the rows it hands over)"""
        if self._dispatch is None:
            self._dispatch = {
                "kubernetes_pod": self.pod,
                "deploy_change": self.deploy,
                "image_change": self.image,
                "log_signal": self.log,
                "metric_signal": self.metric,
                "kubernetes_node": self.node,
            }
        return self._dispatch

    # each returns (flags, vocab, node_key, err)
    def pod(self, data):
        flags = vocab = 0
        wr = data.get("waiting_reason")
        if wr:
            vocab |= self.waiting.get(wr, 0)          # hashes like set.add (:318)
        tr = data.get("terminated_reason")
        if tr:
            vocab |= self.terminated.get(tr, 0)       # (:320)
        rc = data.get("restart_count", 0)
        if not _is_number(rc):                         # max(int, rc) raises (:321)
            raise TypeError(f"'>' not supported between instances of "
                            f"'{type(rc).__name__}' and 'int'")
        node_name = data.get("node_name")
        has_issue = bool(data.get("waiting_reason") or data.get("terminated_reason")
                         or data.get("restart_count", 0) > 0)
        key = L.EGR_NO_NODE
        if node_name and has_issue:                   # dict key, same hash/eq (:330)
            key = self.node_keys.setdefault(node_name, len(self.node_keys))
        ready = next((c for c in data.get("conditions", []) if c.get("type") == "Ready"), None)
        if ready and ready.get("status") != "True" and data.get("phase") == "Running":
            flags |= L.F_NOT_READY
            if ready.get("reason") == "ContainersNotReady":
                flags |= L.F_READINESS_FAIL
        return flags, vocab, key, 0.0

    def row(self, ev):
        """One evidence row: (id, flags, vocab, node_key, err) (rules_engine.py:294-313)."""
        ev_id = ev.get("id")
        ev_type = ev.get("evidence_type")
        data = ev.get("data", {})
        proc = self.dispatch.get(ev_type)
        if proc is None:
            return ev_id, 0, 0, L.EGR_NO_NODE, 0.0
        return (ev_id, *proc(data))

    @staticmethod
    def deploy(data):
        return (L.F_RECENT_DEPLOY if data.get("is_recent_change") else 0), 0, L.EGR_NO_NODE, 0.0

    @staticmethod
    def image(data):
        return (L.F_IMAGE_CHANGED if data.get("image_changed") else 0), 0, L.EGR_NO_NODE, 0.0

    def log(self, data):
        vocab = 0
        for pattern in data.get("patterns_found", []):
            vocab |= self.patterns.get(pattern, 0)    # hashes like set.add (:353)
        ec = data.get("error_count", 0)
        if not _is_number(ec):                        # int += ec raises (:354)
            raise TypeError(f"unsupported operand type(s) for +=: 'int' and '{type(ec).__name__}'")
        flags = 0
        if isinstance(ec, float) and not (ec.is_integer() and abs(ec) < _INT_LIMIT):
            flags = L.F_ERR_FLOAT
        elif abs(ec) >= _INT_LIMIT:
            flags = L.F_ERR_FLOAT
        return flags, vocab, L.EGR_NO_NODE, float(ec)

    @staticmethod
    def metric(data):
        flags = 0
        query_name = data.get("query_name", "")
        if "memory" in query_name and data.get("is_anomalous"):
            current = data.get("current_value")
            if current and current > 90:
                flags |= L.F_MEMORY_HIGH
        if "hpa" in query_name and "max" in query_name and data.get("current_value") == 1:
            flags |= L.F_HPA_AT_MAX
        if "latency" in query_name and data.get("current_value", 0) > 1:
            flags |= L.F_LATENCY_HIGH
        return flags, 0, L.EGR_NO_NODE, 0.0

    @staticmethod
    def node(data):
        name = data.get("name")
        status = data.get("conditions", {}).get("Ready", {}).get("status")
        if status != "True":
            hash(name)                                # node_issues[name] = ... (:376)
            return L.F_NODE_ISSUE, 0, L.EGR_NO_NODE, 0.0
        return 0, 0, L.EGR_NO_NODE, 0.0


def _columns(evidence_lists):
    n = sum(len(ev) for ev in evidence_lists)
    return (np.zeros(n, np.uint32), np.zeros(n, np.uint32), np.full(n, L.EGR_NO_NODE, np.uint32),
            np.zeros(n, np.float64), np.zeros(len(evidence_lists) + 1, np.int64))


def _columns_native(evidence_lists):
    """The five columns as views of ONE uninitialised buffer: encode_rows writes every row's
    flags / vocab / node / err and every seg_off entry (a single-incident call pays one
    allocation instead of five)."""
    n = sum(len(ev) for ev in evidence_lists)
    nb = len(evidence_lists) + 1
    buf = np.empty(8 * (n + nb) + 12 * n, np.uint8)
    err = buf[:8 * n].view(np.float64)
    seg = buf[8 * n:8 * (n + nb)].view(np.int64)
    o = 8 * (n + nb)
    return (buf[o:o + 4 * n].view(np.uint32), buf[o + 4 * n:o + 8 * n].view(np.uint32),
            buf[o + 8 * n:o + 12 * n].view(np.uint32), err, seg)


def encode_threads() -> int:
    """Worker threads of the native encoder's parallel row pass ($EGRAPH_ENCODE_THREADS, else
    this process's CPU share, capped at 16; 1 = serial).  The pass applies to batches of at
    least 4096 rows; single incidents always encode on the calling thread."""
    global _THREADS
    if _THREADS is None:
        env = os.environ.get("EGRAPH_ENCODE_THREADS")
        if env:
            _THREADS = max(1, int(env))
        else:
            share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
            _THREADS = max(1, min(16, share))
    return _THREADS


_THREADS = None


def encode_batch(evidence_lists: list[list[dict]], cat: Catalog, threads: int | None = None,
                 out=None) -> EncodedBatch:
    """Encode B evidence lists (one per incident) into batch columns (native row encoder;
    `threads` workers for large batches, default encode_threads()).  `out(rows, B)`, if given,
    returns the five column arrays to write into (e.g. a launch's pinned staging buffer)."""
    enc = _RowEncoder(cat)
    if out is not None:
        flags, vocab, node, err, seg_off = out(sum(len(ev) for ev in evidence_lists),
                                               len(evidence_lists))
    else:
        flags, vocab, node, err, seg_off = _columns_native(evidence_lists)
    ids, _ = L.pyhost.encode_rows(evidence_lists, enc.waiting, enc.terminated, enc.patterns,
                                  enc.node_keys, enc.row, flags, vocab, node, err, seg_off,
                                  encode_threads() if threads is None else threads)
    return EncodedBatch(flags, vocab, node, err, seg_off, ids)


def encode_batch_py(evidence_lists: list[list[dict]], cat: Catalog) -> EncodedBatch:
    """The same encoding with every row in Python (checker for the native encoder)."""
    enc = _RowEncoder(cat)
    flags, vocab, node, err, seg_off = _columns(evidence_lists)
    ids = []
    r = 0
    for i, evidence in enumerate(evidence_lists):
        first = []
        for ev in evidence:
            ev_id, f, v, k, e = enc.row(ev)
            if len(first) < 5:
                first.append(ev_id)
            flags[r] = f
            vocab[r] = v
            node[r] = k
            if e:
                err[r] = e
            r += 1
        seg_off[i + 1] = r
        ids.append(first)
    return EncodedBatch(flags, vocab, node, err, seg_off, ids)
