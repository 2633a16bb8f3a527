"""Alert-storm front end on the GPU (BASELINE config C5): batched alert
fingerprints and the TTL deduplication table (csrc/alerts.hip through the C-ABI).

Reference:
  src/services/ingestion/normalizer.py:208-218   fingerprint = sha256(f"{source}:{alertname}:
                                                   {namespace}:{service}").hexdigest()[:32]
  src/services/ingestion/deduplicator.py:41-140  Redis GET / SET EX / DEL / EXPIRE on
                                                   "aiops:fingerprint:<fp>" (TTL 4 h)
  src/services/ingestion/main.py:141-170, :392    the webhook loop: check, create, register.

Fingerprints travel as 16-byte digests ([n, 16] uint8 device tensors); `hex` gives the
reference's 32-character strings.  Incident ids inside the table are u32 handles; the host
mirror (src/services/ingestion/deduplicator.py) maps them to the caller's id strings.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from egraph import _lib as L
from egraph.device import require_device, to_device

NO_INCIDENT = 0xFFFFFFFF


def fingerprint_key(source: str, alertname: str, namespace: str, service: str) -> str:
    """The hashed string of normalizer.py:217."""
    return f"{source}:{alertname}:{namespace}:{service}"


def pack_strings(keys: list[str | bytes]) -> tuple[np.ndarray, np.ndarray]:
    """UTF-8 blob + int64 offsets [n+1] (the encoding `key.encode()` of normalizer.py:218)."""
    enc = [k.encode() if isinstance(k, str) else bytes(k) for k in keys]
    off = np.zeros(len(enc) + 1, np.int64)
    if enc:
        off[1:] = np.cumsum([len(b) for b in enc])
    blob = np.frombuffer(b"".join(enc), np.uint8) if off[-1] else np.zeros(1, np.uint8)
    return blob, off


def fingerprints(keys: list[str | bytes], device=None, hex: bool = False, stream=None):
    """SHA-256 prefixes of `keys` on the GPU: ([n, 16] uint8 device tensor, list of 32-char hex
    strings if `hex` else None)."""
    dev = require_device(device)
    n = len(keys)
    blob, off = pack_strings(keys)
    out = torch.empty((max(n, 1), 16), dtype=torch.uint8, device=dev)[:n]
    hx = torch.empty(max(n, 1) * 32, dtype=torch.uint8, device=dev) if hex else None
    with torch.cuda.device(dev):
        d_blob, d_off = to_device(blob, dev), to_device(off, dev)
        st = L.stream_handle(dev) if stream is None else stream
        L.check(L.lib.egr_fingerprint(L.ptr(d_blob), L.ptr(d_off), n, L.ptr(out), L.ptr(hx), st),
                "egr_fingerprint")
    if not hex:
        return out, None
    raw = hx[: n * 32].cpu().numpy().tobytes().decode("ascii")
    return out, [raw[i * 32:(i + 1) * 32] for i in range(n)]


def fingerprints_from_hex(fps: list[str], device=None) -> torch.Tensor:
    """32-char hex fingerprints (the reference's strings) -> [n, 16] uint8 device tensor."""
    dev = require_device(device)
    raw = b"".join(bytes.fromhex(f) for f in fps)
    a = np.frombuffer(raw, np.uint8).reshape(len(fps), 16) if fps else np.zeros((0, 16), np.uint8)
    return to_device(a, dev)


def _fp_arg(fp: torch.Tensor, dev: torch.device) -> torch.Tensor:
    if fp.dtype != torch.uint8 or fp.dim() != 2 or fp.shape[1] != 16:
        raise ValueError("fingerprints must be a [n, 16] uint8 tensor")
    if fp.device != dev:
        raise ValueError(f"fingerprints on {fp.device}, table on {dev}")
    return fp.contiguous()


class DedupTable:
    """The TTL table on one GPU.  Times are integer milliseconds; a key is live while
    now_ms < expiry (Redis EX).  `capacity` = live keys it holds at <= 1/2 load.

    Expired and removed keys keep their slot (probe chains stay intact) until a compaction
    rebuilds the table from the live keys.  With `auto_compact` (default) the table compacts
    itself before an ingest / register could push the used slots past COMPACT_LOAD of the slot
    count, growing when the live keys plus the batch need it -- so, like Redis expiring keys, a
    long-running service never fills it.  Without it a full table raises MemoryError."""

    COMPACT_LOAD = 0.75

    def __init__(self, capacity: int = 1 << 20, device=None, auto_compact: bool = True):
        self.dev = require_device(device)
        h = C.c_void_p()
        L.check(L.lib.egr_dedup_create(self.dev.index, int(capacity), C.byref(h)), "egr_dedup_create")
        self._h = h
        self.capacity = int(capacity)
        self.auto_compact = auto_compact
        self.next_id = 0                 # the next incident handle ingest() hands out
        self.compactions = 0
        self._counts = torch.zeros(2, dtype=torch.int32, device=self.dev)
        self._slots = self.stats(0)["slots"]
        self._used_bound = 0             # >= slots holding a key (each batch adds <= its size)

    def _make_room(self, n: int, now_ms: int) -> None:
        """Before a batch that may occupy up to n fresh slots: compact (and grow) if the used
        slots could pass COMPACT_LOAD.  The exact count is read only when the bound says so."""
        if not self.auto_compact or self._used_bound + n <= self.COMPACT_LOAD * self._slots:
            return
        st = self.stats(now_ms)
        self._used_bound = st["used_slots"]
        if self._used_bound + n <= self.COMPACT_LOAD * self._slots:
            return
        need = st["live"] + n
        cap = self.capacity                   # the rebuilt table has >= 2 * cap slots
        while need > self.COMPACT_LOAD * 2 * cap:
            cap *= 2
        self.compact(now_ms, cap)
        self.capacity = cap
        self.compactions += 1

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and getattr(L, "lib", None) is not None:
            L.lib.egr_dedup_free(h)
            self._h = None

    def _st(self, stream):
        return L.stream_handle(self.dev) if stream is None else stream

    def ingest(self, fp: torch.Tensor, now_ms: int, ttl_ms: int, stream=None):
        """The webhook loop over a batch (see egr_dedup_ingest).  Returns (dup bool [n],
        incident int64 [n] handles, n_new) -- device tensors, n_new an int (synchronises)."""
        fp = _fp_arg(fp, self.dev)
        n = fp.shape[0]
        self._make_room(n, now_ms)
        self._used_bound += n
        dup = torch.empty(max(n, 1), dtype=torch.uint8, device=self.dev)[:n]
        inc = torch.empty(max(n, 1), dtype=torch.int32, device=self.dev)[:n]
        L.check(L.lib.egr_dedup_ingest(self._h, L.ptr(fp), n, int(now_ms), int(ttl_ms),
                                       self.next_id & 0xFFFFFFFF, L.ptr(dup), L.ptr(inc),
                                       L.ptr(self._counts), self._st(stream)), "egr_dedup_ingest")
        full, n_new = (int(x) for x in self._counts.cpu().tolist())
        if full:
            raise MemoryError(f"dedup table full: {full} alerts not registered (compact or grow it)")
        self.next_id += n_new
        return dup.bool(), inc.to(torch.int64) & 0xFFFFFFFF, n_new

    def lookup(self, fp: torch.Tensor, now_ms: int, stream=None):
        """check_duplicate for a batch: (dup bool [n], incident int64 [n]) device tensors."""
        fp = _fp_arg(fp, self.dev)
        n = fp.shape[0]
        dup = torch.empty(max(n, 1), dtype=torch.uint8, device=self.dev)[:n]
        inc = torch.empty(max(n, 1), dtype=torch.int32, device=self.dev)[:n]
        L.check(L.lib.egr_dedup_lookup(self._h, L.ptr(fp), n, int(now_ms), L.ptr(dup), L.ptr(inc),
                                       self._st(stream)), "egr_dedup_lookup")
        return dup.bool(), inc.to(torch.int64) & 0xFFFFFFFF

    def register(self, fp: torch.Tensor, now_ms: int, ttl_ms: int, incident: torch.Tensor,
                 stream=None) -> None:
        fp = _fp_arg(fp, self.dev)
        n = fp.shape[0]
        if incident.numel() != n:
            raise ValueError("one incident handle per fingerprint")
        inc = incident.to(device=self.dev, dtype=torch.int64).to(torch.int32).contiguous()
        self._make_room(n, now_ms)
        self._used_bound += n
        L.check(L.lib.egr_dedup_register(self._h, L.ptr(fp), n, int(now_ms), int(ttl_ms), L.ptr(inc),
                                         L.ptr(self._counts), self._st(stream)), "egr_dedup_register")
        if int(self._counts[0].item()):
            raise MemoryError("dedup table full (compact or grow it)")

    def remove(self, fp: torch.Tensor, stream=None) -> None:
        fp = _fp_arg(fp, self.dev)
        L.check(L.lib.egr_dedup_remove(self._h, L.ptr(fp), fp.shape[0], self._st(stream)),
                "egr_dedup_remove")

    def extend(self, fp: torch.Tensor, now_ms: int, ttl_ms: int, stream=None) -> torch.Tensor:
        """extend_fingerprint for a batch: bool [n] = the key was live (and got the new TTL)."""
        fp = _fp_arg(fp, self.dev)
        n = fp.shape[0]
        ok = torch.empty(max(n, 1), dtype=torch.uint8, device=self.dev)[:n]
        L.check(L.lib.egr_dedup_extend(self._h, L.ptr(fp), n, int(now_ms), int(ttl_ms), L.ptr(ok),
                                       self._st(stream)), "egr_dedup_extend")
        return ok.bool()

    def stats(self, now_ms: int) -> dict:
        out = (C.c_int64 * 3)()
        L.check(L.lib.egr_dedup_stats(self._h, int(now_ms), out), "egr_dedup_stats")
        return {"used_slots": out[0], "live": out[1], "slots": out[2]}

    def compact(self, now_ms: int, capacity: int = 0) -> None:
        """Rebuild from the live keys (expired / removed ones drop out), with room for at
        least max(capacity, live) keys at <= 1/2 load."""
        L.check(L.lib.egr_dedup_compact(self._h, int(now_ms), int(capacity)), "egr_dedup_compact")
        st = self.stats(now_ms)
        self._slots, self._used_bound = st["slots"], st["used_slots"]
