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


class ShardedDedup:
    """The TTL table sharded by fingerprint range over the ranks of a process group (BASELINE
    C5 across GPUs).  The reference keeps one Redis (deduplicator.py:41-104) that every webhook
    replica shares; here rank r owns the fingerprints whose first digest byte b has
    b * world >> 8 == r, in its own DedupTable on its own GPU.

    ingest() runs the webhook loop (main.py:141-170) over a GLOBAL batch whose alerts arrive
    spread over the ranks, each alert carrying its global arrival number `seq`:
      1. every rank routes its alerts' (fingerprint, seq) to the owner ranks (all-to-all; RCCL
         over xGMI between GPUs);
      2. each owner runs its table's ingest over the alerts it owns IN ARRIVAL ORDER -- the loop
         is per key (get / set of one fingerprint), so the owners' loops together make exactly
         the single table's decisions;
      3. the owners' (seq, duplicate, owner-local handle) are all-gathered, and every rank
         numbers the new incidents globally in arrival order (the single table's numbering)
         and maps each owner-local handle to its global one.
    Every rank ends with the whole batch's decisions; the host state (the handle maps) is
    identical on all ranks.  `table` is a DedupTable (or any object with its ingest / remove /
    extend methods; the CPU tests use the oracle's TTL store), `comm` an egraph.shard.TorchComm."""

    def __init__(self, table, comm, rank: int):
        self.table, self.comm, self.rank, self.world = table, comm, rank, comm.P
        self.dev = table.dev
        self.next_id = 0                                  # the next global incident handle
        self._g_of = [np.zeros(0, np.int64) for _ in range(self.world)]   # owner-local -> global

    def owner(self, fp: torch.Tensor) -> torch.Tensor:
        """Owning rank of each [n, 16] fingerprint (range partition of the first byte)."""
        return (fp[:, 0].to(torch.int64) * self.world) >> 8

    def owns(self, fp: torch.Tensor) -> torch.Tensor:
        return self.owner(fp) == self.rank

    def _all_gather_v(self, x: torch.Tensor) -> list[torch.Tensor]:
        """Variable-length all-gather of a 1-D int64 tensor -> one tensor per rank."""
        n = torch.tensor([x.numel()], dtype=torch.int64, device=x.device)
        (counts,) = self.comm.all_gather([n])
        counts = counts.cpu().tolist()
        m = max(max(counts), 1)
        pad = torch.zeros(m, dtype=torch.int64, device=x.device)
        pad[: x.numel()] = x
        (allx,) = self.comm.all_gather([pad])
        return [allx[r * m: r * m + counts[r]] for r in range(self.world)]

    def ingest(self, fp: torch.Tensor, seq: torch.Tensor, now_ms: int, ttl_ms: int):
        """This rank's alerts ([n, 16] uint8 fingerprints, int64 global arrival numbers) ->
        (dup bool [N], incident int64 [N], n_new) for ALL N alerts of the global batch, in
        arrival order (numpy arrays; seq must number the global batch 0..N-1)."""
        fp = _fp_arg(fp, self.dev)
        seq = seq.to(device=self.dev, dtype=torch.int64)
        own = self.owner(fp)
        order = torch.argsort(own, stable=True)
        words = fp.reshape(-1).view(torch.int64).reshape(-1, 2)[order]             # 16 B = 2 int64
        payload = torch.cat([words, seq[order, None]], dim=1).reshape(-1)
        counts = torch.bincount(own, minlength=self.world).cpu().tolist()
        ((recv, rc),) = self.comm.all_to_all_v([(payload.contiguous(), [3 * c for c in counts])])
        recv = recv.reshape(-1, 3)
        rseq = recv[:, 2]
        o = torch.argsort(rseq)                                         # arrival order
        mine_fp = recv[o, :2].contiguous().reshape(-1).view(torch.uint8).reshape(-1, 16)
        mine_seq = rseq[o]
        dup, local, _ = self.table.ingest(mine_fp, now_ms, ttl_ms)
        rec = torch.stack([mine_seq, dup.to(torch.int64), local.to(torch.int64)], dim=1).reshape(-1)
        parts = [p.cpu().numpy().reshape(-1, 3) for p in self._all_gather_v(rec)]
        N = sum(len(p) for p in parts)
        dup_all = np.zeros(N, bool)
        inc_all = np.zeros(N, np.int64)
        owner_all = np.zeros(N, np.int64)
        local_all = np.zeros(N, np.int64)
        for r, p in enumerate(parts):
            s = p[:, 0]
            if len(s) and (s.min() < 0 or s.max() >= N):
                raise ValueError("seq must number the global batch 0..N-1")
            dup_all[s], owner_all[s], local_all[s] = p[:, 1] != 0, r, p[:, 2]
        new = np.flatnonzero(~dup_all)
        g = self.next_id + np.arange(len(new), dtype=np.int64)
        for r in range(self.world):                     # owner-local handles of the new ones
            sel = owner_all[new] == r
            if sel.any():
                loc = local_all[new][sel]
                need = int(loc.max()) + 1
                if need > len(self._g_of[r]):
                    grown = np.full(max(need, 2 * len(self._g_of[r])), -1, np.int64)
                    grown[: len(self._g_of[r])] = self._g_of[r]
                    self._g_of[r] = grown
                self._g_of[r][loc] = g[sel]
        inc_all[new] = g
        d = np.flatnonzero(dup_all)
        for r in range(self.world):
            sel = d[owner_all[d] == r]
            if len(sel):
                inc_all[sel] = self._g_of[r][local_all[sel]]
        self.next_id += len(new)
        return dup_all, inc_all, len(new)

    def remove(self, fp: torch.Tensor) -> None:
        """DEL of every fingerprint in fp (each rank passes the same list; owners apply)."""
        fp = _fp_arg(fp, self.dev)
        m = self.owns(fp)
        if bool(m.any()):
            self.table.remove(fp[m].contiguous())

    def extend(self, fp: torch.Tensor, now_ms: int, ttl_ms: int) -> np.ndarray:
        """EXPIRE of every fingerprint in fp (same list on every rank): bool [n], the key was
        live, gathered from the owners."""
        fp = _fp_arg(fp, self.dev)
        n = fp.shape[0]
        m = self.owns(fp)
        ok = torch.zeros(n, dtype=torch.int64, device=self.dev)
        if bool(m.any()):
            ok[m] = self.table.extend(fp[m].contiguous(), now_ms, ttl_ms).to(torch.int64)
        parts = self._all_gather_v(ok)
        return (torch.stack([p.cpu() for p in parts]).sum(0) != 0).numpy()
