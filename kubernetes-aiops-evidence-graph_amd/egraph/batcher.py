"""Low-latency rules launches and the aggregator that batches concurrent RulesEngine calls.

The reference runs one RulesEngine.generate_hypotheses + HypothesisRanker.rank per incident
inside each Temporal activity (src/services/workflow/activities.py:124-170); activities run
concurrently in one worker.  Here:

  RulesRunner   one egr_rules_eval launch per call.  A single incident of at most 1024 rows
                (the activities' calls) goes to the resident rules server (egr_rules_server_*):
                a one-wave kernel polling a mailbox in mapped host memory, so the call is two
                PCIe round trips and no kernel launch.  Other small batches are ZERO-COPY: the
                kernel reads the encoded rows from, and writes its outputs to, pinned host memory
                mapped into the GPU address space (egr_host_alloc).  Large
                batches go through a device buffer: the columns go up in ONE host-to-device copy
                and the seven outputs come back in ONE device-to-host copy, issued with the
                kernel in one library call (egr_rules_eval_staged).  Either way the caller waits
                on a HIP event by polling it from the event loop (no thread hop, the loop is
                never blocked).
  RulesBatcher  adaptive batching: a call that finds no launch in flight starts one at once
                from its own task (no added latency when idle); calls arriving while a launch
                runs are collected and go out together in the next one.  Each call gets exactly the dicts a
                single call would (the kernel is per incident), and an input that makes the
                reference raise raises in its own call only.
"""
from __future__ import annotations

import asyncio
import contextlib
import gc
import os
import time

import numpy as np
import torch

from . import _lib as L
from .catalog import Catalog
from .device import MappedBuffer, require_device
from .encode import EncodedBatch, encode_batch
from .ranker import FUSED
from .rca import RulesResult, hypothesis_lists


def _align(n: int, a: int = 256) -> int:
    return (n + a - 1) // a * a


@contextlib.contextmanager
def gc_paused():
    """Defer the cyclic GC while a batch's dicts are built.  Assembling thousands of
    hypothesis dicts triggers collections that traverse every live object -- the callers' large
    evidence structures included -- and doubled the assembly time of a 1024-incident batch on
    the C3 workload; the deferred collection runs once, on the next allocation after it."""
    on = gc.isenabled()
    if on:
        gc.disable()
    try:
        yield
    finally:
        if on:
            gc.enable()


class RulesRunner:
    """egr_rules_eval over persistent buffers (grown on demand) on one stream.  One launch at
    a time: the next launch reuses the buffers, so read results() before launching again."""

    # batches up to this many rows are zero-copy (mapped host memory; about 0.4 MB read over
    # PCIe at the limit); above it the staged device buffer and its two DMA copies win
    ZERO_COPY_ROWS = 16384

    def __init__(self, cat: Catalog, device=None):
        self.cat = cat
        self.dev = require_device(device)
        self.S = cat.n_rules + 1
        self.stream = torch.cuda.Stream(self.dev)
        self.cap_rows = self.cap_inc = -1
        self.event = torch.cuda.Event()
        self._offs = np.zeros(12, np.int64)
        self.mapped: MappedBuffer | None = None
        self.zero_copy = False                        # the last launch's outputs in mapped memory
        self.mode = ""                                # "small" / "zero_copy" / "staged"
        self._layouts: dict = {}
        self._small_out = None                        # EgrRulesOut of the single-incident layout
        self._srv = None                              # the rules server (created on first use)
        self._srv_wait = None

    # a single incident of at most this many rows travels in the kernel's arguments
    # (egr_rules_eval_small): one launch, no copies, no PCIe reads by the kernel
    SMALL_ROWS = 128

    # the single-incident path through the resident rules server (False: one small kernel
    # launch per call, egr_rules_eval_small; $EGRAPH_RULES_SERVER=0 for A/B runs)
    USE_SERVER = os.environ.get("EGRAPH_RULES_SERVER", "1") != "0"
    SERVER_ROWS = 1024                            # the server's mailbox (egr_rules_server_post)

    def _server(self):
        if self._srv is None:
            import ctypes as C
            h = C.c_void_p()
            L.check(L.lib.egr_rules_server_create(self.cat.table, self.dev.index or 0, C.byref(h)),
                    "egr_rules_server_create")
            self._srv = h
            S = self.S
            a8 = (S + 7) // 8 * 8
            # one output block per call: mask u32 @0, n_hyp u8 @8, order_conf / order_rank (S
            # bytes each), confidence / final_score / strength (S doubles each)
            self._srv_off = (0, 8, 16, 16 + a8, 16 + 2 * a8, 16 + 2 * a8 + 8 * S, 16 + 2 * a8 + 16 * S)
            self._srv_bytes = 16 + 2 * a8 + 24 * S
            self._srv_wait = _ServerWait(self)
        return self._srv

    def __del__(self):
        h = getattr(self, "_srv", None)
        if h is not None and getattr(L, "lib", None) is not None:
            self._srv = None
            L.lib.egr_rules_server_free(h)

    def _server_failed(self) -> None:
        """A server request went unanswered past _ServerWait.TIMEOUT_S (its wave faulted or
        never ran): drop the handle -- free() stops the wave, which leaves at its next poll --
        so the next single call creates a fresh server instead of being refused forever."""
        h, self._srv, self._srv_wait = self._srv, None, None
        if h is not None:
            L.lib.egr_rules_server_free(h)

    def _layout(self, rows: int, B: int):
        key = (rows, B)
        hit = self._layouts.get(key)
        if hit is None:
            if len(self._layouts) > 4096:
                self._layouts.clear()
            hit = self._layouts[key] = self._layout_new(rows, B)
        return hit

    def _layout_new(self, rows: int, B: int):
        S = self.S
        inp = [("flags", 4 * rows), ("vocab", 4 * rows), ("node", 4 * rows), ("err", 8 * rows),
               ("seg", 8 * (B + 1))]
        outp = [("mask", 4 * B), ("n_hyp", B), ("oc", B * S), ("orank", B * S),
                ("conf", 8 * B * S), ("fin", 8 * B * S), ("str", 8 * B * S)]
        off, o = {}, 0
        for name, nb in inp:
            off[name] = (o, nb)
            o = _align(o + nb)
        in_bytes = o
        for name, nb in outp:
            off[name] = (o, nb)
            o = _align(o + nb)
        return off, in_bytes, o

    def _ensure(self, rows: int, B: int) -> None:
        if rows <= self.cap_rows and B <= self.cap_inc:
            return
        rows, B = max(rows, 2 * self.cap_rows, 1024), max(B, 2 * self.cap_inc, 64)
        _, _, total = self._layout(rows, B)
        self.dbuf = torch.empty(total, dtype=torch.uint8, device=self.dev)
        self.hbuf = torch.empty(total, dtype=torch.uint8).pin_memory()
        self.cap_rows, self.cap_inc = rows, B

    def _h(self, name, dtype, n):
        o, _ = self.off[name]
        return self.hnp[o:o + n * np.dtype(dtype).itemsize].view(dtype)

    def _d(self, name) -> int:
        return self.dbuf.data_ptr() + self.off[name][0]

    def input_views(self, rows: int, B: int):
        """(flags, vocab, node, err, seg_off) arrays inside the buffer the next launch of this
        size reads its inputs from: an encoder writing into them saves launch() the staging
        copy (launch() recognises them and skips it)."""
        if B == 1 and rows <= self.SMALL_ROWS:
            # (a single small incident travels in the kernel's arguments; its outputs land
            # where these inputs would sit, so it gets arrays of its own)
            return (np.empty(rows, np.uint32), np.empty(rows, np.uint32), np.empty(rows, np.uint32),
                    np.empty(rows, np.float64), np.empty(B + 1, np.int64))
        off, _, total = self._layout(rows, B)
        if rows <= self.ZERO_COPY_ROWS:
            if self.mapped is None or self.mapped.nbytes < total:
                self.mapped = MappedBuffer(max(total, 1 << 20))
                self._small_out = None
            h = self.mapped.np
        else:
            self._ensure(rows, B)
            h = self.hbuf.numpy()

        def v(name, dt, n):
            o = off[name][0]
            return h[o:o + n * np.dtype(dt).itemsize].view(dt)
        return (v("flags", np.uint32, rows), v("vocab", np.uint32, rows), v("node", np.uint32, rows),
                v("err", np.float64, rows), v("seg", np.int64, B + 1))

    def _staged_in_place(self, enc: EncodedBatch, h) -> bool:
        """The encoded columns already sit where this launch reads them (input_views)."""
        base = h.ctypes.data
        return all(len(a) == 0 or a.ctypes.data == base + self.off[name][0]
                   for name, a in (("flags", enc.flags), ("vocab", enc.vocab), ("node", enc.node),
                                   ("err", enc.err), ("seg", enc.seg_off)))

    def _stage_inputs(self, enc: EncodedBatch) -> None:
        if self._staged_in_place(enc, self.hnp):
            return
        for name, arr, dt in (("flags", enc.flags, np.uint32), ("vocab", enc.vocab, np.uint32),
                              ("node", enc.node, np.uint32), ("err", enc.err, np.float64),
                              ("seg", enc.seg_off, np.int64)):
            if len(arr):
                self._h(name, dt, len(arr))[:] = arr

    def launch(self, enc: EncodedBatch) -> torch.cuda.Event:
        """Enqueue one encoded batch; returns the event that marks the results as ready in host
        memory (read them with results())."""
        B, rows = enc.n_incidents, enc.n_rows
        self._B, self._rows = B, rows
        # this launch's layout inside the buffers: only its own bytes are touched
        self.off, self.in_bytes, self.total = self._layout(rows, B)
        st = self.stream
        small = B == 1 and rows <= self.SMALL_ROWS
        if B == 1 and rows <= self.SERVER_ROWS and self.USE_SERVER:
            srv = self._server()
            f = enc.flags.ctypes.data if rows else None
            L.check(L.lib.egr_rules_server_post(srv, f, enc.vocab.ctypes.data if rows else None,
                                                enc.node.ctypes.data if rows else None,
                                                enc.err.ctypes.data if rows else None, rows),
                    "egr_rules_server_post")
            self.mode = "server"
            return self._srv_wait.arm()
        if (small or rows <= self.ZERO_COPY_ROWS) and (self.mapped is None or self.mapped.nbytes < self.total):
            self.mapped = MappedBuffer(max(self.total, 1 << 20))
            self._small_out = None
        if small:
            # the rows in the kernel arguments, the outputs into mapped host memory
            self.hnp, self.zero_copy = self.mapped.np, True
            if self._small_out is None:
                base = self.mapped.dev
                so = self._layout(0, 1)[0]                # output offsets do not depend on rows
                self._small_out = (so, L.EgrRulesOut(*(base + so[k][0] for k in (
                    "mask", "n_hyp", "oc", "orank", "conf", "fin", "str"))))
            self.off, self.mode = self._small_out[0], "small"
            f = enc.flags.ctypes.data if rows else None
            L.check(L.lib.egr_rules_eval_small(
                self.cat.table, f, enc.vocab.ctypes.data if rows else None,
                enc.node.ctypes.data if rows else None, enc.err.ctypes.data if rows else None,
                rows, self._small_out[1], st.cuda_stream), "egr_rules_eval_small")
            self.event.record(st)
            return self.event
        if rows <= self.ZERO_COPY_ROWS:
            self.hnp, self.zero_copy, self.mode = self.mapped.np, True, "zero_copy"
            self._stage_inputs(enc)
            base = self.mapped.dev
            d = {k: base + o for k, (o, _) in self.off.items()}
            o = L.EgrRulesOut(d["mask"], d["n_hyp"], d["oc"], d["orank"], d["conf"], d["fin"], d["str"])
            L.check(L.lib.egr_rules_eval(self.cat.table, d["flags"], d["vocab"], d["node"], d["err"],
                                         d["seg"], B, o, st.cuda_stream), "egr_rules_eval")
            self.event.record(st)
            return self.event
        self._ensure(rows, B)
        self.hnp, self.zero_copy, self.mode = self.hbuf.numpy(), False, "staged"
        self._stage_inputs(enc)
        out_lo = self.off["mask"][0]
        self._offs[:] = [self.off[k][0] for k in ("flags", "vocab", "node", "err", "seg", "mask",
                                                   "n_hyp", "oc", "orank", "conf", "fin", "str")]
        # upload, kernel and download in ONE library call (egr_rules_eval_staged)
        hp = self.hbuf.data_ptr()
        L.check(L.lib.egr_rules_eval_staged(self.cat.table, hp, self.dbuf.data_ptr(), hp,
                                            self._offs.ctypes.data, self.in_bytes, out_lo,
                                            self.total, B, st.cuda_stream), "egr_rules_eval_staged")
        self.event.record(st)
        return self.event

    def results(self) -> RulesResult:
        """Host copies of the last launch's outputs (after its event completed): the output
        block is copied once and the seven arrays are views of that copy."""
        B, S = self._B, self.S
        if self.mode == "server":
            return self._srv_wait.result()
        lo = self.off["mask"][0]
        o, nb = self.off["str"]
        blk = self.hnp[lo:o + nb].copy()

        def g(name, dtype, n):
            a = self.off[name][0] - lo
            return blk[a:a + n * np.dtype(dtype).itemsize].view(dtype)
        return RulesResult(g("mask", np.uint32, B), g("n_hyp", np.uint8, B),
                           g("oc", np.uint8, B * S).reshape(B, S),
                           g("orank", np.uint8, B * S).reshape(B, S),
                           g("conf", np.float64, B * S).reshape(B, S),
                           g("fin", np.float64, B * S).reshape(B, S),
                           g("str", np.float64, B * S).reshape(B, S))

    def run_sync(self, enc: EncodedBatch) -> RulesResult:
        self.launch(enc).synchronize()
        return self.results()

    def sync_last(self) -> None:
        """Wait for the last launch (whichever path it took)."""
        (self._srv_wait if self.mode == "server" else self.event).synchronize()

    # the first SPIN_S of a launch's wait spin on its event without yielding (a single
    # incident's round trip is ~25-30 us, and every event-loop hop adds several us); past it
    # the wait yields to the loop between polls.  The reference runs its rules inline in the
    # coroutine (~65 us per incident), so a bounded spin blocks the loop no longer than it did.
    SPIN_S = 100e-6

    async def run(self, enc: EncodedBatch) -> RulesResult:
        ev = self.launch(enc)
        # one loop turn while the kernel runs: calls made in this turn (e.g. the rest of an
        # asyncio.gather) queue up for the next launch instead of waiting behind a spin.  When
        # no other callback is ready (a lone call: the loop's ready queue is empty) the turn
        # would only cost the loop's select and task bookkeeping, so it is skipped.
        ready = getattr(asyncio.get_running_loop(), "_ready", None)
        if ready is None or len(ready):
            await asyncio.sleep(0)
        t0 = time.perf_counter()
        while not ev.query():
            dt = time.perf_counter() - t0
            if dt > self.SPIN_S:
                if self.mode == "server" and dt > _ServerWait.TIMEOUT_S:
                    ev.expire()                     # raises; the next call gets a new server
                await asyncio.sleep(0)              # long launch: poll from the loop
        return self.results()


class _ServerWait:
    """The event-like handle of a rules-server call (query / synchronize, as a torch.cuda.Event
    is used by RulesRunner.run / run_sync): query() polls the mailbox and, once the incident is
    done, holds its outputs in a fresh block (the arrays of the RulesResult are views of it)."""
    __slots__ = ("r", "blk", "done", "_args")

    def __init__(self, runner: RulesRunner):
        self.r, self.blk, self.done, self._args = runner, None, False, None

    def arm(self) -> "_ServerWait":
        r = self.r
        self.blk = np.empty(r._srv_bytes, np.uint8)
        base = self.blk.ctypes.data
        self._args = tuple(base + o for o in r._srv_off)
        self.done = False
        return self

    def query(self) -> bool:
        if not self.done:
            rc = L.lib.egr_rules_server_poll(self.r._srv, *self._args)
            if rc < 0:
                L.check(rc, "egr_rules_server_poll")
            self.done = rc == 1
        return self.done

    # a request unanswered this long is lost: the wave polls its mailbox every few us while
    # resident and is relaunched when it has left, so only a faulted wave gets here
    TIMEOUT_S = 5.0

    def synchronize(self) -> None:
        t0 = time.perf_counter()
        while not self.query():
            if time.perf_counter() - t0 > self.TIMEOUT_S:
                self.expire()

    def expire(self) -> None:
        self.r._server_failed()
        raise RuntimeError(f"egr_rules_server: no answer within {self.TIMEOUT_S} s "
                           "(the server was dropped; the next call starts a new one)")

    def result(self) -> RulesResult:
        S, o, b = self.r.S, self.r._srv_off, self.blk
        return RulesResult(b[o[0]:o[0] + 4].view(np.uint32), b[o[1]:o[1] + 1],
                           b[o[2]:o[2] + S].reshape(1, S), b[o[3]:o[3] + S].reshape(1, S),
                           b[o[4]:o[4] + 8 * S].view(np.float64).reshape(1, S),
                           b[o[5]:o[5] + 8 * S].view(np.float64).reshape(1, S),
                           b[o[6]:o[6] + 8 * S].view(np.float64).reshape(1, S))


def concat(encs: list[EncodedBatch]) -> EncodedBatch:
    """One batch of several encoded batches (segments re-based; node keys only ever meet
    inside one incident's segment, so per-batch key numberings do not collide)."""
    if len(encs) == 1:
        return encs[0]
    seg = [np.zeros(1, np.int64)]
    base = 0
    for e in encs:
        seg.append(e.seg_off[1:] + base)
        base += e.n_rows
    return EncodedBatch(np.concatenate([e.flags for e in encs]), np.concatenate([e.vocab for e in encs]),
                        np.concatenate([e.node for e in encs]), np.concatenate([e.err for e in encs]),
                        np.concatenate(seg), [i for e in encs for i in e.evidence_ids])


class _Call:
    """One caller's incidents; `single`: submit() of one incident (its future gets the list
    itself, not a list of one list)."""
    __slots__ = ("incident_ids", "evidence_lists", "ranked", "fut", "single")

    def __init__(self, incident_ids: list, evidence_lists: list, ranked: bool, fut, single=False):
        self.incident_ids, self.evidence_lists, self.ranked = incident_ids, evidence_lists, ranked
        self.fut, self.single = fut, single


class RulesBatcher:
    """Coalesces concurrent rules calls into launches of up to max_batch incidents."""

    def __init__(self, cat: Catalog, device=None, max_batch: int = 16384):
        self.cat = cat
        self.runner = RulesRunner(cat, device)
        self.max_batch = max_batch
        self.queue: list[_Call] = []
        self.busy = False
        self.launches = 0                             # diagnostics: launches / calls
        self.calls = 0

    async def submit(self, incident_id, evidence: list[dict], ranked: bool) -> list[dict]:
        """One incident's hypothesis list (generate_hypotheses, ranked or not)."""
        self.calls += 1
        if not self.busy:
            return await self._single_idle(str(incident_id), evidence, ranked)
        # (a launch is running: this call joins the next one)
        loop = asyncio.get_running_loop()
        call = _Call([str(incident_id)], [evidence], ranked, loop.create_future(), True)
        self.queue.append(call)
        return await call.fut

    def queued(self, incident_id, evidence: list[dict], ranked: bool) -> asyncio.Future:
        """submit()'s path while a launch runs, as a plain call: the future of a call queued for
        the next launch (the caller awaits it -- one coroutine frame fewer per concurrent call
        than awaiting submit()).  Only while self.busy."""
        self.calls += 1
        fut = asyncio.get_running_loop().create_future()
        self.queue.append(_Call([str(incident_id)], [evidence], ranked, fut, True))
        return fut

    async def _single_idle(self, incident_id: str, evidence: list[dict], ranked: bool) -> list[dict]:
        """An idle batcher's lone call, run in the caller's task with no queue entry, future or
        second task: encode (raising what the reference raises, to this caller only), the
        launch (the rules server for a single incident), the dicts.  Calls that arrive while it
        runs queue up and go out together from a drain task afterwards.  (Fewer objects per call
        than the queued path: the activities' one-incident calls see fewer collector pauses.)"""
        self.busy = True
        launched = False
        try:
            enc = encode_batch([evidence], self.cat, out=self.runner.input_views)
            self.launches += 1
            launched = True
            res = await self.runner.run(enc)
            launched = False
            with gc_paused():
                lists = hypothesis_lists(self.cat, res, [incident_id], enc.evidence_ids, ranked)
                if not ranked:
                    FUSED.register(self.cat, res, lists, (0,))
            return lists[0]
        except asyncio.CancelledError:
            if launched:                     # (the next launch reuses the buffers / mailbox)
                self.runner.sync_last()
            raise
        finally:
            if self.queue:
                asyncio.get_running_loop().create_task(self._drain())   # stays busy until empty
            else:
                self.busy = False

    async def submit_many(self, incident_ids: list, evidence_lists: list, ranked: bool
                          ) -> list[list[dict]]:
        """Several incidents as ONE call (it raises as a whole if any row makes the
        reference raise, as the reference's loop over them would).  No incidents: [] at once
        (a call with nothing to launch never joins a batch)."""
        if not incident_ids and not evidence_lists:
            return []
        loop = asyncio.get_running_loop()
        call = _Call([str(i) for i in incident_ids], list(evidence_lists), ranked, loop.create_future())
        self.calls += 1
        self.queue.append(call)
        if self.busy:
            return await call.fut
        return await self._launch_idle(loop, call)

    async def _launch_idle(self, loop, call: "_Call"):
        # idle: this call launches at once from its own task; calls arriving while it runs
        # (its wait yields one loop turn) go out together from a drain task afterwards
        self.busy = True
        try:
            await self._run(self._take())
        finally:
            if self.queue:
                loop.create_task(self._drain())          # stays busy until the queue is empty
            else:
                self.busy = False
        return await call.fut

    def _take(self) -> list[_Call]:
        """The next launch's calls: queue order, up to max_batch incidents (at least one call)."""
        take, n = 0, 0
        while take < len(self.queue) and (take == 0 or n + len(self.queue[take].incident_ids)
                                          <= self.max_batch):
            n += len(self.queue[take].incident_ids)
            take += 1
        calls, self.queue = self.queue[:take], self.queue[take:]
        return calls

    async def _drain(self) -> None:
        try:
            while self.queue:
                await self._run(self._take())
        finally:
            self.busy = False

    async def _run(self, calls: list[_Call]) -> None:
        # encode: the whole batch at once; if a row raises, call by call, so that only the
        # calls whose evidence makes the reference raise get the exception
        try:
            encs = [encode_batch([ev for c in calls for ev in c.evidence_lists], self.cat,
                                 out=self.runner.input_views)]
            ok = calls
        except Exception:
            encs, ok = [], []
            for c in calls:
                try:
                    encs.append(encode_batch(c.evidence_lists, self.cat))
                    ok.append(c)
                except Exception as e:                      # noqa: BLE001 (re-raised per call)
                    if not c.fut.done():
                        c.fut.set_exception(e)
        if not ok:
            return
        enc = concat(encs)
        self.launches += 1
        try:
            res = await self.runner.run(enc)
        except asyncio.CancelledError:
            # the task that launched this batch was cancelled (e.g. an activity timeout) while
            # its kernel runs: finish the launch here -- the next launch reuses its buffers --
            # and serve the other calls of the batch, then let the cancellation through
            try:
                self.runner.sync_last()
                res = self.runner.results()
            except BaseException as e:                      # noqa: BLE001 (re-raised below)
                self._fail(ok, e)
                raise
            self._finish(ok, enc, res)
            raise
        except Exception as e:                              # noqa: BLE001 (device failure)
            self._fail(ok, e)
            return
        self._finish(ok, enc, res)

    @staticmethod
    def _fail(calls: list, e: BaseException) -> None:
        for c in calls:
            if not c.fut.done():
                c.fut.set_exception(e)

    def _finish(self, ok: list, enc: EncodedBatch, res: RulesResult) -> None:
        """Deliver a finished launch's lists; a failure while assembling them goes to every call
        still waiting (none is left pending)."""
        try:
            with gc_paused():
                if enc.n_incidents == len(ok):
                    # every call is one incident (concurrent single calls): one assembly, one
                    # registration, one future per call, no per-call bookkeeping arrays
                    r0 = ok[0].ranked
                    if all(c.ranked == r0 for c in ok):
                        lists = hypothesis_lists(self.cat, res, [c.incident_ids[0] for c in ok],
                                                 enc.evidence_ids, r0)
                        if not r0:
                            FUSED.register(self.cat, res, lists, range(len(lists)))
                        for c, lst in zip(ok, lists):
                            f = c.fut
                            if not f.done():
                                f.set_result(lst if c.single else [lst])
                        return
                if len(ok) == 1:               # (a lone call: its lists are the whole result)
                    c = ok[0]
                    lists = hypothesis_lists(self.cat, res, c.incident_ids, enc.evidence_ids, c.ranked)
                    if not c.ranked:
                        FUSED.register(self.cat, res, lists, range(len(lists)))
                    if not c.fut.done():
                        c.fut.set_result(lists[0] if c.single else lists)
                    return
                # incident rows of every call, then one native assembly per ranking mode
                starts = np.cumsum([0] + [len(c.incident_ids) for c in ok])
                self._deliver(ok, starts, enc, res)
        except BaseException as e:                          # noqa: BLE001
            self._fail(ok, e)
            if not isinstance(e, Exception):
                raise

    def _deliver(self, ok: list, starts, enc: EncodedBatch, res: RulesResult) -> None:
        modes = np.fromiter((c.ranked for c in ok), bool, len(ok))
        counts = np.diff(starts)
        for ranked in (False, True):
            sel = modes == ranked
            if not sel.any():
                continue
            if sel.all():                  # (the common case: every call in one mode)
                cs, sub, eids = ok, res, enc.evidence_ids
            else:
                cs = [c for c, m in zip(ok, sel) if m]
                idx = np.flatnonzero(np.repeat(sel, counts))
                sub = RulesResult(*(a[idx] for a in (
                    res.mask, res.n_hyp, res.order_conf, res.order_rank, res.confidence,
                    res.final_score, res.strength)))
                eids = [enc.evidence_ids[i] for i in idx.tolist()]
            ids = [i for c in cs for i in c.incident_ids]
            lists = hypothesis_lists(self.cat, sub, ids, eids, ranked)
            if not ranked:             # the kernel ranked them too: HypothesisRanker.rank reuses it
                FUSED.register(self.cat, sub, lists, range(len(lists)))
            if all(len(c.incident_ids) == 1 for c in cs):   # (concurrent single calls)
                for c, lst in zip(cs, lists):
                    f = c.fut
                    if not f.done():
                        f.set_result(lst if c.single else [lst])
                continue
            pos = 0
            for c in cs:
                n = len(c.incident_ids)
                if not c.fut.done():
                    c.fut.set_result(lists[pos] if n == 1 and c.single else lists[pos:pos + n])
                pos += n
