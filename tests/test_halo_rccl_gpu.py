"""egr_plan_halo_exchange -- the halo exchange as ONE C-ABI call over an RCCL communicator (pack
into fixed peer slots, ncclAllToAll, unpack), for callers of libegraph.so without torch.  RCCL
refuses two ranks on one GPU, so on the test box the communicator has one rank
(ncclCommInitAll over device 0, created through librccl itself, not torch) and the exchange
sends a set of rows to itself: after it, every "received" row holds exactly the sent row's
scores / reach words, bit for bit, and no other row changed; a communicator whose size is not
the partition count is refused.  Runs in a child process so the communicator never lives in the
pytest process.  (The multi-rank protocol is the one tests/test_shard.py runs over gloo.)"""
from __future__ import annotations

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _main(q):
    try:
        _body(q)
    except BaseException as e:                 # noqa: BLE001 (reported to the parent)
        q.put({"error": repr(e)})


def _body(q):
    import ctypes as C

    import torch
    from egraph import _lib as L
    from egraph import synth
    from egraph.graph import EvidenceGraph
    out = {}
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    rccl = C.CDLL("librccl.so.1")
    comm = C.c_void_p()
    devs = (C.c_int * 1)(0)
    out["init"] = rccl.ncclCommInitAll(C.byref(comm), 1, devs)
    try:
        cfg = synth.ClusterConfig(pods=1200, namespaces=4, nodes=20, deployments=120,
                                  services=80, attach_fraction=0.3, seed=9)
        c = synth.build_cluster(cfg)
        cases = synth.make_incidents(c, 40, seed=10)
        synth.add_incidents(c, cases)
        g = EvidenceGraph()
        g.merge_nodes(c.ids, c.labels)
        g.merge_edges(c.src, c.dst, c.types)
        sv, sc, ss = synth.seeds_for_batch(g, [k.evidence for k in cases])
        src = g.lookup([f"incident:{k.incident['id']}" for k in cases]).astype(np.uint32)
        B = len(src)

        def t(a):
            return torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        plan = g.snapshot().plan(B, max_seeds=len(sv), k=5)
        plan.set_seeds(t(sv), t(sc), t(ss))
        plan.set_sources(t(src))
        for _ in range(2):
            plan.hop()
            plan.reach_hop()
        torch.cuda.synchronize()
        x0 = plan.read_scores().cpu().numpy().copy()
        r0 = plan.read_reach().cpu().numpy().copy()
        V = x0.shape[0]
        nz = np.flatnonzero(x0.any(axis=1))
        rng = np.random.default_rng(3)
        send = np.sort(rng.choice(nz, size=min(60, len(nz) // 2), replace=False)).astype(np.uint32)
        rest = np.setdiff1d(np.arange(V), send)
        recv = np.sort(rng.choice(rest, size=len(send), replace=False)).astype(np.uint32)
        seg = t(np.array([0, len(send)], np.int64))
        rbase = t(np.array([0], np.int64))
        ovf = torch.zeros(1, dtype=torch.int32, device=dev)
        ok = {}
        for what in ("scores", "reach"):
            cap = B * 64 + 16
            words = plan.slot_words(what, cap)
            sbuf = torch.zeros(words, dtype=torch.int64, device=dev)
            rbuf = torch.zeros(words, dtype=torch.int64, device=dev)
            plan.halo_exchange_rccl(what, t(send), seg, cap, sbuf, rbuf, t(recv), rbase, ovf,
                                    comm.value)
            torch.cuda.synchronize()
            ok[what + "_slots_equal"] = bool(torch.equal(sbuf, rbuf))
        x1 = plan.read_scores().cpu().numpy()
        r1 = plan.read_reach().cpu().numpy()
        exp_x = x0.copy()
        exp_x[recv] = x0[send]
        out["scores"] = x1.tobytes() == exp_x.tobytes()
        exp_r = r0.copy()
        exp_r[:, recv] = r0[:, send]
        out["reach"] = np.array_equal(r1, exp_r)
        out["overflow"] = int(ovf.item())
        out.update(ok)
        out["moved_nonzero"] = bool(x0[send].any())
        # a communicator of 1 rank for a 2-partition exchange: refused
        seg2 = t(np.array([0, len(send), len(send)], np.int64))
        rb2 = t(np.array([0, len(send)], np.int64))
        rc = L.lib.egr_plan_halo_exchange(plan._h, 0, L.ptr(t(send)), len(send), L.ptr(seg2), 2, 8,
                                          L.ptr(sbuf), L.ptr(rbuf), L.ptr(t(recv)), len(recv),
                                          L.ptr(rb2), L.ptr(ovf), comm.value, None)
        out["mismatch_rc"] = rc
        out["EINVAL"] = L.EGR_EINVAL
    finally:
        if comm.value:
            rccl.ncclCommDestroy(comm)
    q.put(out)


def test_halo_exchange_over_rccl():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_main, args=(q,))
    p.start()
    out = q.get(timeout=240)
    p.join(60)
    assert p.exitcode == 0, out
    assert out["init"] == 0, out
    assert out["moved_nonzero"] and out["overflow"] == 0, out
    assert out["scores_slots_equal"] and out["reach_slots_equal"], out
    assert out["scores"] and out["reach"], out
    assert out["mismatch_rc"] == out["EINVAL"], out
