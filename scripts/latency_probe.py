"""Single-incident latency of the drop-in rules path, piece by piece (diagnostic; GPU box).
Prints p50 / p99 (us) of: the reference restatement, encode, the zero-copy and staged runner
round trips (sync and polled from asyncio), generate_hypotheses, generate + rank."""
import asyncio
import sys
import time
from pathlib import Path
from types import SimpleNamespace

REPO = Path(__file__).resolve().parents[1]
for p in (REPO / "kubernetes-aiops-evidence-graph_amd", REPO / "oracle", REPO / "tests"):
    sys.path.insert(0, str(p))
import numpy as np
import torch

import rca_oracle
from egraph import catalog, synth
from egraph.batcher import RulesRunner
from egraph.encode import encode_batch
from egraph.rca import hypothesis_lists
from src.services.rca import rules_engine as RE
from src.services.rca.hypothesis_ranker import HypothesisRanker

N = 300
cat = catalog.default()
c = synth.build_cluster(synth.CONFIGS["C3"])
cases = synth.make_incidents(c, N, seed=1000)
ev = [x.evidence for x in cases]
incs = [SimpleNamespace(id=f"inc-{i}") for i in range(N)]
encs = [encode_batch([e], cat) for e in ev]


def stat(name, f, n=N):
    f(0)
    t = []
    for i in range(n):
        a = time.perf_counter()
        f(i)
        t.append(time.perf_counter() - a)
    t = np.array(t) * 1e6
    print(f"{name:42s} p50 {np.percentile(t, 50):8.1f}  p99 {np.percentile(t, 99):8.1f}", flush=True)


stat("reference (rca_oracle.rca)", lambda i: rca_oracle.rca(incs[i].id, ev[i]))
stat("encode_batch (1 incident)", lambda i: encode_batch([ev[i]], cat))
r = RulesRunner(cat)
stat("runner zero-copy run_sync", lambda i: r.run_sync(encs[i]))
r2 = RulesRunner(cat)
r2.ZERO_COPY_ROWS = -1
stat("runner staged run_sync", lambda i: r2.run_sync(encs[i]))
res = r.run_sync(encs[0])
stat("assemble (hypothesis_lists)", lambda i: hypothesis_lists(cat, res, ["x"], encs[0].evidence_ids, False))
st = torch.cuda.Stream()
ev0 = torch.cuda.Event()


def empty(i):
    with torch.cuda.stream(st):
        torch.cuda._sleep(0)
    ev0.record(st)
    ev0.synchronize()


stat("empty kernel + event sync", empty)


def empty_spin(i):
    with torch.cuda.stream(st):
        torch.cuda._sleep(0)
    ev0.record(st)
    while not ev0.query():
        pass


stat("empty kernel + event query spin", empty_spin)
stat("runner launch only (host enqueue)", lambda i: r.launch(encs[i]) and torch.cuda.synchronize())
stat("runner zero-copy launch+query spin", lambda i: [None for _ in iter(r.launch(encs[i]).query, True)])


async def poll(i):
    return await r.run(encs[i])
stat("runner zero-copy asyncio run", lambda i: asyncio.run(poll(i)))
eng = RE.RulesEngine()
rk = HypothesisRanker()


async def many(fn):
    t = []
    for i in range(N):
        a = time.perf_counter()
        await fn(i)
        t.append(time.perf_counter() - a)
    return np.array(t) * 1e6


async def gen(i):
    return await eng.generate_hypotheses(incs[i], ev[i])


async def gen_rank(i):
    return rk.rank(await eng.generate_hypotheses(incs[i], ev[i]))


for name, fn in (("generate_hypotheses (one loop)", gen), ("generate + rank (one loop)", gen_rank)):
    asyncio.run(many(fn))
    t = asyncio.run(many(fn))
    print(f"{name:42s} p50 {np.percentile(t, 50):8.1f}  p99 {np.percentile(t, 99):8.1f}", flush=True)
hyps = [asyncio.run(gen(i)) for i in range(N)]
import copy
from egraph import ranker


def stat_pre(name, f, prep):
    """like stat(), with an untimed per-call input built by prep(i)"""
    t = []
    for i in range(N):
        x = prep(i)
        a = time.perf_counter()
        f(x)
        t.append(time.perf_counter() - a)
    t = np.array(t) * 1e6
    print(f"{name:42s} p50 {np.percentile(t, 50):8.1f}  p99 {np.percentile(t, 99):8.1f}", flush=True)


stat("runner small launch+spin+results", lambda i: (lambda e: ([None for _ in iter(e.query, True)], r.results()))(r.launch(encs[i])))
r.launch(encs[0]).synchronize()
stat("runner results() copy", lambda i: r.results())
stat("FUSED.register (1 list)", lambda i: ranker.FUSED.register(cat, res, [hyps[i]], [0]))
for i in range(N):                                  # re-register the generated lists
    asyncio.run(gen(i))
hyps = [asyncio.run(gen(i)) for i in range(N)]
stat_pre("rank via fused record", rk.rank, lambda i: copy.deepcopy(hyps[i]))
ranker.FUSED.recs.clear()
stat_pre("rank via egr_rank (zero-copy)", rk.rank, lambda i: copy.deepcopy(hyps[i]))
