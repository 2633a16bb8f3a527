"""Benchmark: incidents RCA-ranked/s + edges/s (3-hop propagation) on the 100k-pod graph.

One step = one pass of the hot path over one batch of B incidents whose inputs are already
resident in HBM (encoded evidence rows, seed triples, incident vertices):
  --engine frontier (default):
    egr_rules_eval (A1-A6, fused ranker)  ->  egr_frontier_set_seeds (radix sort by (column,
    vertex) + max-combine)  ->  egr_frontier_run (per column: 3-hop reach + 3-hop propagation
    + top-k in one workgroup, LDS hash table; overflow columns in the global-memory variant)
  --engine dense:
    egr_rules_eval  ->  egr_plan_set_seeds  ->  egr_plan_set_sources
    ->  3 x (egr_plan_hop + egr_plan_reach_hop)  ->  egr_plan_candidates  ->  egr_plan_topk.
Both engines produce bit-identical scores, reach sets and top-k (tests/test_frontier_gpu.py).
Frontier batches are scheduled explicitly on ONE stream (--merge, default: the largest divisor
of --steps up to 50): a launch carries M consecutive batches (M x B columns, each batch's seeds
at its own column offset, rules over the M batches' rows) and the hardware dispatcher hands its
workgroups out costliest column first across all M batches, so one batch's tail (its last,
unevenly long columns) runs beside the next batch's columns inside the same launch.  Nothing
depends on how streams map to HIP's hardware queues (GPU_MAX_HW_QUEUES 1 / 2 / 4 within 1 %;
round 2's three lanes on four queues was an accident of that mapping: 35-140 % slower on any
other setting, profiles/r03_ab_merge_schedule.txt).  --pipeline P > 1 still runs P such lanes
on their own streams.  Every batch is computed in full; `value` = batches x B / wall time of
the timed region.
The default run also times a few dense steps after the timed region and reports them under
"dense_engine" (with the dense hop kernel's HBM roofline) for comparison.
Workload: BASELINE.json configs[2] (C3: 100k pods / 100 namespaces / 2k nodes / 10k
deployments / 10k services, Event/LogPattern/MetricAnomaly vertices; synthetic, seeded).
Multi-GPU (torchrun): every rank holds the snapshot and ranks its own B incidents -- incidents
are independent, so there is no collective on the data path (weak scaling); the barrier and
the max-over-ranks timing are the only communication.

--shard graph (BASELINE configs[3], C4: the 1M-vertex graph edge-cut across the ranks,
egraph/shard.py): each rank owns a partition (local snapshot + dense plan) and the whole job
ranks ONE batch of B incidents per step; per hop the boundary rows are exchanged point-to-point
(RCCL all_to_all_single over xGMI), the candidate lists are all-gathered and merged (strong
scaling).  `--partitions P` on one GPU runs P partitions in one process (device-copy exchange).
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "kubernetes-aiops-evidence-graph_amd"))

METRIC = "incidents RCA-ranked/sec + edges/sec (3-hop propagation), 100k-pod graph"
XGMI_LINK_GBS = 153.0          # one xGMI link, GB/s (MI355X_MICROARCH.md)
# The edge-cut projection's charge per RCCL collective on the critical path (a stated assumption,
# not a measurement: RCCL refuses two ranks on one GPU, so the 8-GPU latency cannot be timed on
# the 1-GPU box; small-message all-to-all / all-gather over 8 MI355X on xGMI are tens of us).
# The JSON also carries the projection at 10 and 60 us.
RCCL_COLL_LATENCY_US = 30.0
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
L2_PEAK_GBS = 34500.0   # MI355X_MICROARCH.md: the eight XCD L2s together, ~34.5 TB/s
# --merge default cap: a launch costs ~0.12 ms of tail + ~0.055 ms per C3 batch (0.0734 / 0.0653 /
# 0.0626 ms per batch at 8 / 16 / 24 batches, profiles/r03_ab_merge_schedule.txt).  The M batches
# of a launch are M different incident sets, all open in the graph (M x B incidents): 20 sets
# (20,480 incidents) bring C3 to 254k vertices / 1.13M CSR entries, SURVEY §8d's ~250k vertices
MERGE_MAX = 20


BACKEND = os.environ.get("EGRAPH_BENCH_BACKEND", "nccl")
# --seed-input (main sets it): "grouped" = the seed triples arrive grouped by incident with
# their column offsets (the host's seed attachment emits them incident by incident;
# egr_frontier_run_grouped) and the costliest-first launch order is computed on the device in
# every step (two small kernels in the captured step); "grouped-host-order" (A/B) = the same with
# the order computed once on the host outside the timed region; "sort" = unordered triples,
# sorted by column on the device in every step (egr_frontier_set_seeds: count, scan, scatter)
GROUPED = "device"


def max_over_ranks(dist, x: float, dev) -> float:
    t = torch.tensor([x], dtype=torch.float64, device=dev if BACKEND == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def timed_steps(one_step, steps: int, dist, rank: int, sync, dev) -> float:
    """The timed region of the contract: barrier + device sync, exactly `steps` steps, device
    sync + barrier; returns the MAX over ranks of the elapsed seconds (every rank returns it).
    `sync` waits for this rank's device work (torch.cuda.synchronize on the GPU)."""
    if dist:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        one_step()
    t_enq = time.perf_counter() - t0
    sync()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    log(f"[rank {rank}] host enqueue {t_enq / steps * 1e3:.4f} ms/step, "
        f"wall {elapsed / steps * 1e3:.4f} ms/step")
    if dist:
        elapsed = max_over_ranks(dist, elapsed, dev)
    return elapsed


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def launch_ranks(n: int) -> int:
    """Run this command line as n ranks under torch.distributed.run (child process; the caller
    has not touched the GPU); returns its exit status."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)]
    log(f"bench.py: launching {n} ranks: {' '.join(cmd)} {' '.join(sys.argv[1:])}")
    return subprocess.call(cmd + sys.argv[1:])


def setup(config: str, B: int, k: int, rank: int, dev: torch.device, pipeline: int = 1,
          pool_entries: int = 0, merge: int = 1, replicate: bool = False):
    from egraph import catalog
    from egraph.device import to_device
    from egraph.encode import encode_batch
    from egraph.rca import RulesDeviceBatch
    t0 = time.time()
    # --merge M: the M batches of one launch are M DIFFERENT incident sets (distinct_batches);
    # every one of them is open in the graph, so the graph holds M x B incidents.  --pipeline P
    # lanes: each lane's launches carry their OWN M sets (P x M distinct sets in all -- lanes
    # in flight at once never share columns, whose common rows would meet in L2).  Each rank
    # builds its own graph with its own incident sets (per-GPU work fixed: weak scaling)
    per_lane = merge if merge > 1 else 1
    n_sets = 1 if replicate else per_lane * max(pipeline, 1)
    g, batches = make_world(config, B, n_sets, seed0=1000 + rank * n_sets)
    evidence, sv, sc, ss, src = batches[0]
    enc = encode_batch(evidence, catalog.default())
    log(f"[rank {rank}] built {config}: V={g.num_vertices} E={g.num_edges} rows={enc.n_rows} "
        f"seeds={len(sv)} incident sets={n_sets} in {time.time() - t0:.1f}s")
    with torch.cuda.device(dev):
        snap = g.snapshot(device=dev)
        plan = snap.plan(B, max_seeds=len(sv), k=k)
        rules = RulesDeviceBatch(enc, catalog.default(), dev)
        seeds = tuple(to_device(a, dev) for a in (sv, sc, ss))
        sources = to_device(src, dev)
        # --merge M: a lane's launch carries M consecutive batches (M x B columns, each batch's
        # seeds at its own column offset, the rules over the M batches' rows): the hardware
        # dispatcher hands the columns out costliest-first across all M batches, so batch i's
        # tail runs beside batch i+1's columns inside one launch on one stream
        # (lane l's batch i = batches[l * M + i]; --replicate-batches (A/B only): M copies of
        # batch 0, round 3's launch, whose adjacent copies share L2 lines)
        Bm = B * merge
        lane_in = []
        for ln in range(max(pipeline, 1)):
            if merge > 1:
                parts = [batches[(ln * merge + i) % n_sets] for i in range(merge)]
                msv, msc, mss, msrc = merge_batches([p[1:] for p in parts], B)
                lane_in.append((tuple(to_device(a, dev) for a in (msv, msc, mss)), to_device(msrc, dev),
                                encode_batch([ev for p in parts for ev in p[0]], catalog.default()),
                                (msv, msc, mss, msrc)))
            else:
                ev_l, sv_l, sc_l, ss_l, src_l = batches[ln % n_sets]
                if ln == 0:
                    lane_in.append((seeds, sources, rules, (sv, sc, ss, src)))
                else:
                    lane_in.append((tuple(to_device(a, dev) for a in (sv_l, sc_l, ss_l)),
                                    to_device(src_l, dev), encode_batch(ev_l, catalog.default()),
                                    (sv_l, sc_l, ss_l, src_l)))
        n_seeds = max(len(x[3][0]) for x in lane_in)
        lane_enc = lane_in[0][2] if merge > 1 else enc
        lane_host = lane_in[0][3]
        # pool_entries=-1: top-k only, as GraphService runs it (the last pull then skips the
        # members outside the candidate set); 0 keeps every member's score for inspection
        fr = snap.frontier(Bm, max_seeds=n_seeds, k=k, pool_entries=pool_entries)
        lanes = build_lanes(snap, Bm, n_seeds, k, pipeline, pool_entries, dev,
                            [(fr if ln == 0 else None, x[2], x[0], x[1]) for ln, x in enumerate(lane_in)])
        torch.cuda.synchronize(dev)
    inc_label = g.labels().index("Incident")
    return dict(config=config, graph=g, snap=snap, plan=plan, frontier=fr, rules=rules, seeds=seeds, sources=sources,
                lanes=lanes, tick=0, merge=merge, sub=0, enc=enc, seed_host=(sv, sc, ss), src_host=src, inc_label=inc_label,
                evidence=evidence, incident_ids=[str(e[0]["incident_id"]) for e in evidence],
                distinct_batches=min(n_sets, per_lane), incidents_in_graph=n_sets * B,
                distinct_sets=n_sets,
                # lane 0's launch input on the host (all M batches: seeds, incident vertices,
                # encoded rows): what the parity test of the headline launch checks against
                lane_host=lane_host, lane_enc=lane_enc)


def make_world(config: str, B: int, n_sets: int, seed0: int = 1000, cfg=None):
    """The config's cluster with n_sets incident sets of B incidents each (make_incidents seeds
    seed0, seed0 + 1, ...) all added to ONE graph; per set (evidence lists, seed vertex, seed
    column, seed strength, incident vertex per column).  `cfg` overrides the cluster config."""
    from egraph import synth
    cl = synth.build_cluster(cfg or synth.CONFIGS[config])
    sets = []
    for i in range(n_sets):
        cases = synth.make_incidents(cl, B, seed=seed0 + i)
        synth.add_incidents(cl, cases)
        sets.append(cases)
    g = synth.build_graph(cl)                 # C4: with its dense telemetry links (~10M entries)
    if os.environ.get("EGRAPH_BENCH_HUB_ORDER"):
        # (experiment: the same graph MERGEd in egraph.graph.locality_order's vertex order)
        from egraph.graph import EvidenceGraph, locality_order
        csr = g.csr()
        o = locality_order(csr["row_ptr"], csr["col"])
        ids, labels = g.vertex_ids(), g.labels()
        vl, es, ed, et = g.export()
        g2 = EvidenceGraph()
        g2.merge_nodes([ids[v] for v in o], [labels[vl[v]] for v in o])
        pos = np.empty(len(o), np.int64)
        pos[o] = np.arange(len(o))
        g2.add_edges_indexed(pos[es], pos[ed], et.astype(np.int32), g.rel_types())
        g = g2
    out = []
    for cases in sets:
        evidence = [x.evidence for x in cases]
        sv, sc, ss = synth.seeds_for_batch(g, evidence)
        src = g.lookup([f"incident:{x.incident['id']}" for x in cases]).astype(np.uint32)
        out.append((evidence, sv, sc, ss, src))
    return g, out


def merge_batches(batches: list, B: int) -> tuple:
    """One launch's input from M batches of B incidents, each (seed vertex, seed column, seed
    strength, source vertex per column): batch i's columns become columns i*B .. i*B + B - 1."""
    sv = np.concatenate([np.asarray(b[0]) for b in batches])
    sc = np.concatenate([np.asarray(b[1], np.int64) + i * B for i, b in enumerate(batches)])
    ss = np.concatenate([np.asarray(b[2]) for b in batches])
    src = np.concatenate([np.asarray(b[3]) for b in batches])
    return sv, sc.astype(np.asarray(batches[0][1]).dtype), ss, src


def build_lanes(snap, B: int, max_seeds: int, k: int, pipeline: int, pool_entries: int, dev,
                inputs: list) -> list[dict]:
    """--pipeline P: P independent frontier + rules states, each on its own pair of streams;
    consecutive batches alternate between them so one batch's tail overlaps the next batch's
    start (every batch is still computed in full).  inputs[i] = (frontier or None, rules batch
    or the encoded rows to build one from, seed tensors, source tensor) of lane i."""
    from egraph import catalog
    from egraph.rca import RulesDeviceBatch
    lanes = []
    # $EGRAPH_BENCH_LANE_STREAMS=S (A/B): the lanes share S stream pairs round-robin (lanes on
    # one stream run their batches in order); default: a pair per lane
    share = int(os.environ.get("EGRAPH_BENCH_LANE_STREAMS", "0") or 0)
    pairs: list = []
    for i, (fr, rules, seeds, sources) in enumerate(inputs):
        if fr is None:
            fr = snap.frontier(B, max_seeds=max_seeds, k=k, pool_entries=pool_entries)
        if not isinstance(rules, RulesDeviceBatch):
            rules = RulesDeviceBatch(rules, catalog.default(), dev)
        if share <= 0 or len(pairs) < share:
            pairs.append((torch.cuda.Stream(dev) if pipeline > 1 else None,
                          None if os.environ.get("EGRAPH_BENCH_ONE_STREAM") else torch.cuda.Stream(dev)))
        main, side = pairs[i % share] if share > 0 else pairs[-1]
        lane = dict(frontier=fr, rules=rules, seeds=seeds, sources=sources, main=main, side=side)
        set_lane_seeds(lane, seeds, B, snap, dev)
        lanes.append(lane)
    return lanes


def set_lane_seeds(lane: dict, seeds: tuple, B: int, snap, dev, row_ptr=None) -> None:
    """A lane's seed input: the device triples, and for --seed-input grouped their grouping by
    column (offsets) and the costliest-first launch order, built on the host."""
    lane["seeds"] = seeds
    lane.pop("grouped", None)
    lane["order"] = None
    if GROUPED:
        from egraph.graph import group_seeds, launch_order
        gp, gv, gs = group_seeds(*(a.cpu().numpy() for a in seeds), B)
        lane["grouped"] = tuple(torch.from_numpy(x).to(dev) for x in
                                (gp.view(np.int32), gv.view(np.int32), gs))
        if GROUPED == "order":          # (A/B: --seed-input grouped-host-order)
            rp = row_ptr if row_ptr is not None else snap.download()["row_ptr"]
            lane["order"] = torch.from_numpy(launch_order(gp, gv, rp).view(np.int32)).to(dev)


GRAPH_MERGE_MAX = 8      # eager launches from this many batches per launch up (main())


def warm_up(ctx, hops: int, warmup: int, dev, rank: int = 0, engine: str = "frontier",
            graphs: bool = True):
    """The untimed part of a run, as main() does it: `warmup` eager steps (at least one per lane
    and launch group), then -- frontier -- two looks of Frontier.adapt() at the stats (overflow
    handling for graphs whose columns overflow the narrow table: continuation regions, the wide
    retry behind them; mid- or wide-first when most do) with warm-up steps after each, then the
    lanes captured as HIP graphs and replayed
    `warmup` times.  Returns the step function of the timed region."""
    M = ctx.get("merge", 1)
    run_step = step_frontier if engine == "frontier" else step
    # (at least one step per lane: every lane's frontier has run before adapt() reads its stats)
    for _ in range(max(warmup, len(ctx.get("lanes", ())) * M)):
        run_step(ctx, hops)
    torch.cuda.synchronize(dev)
    if engine == "frontier":
        # graphs with large 3-hop neighbourhoods: columns that overflow the narrow table continue
        # in global-memory regions inside the grid from here on, the wide-table retry behind
        # them (egraph.graph.Frontier.adapt)
        # most columns overflowing the narrow table: the mid table first; a second look after the
        # next warm-up steps moves to wide-first if most columns overflow that one too
        for check in range(2):
            for lane in ctx["lanes"]:
                fr = lane["frontier"]
                if fr.adapt(fr.stats()):
                    log(f"[rank {rank}] overflow handling on (wide retry {fr.retry_blocks} blocks, "
                        f"{fr.continuation_regions} continuation regions), first table "
                        f"{FIRST_TABLE[fr.wide_first]}")
            for _ in range(max(warmup, 1)):
                run_step(ctx, hops)
            torch.cuda.synchronize(dev)
    if graphs and engine == "frontier":
        capture_lanes(ctx, hops)
        run_step = step_graph
        for _ in range(warmup):
            run_step(ctx, hops)
        torch.cuda.synchronize(dev)
    return run_step


def _launch_due(ctx) -> bool:
    """--merge M: batch t is launched by the launch of batch t - t % M (the first of its group);
    the other M - 1 calls enqueue nothing.  A timed region of K steps with K % M != 0 computes
    the whole last group (more work than it counts)."""
    m = ctx.get("merge", 1)
    if m <= 1:
        return True
    due = ctx["sub"] == 0
    ctx["sub"] = (ctx["sub"] + 1) % m
    return due


_GRAPH_NAME = {"C2": "10k-pod", "C3": "100k-pod", "C4": "400k-pod (1M-vertex)"}


def step_frontier(ctx, hops: int, ev=None):
    """One pass; `ev` (EventPool) times the frontier run on its stream.  The rules launch does
    not depend on the graph stages (nor they on it), so it goes to a second stream, enqueued
    first: its waves (35 VGPRs, no LDS) run while the host enqueues the frontier chain and the
    cost / order kernels run, ahead of the narrow kernel, whose workgroups (72 VGPRs, seven
    waves per SIMD) then fill the CUs (the launch chain).  The timed region ends
    with a device-wide synchronize, which joins every stream."""
    if not _launch_due(ctx):
        return None
    lane = ctx["lanes"][ctx["tick"] % len(ctx["lanes"])]
    ctx["tick"] += 1
    # (the lane's stream by handle: no stream context to enter and leave)
    lane_step(lane, hops, ctx["inc_label"], ev, cur=lane["main"])
    return lane


def lane_step(lane, hops: int, inc_label: int, ev=None, fork_join: bool = False, cur=None):
    """One batch on one lane (the current stream): the rules on the lane's side stream, then the
    seed preparation and the frontier run.  Eager: launched with stream handles, not stream
    contexts (those cost ~40 us of host time ahead of the frontier's chain,
    profiles/r05_timeline_eager.txt); the rules kernel runs while the host enqueues that chain
    -- enqueued after it instead, it shares the CUs with the frontier kernel and slows it more
    than it saves, with the frontier on a high-priority stream and the rules on a low-priority
    one too (profiles/r05_ab_rules_last.txt).  fork_join (graph capture): the side stream forks from the current stream
    and joins it again after the frontier launch."""
    fr = lane["frontier"]
    side = lane["side"]
    if cur is None:
        cur = torch.cuda.current_stream()
    st = cur.cuda_stream
    if fork_join:
        if side is not None:
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                lane["rules"].launch()
        else:
            lane["rules"].launch()
    else:
        lane["rules"].launch(side.cuda_stream if side is not None else st)

    def run():
        if "grouped" in lane:
            fr.run_grouped(*lane["grouped"], lane["sources"], hops, inc_label, order=lane["order"],
                           stream=st)
        else:
            fr.run(lane["sources"], hops, inc_label, stream=st)
    if "grouped" not in lane:
        fr.set_seeds(*lane["seeds"], stream=st)
    if ev is not None:
        a, b = ev.pop()
        a.record(cur)
        run()
        b.record(cur)
        ev.done.append((a, b))
    else:
        run()
    if fork_join and side is not None:
        cur.wait_stream(side)


def capture_lanes(ctx, hops: int, inline_rules: bool | None = None) -> None:
    """Capture each lane's batch (rules on the side stream, seed count / scan / scatter, the
    frontier kernel and the overflow grid) as one HIP graph: a step then costs one graph launch
    of host time instead of seven library calls.  The captured kernels are exactly the eager
    ones (same arguments, same buffers); the host-side state they depend on (the frontier's
    clean-counter flags) is constant in steady state, which one eager warm-up step settles."""
    inc = ctx["inc_label"]
    if inline_rules is None:
        # rules inline on the lane's stream (default): a captured fork / join to a side stream
        # made replays slower on ROCm 7 (0.113 vs 0.0745 ms per step, profiles/r02_graph_ab.txt)
        inline_rules = os.environ.get("EGRAPH_BENCH_GRAPH_FORK_RULES") is None
    for lane in ctx["lanes"]:
        if inline_rules:
            lane["side"] = None                        # rules on the lane's own stream
        st = lane["main"] if lane["main"] is not None else torch.cuda.Stream()
        lane["cap_stream"] = st
        with torch.cuda.stream(st):
            lane_step(lane, hops, inc)                 # settles the clean flags
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            lane_step(lane, hops, inc, fork_join=True)
        torch.cuda.synchronize()
        lane["graph"] = g


def step_graph(ctx, hops: int, ev=None):
    """One batch = one replay of the next lane's captured graph on that lane's stream (with
    --merge M, one replay per M batches: the call that starts a group of M launches them all)."""
    if not _launch_due(ctx):
        return None
    lane = ctx["lanes"][ctx["tick"] % len(ctx["lanes"])]
    ctx["tick"] += 1
    with torch.cuda.stream(lane["cap_stream"]):
        if ev is not None:
            # HIP events on the lane's stream around the replay: its span on the GPU (from its
            # first kernel's start to its last kernel's end, the wait for CUs held by the other
            # batches in flight included)
            a, b = ev.pop()
            a.record()
            lane["graph"].replay()
            b.record()
            ev.done.append((a, b))
        else:
            lane["graph"].replay()
    return lane


class EventPool(list):
    """Pre-created timing events (creating them inside the timed loop costs host time)."""

    def __init__(self, n: int):
        super().__init__((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                         for _ in range(n))
        self.done: list = []
        # (torch creates an event's HIP event at its first record: do that here, not in the
        # timed region)
        for a, b in self:
            a.record()
            b.record()
        torch.cuda.synchronize()


def step(ctx, hops: int, ev=None):
    """One pass; `ev` (list) collects (start, end) events around the dense hop launches."""
    plan = ctx["plan"]
    ctx["rules"].launch()
    plan.set_seeds(*ctx["seeds"])
    plan.set_sources(ctx["sources"])
    for h in range(hops):
        if ev is not None and h > 0:                      # dense (non-seed) hops are timed
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            plan.hop()
            b.record()
            ev.append((a, b))
        else:
            plan.hop()
        plan.reach_hop()
    # candidate lists from the final reach sets, so top-k reads only the reached vertices
    plan.candidates(ctx["inc_label"])
    plan.topk(ctx["inc_label"])


def dropin_rules(ctx, dev, reps: int = 5, n_single: int = 1024) -> dict:
    """The drop-in API end to end (host-bound; reported beside `value`, never as it):
      * batch: RulesEngine.rank_incidents_batch on the bench batch (evidence dicts in, ranked
        hypothesis dicts out: native encode, one packed upload, egr_rules_eval, one packed
        download, native dict assembly);
      * single-call latency: generate_hypotheses + HypothesisRanker.rank for one incident at a
        time (the reference activities' pattern), p50 / p99, beside the reference's own path
        (the pure-Python restatement) on the same incidents;
      * concurrent: every incident of the batch as its own generate_hypotheses +
        rank call, all in flight at once (concurrent activities): the batcher coalesces them."""
    import asyncio
    from types import SimpleNamespace

    sys.path.insert(0, str(REPO / "oracle"))
    import rca_oracle
    from egraph import catalog
    from egraph.batcher import RulesRunner, gc_paused
    from egraph.encode import encode_batch
    from egraph.rca import hypothesis_lists
    from src.services.rca import rules_engine as RE
    from src.services.rca.hypothesis_ranker import HypothesisRanker
    ev = ctx["evidence"]
    incs = [SimpleNamespace(id=f"inc-{i}") for i in range(len(ev))]
    eng = RE.RulesEngine(device=dev)
    cat = catalog.default()
    ranker = HypothesisRanker()

    async def batches(n):
        # one event loop for all the calls, as in a service (asyncio.run per call would add
        # the loop's creation and teardown to every batch)
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            await eng.rank_incidents_batch(incs, ev)
            ts.append(time.perf_counter() - t0)
        return ts

    asyncio.run(batches(1))                                   # warm
    t = asyncio.run(batches(reps))
    parts = np.zeros(3)
    runner = RulesRunner(cat, dev)
    for _ in range(reps):
        a = time.perf_counter()
        enc = encode_batch(ev, cat)
        b = time.perf_counter()
        res = runner.run_sync(enc)
        c = time.perf_counter()
        with gc_paused():                        # as the batcher assembles (egraph/batcher.py)
            hypothesis_lists(cat, res, [x.id for x in incs], enc.evidence_ids, True)
        parts += (b - a, c - b, time.perf_counter() - c)
    best = min(t)
    n1 = min(n_single, len(ev))

    async def single():
        lat = []
        for i in range(n1):
            t0 = time.perf_counter()
            ranker.rank(await eng.generate_hypotheses(incs[i], ev[i]))
            lat.append(time.perf_counter() - t0)
        return lat

    asyncio.run(single())                                          # warm
    gc.collect()               # (both single-call loops start from a collected heap)
    lat = np.array(asyncio.run(single())) * 1e6
    gc.collect()
    ref = []
    for i in range(n1):
        t0 = time.perf_counter()
        rca_oracle.rca(incs[i].id, ev[i])
        ref.append(time.perf_counter() - t0)
    ref = np.array(ref) * 1e6

    async def concurrent():
        # one event loop, as in a worker: a warm-up round, then the best of five rounds, each
        # from a collected heap
        async def one(i):
            return ranker.rank(await eng.generate_hypotheses(incs[i], ev[i]))
        b0 = RE._batcher(eng.catalog, eng.device)
        await asyncio.gather(*[one(i) for i in range(len(ev))])
        l0, ts = b0.launches, []
        for _ in range(5):
            gc.collect()
            t0 = time.perf_counter()
            await asyncio.gather(*[one(i) for i in range(len(ev))])
            ts.append(time.perf_counter() - t0)
        log(f"concurrent drop-in rounds (ms): {[round(t * 1e3, 2) for t in ts]}")
        return min(ts), (b0.launches - l0) // 5

    t_conc, conc_launches = asyncio.run(concurrent())

    async def floor():
        # the event loop's own cost for the same pattern: len(ev) tasks, each awaiting a future
        # that one batch resolves (no rules, no ranking) -- the bound on `concurrent`
        loop = asyncio.get_running_loop()
        futs: list = []

        async def wait_one():
            f = loop.create_future()
            futs.append(f)
            return await f

        async def resolve():
            await asyncio.sleep(0)
            for f in futs:
                f.set_result(None)
        ts = []
        for _ in range(3):
            futs.clear()
            gc.collect()
            t0 = time.perf_counter()
            await asyncio.gather(resolve(), *[wait_one() for _ in range(len(ev))])
            ts.append(time.perf_counter() - t0)
        return min(ts)
    t_floor = asyncio.run(floor())
    from egraph.encode import encode_threads
    return {"value": len(ev) / best, "unit": "incidents/s",
            "cores": encode_threads(), "cores_note": "the encoder's parallel row pass; assembly "
                                                     "and the rest on the calling thread",
            "ms_per_batch": best * 1e3, "incidents": len(ev),
            "encode_ms": parts[0] / reps * 1e3, "device_ms": parts[1] / reps * 1e3,
            "assemble_ms": parts[2] / reps * 1e3,
            "what": "RulesEngine.rank_incidents_batch, evidence dicts -> ranked hypothesis dicts",
            "single_call_us": {"p50": float(np.percentile(lat, 50)), "p99": float(np.percentile(lat, 99)),
                               "calls": n1,
                               "what": "generate_hypotheses + HypothesisRanker.rank, one incident "
                                       "at a time (idle engine: launched at once)"},
            "reference_single_call_us": {"p50": float(np.percentile(ref, 50)),
                                         "p99": float(np.percentile(ref, 99)),
                                         "what": "the reference's Python path (oracle/rca_oracle.py "
                                                 "restatement), same incidents, 1 core"},
            "concurrent": {"value": len(ev) / t_conc, "unit": "incidents/s",
                           "calls": len(ev), "launches": conc_launches,
                           "asyncio_floor": len(ev) / t_floor,
                           "asyncio_floor_what": "the same number of tasks awaiting futures one "
                                                 "batch resolves, nothing else: CPython's own cost "
                                                 "for one task per call on this host",
                           "what": "every incident its own generate_hypotheses + rank call, all "
                                   "in flight at once; the batcher coalesces them"}}


def dropin_graph(ctx, dev, hops: int, k: int, reps: int = 5) -> dict:
    """The graph half of the drop-in end to end (host buffers; reported beside `value`, never as
    it): activities.rank_root_causes_batch on the bench batch -- evidence dicts in, seed
    attachment on the host (egraph.seeds.seeds_for_batch), seed upload, the frontier through
    torch.ops.egraph.frontier_run, download, ranked root-cause entity dicts out -- over the
    bench's own graph and snapshot installed in GraphService (src/database/graph.py)."""
    import asyncio

    from src.database import GraphService
    from src.services.workflow import activities
    GraphService.reset()
    GraphService._graph, GraphService._snapshot, GraphService.device = ctx["graph"], ctx["snap"], dev
    data = [{"incident": {"id": i}, "evidence": {"evidence": ev}, "k": k}
            for i, ev in zip(ctx["incident_ids"], ctx["evidence"])]

    async def go(n):
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            out = await activities.rank_root_causes_batch(data)
            ts.append(time.perf_counter() - t0)
        return ts, out

    asyncio.run(go(1))                                            # warm (frontier creation)
    ts, out = asyncio.run(go(reps))
    # the same call's stages (GraphService.rank_root_causes_sync(stages=...): the device is
    # synchronised between stages, so the parts add up to the call; untimed in `value`)
    stages: dict = {}
    for _ in range(reps):
        GraphService.rank_root_causes_sync([d["incident"]["id"] for d in data], ctx["evidence"],
                                           hops, k, stages=stages)
    stages_ms = {name: t / reps * 1e3 for name, t in stages.items()}
    t_seed = stages_ms["seed_attach"] / 1e3
    best = min(ts)
    # the same batch's ids from the bench's own frontier (lane 0 ran the same evidence): the
    # drop-in's entities must be the engine's top-k
    g = ctx["graph"]
    # (--merge: the lane's first len(data) columns are this batch)
    ids0 = ctx["lanes"][0]["frontier"].out_ids.view(-1, k)[:len(data)].cpu().numpy().view(np.uint32)
    same = all([e["id"] for e in row] == [g.vertex_id(int(v)) for v in ids0[b] if v != 0xFFFFFFFF]
               for b, row in enumerate(out))
    GraphService.reset()
    return {"value": len(data) / best, "unit": "incidents/s", "ms_per_batch": best * 1e3,
            "incidents": len(data), "seed_attach_ms": t_seed * 1e3, "matches_engine_topk": same,
            "stages_ms": stages_ms,
            "stages_note": "GraphService.rank_root_causes_sync with the device synchronised between "
                           "stages (sum ~ one call without the activity's to_thread hop)",
            "what": "activities.rank_root_causes_batch: evidence dicts -> host seed attachment -> "
                    "torch.ops.egraph.frontier_run (3-hop propagation + reach + top-k) -> ranked "
                    "root-cause entity dicts"}


def cpu_baseline(ctx, hops: int, k: int, threads: int, seconds: float = 8.0) -> dict:
    """The same step on the host cores: oracle/egraph_oracle.c's rules restatement plus
    orc_frontier (the frontier engine's algorithm per column: touched vertices only, pruned last
    hop; bit-identical results, tests/test_oracle_frontier.py), OpenMP `threads`, repeated for
    about `seconds`.  Context beside it: the reference's own CPU path (the Python rules engine +
    ranker, restated in oracle/rca_oracle.py) on one core, and the dense C port (V x B sweep
    per hop) once."""
    sys.path.insert(0, str(REPO / "oracle"))
    import oracle
    from egraph import catalog
    g, enc = ctx["graph"], ctx["enc"]
    sv, sc, ss = ctx["seed_host"]
    csr = g.csr()
    vl, _, _, _ = g.export()
    B = enc.n_incidents
    table = catalog.default().table
    reps, t_rules, t_graph = 0, 0.0, 0.0
    work = None
    t_start = time.perf_counter()
    while reps < 3 or time.perf_counter() - t_start < seconds:
        t0 = time.perf_counter()
        oracle.rules_eval(table, enc.flags, enc.vocab, enc.node, enc.err, enc.seg_off)
        t1 = time.perf_counter()
        _, _, work = oracle.frontier(csr["row_ptr"], csr["col"], csr["val"], vl, sv, sc, ss,
                                     ctx["src_host"], hops, ctx["inc_label"], k, threads)
        t_graph += time.perf_counter() - t1
        t_rules += t1 - t0
        reps += 1
    per_step = (t_rules + t_graph) / reps
    # the reference's own CPU path: the Python rules engine + ranker (restated in
    # oracle/rca_oracle.py, pinned to the reference goldens by tests/test_oracle_golden.py)
    import rca_oracle
    n_py = min(B, 200)
    t3 = time.perf_counter()
    for ev in ctx["evidence"][:n_py]:
        rca_oracle.rca("x", ev)
    t4 = time.perf_counter()
    # the dense C port, once (every V x B value per hop, > 99 % exact zeros)
    t5 = time.perf_counter()
    scores = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, B, hops, threads)
    reach = oracle.reach(csr["row_ptr"], csr["col"], ctx["src_host"], hops, threads)
    oracle.topk(scores, reach, vl, ctx["inc_label"], k)
    t6 = time.perf_counter()
    del scores, reach
    return {"value": B / per_step, "unit": "incidents/s", "cores": threads, "kind": "port",
            "sample": f"{reps} full steps of the same batch (B={B}: rules + {hops}-hop propagation "
                      f"+ reach + top-{k}), orc_rules_eval + orc_frontier (per column over the "
                      f"touched vertices, pruned last hop) with OpenMP {threads} threads; per step "
                      f"rules {t_rules / reps * 1e3:.2f} ms, graph {t_graph / reps * 1e3:.1f} ms, "
                      f"{work[0]} CSR entries read",
            "csr_entries_read_per_step": work[0],
            "python_rules_path": {"value": n_py / (t4 - t3), "unit": "incidents/s", "cores": 1,
                                  "sample": f"{n_py} incidents through oracle/rca_oracle.py "
                                            "(pure-Python restatement of RulesEngine + "
                                            "HypothesisRanker: the reference's CPU path; it "
                                            "has no graph stage to time without Neo4j)"},
            "dense_port": {"value": B / (t6 - t5), "unit": "incidents/s", "cores": threads,
                           "sample": "one step through orc_propagate + orc_reach + orc_topk "
                                     "(dense V x B sweep per hop; context only)"}}


def _lib_hash() -> str:
    from egraph import _lib
    return _lib.build_hash()


def _stamped(pmc: Path, d: dict):
    """(bytes, source note) of a counter summary if it was taken on the loaded libegraph.so
    (its `lib_hash` stamp, scripts/pmc_rdreq.py / pmc_traffic.py), else (None, why not): a
    figure from another build is never reported as this one's."""
    h = _lib_hash()
    if d.get("lib_hash") != h:
        return None, (f"{pmc.name} was taken on build {d.get('lib_hash')}, this run loads {h}: "
                      "no current counter pass, traffic not reported")
    return d.get("hbm_bytes_per_launch"), f"{pmc.name} (build {h})"


def _traffic(name: str):
    """HBM bytes per launch from a committed PMC summary (scripts/gpu_pmc.sh) of this build,
    else None; returns (bytes, note)."""
    pmc = REPO / "profiles" / f"pmc_{name}.json"
    if pmc.is_file():
        return _stamped(pmc, json.loads(pmc.read_text()))
    return None, f"no {pmc.name}"


# the table a frontier column tries first (egraph.graph.Frontier.FIRST_*)
FIRST_TABLE = ("narrow", "wide", "mid")


def frontier_layout_on() -> bool:
    """The snapshot lays the frontier's CSR out in locality order (csrc/layout.hip) unless
    $EGRAPH_FRONTIER_LAYOUT is "0"."""
    return not os.environ.get("EGRAPH_FRONTIER_LAYOUT", "1").startswith("0")


def _frontier_traffic(ctx, B: int):
    """Bytes past L2 per frontier launch (profiles/pmc_frontier_calibrated*.json, one per
    collected workload), when this run is a workload the counters were collected on (config,
    batch, batches per launch, layout) AND on this build (lib_hash); returns (bytes or None, note)."""
    M = ctx.get("merge", 1)
    note = "no counter pass of this workload in profiles/"
    for pmc in sorted((REPO / "profiles").glob("pmc_frontier_calibrated*.json")):
        d = json.loads(pmc.read_text())
        w = d.get("workload", {})
        if (w.get("config") == ctx.get("config") and w.get("batch") == B // M
                and w.get("batches_per_launch", 1) == M
                and w.get("distinct_batches", 1) == ctx.get("distinct_batches", 1)
                and w.get("layout", False) == frontier_layout_on()):
            v, note = _stamped(pmc, d)
            if v is not None:
                return v, note
    return None, note


def dense_roofline(ctx, hop_ms: float, B: int, V: int, nnz: int) -> dict:
    # SURVEY §8d compulsory bytes of one propagation hop: CSR (col + type) once, row_ptr,
    # scores read once and written once; gathers beyond the one compulsory read are not counted
    hop_bytes = nnz * 5 + (V + 1) * 4 + 2 * V * B * 4
    achieved = hop_bytes / (hop_ms * 1e-3) / 1e9
    traffic, src = _traffic("hop")
    return {"bound": "hbm", "kernel": f"hop_kernel<{ctx['plan'].tile_width // 4},false> "
                                      "(dense propagation hop + seed_add)",
            "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": src,
            "avg_launch_ms": hop_ms, "algorithmic_bytes_per_launch": hop_bytes}


def roofline_probe(ctx, hops: int, reps: int) -> float:
    """Mean duration (ms) of `reps` isolated egr_frontier_run launches of lane 0's batch, each
    alone on the GPU (synchronised before and after), bracketed by HIP events on its stream."""
    lane = ctx["lanes"][0]
    fr = lane["frontier"]
    ms = []
    torch.cuda.synchronize()
    for _ in range(max(reps, 1)):
        if "grouped" not in lane:
            fr.set_seeds(*lane["seeds"])
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        if "grouped" in lane:
            fr.run_grouped(*lane["grouped"], lane["sources"], hops, ctx["inc_label"],
                           order=lane["order"])
        else:
            fr.run(lane["sources"], hops, ctx["inc_label"])
        b.record()
        b.synchronize()
        ms.append(a.elapsed_time(b))
    return float(np.mean(ms))


def rules_probe(ctx, reps: int = 50) -> dict:
    """egr_rules_eval alone on the GPU: the bench batch's launch timed `reps` times with HIP
    events on its stream, one at a time (in the timed region it shares the CUs with the
    frontier launches of the other batches in flight)."""
    rules = ctx["rules"]
    st = torch.cuda.Stream()
    ms = []
    torch.cuda.synchronize()
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        rules.launch(st.cuda_stream)
        b.record(st)
        b.synchronize()
        ms.append(a.elapsed_time(b))
    rows = ctx["enc"].n_rows
    B = rules.B
    # algorithmic bytes: the rows once (20 B: flags, vocab, node, err), the segment offsets,
    # and the outputs (mask, n_hyp, 2 x S order bytes, 3 x S doubles per incident)
    S = 11
    nbytes = 20 * rows + 8 * (B + 1) + B * (5 + 2 * S + 24 * S)
    us = float(np.median(ms)) * 1e3
    return {"kernel": "rules_eval_kernel", "isolated_us_median": us,
            "isolated_us_min": float(np.min(ms)) * 1e3, "launches": reps,
            "incidents": B, "rows": rows, "algorithmic_bytes": nbytes,
            "achieved_GBps": nbytes / (us * 1e-6) / 1e9}


def frontier_roofline(ctx, run_ms: float, B: int, k: int, step_ms: float) -> tuple[dict, dict]:
    """Algorithmic bytes of one egr_frontier_run: every CSR entry a pull reads
    (col + val, 8 B), every entry an expansion reads (col, 4 B), a row_ptr pair per row walk
    (8 B), the seed entries (vertex + value, 8 B), the member pool written when there is one
    (vertex, score, depth: 9 B) and the top-k output (8 B per slot)."""
    work = ctx["frontier"].stats()
    n_seeds = work["seed_entries"]
    nbytes = (8 * work["pull_entries"] + 4 * work["expand_entries"] + 8 * work["rows"]
              + 8 * n_seeds + (9 * work["members"] if ctx["frontier"].pool_entries >= 0 else 0) + 8 * B * k)
    achieved = nbytes / (run_ms * 1e-3) / 1e9
    traffic, traffic_src = _frontier_traffic(ctx, B)
    return ({"bound": "hbm", "kernel": "frontier_lds_kernel + frontier_global_kernel "
                                       "(egr_frontier_run: reach + propagation + top-k)",
             "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": achieved / HBM_PEAK_GBS,
             # bytes fetched past L2 per launch from the committed counter passes at the bench
             # workload (C3, B = 1024): TCC_EA0_RDREQ x 128 B, the request size calibrated for
             # this kernel's 8-B gathers by scripts/calib_gather.hip, + the write requests.
             # Infinity-Cache hits count as fetched: an upper bound on HBM bytes.
             "traffic": traffic, "traffic_source": traffic_src,
             "traffic_note": "TCC_EA0_RDREQ x 128 B (calibrated: profiles/r02_calib_gather.txt) + "
                             "write requests, profiles/pmc_frontier_calibrated*.json; counts "
                             "Infinity-Cache hits (C3 CSR resident there): upper bound on HBM bytes",
             "avg_launch_ms": run_ms, "algorithmic_bytes_per_launch": nbytes,
             # the same bytes against the L2 roof: the C3 CSR (~5.5 MB) is re-read by every
             # column from L2 / the Infinity Cache, so neither bandwidth binds -- the kernel is
             # bound by dependent-load latency and issue (the stall counters in
             # profiles/r05_pmc_*.txt)
             "l2_roof": {"achieved": achieved, "peak": L2_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / L2_PEAK_GBS},
             # with batches in flight, launches overlap: per batch the GPU delivers nbytes
             # in one step's wall time
             "achieved_per_step": nbytes / (step_ms * 1e-3) / 1e9,
             "lanes": len(ctx["lanes"]), "batches_per_launch": ctx.get("merge", 1)}, work)


def time_dense(ctx, hops: int, steps: int, B: int, V: int, nnz: int, dev) -> dict:
    """A few dense-engine steps after the timed region, for comparison (not `value`)."""
    step(ctx, hops)
    torch.cuda.synchronize(dev)
    ev: list = []
    t0 = time.perf_counter()
    for _ in range(steps):
        step(ctx, hops, ev)
    torch.cuda.synchronize(dev)
    ms = (time.perf_counter() - t0) / steps * 1e3
    hop_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    return {"ms_per_step": ms, "incidents_per_sec": B / (ms * 1e-3), "steps": steps,
            "roofline": dense_roofline(ctx, hop_ms, B, V, nnz)}


class _TimedPlan:
    """Delegates to a Plan, recording HIP events around the non-seed propagation hops (`ev`)
    and, per partition (`part`: a list collecting this partition's (start, end) pairs), around
    every kernel of the partition's own compute (hops, reach hops, candidates, top-k)."""

    def __init__(self, plan, ev, part=None):
        self._p, self._ev, self._h, self._part = plan, ev, 0, part

    def __getattr__(self, name):
        return getattr(self._p, name)

    def _timed(self, fn, *a, tail: bool = False, what: str = ""):
        if self._part is None:
            return fn(*a)
        x, y = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        x.record()
        r = fn(*a)
        y.record()
        # which chain the call belongs to: the side stream's (reach), the main stream's
        # (propagation), or the tail after both joined (candidates, top-k)
        from egraph import shard
        side = shard._SIDE.get(torch.cuda.current_device())
        chain = "tail" if tail else ("side" if side is not None and torch.cuda.current_stream() == side
                                     else "main")
        self._part.append((x, y, chain, what or getattr(fn, "__name__", "?")))
        return r

    def hop(self):
        if self._ev is not None and self._h > 0:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            self._timed(self._p.hop)
            b.record()
            self._ev.append((a, b))
        else:
            self._timed(self._p.hop)
        self._h += 1

    def reach_hop(self):
        return self._timed(self._p.reach_hop)

    def candidates(self, *a):
        return self._timed(self._p.candidates, *a, tail=True)

    def topk(self, *a):
        return self._timed(self._p.topk, *a, tail=True)

    # the halo exchange's own device work (pack before, unpack after the transfer) runs on the
    # partition's GPU too: counted in its compute (the pack's host read of the peer sizes included)
    def pack_sparse(self, *a, **k):
        return self._timed(lambda: self._p.pack_sparse(*a, **k), what="pack_sparse")

    def unpack_sparse(self, *a, **k):
        return self._timed(lambda: self._p.unpack_sparse(*a, **k), what="unpack_sparse")

    def pack_sparse_cap(self, *a, **k):
        return self._timed(lambda: self._p.pack_sparse_cap(*a, **k), what="pack_sparse_cap")

    def unpack_sparse_cap(self, *a, **k):
        return self._timed(lambda: self._p.unpack_sparse_cap(*a, **k), what="unpack_sparse_cap")

    def pack_scores(self, *a):
        return self._timed(self._p.pack_scores, *a)

    def unpack_scores(self, *a):
        return self._timed(self._p.unpack_scores, *a)

    def pack_reach(self, *a):
        return self._timed(self._p.pack_reach, *a)

    def unpack_reach(self, *a):
        return self._timed(self._p.unpack_reach, *a)


def shard_setup(args, world: int, rank: int, dev: torch.device):
    from egraph import catalog, shard, synth
    from egraph.device import to_device
    from egraph.encode import encode_batch
    from egraph.graph import Snapshot
    from egraph.rca import RulesDeviceBatch
    t0 = time.time()
    B = args.batch
    cl = synth.build_cluster(synth.CONFIGS[args.config])
    cases = synth.make_incidents(cl, B, seed=1000)       # one global batch, same on every rank
    synth.add_incidents(cl, cases)
    g = synth.build_graph(cl)
    csr = g.csr()
    vl, _, _, _ = g.export()
    V = g.num_vertices
    evidence = [x.evidence for x in cases]
    sv, sc, ss = synth.seeds_for_batch(g, evidence)
    src = g.lookup([f"incident:{x.incident['id']}" for x in cases]).astype(np.uint32)
    P = world if world > 1 else max(args.partitions, 1)
    mine = [rank] if world > 1 else list(range(P))
    owner = shard.partition_vertices(csr["row_ptr"], vl, g.labels(), P)
    # rules: each rank evaluates its slice of the batch (incidents are independent)
    lo, hi = rank * B // world, (rank + 1) * B // world
    enc = encode_batch(evidence[lo:hi], catalog.default())
    runs, plans = [], []
    with torch.cuda.device(dev):
        rules = RulesDeviceBatch(enc, catalog.default(), dev)
        for r in mine:
            lg = shard.build_local(csr, vl, owner, r, P)
            snap = Snapshot.from_csr(lg.row_ptr, lg.col, lg.meta, lg.val, lg.vlabel, g.labels(), dev)
            lv, lc, ls = shard.local_seeds(lg, V, sv, sc, ss)
            plan = snap.plan(B, max_seeds=max(len(lv), 1), k=args.k)
            seeds = tuple(to_device(np.ascontiguousarray(a), dev) for a in (lv, lc, ls))
            sources = to_device(shard.local_sources(lg, V, src), dev)
            runs.append(shard.RankRun(lg, plan, dev))
            runs[-1].snap = snap
            plans.append((plan, seeds, sources))
        torch.cuda.synchronize(dev)
    comm = shard.TorchComm() if world > 1 else shard.LocalComm()
    log(f"[rank {rank}] built {args.config}: V={V} entries={len(csr['col'])} P={P} "
        f"owned={[r.lg.n_owned for r in runs]} halo={[len(r.lg.halo_rows) for r in runs]} "
        f"in {time.time() - t0:.1f}s")
    return dict(graph=g, csr=csr, vl=vl, runs=runs, plans=plans, comm=comm, rules=rules, P=P,
                inc_label=g.labels().index("Incident"), seed_host=(sv, sc, ss), src_host=src,
                enc_full=encode_batch(evidence, catalog.default()), evidence=evidence, V=V)


def shard_step(ctx, hops: int, k: int, ev=None, parts=None):
    from egraph import shard
    ctx["rules"].launch()
    for i, (run, (plan, seeds, sources)) in enumerate(zip(ctx["runs"], ctx["plans"])):
        plan.set_seeds(*seeds)
        plan.set_sources(sources)
        run.eng = _TimedPlan(plan, ev, parts[i] if parts is not None else None)
    if ctx.get("dense_halo") or ctx.get("host_counts"):
        return shard.run_partitioned(ctx["runs"], ctx["comm"], hops, ctx["inc_label"], k,
                                     sparse=not ctx.get("dense_halo", False),
                                     overlap=not ctx.get("no_overlap", False))

    def reset():                   # a pass that overflowed its slots re-runs (recalibrating)
        for run, (plan, seeds, sources) in zip(ctx["runs"], ctx["plans"]):
            plan.set_seeds(*seeds)
            plan.set_sources(sources)
    return shard.run_partitioned_retry(ctx["runs"], ctx["comm"], hops, ctx["inc_label"], k, reset,
                                       overlap=not ctx.get("no_overlap", False))


def shard_main(args, world: int, rank: int, dev: torch.device, dist) -> None:
    ctx = shard_setup(args, world, rank, dev)
    ctx["dense_halo"] = args.dense_halo
    ctx["host_counts"] = args.halo_host_counts
    ctx["no_overlap"] = args.no_overlap
    for _ in range(args.warmup):
        shard_step(ctx, args.hops, args.k)
    torch.cuda.synchronize(dev)
    events: list = []
    for r in ctx["runs"]:
        r.sent_bytes, r.exchanges, r.link_bytes = 0, 0, 0
    calls0 = ctx["comm"].calls
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        shard_step(ctx, args.hops, args.k, events)
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    coll_per_step = (ctx["comm"].calls - calls0) / max(args.steps, 1)
    if dist:
        elapsed = max_over_ranks(dist, elapsed, dev)
    # untimed: each partition's own compute (its kernels only, no exchange) per step, from HIP
    # events -- the per-GPU time of P GPUs running their partitions side by side
    # the timed steps' wire bytes (the untimed steps below exchange too)
    sent_t = max(r.sent_bytes for r in ctx["runs"])
    link_t = max(r.link_bytes for r in ctx["runs"])
    parts = [[] for _ in ctx["runs"]]
    for _ in range(3):
        shard_step(ctx, args.hops, args.k, None, parts)
    torch.cuda.synchronize(dev)
    part_ms = [sum(a.elapsed_time(b) for a, b, _, _ in q) / 3 for q in parts]
    # the critical path of a partition with the reach chain on its own stream: the longer of the
    # two chains, then the tail (what one GPU running the partition waits for, if the chains
    # overlap; the in-process ms_per_step with and without --no-overlap measures that they do)
    def chain_ms(q, c):
        return sum(a.elapsed_time(b) for a, b, t, _ in q if t == c) / 3
    crit_ms = [max(chain_ms(q, "main"), chain_ms(q, "side")) + chain_ms(q, "tail") for q in parts]
    # the slowest partition's calls by chain and kind (ms per step)
    slow = parts[int(np.argmax(crit_ms))]
    breakdown: dict = {}
    for a, b, t, w in slow:
        key = f"{t}:{w}"
        breakdown[key] = breakdown.get(key, 0.0) + a.elapsed_time(b) / 3
    B = args.batch
    ms = elapsed / args.steps * 1e3
    hop_ms = float(np.mean([a.elapsed_time(b) for a, b in events]))
    # the dense hop kernel of the largest local partition (SURVEY §8d bytes, local sizes)
    big = max(ctx["runs"], key=lambda r: len(r.lg.gid))
    Vl, nnzl = len(big.lg.gid), len(big.lg.col)
    hop_bytes = nnzl * 5 + (Vl + 1) * 4 + 2 * Vl * B * 4
    achieved = hop_bytes / (hop_ms * 1e-3) / 1e9
    nnz = len(ctx["csr"]["col"])
    halo = max(r.halo_bytes_per_hop for r in ctx["runs"])
    # collectives a GPU waits for on its critical path per step: with the reach chain on its own
    # stream, one chain's exchanges (hops - 1; the other chain's overlap them) + the all-gather;
    # serial, all of them.  (Steady state: one all-to-all per exchange; a calibrating or re-run
    # pass issues more, which coll_per_step -- the timed steps' own count -- would show.)
    overlap_on = not args.no_overlap
    coll_crit = (args.hops - 1 + 1) if overlap_on else coll_per_step
    per_hop = max(1, args.steps * max(args.hops - 1, 1))
    sent = sent_t / per_hop
    link = link_t / max(args.steps, 1)
    out = {
        "metric": METRIC, "value": B / (ms * 1e-3), "unit": "incidents/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "fp32", "data": "synthetic",
        "edges_per_sec": args.hops * nnz * B / (ms * 1e-3),
        "config": {
            "workload": f"{args.config}: {ctx['V']}-vertex graph edge-cut into {ctx['P']} "
                        f"partitions, {args.hops}-hop typed propagation + reach + top-{args.k}, "
                        f"one batch of {B} incidents per step (whole job)",
            "engine": "dense (partitioned)", "vertices": ctx["V"], "csr_entries": nnz,
            "partitions": ctx["P"], "incidents": B, "hops": args.hops, "k": args.k,
            "parallelism": f"edge-cut x{ctx['P']}" + (" (one process)" if world == 1 else ""),
            "local_vertices": [len(r.lg.gid) for r in ctx["runs"]],
            "owned_vertices": [int(r.lg.n_owned) for r in ctx["runs"]],
            "halo_over_owned": [round(len(r.lg.halo_rows) / max(r.lg.n_owned, 1), 3) for r in ctx["runs"]],
            "slowest_partition_breakdown_ms": {k: round(v, 4) for k, v in sorted(breakdown.items())},
            "halo_bytes_per_hop_max_rank": halo,
            "halo_exchange": "dense" if args.dense_halo else
                             "sparse, host-read peer counts" if args.halo_host_counts else
                             "sparse, fixed-capacity device slots (no host read per exchange)",
            "halo_slot_entries": None if args.dense_halo or args.halo_host_counts else
                                 {w: ctx["runs"][0].cap.get(w) for w in ("scores", "reach")},
            "halo_overflow_reruns": ctx["runs"][0].overflows,
            "halo_bytes_sent_per_hop_max_rank": sent,
            "halo_reduction_vs_dense": halo / sent if sent else None,
            "partition_compute_ms": part_ms,
            "link_bytes_per_step_max_rank": link,
            "reach_chain_overlap": overlap_on,
            "partition_critical_ms": crit_ms if overlap_on else part_ms,
            "collectives_per_step": coll_per_step,
            "collectives_on_critical_path": coll_crit,
            "collective_latency_us": RCCL_COLL_LATENCY_US,
            "collective_latency_note": "bench.RCCL_COLL_LATENCY_US: a stated charge per RCCL "
                                       "collective (not measured: RCCL refuses two ranks on one GPU)",
            "projected_ms_per_gpu": max(crit_ms if overlap_on else part_ms) + link / (XGMI_LINK_GBS * 1e6)
                                    + coll_crit * RCCL_COLL_LATENCY_US * 1e-3,
            "projected_ms_per_gpu_at_latency_us": {
                str(us): max(crit_ms if overlap_on else part_ms) + link / (XGMI_LINK_GBS * 1e6)
                         + coll_crit * us * 1e-3 for us in (0, 10, 30, 60)},
            "projected_serial_ms_per_gpu": max(part_ms) + link / (XGMI_LINK_GBS * 1e6)
                                           + coll_per_step * RCCL_COLL_LATENCY_US * 1e-3,
            "projected_note": "max over partitions of their own device work per step (hops, reach "
                              "hops, candidates, top-k and the halo pack / unpack kernels; HIP events, "
                              "untimed steps) -- with the reach chain on its own stream, the longer "
                              "chain plus the top-k tail (partition_critical_ms; the serial sum is "
                              "projected_serial_ms_per_gpu) -- + per exchange the largest transfer "
                              "from one rank to ONE peer over its xGMI link (point to point: the "
                              "peers' transfers run on separate links at once); what P GPUs running "
                              "one partition each would take per step (the in-process ms_per_step "
                              "runs them one after another on one GPU) + the collectives on the "
                              "critical path x collective_latency_us",
        },
        "roofline": {"bound": "hbm", "kernel": "hop_kernel (dense propagation hop, local partition)",
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None, "avg_launch_ms": hop_ms,
                     "algorithmic_bytes_per_launch": hop_bytes},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, str(REPO / "oracle"))
        import oracle
        from egraph import catalog
        threads = args.cpu_threads or min(16, len(os.sched_getaffinity(0)))
        csr, enc = ctx["csr"], ctx["enc_full"]
        sv, sc, ss = ctx["seed_host"]
        t0 = time.perf_counter()
        oracle.rules_eval(catalog.default().table, enc.flags, enc.vocab, enc.node, enc.err, enc.seg_off)
        scores = oracle.propagate(csr["row_ptr"], csr["col"], csr["val"], sv, sc, ss, B, args.hops, threads)
        reach = oracle.reach(csr["row_ptr"], csr["col"], ctx["src_host"], args.hops, threads)
        oracle.topk(scores, reach, ctx["vl"], ctx["inc_label"], args.k)
        t1 = time.perf_counter()
        out["cpu_baseline"] = {"value": B / (t1 - t0), "unit": "incidents/s", "cores": threads,
                               "kind": "port", "sample": f"one full step of the same batch (B={B}) "
                               f"on the unpartitioned graph by oracle/egraph_oracle.c, OpenMP "
                               f"{threads} threads"}
    if rank == 0:
        print(json.dumps(out), flush=True)


def storm_main(args, world: int, rank: int, dev: torch.device) -> None:
    """BASELINE configs[4] (C5): the alert storm on the C3 graph -- 100k alerts/min, Zipf(1.1)
    over 10k (alertname, namespace, service) keys; one step = one tick = one second of the
    stream: fingerprints + TTL dedup, MERGE of the new incidents and topology delta, incremental
    CSR update, affected-incident BFS and re-rank (egraph/storm.py)."""
    from egraph import synth
    from egraph.storm import StormEngine
    t0 = time.time()
    cl = synth.build_cluster(synth.CONFIGS[args.config])
    g = synth.build_graph(cl)
    # every rank replays the same global stream (same seed): the alerts of a tick arrive spread
    # over the ranks (alert i at rank i % world) and each rank's webhook share stays at
    # storm_rate / 60 per tick (weak scaling); the table is fingerprint-sharded, the graph
    # replicated, incident h ranked on rank h % world (egraph/storm.py)
    wl = synth.StormWorkload(cl, n_keys=args.storm_keys, seed=20260826)
    comm = None
    if world > 1:
        from egraph.shard import TorchComm
        comm = TorchComm()
    eng = StormEngine(g, device=dev, hops=args.hops, k=args.k, dedup_capacity=1 << 17,
                      comm=comm, rank=rank, keep_evidence=args.storm_keep_evidence)
    per_tick = args.storm_rate // 60
    n_tick = per_tick * world
    log(f"[rank {rank}] built {args.config} + storm: V={g.num_vertices} keys={args.storm_keys} "
        f"alerts/tick={n_tick} ({per_tick} per rank) in {time.time() - t0:.1f}s")
    now = 1_790_000_000_000
    stats = []
    mine = np.arange(rank, n_tick, world, dtype=np.int64)
    # cyclic-GC time inside the timed part of a tick (not while the collector stand-in runs)
    gc_t = [0.0, 0.0, False]

    def _gc_cb(phase, info):
        if phase == "start":
            gc_t[0] = time.perf_counter()
        elif not gc_t[2]:
            gc_t[1] += time.perf_counter() - gc_t[0]
    gc.callbacks.append(_gc_cb)

    def make_case(h, i):
        gc_t[2] = True
        try:
            return wl.make_case(h, i)
        finally:
            gc_t[2] = False
    for i in range(args.warmup + args.steps):
        now += 1000
        keys = wl.alerts(n_tick)
        topo = wl.topology(args.storm_events)
        local = [keys[j] for j in mine]
        torch.cuda.synchronize(dev)
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
        import resource
        f0 = resource.getrusage(resource.RUSAGE_SELF)
        a = time.perf_counter()
        gc_t[1] = 0.0
        st = eng.tick(local, now, make_case, topology=topo, seq=mine if world > 1 else None)
        torch.cuda.synchronize(dev)
        st["wall_ms"] = (time.perf_counter() - a) * 1e3 - st["collect_ms"]
        st["gc_ms"] = gc_t[1] * 1e3
        f1 = resource.getrusage(resource.RUSAGE_SELF)
        st["minflt"] = f1.ru_minflt - f0.ru_minflt          # (collector stand-in included)
        st["invol_cs"] = f1.ru_nivcsw - f0.ru_nivcsw
        if world > 1:
            import torch.distributed as dist
            st["wall_ms"] = max_over_ranks(dist, st["wall_ms"], dev)
        if i >= args.warmup:
            stats.append(st)
        if rank == 0:
            log(f"tick {i}: {st['new_incidents']} new, {st['affected']} affected (rank 0) / "
                f"{st['open_incidents']} open, {st['new_edges']} edges, {st['wall_ms']:.2f} ms")
    wall = np.array([s_["wall_ms"] for s_ in stats])
    total_alerts = sum(s_["alerts"] for s_ in stats)
    stage = {k_: float(np.mean([s_["ms"][k_] for s_ in stats])) for k_ in stats[0]["ms"]}
    out = {
        "metric": "alerts/sec through dedup + incremental CSR update + re-ranking (alert storm)",
        "value": total_alerts / (wall.sum() * 1e-3), "unit": "alerts/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": float(wall.mean()),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8/u32/fp32",
        "data": "synthetic",
        "config": {"workload": f"C5: {args.storm_rate} alerts/min per GPU (one tick = 1 s of stream = "
                               f"{n_tick} alerts over {world} GPU(s)), Zipf(1.1) over {args.storm_keys} keys, "
                               f"{args.config} graph, {args.storm_events} topology events/tick, "
                               f"{args.hops}-hop re-rank top-{args.k}",
                   "tick_ms_p50": float(np.percentile(wall, 50)),
                   "tick_ms_p99": float(np.percentile(wall, 99)),
                   "stage_ms_mean": stage,
                   "gc_ms_per_tick": float(np.mean([s_["gc_ms"] for s_ in stats])),
                   "minor_faults_per_tick": float(np.mean([s_["minflt"] for s_ in stats])),
                   "involuntary_switches_per_tick": float(np.mean([s_["invol_cs"] for s_ in stats])),
                   "new_incidents_per_tick": float(np.mean([s_["new_incidents"] for s_ in stats])),
                   "affected_per_tick": float(np.mean([s_["affected"] for s_ in stats])),
                   "reseed_per_tick": {k_: float(np.mean([s_["reseed"].get(k_, 0) for s_ in stats]))
                                       for k_ in ("incidents", "new", "candidates_ms", "attach_ms",
                                                  "pending_ms")},
                   "open_incidents_end": stats[-1]["open_incidents"],
                   "parallelism": (f"fingerprint-sharded dedup x{world}, replicated graph, "
                                   f"incidents re-ranked by owner rank") if world > 1 else "one GPU",
                   "realtime_headroom": 1000.0 / float(wall.mean())},
        "note": "value = alerts of the timed ticks / pipeline time (collector-side evidence "
                "generation excluded); a tick covers 1 s of stream, so realtime_headroom = "
                "1000 ms / mean tick time",
    }
    if rank == 0:
        print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default: 400 for the incident-sharded rank workload, whose "
                         "step is ~0.07 ms; 20 for the storm and the edge-cut graph)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 10 / 3)")
    ap.add_argument("--config", default="C3", choices=["C2", "C3", "C4"])
    ap.add_argument("--batch", type=int, default=1024, help="incidents per GPU per step")
    ap.add_argument("--hops", type=int, default=3)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="frontier lanes in flight (independent states on their own streams)")
    ap.add_argument("--merge", type=int, default=0,
                    help="frontier batches per launch: each lane's launch carries this many "
                         "consecutive batches (one costliest-first column order across them); "
                         f"0 = the largest divisor of --steps up to {MERGE_MAX}")
    ap.add_argument("--replicate-batches", action="store_true",
                    help="A/B only: a launch's M batches are M copies of one incident set (round "
                         "3's launch) instead of M different incident sets")
    ap.add_argument("--no-dropin", action="store_true",
                    help="skip the end-to-end drop-in RulesEngine measurement")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--engine", default="frontier", choices=["frontier", "dense"])
    ap.add_argument("--pool", action="store_true",
                    help="frontier keeps every member's score (inspection mode: no last-pull pruning)")
    ap.add_argument("--dense-steps", type=int, default=5,
                    help="dense-engine steps timed after the main run for comparison (0: skip)")
    ap.add_argument("--shard", default="incidents", choices=["incidents", "graph"],
                    help="incidents: replicated snapshot, incident-sharded (default); graph: "
                         "edge-cut partitioned graph with halo exchange (C4)")
    ap.add_argument("--dense-halo", action="store_true",
                    help="--shard graph: exchange whole boundary rows instead of their non-zero entries")
    ap.add_argument("--halo-host-counts", action="store_true",
                    help="--shard graph: sparse exchange with a host read of the peer counts per "
                         "exchange (the round-3 path) instead of fixed-capacity device slots")
    ap.add_argument("--no-overlap", action="store_true",
                    help="--shard graph: run the reach chain on the main stream too (A/B)")
    ap.add_argument("--partitions", type=int, default=1,
                    help="--shard graph on one process: partitions run on this GPU")
    ap.add_argument("--workload", default="rank", choices=["rank", "storm"],
                    help="rank: the headline incident-ranking step; storm: BASELINE C5 alert storm")
    ap.add_argument("--storm-rate", type=int, default=100_000, help="alerts per minute")
    ap.add_argument("--storm-keys", type=int, default=10_000)
    ap.add_argument("--storm-events", type=int, default=100, help="topology events per tick")
    ap.add_argument("--storm-keep-evidence", action="store_true",
                    help="A/B: the engine keeps every incident's evidence rows (no release)")
    ap.add_argument("--no-graph", action="store_true",
                    help="frontier: enqueue each launch eagerly instead of replaying the lane's "
                         "captured HIP graph (the default from --merge 8 up: five kernel launches "
                         "per M batches cost less than a graph launch, -1.5 %% per step at M=20, "
                         "profiles/r05_ab_graph_eager.txt)")
    ap.add_argument("--graph", action="store_true",
                    help="frontier: replay captured HIP graphs at any --merge (A/B)")
    ap.add_argument("--seed-input", default="grouped", choices=["grouped", "grouped-host-order", "sort"],
                    help="grouped: seeds grouped by incident as resident input, launch order on "
                         "the device per step (egr_frontier_run_grouped); grouped-host-order: the "
                         "order computed once on the host (A/B); sort: device counting sort per step")
    ap.add_argument("--roofline-reps", type=int, default=20,
                    help="isolated frontier launches timed after the run for the roofline")
    args = ap.parse_args()
    short = args.workload == "rank" and args.shard == "incidents"
    if args.steps is None:
        args.steps = 400 if short else 20
    if args.warmup is None:
        args.warmup = 10 if short else 3
    if args.merge <= 0:
        args.merge = max(m for m in range(1, MERGE_MAX + 1) if args.steps % m == 0)

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # `bench.py --gpus N` outside a launcher: start the N ranks ourselves (one per GPU,
        # torch.distributed.run over 127.0.0.1) before anything here touches the GPU, as a child
        # process, and exit with its status
        raise SystemExit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank "
                         f"per GPU (torch.distributed.run --nproc-per-node {args.gpus}) or pass "
                         f"--gpus {world}")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    global GROUPED
    GROUPED = {"grouped": "device", "grouped-host-order": "order"}.get(args.seed_input)
    if not torch.cuda.is_available():
        raise SystemExit("bench.py needs a ROCm GPU")
    # EGRAPH_BENCH_BACKEND=gloo rehearses N ranks on fewer GPUs (ranks share a device); the
    # driver's runs use RCCL ("nccl"), one rank per GPU
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count()))
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if BACKEND == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(BACKEND)

    if args.workload == "storm":
        storm_main(args, world, rank, dev)
        if dist:
            dist.destroy_process_group()
        return
    if args.shard == "graph":
        shard_main(args, world, rank, dev, dist)
        if dist:
            dist.destroy_process_group()
        return
    ctx = setup(args.config, args.batch, args.k, rank, dev,
                args.pipeline if args.engine == "frontier" else 1,
                pool_entries=0 if args.pool else -1,
                merge=max(1, args.merge) if args.engine == "frontier" else 1,
                replicate=args.replicate_batches)
    M = ctx["merge"]
    # captured graphs pay off while a launch carries few batches; at M >= 8 the eager launch's
    # five kernel launches are cheaper than hipGraphLaunch (profiles/r05_ab_graph_eager.txt)
    graphs = args.engine == "frontier" and not args.no_graph and (args.graph or M < GRAPH_MERGE_MAX)
    run_step = warm_up(ctx, args.hops, args.warmup, dev, rank,
                       engine=args.engine, graphs=graphs)

    events: list = EventPool(args.steps) if args.engine == "frontier" else []
    ctx["sub"] = 0                  # the timed region starts a group of M batches
    if args.steps % M:
        log(f"[rank {rank}] --steps {args.steps} is not a multiple of --merge {M}: the last "
            f"launch computes {M - args.steps % M} batches more than the region counts")
    elapsed = timed_steps(lambda: run_step(ctx, args.hops, events), args.steps, dist, rank,
                          lambda: torch.cuda.synchronize(dev), dev)

    B, V = args.batch, ctx["snap"].n_vertices
    nnz = ctx["snap"].n_entries
    ms = elapsed / args.steps * 1e3
    timed = events.done if isinstance(events, EventPool) else events
    if args.engine == "frontier":
        # the dominant kernel's duration: isolated launches (one at a time, HIP events on the
        # launching stream) after the timed region -- in the timed region launches overlap
        # across the lanes, so an event pair there also times the wait for CUs held by the
        # other batches (reported as avg_launch_ms_in_flight when the run was eager)
        launch_ms = roofline_probe(ctx, args.hops, args.roofline_reps)
        roof, work = frontier_roofline(ctx, launch_ms, B * M, args.k, ms * M)
        roof["isolated_launches"] = args.roofline_reps
        rules_iso = rules_probe(ctx)
        if timed:
            spans = np.array([a.elapsed_time(b) for a, b in timed])
            # in the timed region: each batch's span on its lane's stream (graph replay: the
            # whole captured batch; eager: the frontier run), their sum per step, and the mean
            # number of batches in flight (sum of spans / wall time) -- so the isolated launch
            # time, the overlap and ms_per_step can be reconciled from this line alone
            roof["in_region"] = {
                "what": "graph replay span (rules + frontier + fallback)" if graphs
                        else "egr_frontier_run span",
                "span_ms_mean": float(spans.mean()), "span_ms_p50": float(np.median(spans)),
                "span_ms_sum_per_step": float(spans.sum() / args.steps),
                "launches_in_flight_mean": float(spans.sum() / (elapsed * 1e3)),
                "batches_per_launch": M,
                "isolated_launch_ms_over_launch_group_ms": launch_ms / (ms * M)}
        out_graph = graphs
    else:
        launch_ms = float(np.mean([a.elapsed_time(b) for a, b in timed]))
        roof, work = dense_roofline(ctx, launch_ms, B, V, nnz), None
        out_graph = False
    out = {
        "metric": METRIC,
        "value": world * B / (ms * 1e-3),
        "unit": "incidents/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp32",
        "data": "synthetic",
        # edge = one directed CSR entry processed in one hop for one column.
        # edges_per_sec counts the entries the engine actually read (pulls + expansions, from
        # the kernel's own counters); the dense-equivalent 3*nnz*B figure -- work a dense sweep
        # would do, most of it on exact zeros, which this engine skips -- is kept apart
        "edges_per_sec": None,
        "edges_per_sec_dense_equivalent": world * args.hops * nnz * B / (ms * 1e-3),
        "config": {
            "workload": f"{args.config}: {_GRAPH_NAME.get(args.config, args.config)} multi-namespace graph, full rule set + "
                        f"{args.hops}-hop typed propagation + reach + top-{args.k}, "
                        f"{B} incidents per GPU per step",
            "engine": args.engine,
            "vertices": V, "csr_entries": nnz, "incidents_per_gpu": B,
            "evidence_rows_per_gpu": ctx["enc"].n_rows, "seeds_per_gpu": int(len(ctx["seed_host"][0])),
            "hops": args.hops, "k": args.k, "parallelism": f"incident-sharded x{world}",
            "lanes": args.pipeline if args.engine == "frontier" else 1,
            "batches_per_launch": M,
            "distinct_batches_per_launch": ctx["distinct_batches"],
            "distinct_incident_sets": ctx["distinct_sets"],
            "frontier_layout": "locality order (csrc/layout.hip)" if frontier_layout_on() else "canonical",
            "first_table": (FIRST_TABLE[ctx["lanes"][0]["frontier"].wide_first]
                            if args.engine == "frontier" else None),
            "incidents_in_graph": ctx["incidents_in_graph"],
            "hip_graph_replay": out_graph,
            "seed_input": ("grouped by incident + column offsets, resident; costliest-first launch "
                           "order computed on the device in every step (egr_frontier_run_grouped)"
                           if GROUPED == "device" and args.engine == "frontier" else
                           "grouped by incident + column offsets + a launch order computed once on "
                           "the host (A/B)" if GROUPED == "order" and args.engine == "frontier"
                           else "unordered triples, device counting sort per step"),
        },
        "roofline": roof,
    }
    if args.engine == "frontier":
        out["rules_kernel"] = rules_iso
    if work is not None:
        out["edges_per_sec"] = world * (work["pull_entries"] + work["expand_entries"]) / (ms * 1e-3)
        out["frontier_work"] = work
    else:
        out["edges_per_sec"] = out["edges_per_sec_dense_equivalent"]   # the dense engine reads them all
    if args.engine == "frontier" and args.dense_steps > 0:
        out["dense_engine"] = time_dense(ctx, args.hops, args.dense_steps, B, V, nnz, dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = args.cpu_threads or min(16, len(os.sched_getaffinity(0)))
        out["cpu_baseline"] = cpu_baseline(ctx, args.hops, args.k, threads)
    if rank == 0 and args.engine == "frontier" and not args.no_dropin:
        out["dropin_rules"] = dropin_rules(ctx, dev)
        out["dropin_graph"] = dropin_graph(ctx, dev, args.hops, args.k)
    if "cpu_baseline" in out:
        reference_speedups(out)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


CALIBRATION = REPO / "profiles" / "r06_standin_calibration.json"


def reference_speedups(out: dict) -> None:
    """cpu_baseline.speedup_vs_reference and .end_to_end_speedup: the GPU figures over the
    reference's own Python rules path on this host's cores.  That path cannot run here (the
    reference does not travel to the GPU box); its pinned restatement oracle/rca_oracle.py is
    timed instead (python_rules_path), and oracle/calibrate_standin.py measured, in the build
    container, how much longer the real reference takes on the same C3-shaped incidents: the
    median over interleaved pairs of rounds with a distribution-free 95 % interval
    (profiles/r06_standin_calibration.json).  reference rate = stand-in rate / that ratio; the
    interval of each speed-up is the ratio's interval carried through."""
    cb = out["cpu_baseline"]
    try:
        cal = json.loads(CALIBRATION.read_text())
        r = float(cal["bench_workload_ratio"])
        lo, hi = (float(x) for x in cal["bench_workload_ratio_ci95"])
    except (OSError, KeyError, ValueError) as e:
        cb["speedup_vs_reference"] = {"value": None, "note": f"no calibration: {e}"}
        return
    py = cb["python_rules_path"]["value"]
    ref, ref_lo, ref_hi = py / r, py / hi, py / lo       # the reference's incidents/s, interval
    cb["reference_rules_path"] = {
        "value": ref, "ci95": [ref_lo, ref_hi], "unit": "incidents/s", "cores": 1,
        "derivation": f"python_rules_path {py:.0f}/s / calibration ratio {r:.4f} "
                      f"(95 % CI {lo:.4f} .. {hi:.4f}, {CALIBRATION.name})"}

    def ratio(x: float) -> dict:
        return {"value": x / ref, "ci95": [x / ref_hi, x / ref_lo]}
    cb["speedup_vs_reference"] = {
        **ratio(out["value"]),
        "what": "the headline (GPU stage on resident, pre-encoded columns: rules + 3-hop "
                "propagation + reach + top-k per incident) over the reference's Python rules path "
                "(dicts in, dicts out; it has no graph stage without Neo4j)"}
    e2e: dict = {"what": "the drop-in's Python API end to end (evidence dicts in, hypothesis "
                         "dicts out) against the reference's rules path, same host"}
    dr = out.get("dropin_rules")
    if dr:
        e2e["rules_batch"] = {**ratio(dr["value"]), "what": "RulesEngine.rank_incidents_batch, 1024 "
                                                           "incidents per call"}
        conc = dr.get("concurrent", {}).get("value")
        if conc:
            e2e["concurrent_single_calls"] = {**ratio(conc), "what": "1024 concurrent "
                                              "generate_hypotheses + rank calls"}
        one, ref_one = dr.get("single_call_us", {}).get("p50"), dr.get("reference_single_call_us", {}).get("p50")
        if one and ref_one:
            # the reference's per-call time = the stand-in's measured p50 x the ratio
            e2e["single_call_p50"] = {"value": ref_one * r / one, "ci95": [ref_one * lo / one, ref_one * hi / one],
                                      "what": "one incident per call, idle engine (the activity's "
                                              "pattern, activities.py:124-170): reference p50 / drop-in p50"}
    cb["end_to_end_speedup"] = e2e


if __name__ == "__main__":
    main()
