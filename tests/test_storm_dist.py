"""The fingerprint-sharded dedup protocol (egraph.alerts.ShardedDedup, BASELINE C5 across GPUs)
on CPU: world-size 2 and 3 gloo process groups replay the reference's 60-tick webhook storm
(tests/golden/storm_cases.json, recorded from the reference with TTL expiry, DEL and EXPIRE).
The alerts of each tick arrive spread over the ranks (alert i at rank i % world); every rank
must end with the reference's decision and incident for every alert, and EXPIRE's result.
The owners' tables are the oracle's TTL store here (tests/storm_cpu_table.py); the GPU runs
the same protocol over DedupTable (tests/test_storm_gpu.py)."""
from __future__ import annotations

import os
import socket

import pytest


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, q):
    import json

    import torch
    import torch.distributed as dist

    from conftest import REPO
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from egraph.alerts import ShardedDedup
        from egraph.shard import TorchComm
        from storm_cpu_table import CpuTable
        storm = json.loads((REPO / "tests" / "golden" / "storm_cases.json").read_text())
        sd = ShardedDedup(CpuTable(), TorchComm(), rank)
        ttl_ms = storm["ttl_s"] * 1000
        owned_keys = 0

        def fps(hexes):
            import numpy as np
            raw = b"".join(bytes.fromhex(h) for h in hexes)
            a = np.frombuffer(raw, np.uint8).reshape(len(hexes), 16) if hexes else np.zeros((0, 16), np.uint8)
            return torch.from_numpy(a.copy())

        for tick in storm["ticks"]:
            now = tick["now_ms"]
            for op in tick["ops"]:
                k = fps([op["fingerprint"]])
                if op["op"] == "remove":
                    sd.remove(k)
                else:
                    assert bool(sd.extend(k, now, op["ttl_s"] * 1000)[0]) == op["ok"]
            firing = [e for e in tick["expected"] if e is not None]
            mine = list(range(rank, len(firing), world))
            f = fps([firing[i]["fingerprint"] for i in mine])
            owned_keys += int(sd.owns(f).sum())
            dup, inc, n_new = sd.ingest(f, torch.tensor(mine, dtype=torch.int64), now, ttl_ms)
            assert len(dup) == len(firing)
            for e, d, i in zip(firing, dup.tolist(), inc.tolist()):
                assert d == e["dup"] and f"inc-{i}" == e["incident"]
        q.put((rank, sd.next_id, sd.table.next_id, owned_keys))
    except BaseException as e:                      # noqa: BLE001 (reported to the parent)
        q.put((rank, repr(e), None, None))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_dedup_replays_reference_storm(world):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0, res
    assert all(r[1] == 225 for r in res), res               # global incidents, every rank
    assert sum(r[2] for r in res) == 225                     # each opened on exactly one owner
    assert all(r[2] > 0 for r in res)                        # every shard holds keys
