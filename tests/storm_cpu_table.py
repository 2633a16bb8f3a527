"""TEST INFRASTRUCTURE: a CPU stand-in for egraph.alerts.DedupTable (ingest / remove / extend
with the same tensor shapes and handle numbering) over the oracle's TTL store
(oracle/alerts_oracle.py).  It lets the fingerprint-sharded dedup protocol
(egraph.alerts.ShardedDedup) run under gloo on CPU; the HIP table runs the same protocol on
the GPU (tests/test_storm_gpu.py).  Never imported by the package."""
from __future__ import annotations

import numpy as np
import torch

import alerts_oracle as AO


class CpuTable:
    def __init__(self):
        self.dev = torch.device("cpu")
        self.store = AO.TTLStore()
        self.next_id = 0

    @staticmethod
    def _hex(fp: torch.Tensor) -> list[str]:
        return [bytes(r).hex() for r in fp.numpy()]

    def ingest(self, fp, now_ms, ttl_ms):
        dup, inc, n = AO.webhook_loop(self.store, self._hex(fp), now_ms, ttl_ms // 1000, self.next_id)
        self.next_id += n
        return (torch.tensor(dup, dtype=torch.bool), torch.tensor(inc, dtype=torch.int64), n)

    def remove(self, fp):
        for k in self._hex(fp):
            self.store.delete(k)

    def extend(self, fp, now_ms, ttl_ms):
        return torch.tensor([self.store.expire(k, now_ms, ttl_ms // 1000) for k in self._hex(fp)],
                            dtype=torch.bool)
