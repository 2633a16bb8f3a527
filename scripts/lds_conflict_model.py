"""Bank conflicts that uniformly random LDS addresses cost, against the narrow frontier kernel's
measured ones (profiles/r06_pmc_final_s20.txt, the `lanes` pass of scripts/gpu_pmc.sh).

A ds_read_b32 / ds_write_b32 of a wave64 is serviced in two 32-lane groups; its bank is
(address / 4) mod 32 (MI355X_MICROARCH.md, LDS).  A group of m active lanes with distinct random
addresses takes max-load cycles, so it adds E[max load] - 1 conflict cycles; lanes with the same
address broadcast.  The frontier's hash-table probes (keys[slot], s[slot], the filter words)
are such addresses: the slot is a hash of a vertex id.  A per-lane XOR swizzle of the slot
(the round-4 ask) maps a uniformly random bank to another uniformly random bank -- the
distribution of the max load, and so the conflicts, do not change; only fewer distinct
addresses per instruction (fewer active lanes, or several keys per wider access) would.

Usage: python scripts/lds_conflict_model.py [active_lane_fraction]"""
from __future__ import annotations

import sys

import numpy as np


def extra_cycles(m: int, banks: int = 32, trials: int = 20000, seed: int = 1) -> float:
    """E[max bank load] - 1 for m random addresses over `banks` banks (m >= 1)."""
    if m <= 1:
        return 0.0
    rng = np.random.default_rng(seed)
    b = rng.integers(0, banks, size=(trials, m))
    loads = np.zeros((trials, banks), np.int32)
    np.add.at(loads, (np.repeat(np.arange(trials), m), b.ravel()), 1)
    return float(loads.max(axis=1).mean() - 1.0)


def main() -> None:
    frac = float(sys.argv[1]) if len(sys.argv) > 1 else None
    print("active lanes per 32-lane group -> conflict cycles per group / per wave-instruction "
          "(two groups), uniformly random addresses")
    for m in (1, 2, 4, 8, 12, 16, 24, 32):
        e = extra_cycles(m)
        print(f"  {m:2d} lanes: {e:5.2f} / {2 * e:5.2f}")
    if frac is not None:
        m = max(1, round(32 * frac))
        print(f"at the measured active-lane fraction {frac:.3f} (~{m} lanes per group): "
              f"{2 * extra_cycles(m):.2f} conflict cycles per random-address wave-instruction")


if __name__ == "__main__":
    main()
