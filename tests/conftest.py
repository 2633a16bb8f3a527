"""Shared test setup: import paths, the `gpu` marker, native libraries built on demand."""
from __future__ import annotations

import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
PKG = REPO / "kubernetes-aiops-evidence-graph_amd"
for p in (REPO, PKG, REPO / "oracle", REPO / "tests"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

if not (PKG / "lib" / "libegraph.so").is_file():
    subprocess.run(["make", "-C", str(PKG), "-j4"], check=True)
if not (REPO / "oracle" / "liboracle.so").is_file():
    subprocess.run(["make", "-C", str(REPO / "oracle")], check=True)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")


def gpu_available() -> bool:
    import torch
    return torch.cuda.is_available()


@pytest.fixture(scope="session")
def golden():
    import json
    g = REPO / "tests" / "golden"
    return {
        "rules": json.loads((g / "rules_cases.json").read_text()),
        "errors": json.loads((g / "rules_errors.json").read_text()),
        "lut": json.loads((g / "mask_lut.json").read_text()),
        "ranker": json.loads((g / "ranker_cases.json").read_text()),
        "fingerprints": json.loads((g / "fingerprints.json").read_text()),
        "normalizer": json.loads((g / "normalizer_cases.json").read_text()),
        "storm": json.loads((g / "storm_cases.json").read_text()),
    }
