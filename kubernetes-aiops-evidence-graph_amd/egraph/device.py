"""Device selection for the egraph ops: the GPU path or a loud failure, never a CPU fallback."""
from __future__ import annotations

import os

import numpy as np
import torch


def require_device(device: int | str | torch.device | None = None) -> torch.device:
    """The HIP device the ops run on (default: torch's current device, or $EGRAPH_DEVICE)."""
    if not torch.cuda.is_available():
        raise RuntimeError(
            "egraph needs a ROCm GPU (MI355X / gfx950): torch.cuda.is_available() is False. "
            "There is no CPU fallback; the CPU restatement under oracle/ is test infrastructure.")
    if device is None:
        env = os.environ.get("EGRAPH_DEVICE")
        device = int(env) if env is not None else torch.cuda.current_device()
    dev = torch.device("cuda", device) if isinstance(device, int) else torch.device(device)
    if dev.type != "cuda":
        raise ValueError(f"egraph ops run on a cuda (HIP) device, got {dev}")
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    return dev


def to_device(a, dev: torch.device) -> torch.Tensor:
    """numpy array -> device tensor through pinned memory (asynchronous on the current stream)."""
    if a.dtype == np.uint32:      # torch's unsigned types are storage-only: move the bits
        a = a.view(np.int32)
    elif a.dtype == np.uint64:
        a = a.view(np.int64)
    a = np.ascontiguousarray(a)
    if not a.flags.writeable:     # e.g. np.frombuffer over bytes
        a = a.copy()
    t = torch.from_numpy(a)
    if t.numel() == 0:
        return torch.empty(t.shape, dtype=t.dtype, device=dev)
    return t.pin_memory().to(dev, non_blocking=True)


class MappedBuffer:
    """Pinned host memory mapped into the GPU address space (egr_host_alloc): `np` is the host
    view, `dev` the address kernels read and write.  The drop-in's small launches use it so
    that a call is one kernel launch with no DMA copies (egraph/batcher.py, egraph/ranker.py)."""

    def __init__(self, nbytes: int):
        import ctypes as C

        from . import _lib as L
        h, d = C.c_void_p(), C.c_void_p()
        L.check(L.lib.egr_host_alloc(int(nbytes), C.byref(h), C.byref(d)), "egr_host_alloc")
        self._free = L.lib.egr_host_free
        self.host, self.dev, self.nbytes = h.value, d.value, int(nbytes)
        self.np = np.ctypeslib.as_array((C.c_uint8 * self.nbytes).from_address(self.host))

    def __del__(self):
        h, self.host = getattr(self, "host", None), None
        if h:
            self.np = None
            self._free(h)
