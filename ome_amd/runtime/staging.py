"""Pinned host staging for the per-step host->device metadata copies.

Every eager step ships its packed metadata (token ids, positions, KV slots, attention plan,
sampling parameters) and the request page-table updates to the GPU.  ``Tensor.pin_memory()``
per step goes through the caching host allocator, whose misses pin fresh pages (a blocking
runtime call that can serialise with the device); a small ring of persistent pinned buffers
avoids that entirely.  A buffer is rewritten only after the copy that last read it has executed
(its event), which in steady state has long happened: the ring is several steps deep.

The copy itself is a kernel reading the mapped pinned pages (:func:`copy_h2d`), not
``hipMemcpyAsync``: every per-step transfer stays a plain dispatch on the compute stream.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

_TORCH = {np.dtype(np.int32): torch.int32, np.dtype(np.int64): torch.int64, np.dtype(np.float32): torch.float32,
          np.dtype(np.uint8): torch.uint8}


_DEV_PTR: dict[int, int] = {}


def mapped_ptr(host: torch.Tensor) -> int:
    """Device address of a pinned host tensor's storage (cached per allocation)."""
    from ome_amd.ops._native import call

    base = host.untyped_storage().data_ptr()
    d = _DEV_PTR.get(base)
    if d is None:
        out = ctypes.c_void_p()
        call("ome_host_device_ptr", ctypes.c_void_p(base), ctypes.byref(out))
        d = _DEV_PTR[base] = int(out.value or 0)
    return d + (host.data_ptr() - base)


def copy_h2d(dst: torch.Tensor, src_pinned: torch.Tensor) -> None:
    """``dst.copy_(src, non_blocking=True)`` as a kernel on the current stream (contiguous, same bytes)."""
    from ome_amd.ops._native import call, stream_ptr

    nb = src_pinned.numel() * src_pinned.element_size()
    assert dst.is_contiguous() and src_pinned.is_contiguous() and dst.numel() * dst.element_size() == nb
    call("ome_copy_mapped", ctypes.c_void_p(mapped_ptr(src_pinned)), ctypes.c_void_p(dst.data_ptr()), nb,
         ctypes.c_void_p(stream_ptr(dst.device)))


def copy_d2h(dst_pinned: torch.Tensor, src: torch.Tensor) -> None:
    """Device -> pinned host as a kernel on the current stream (the host reads it after an event)."""
    from ome_amd.ops._native import call, stream_ptr

    nb = src.numel() * src.element_size()
    assert src.is_contiguous() and dst_pinned.is_contiguous() and dst_pinned.numel() * dst_pinned.element_size() == nb
    call("ome_copy_mapped", ctypes.c_void_p(src.data_ptr()), ctypes.c_void_p(mapped_ptr(dst_pinned)), nb,
         ctypes.c_void_p(stream_ptr(src.device)))


class H2DStaging:
    def __init__(self, device, slots: int = 8, init_bytes: int = 1 << 20):
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.bufs: list[torch.Tensor | None] = [None] * slots
        self.events: list = [None] * slots
        self.init_bytes = init_bytes
        self.i = 0

    def to_device(self, arr: np.ndarray) -> torch.Tensor:
        """Asynchronous copy of ``arr`` (C-contiguous) to the device on the current stream."""
        arr = np.ascontiguousarray(arr)
        dt = _TORCH[arr.dtype]
        if not self.cuda:
            return torch.from_numpy(arr.copy())
        nb = arr.nbytes
        i = self.i
        self.i = (i + 1) % len(self.bufs)
        ev = self.events[i]
        if ev is not None:
            ev.synchronize()
        buf = self.bufs[i]
        if buf is None or buf.numel() < nb:
            size = max(nb, self.init_bytes, 2 * (buf.numel() if buf is not None else 0))
            buf = self.bufs[i] = torch.empty(size, dtype=torch.uint8, pin_memory=True)
        hv = buf[:nb]
        if nb:
            hv.numpy()[:] = arr.reshape(-1).view(np.uint8)
        dev = torch.empty(nb, dtype=torch.uint8, device=self.device)
        if nb:
            copy_h2d(dev, hv)
        ev = torch.cuda.Event()
        ev.record()
        self.events[i] = ev
        return dev.view(dt).view(arr.shape)
