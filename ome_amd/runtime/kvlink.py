"""Same-node xGMI fast path for PD KV hand-off (``csrc/comm/kvlink.hip``).

Decode side: a *landing pool* — per-layer K/V page tensors with the decode cache's exact page
layout — is allocated once and exported through hipIpc handles.  Prefill side: the handles are
mapped once per decode engine, and each finished prompt's pages are written straight into
reserved landing slots by a copy kernel on the prefill GPU (remote stores over xGMI); the decode
engine then moves them from the landing slots into freshly allocated cache pages with an
on-device copy.  The landing indirection keeps page allocation on the decode engine's thread
(the scheduler owns the page pool) and costs one HBM->HBM copy of the prompt's KV.

The TCP path of :mod:`ome_amd.runtime.disagg` remains the fallback (other node, CPU engines,
IPC unavailable).
"""
from __future__ import annotations

import ctypes as C
import logging
import threading
import uuid

import torch

from ome_amd.ops import _native

log = logging.getLogger("ome_amd.kvlink")


def _lib():
    return _native.load("ome_comm")


def available(device: torch.device) -> bool:
    return device.type == "cuda" and _native.available("ome_comm")


def export(t: torch.Tensor) -> tuple[str, int]:
    """(hex IPC handle of the owning allocation, byte offset of ``t`` inside it)."""
    lib = _lib()
    h = (C.c_char * lib.ome_kvlink_handle_size())()
    off = C.c_int64()
    rc = lib.ome_kvlink_export(C.c_void_p(t.data_ptr()), h, C.byref(off))
    if rc != 0:
        raise _native.NativeError(f"ome_kvlink_export failed ({rc})")
    return bytes(h).hex(), int(off.value)


class LandingPool:
    """Decode side: exported page tensors + a slot allocator (thread-safe)."""

    def __init__(self, kv, n_pages: int):
        self.kv, self.n_pages = kv, n_pages
        dev = next(t for t in kv.k if t is not None).device
        self.k = {i: torch.zeros((n_pages, *kv.k[i].shape[1:]), dtype=kv.dtype, device=dev) for i in kv.local_layers}
        self.v = {i: torch.zeros((n_pages, *kv.v[i].shape[1:]), dtype=kv.dtype, device=dev) for i in kv.local_layers}
        self.free = list(range(n_pages))
        self.lock = threading.Lock()
        self.session = uuid.uuid4().hex
        self.handles = {"k": [export(self.k[i]) for i in kv.local_layers],
                        "v": [export(self.v[i]) for i in kv.local_layers if self.v[i].numel()]}
        ek = self.k[kv.local_layers[0]]
        ev = self.v[kv.local_layers[0]]
        self.k_page_bytes = ek[0].numel() * ek.element_size()
        self.v_page_bytes = ev[0].numel() * ev.element_size()

    def describe(self) -> dict:
        return {"session": self.session, "handles": self.handles, "k_page_bytes": self.k_page_bytes,
                "v_page_bytes": self.v_page_bytes, "dtype": str(self.kv.dtype), "n_pages": self.n_pages}

    def reserve(self, n: int) -> list[int] | None:
        with self.lock:
            if len(self.free) < n:
                return None
            out, self.free = self.free[:n], self.free[n:]
            return out

    def release(self, slots: list[int]) -> None:
        with self.lock:
            self.free.extend(slots)

    def install(self, slots: list[int], pages: list[int]) -> None:
        """Landing slots -> cache pages (on the decode device, in the current stream)."""
        dev = self.k[self.kv.local_layers[0]].device
        src = torch.tensor(slots, dtype=torch.long, device=dev)
        dst = torch.tensor(pages, dtype=torch.long, device=dev)
        for i in self.kv.local_layers:
            self.kv.k[i].index_copy_(0, dst, self.k[i].index_select(0, src))
            if self.v[i].numel():
                self.kv.v[i].index_copy_(0, dst, self.v[i].index_select(0, src))


class PeerMapping:
    """Prefill side: the decode engine's landing pool mapped into this process."""

    def __init__(self, desc: dict, device: torch.device):
        lib = _lib()
        self.session = desc["session"]
        self.device = device
        self.k_page_bytes, self.v_page_bytes = int(desc["k_page_bytes"]), int(desc["v_page_bytes"])
        self._bases: list[C.c_void_p] = []
        opened: dict[str, int] = {}

        def open_ptr(hexh: str, off: int) -> int:
            if hexh not in opened:  # several layer tensors may share one allocation
                base = C.c_void_p()
                h = bytes.fromhex(hexh)
                with torch.cuda.device(device):
                    rc = lib.ome_kvlink_open(h, C.byref(base))
                if rc != 0:
                    raise _native.NativeError(f"ome_kvlink_open failed ({rc})")
                self._bases.append(base)
                opened[hexh] = int(base.value)
            return opened[hexh] + off

        self.k_ptrs = [open_ptr(h, o) for h, o in desc["handles"]["k"]]
        self.v_ptrs = [open_ptr(h, o) for h, o in desc["handles"]["v"]]
        self.k_dev = torch.tensor(self.k_ptrs, dtype=torch.int64, device=device)
        self.v_dev = torch.tensor(self.v_ptrs, dtype=torch.int64, device=device) if self.v_ptrs else None

    def write(self, k_pages: list[torch.Tensor], v_pages: list[torch.Tensor], slots: list[int],
              stream: torch.cuda.Stream) -> None:
        """Copy staged page images (one [n, ...] tensor per layer) into landing ``slots``."""
        lib = _lib()
        n = len(slots)
        dev = self.device
        with torch.cuda.stream(stream):
            src_idx = torch.arange(n, dtype=torch.int32, device=dev)
            dst_idx = torch.tensor(slots, dtype=torch.int32, device=dev)
            groups = [(k_pages, self.k_dev, self.k_page_bytes)]
            if self.v_dev is not None:
                groups.append(([v for v in v_pages if v.numel()], self.v_dev, self.v_page_bytes))
            for tensors, dst_dev, pb in groups:
                if not tensors:
                    continue
                src_dev = torch.tensor([t.data_ptr() for t in tensors], dtype=torch.int64, device=dev)
                rc = lib.ome_kvlink_copy(C.c_void_p(src_dev.data_ptr()), C.c_void_p(dst_dev.data_ptr()),
                                         C.c_void_p(src_idx.data_ptr()), C.c_void_p(dst_idx.data_ptr()), n,
                                         len(tensors), pb, pb, C.c_void_p(stream.cuda_stream))
                if rc != 0:
                    raise _native.NativeError(f"ome_kvlink_copy failed ({rc})")
            stream.synchronize()

    def close(self) -> None:
        lib = _lib()
        for b in self._bases:
            lib.ome_kvlink_close(b)
        self._bases = []
