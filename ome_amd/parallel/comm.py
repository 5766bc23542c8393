"""TP all-reduce for one 8x MI355X node: custom xGMI peer kernels for the decode/prefill message
sizes, RCCL for everything else.

The reference's runtimes get this from SGLang's custom all-reduce on NVLink; here every GPU of
the node has a direct xGMI link to every other one, so ``csrc/comm/allreduce.hip`` reads the
peers' buffers directly through hipIpc mappings:

* one-shot (each rank reads all N inputs, one kernel, two block-level barriers) up to
  ``one_shot_max`` bytes -- the per-layer decode messages ([B, H] bf16: 8 KiB x B for 8B models);
* two-shot (reduce-scatter then all-gather over the same mappings) up to the registered buffer
  size -- prefill-sized messages move (N-1)/N of the bytes per link;
* RCCL ``all_reduce`` above that, for non-bf16 tensors, and when the peers are not on one node.

Handles are exchanged once over a CPU (gloo) group; the kernels keep their epoch counters in
device memory, so the call is HIP-graph capturable.
"""
from __future__ import annotations

import ctypes as C
import logging
import os

import torch
import torch.distributed as dist

from ome_amd.ops import _native

log = logging.getLogger("ome_amd.comm")


class CustomAllReduce:
    def __init__(self, group=None, max_bytes: int = 64 << 20, one_shot_max: int = 512 << 10,
                 cpu_group=None, blocks: int = 64):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if self.world not in (2, 4, 8):
            raise ValueError(f"custom all-reduce supports 2/4/8 ranks, got {self.world}")
        self.max_bytes, self.one_shot_max, self.blocks = max_bytes, one_shot_max, blocks
        # one-shot: 16-B vectors per lane before another workgroup is added (grid sizing);
        # 0 = the measured per-size rule in _grid
        self.vpt = int(os.environ.get("OME_AR_VPT", "0"))
        lib = _native.load("ome_comm")
        hs = lib.ome_comm_handle_size()
        sig_h, dat_h = (C.c_char * hs)(), (C.c_char * hs)()
        ctx = C.c_void_p()
        rc = lib.ome_comm_create(self.rank, self.world, max_bytes, C.byref(ctx), sig_h, dat_h)
        if rc != 0:
            raise _native.NativeError(f"ome_comm_create failed ({rc})")
        self._lib, self._ctx = lib, ctx
        lib.ome_comm_buffer.argtypes = [C.c_void_p]
        lib.ome_comm_buffer.restype = C.c_void_p
        self._buf_ptr = int(lib.ome_comm_buffer(ctx))
        self._buf = None
        mine = (bytes(sig_h), bytes(dat_h))
        allh = [None] * self.world
        dist.all_gather_object(allh, mine, group=cpu_group)
        sig_all = b"".join(h[0] for h in allh)
        dat_all = b"".join(h[1] for h in allh)
        rc = lib.ome_comm_open(ctx, sig_all, dat_all)
        if rc != 0:
            raise _native.NativeError(f"ome_comm_open failed ({rc}): peers not reachable over xGMI/IPC")
        # bounded-wait expiries land in a host-mapped word the engine watchdog polls (no HIP call)
        from ome_amd.runtime import watchdog

        watchdog.register_comm(f"allreduce(rank {self.rank}/{self.world})", self.host_error, self.set_fault)

    def _grid(self, n: int, two_shot: bool) -> int:
        """Workgroups for an n-element reduction: each one costs a flag hand-off with every peer
        (system-scope release + acquire spin), about 0.35 us per workgroup measured with 2 ranks
        (profiles/r03_comm_latency.txt: 1 row 6.6 us, 64 rows 28.8 us), so small messages use
        few of them -- at least 4 16-B vectors per lane (2 per lane and rank's chunk in two-shot)."""
        vec = n // 8
        vpt = self.vpt
        if vpt <= 0:   # measured per size (profiles/r04_comm_latency.txt: one-shot grid sweep)
            nb = n * 2
            vpt = 1 if nb <= 64 << 10 else 2 if nb <= 128 << 10 else 4
        per = 512 * (2 * self.world if two_shot else vpt)
        return max(1, min(self.blocks, -(-vec // per)))

    def usable(self, x: torch.Tensor) -> bool:
        n = x.numel()
        return (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and n % 8 == 0 and
                n * 2 <= self.max_bytes)

    def all_reduce(self, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """Sum of ``x`` over the group (in place unless ``out`` is given; callers use the returned
        tensor).  One-shot never writes into the registered IPC buffer: peers read every index of
        it while this rank writes, so an in-place result there (``x`` produced straight into
        :meth:`staging`) could be re-added by a slower peer.  Such calls get a fresh output."""
        out = x if out is None else out
        two = x.numel() * 2 > self.one_shot_max
        if not two and self._in_buffer(out):
            out = torch.empty_like(x)
        rc = self._lib.ome_comm_all_reduce(self._ctx, C.c_void_p(x.data_ptr()), C.c_void_p(out.data_ptr()),
                                           x.numel(), int(two), self._grid(x.numel(), two),
                                           C.c_void_p(torch.cuda.current_stream(x.device).cuda_stream))
        if rc != 0:
            raise _native.NativeError(f"ome_comm_all_reduce failed ({rc})")
        return out

    def _in_buffer(self, t: torch.Tensor) -> bool:
        p = t.data_ptr()
        return self._buf_ptr <= p < self._buf_ptr + self.max_bytes

    def staging(self, shape, dtype=torch.bfloat16, device=None) -> torch.Tensor | None:
        """A tensor view of this rank's registered IPC input buffer: a producer (the row-parallel
        GEMM) that writes its output here lets the next :meth:`all_reduce` skip the staging copy.
        None when the shape does not fit."""
        n = 1
        for d in shape:
            n *= int(d)
        if dtype != torch.bfloat16 or n * 2 > self.max_bytes or n % 8:
            return None
        if self._buf is None:
            try:
                self._buf = _wrap_device_ptr(self._buf_ptr, self.max_bytes // 2, torch.bfloat16,
                                             device or torch.device("cuda", torch.cuda.current_device()))
            except Exception as e:  # noqa: BLE001 — the staged-copy path stays correct
                log.warning("IPC staging buffer not wrappable as a tensor (%s); all-reduce keeps its copy", e)
                self._buf = False
        if self._buf is False:
            return None
        return self._buf[:n].view(*shape)

    def all_reduce_add_rmsnorm(self, x: torch.Tensor, residual: torch.Tensor, weight: torch.Tensor,
                               eps: float) -> torch.Tensor | None:
        """``residual += allreduce(x); return rmsnorm(residual) * weight`` in ONE kernel (one-shot
        sizes only; ``x`` may be the :meth:`staging` buffer).  None (nothing done) when the message
        is too large for one-shot.  The normed rows go to a fresh tensor: writing them over the
        staged input would race with peers still reading it."""
        rows, H = x.shape
        if x.numel() * 2 > self.one_shot_max or H % 8 or H > 512 * 8 * 4 or not residual.is_contiguous():
            return None
        out = torch.empty_like(x)
        rc = self._lib.ome_comm_all_reduce_add_rmsnorm(
            self._ctx, C.c_void_p(x.data_ptr()), C.c_void_p(out.data_ptr()), C.c_void_p(residual.data_ptr()),
            C.c_void_p(weight.data_ptr()), rows, H, float(eps), max(1, min(self.blocks, -(-rows // 4))),
            C.c_void_p(torch.cuda.current_stream(x.device).cuda_stream))
        if rc != 0:
            raise _native.NativeError(f"ome_comm_all_reduce_add_rmsnorm failed ({rc})")
        return out

    def all_gather_last(self, x: torch.Tensor) -> torch.Tensor | None:
        """concat over ranks along the last dim (x: [rows, cols] bf16 contiguous), or None when the
        shape does not fit the one-shot gather."""
        if x.dtype not in (torch.bfloat16, torch.float16) or not x.is_contiguous() or x.dim() != 2:
            return None
        rows, cols = x.shape
        if (cols * 2) % 16 or rows * cols * 2 > self.max_bytes:
            return None
        out = torch.empty(rows, cols * self.world, dtype=x.dtype, device=x.device)
        rc = self._lib.ome_comm_all_gather(self._ctx, C.c_void_p(x.data_ptr()), C.c_void_p(out.data_ptr()), rows,
                                           cols, self.blocks, C.c_void_p(torch.cuda.current_stream(x.device).cuda_stream))
        if rc != 0:
            raise _native.NativeError(f"ome_comm_all_gather failed ({rc})")
        return out

    def error(self) -> int:
        return self._lib.ome_comm_error(self._ctx)

    def host_error(self) -> int:
        """The error word the kernels mirror into host memory: no HIP call, safe while the GPU is busy."""
        return self._lib.ome_comm_host_error(self._ctx) if self._ctx else 0

    def set_fault(self, stall: int) -> int:
        """Fault injection (OME_COMM_FAULT set before creation): stall the flag publish of every
        following barrier by ``stall`` x s_sleep(127); -1 when injection was not enabled."""
        return self._lib.ome_comm_set_fault(self._ctx, int(stall)) if self._ctx else -1

    def close(self) -> None:
        if self._ctx:
            self._lib.ome_comm_destroy(self._ctx)
            self._ctx = None


def _wrap_device_ptr(ptr: int, numel: int, dtype: torch.dtype, device: torch.device) -> torch.Tensor:
    """A torch tensor over memory this library allocated (the IPC buffer lives as long as the
    communicator; torch never frees it)."""
    class _Holder:
        pass

    h = _Holder()
    itemsize = torch.empty(0, dtype=dtype).element_size()
    h.__cuda_array_interface__ = {"shape": (numel,), "typestr": {torch.bfloat16: "<i2", torch.float16: "<f2"}[dtype],
                                  "data": (ptr, False), "version": 3, "strides": (itemsize,)}
    t = torch.as_tensor(h, device=device)
    return t.view(dtype)


class TPCommunicator:
    """What :func:`ome_amd.parallel.state.tp_all_reduce` calls when installed: the custom kernel
    when it applies, RCCL otherwise."""

    def __init__(self, group, cpu_group=None, **kw):
        self.group = group
        self.custom = None
        try:
            self.custom = CustomAllReduce(group, cpu_group=cpu_group, **kw)
        except Exception as e:  # noqa: BLE001 — multi-node groups etc.: RCCL only, loudly
            log.warning("custom xGMI all-reduce unavailable (%s); using RCCL", e)

    def all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        if self.custom is not None and self.custom.usable(x):
            return self.custom.all_reduce(x)
        dist.all_reduce(x, group=self.group)
        return x

    def staging(self, shape, dtype, device) -> torch.Tensor | None:
        return self.custom.staging(shape, dtype, device) if self.custom is not None else None

    def all_reduce_add_rmsnorm(self, x, residual, weight, eps) -> torch.Tensor | None:
        if self.custom is None or not self.custom.usable(x):
            return None
        return self.custom.all_reduce_add_rmsnorm(x, residual, weight, eps)

    def all_gather_last(self, x: torch.Tensor) -> torch.Tensor:
        if self.custom is not None:
            out = self.custom.all_gather_last(x)
            if out is not None:
                return out
        parts = [torch.empty_like(x) for _ in range(dist.get_world_size(self.group))]
        dist.all_gather(parts, x.contiguous(), group=self.group)
        return torch.cat(parts, dim=-1)
