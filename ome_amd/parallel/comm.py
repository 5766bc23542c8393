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
        lib = _native.load("ome_comm")
        hs = lib.ome_comm_handle_size()
        sig_h, dat_h = (C.c_char * hs)(), (C.c_char * hs)()
        ctx = C.c_void_p()
        rc = lib.ome_comm_create(self.rank, self.world, max_bytes, C.byref(ctx), sig_h, dat_h)
        if rc != 0:
            raise _native.NativeError(f"ome_comm_create failed ({rc})")
        self._lib, self._ctx = lib, ctx
        mine = (bytes(sig_h), bytes(dat_h))
        allh = [None] * self.world
        dist.all_gather_object(allh, mine, group=cpu_group)
        sig_all = b"".join(h[0] for h in allh)
        dat_all = b"".join(h[1] for h in allh)
        rc = lib.ome_comm_open(ctx, sig_all, dat_all)
        if rc != 0:
            raise _native.NativeError(f"ome_comm_open failed ({rc}): peers not reachable over xGMI/IPC")

    def usable(self, x: torch.Tensor) -> bool:
        n = x.numel()
        return (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and n % 8 == 0 and
                n * 2 <= self.max_bytes)

    def all_reduce(self, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """Sum of ``x`` over the group (in place unless ``out`` is given)."""
        out = x if out is None else out
        two = x.numel() * 2 > self.one_shot_max
        rc = self._lib.ome_comm_all_reduce(self._ctx, C.c_void_p(x.data_ptr()), C.c_void_p(out.data_ptr()),
                                           x.numel(), int(two), self.blocks,
                                           C.c_void_p(torch.cuda.current_stream(x.device).cuda_stream))
        if rc != 0:
            raise _native.NativeError(f"ome_comm_all_reduce failed ({rc})")
        return out

    def error(self) -> int:
        return self._lib.ome_comm_error(self._ctx)

    def close(self) -> None:
        if self._ctx:
            self._lib.ome_comm_destroy(self._ctx)
            self._ctx = None


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
