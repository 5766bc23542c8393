"""Low-latency expert-parallel MoE for decode (DeepEP ``low_latency`` equivalent, SURVEY.md §2.9
K17; reference ``config/runtimes/srt/deepseek-rdma-pd-rt.yaml:83-126``).

The normal-mode path (:mod:`ome_amd.parallel.ep`) sizes its all-to-alls from per-layer split
counts pulled to the host (``.tolist()``), which blocks the CPU on every MoE layer and cannot be
captured in a HIP graph.  Here every rank owns fixed-capacity buckets (``cap`` rows per peer) in
an IPC-shared buffer, and the whole exchange runs as device kernels over the xGMI peer mappings
(``csrc/comm/ep_ll.hip``: plan -> pack -> flag -> pull -> experts -> combine pack -> flag -> pull);
split counts never leave the GPU, epochs live in device memory, so a captured decode graph
replays it.  ``cap`` = max tokens per rank x top-k covers the worst case (every assignment to one
rank); DeepSeek's ``SGLANG_DEEPEP_NUM_MAX_DISPATCH_TOKENS_PER_RANK`` plays the same role.
"""
from __future__ import annotations

import ctypes as C
import logging

import torch
import torch.distributed as dist

from ome_amd import ops
from ome_amd.ops import _native

log = logging.getLogger("ome_amd.ep_ll")


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


class LowLatencyEP:
    def __init__(self, group, hidden: int, max_tokens: int, top_k: int, cpu_group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.H, self.max_tokens, self.k = hidden, max_tokens, top_k
        self.cap = max_tokens * top_k
        lib = _native.load("ome_comm")
        hs = lib.ome_comm_handle_size()
        sig_h, buf_h = (C.c_char * hs)(), (C.c_char * hs)()
        ctx = C.c_void_p()
        rc = lib.ome_ep_create(self.rank, self.world, self.cap, hidden, C.byref(ctx), sig_h, buf_h)
        if rc != 0:
            raise _native.NativeError(f"ome_ep_create failed ({rc})")
        self._lib, self._ctx = lib, ctx
        allh = [None] * self.world
        dist.all_gather_object(allh, (bytes(sig_h), bytes(buf_h)), group=cpu_group)
        rc = lib.ome_ep_open(ctx, b"".join(h[0] for h in allh), b"".join(h[1] for h in allh))
        if rc != 0:
            raise _native.NativeError(f"ome_ep_open failed ({rc}): peers not reachable over xGMI/IPC")
        from ome_amd.runtime import watchdog

        watchdog.register_comm(f"ep_ll(rank {self.rank}/{self.world})", self.host_error, self.set_fault)

    def forward(self, x: torch.Tensor, topk_w: torch.Tensor, topk_ids: torch.Tensor, w13, w2, act: int,
                scale: float, e_local: int, tables=None) -> torch.Tensor:
        """x [T, H] this rank's tokens, routing [T, k] over global experts (rank r owns
        [r * e_local, (r + 1) * e_local), or the EPLB replica ``tables``); w13 / w2 this rank's
        expert slots (bf16 or Fp8Experts)."""
        T, H = x.shape
        k = topk_ids.shape[1]
        if T > self.max_tokens or k != self.k or H != self.H:
            raise ValueError(f"low-latency EP sized for {self.max_tokens} tokens x top-{self.k} x {self.H}")
        dev = x.device
        n = T * k
        a_dst = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        a_slot = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        a_local = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
        rr = rs = nr = None
        rmax = 0
        n_experts = e_local * self.world
        if tables is not None:
            rr, rs, nr = (t if t.dtype == torch.int64 else t.long() for t in tables)
            rmax = rr.shape[1]
            n_experts = rr.shape[0]
        R = torch.empty(self.world * self.cap, H, dtype=x.dtype, device=dev)
        rids = torch.empty(self.world * self.cap, dtype=torch.int32, device=dev)
        rcount = torch.empty(self.world, dtype=torch.int32, device=dev)
        ids = topk_ids.to(torch.int32).contiguous()
        s = _native.stream_ptr(dev)
        rc = self._lib.ome_ep_dispatch(self._ctx, C.c_void_p(x.data_ptr()), x.stride(0), C.c_void_p(ids.data_ptr()),
                                       T, k, e_local, n_experts, C.c_void_p(a_dst.data_ptr()), C.c_void_p(a_slot.data_ptr()),
                                       C.c_void_p(a_local.data_ptr()), _ptr(rr), _ptr(rs), _ptr(nr), rmax,
                                       C.c_void_p(R.data_ptr()), C.c_void_p(rids.data_ptr()),
                                       C.c_void_p(rcount.data_ptr()), C.c_void_p(s))
        if rc != 0:
            raise _native.NativeError(f"ome_ep_dispatch failed ({rc})")
        if w13 is None:   # exchange only (latency benchmarks): every received row comes back as is
            y, inv = R, torch.arange(R.shape[0], dtype=torch.int32, device=dev)
        else:
            y, inv = ops.moe_experts_sorted(R, rids, w13, w2, act, e_local)
        out = torch.empty(T, H, dtype=x.dtype, device=dev)
        w = topk_w.float().contiguous()
        rc = self._lib.ome_ep_combine(self._ctx, C.c_void_p(y.data_ptr()), C.c_void_p(inv.data_ptr()),
                                      C.c_void_p(rcount.data_ptr()), C.c_void_p(w.data_ptr()),
                                      C.c_void_p(a_dst.data_ptr()), C.c_void_p(a_slot.data_ptr()), T, k,
                                      float(scale), C.c_void_p(out.data_ptr()), out.stride(0), C.c_void_p(s))
        if rc != 0:
            raise _native.NativeError(f"ome_ep_combine failed ({rc})")
        return out

    def error(self) -> int:
        return self._lib.ome_ep_error(self._ctx)

    def host_error(self) -> int:
        return self._lib.ome_ep_host_error(self._ctx) if self._ctx else 0

    def set_fault(self, stall: int) -> int:
        return self._lib.ome_ep_set_fault(self._ctx, int(stall)) if self._ctx else -1

    def close(self) -> None:
        if self._ctx:
            self._lib.ome_ep_destroy(self._ctx)
            self._ctx = None
