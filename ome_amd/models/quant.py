"""FP8 (OCP e4m3fn) weight-quantised linear layers.

The reference's runtimes serve ``quantization: fp8`` checkpoints two ways, and both are covered:

* **per-channel** (``--quantization fp8`` online quantisation of a bf16 checkpoint, and the
  per-tensor / per-channel ``weight_scale`` FP8 checkpoints such as Llama-3.1-*-FP8): weight
  scale per output row, activation scale per token;
* **block-scaled** (DeepSeek-V3 / Kimi-K2 style ``weight_scale_inv`` with
  ``weight_block_size: [128, 128]``): weight scale per 128x128 block, activation scale per
  1x128 group.

Activations are always quantised dynamically by ``ome_fp8_quant`` (static ``input_scale`` of a
checkpoint is ignored: dynamic scales are at least as accurate and cost one fused pass).  The
GEMM is ``ome_fp8_gemm`` (csrc/kernels/fp8.hip).  FP8 checkpoints are streamed through
:func:`dequant_fp8_stream` so every model loader keeps seeing bf16 tensors, then
:func:`quantize_weight` re-quantises the fused (QKV / gate-up) shards: with the checkpoint's own
block structure and ``amax/448`` scales that round-trip is exact.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.ops import reference as ref


@dataclass
class Fp8Weight:
    q: torch.Tensor        # [N, K] float8_e4m3fn
    scale: torch.Tensor    # [N] (block 0) or [ceil(N/128), K/128] (block 128), float32
    block: int = 0
    # bf16 copy for the row counts where W8A8 was measured slower than bf16 (small N x K
    # projections at decode sizes: activation quant + a few output tiles cost more than the halved
    # weight bytes save -- profiles/r04_fp8_sk_bench.txt); None = always fp8
    bf16: torch.Tensor | None = None
    bf16_max_m: int = 0

    @property
    def shape(self):
        return self.q.shape

    def nbytes(self) -> int:
        n = self.q.numel() + self.scale.numel() * 4
        return n + (self.bf16.numel() * 2 if self.bf16 is not None else 0)

    def dequant(self, dtype=torch.bfloat16) -> torch.Tensor:
        return ref.fp8_dequant_weight(self.q, self.scale, self.block).to(dtype)


# bytes of bf16 copies kept next to fp8 weights in this process (logged once at the end of a
# model's quantisation pass, bounded by OME_FP8_BF16_BUDGET_MB)
_BF16_COPY_BYTES = 0


def fp8_bf16_max_m(N: int, K: int, tp: int = 1) -> int:
    """Rows up to which an fp8 [N, K] projection also runs on a bf16 copy of its own dequantised
    values (0: never).  Only the SMALL projections keep a copy: N <= 2048 with N * K <= 16M
    elements (DeepSeek q_a / kv_a, ~15-22 MB per layer), where activation quantisation plus a few
    output tiles cost more than the halved weight bytes save at decode sizes (r05
    profiles/r05_fp8_routed_bench.txt).  The Llama-size projections (qkv / o / down / gate_up) stay
    fp8-only: a copy there nearly doubled the fp8 footprint.  Under TP the shapes are
    per-rank shards, which were never measured, so no copies are kept; the total is bounded by
    ``OME_FP8_BF16_BUDGET_MB`` (default 2048 MiB) and ``OME_FP8_BF16_FALLBACK=0`` disables it."""
    if os.environ.get("OME_FP8_BF16_FALLBACK", "1") == "0" or tp > 1:
        return 0
    if N <= 2048 and N * K <= (16 << 20):
        budget = int(os.environ.get("OME_FP8_BF16_BUDGET_MB", "2048")) << 20
        if _BF16_COPY_BYTES + N * K * 2 <= budget:
            return 256
    return 0


def fp8_bf16_copy_bytes() -> int:
    return _BF16_COPY_BYTES


@dataclass
class Fp8Experts:
    """MoE expert weights kept in FP8 (``quantization: fp8``, 128x128 block scales): q [E, N, K]
    float8_e4m3fn, scale [E, N/128, K/128] float32.  Consumed by ``ops.fused_moe`` through the
    block-scaled grouped GEMM (csrc/kernels/moe.hip ``ome_moe_gemm_fp8``)."""
    q: torch.Tensor
    scale: torch.Tensor
    block: int = 128

    @property
    def shape(self):
        return self.q.shape

    def nbytes(self) -> int:
        return self.q.numel() + self.scale.numel() * 4

    def dequant(self, dtype=torch.bfloat16) -> torch.Tensor:
        return torch.stack([ref.fp8_dequant_weight(self.q[e], self.scale[e], self.block)
                            for e in range(self.q.shape[0])]).to(dtype)

    def index_select(self, dim: int, idx: torch.Tensor) -> "Fp8Experts":
        assert dim == 0
        return Fp8Experts(self.q.index_select(0, idx), self.scale.index_select(0, idx), self.block)


def quantize_experts(w: torch.Tensor, block: int = 128) -> Fp8Experts:
    """[E, N, K] bf16 -> Fp8Experts with amax/448 scales per 128x128 block of every expert
    (N, K multiples of 128: DeepSeek-V3 2I = 4096 / H = 7168)."""
    E, N, K = w.shape
    if N % block or K % block:
        raise ValueError(f"expert weight {tuple(w.shape)} is not {block}x{block}-tileable")
    blocks = w.float().reshape(E, N // block, block, K // block, block)
    amax = blocks.abs().amax(dim=(2, 4))
    s = torch.where(amax > 0, amax / ref.FP8_MAX, torch.ones_like(amax))
    q = (blocks / s[:, :, None, :, None]).clamp(-ref.FP8_MAX, ref.FP8_MAX).to(torch.float8_e4m3fn)
    return Fp8Experts(q.reshape(E, N, K).contiguous(), s.contiguous(), block)


def quantize_moe_experts(model) -> int:
    """``quantization: fp8`` MoE models: turn every MoE layer's stacked expert weights (w13 / w2,
    bf16 [E_local, N, K]) into :class:`Fp8Experts` with 128x128 block scales, so the experts are
    stored and streamed as fp8 (no load-time dequantisation to bf16).  Returns how many stayed bf16
    (shapes that do not tile by 128)."""
    kept = 0
    for i in getattr(model, "moe_layers", ()):
        for name in ("w13", "w2"):
            lst = getattr(model, name, None)
            w = lst[i] if lst is not None else None
            if isinstance(w, torch.Tensor) and w.dim() == 3 and w.numel():
                if w.shape[1] % 128 == 0 and w.shape[2] % 128 == 0:
                    lst[i] = quantize_experts(w)
                else:
                    kept += 1
    return kept


def quantize_weight(w: torch.Tensor, block: int = 0, tp: int = 1) -> Fp8Weight:
    """bf16/fp32 [N, K] -> Fp8Weight (amax/448 scales per row, or per 128x128 block); ``tp``: the
    tensor-parallel degree the shard belongs to (no bf16 copies under TP)."""
    global _BF16_COPY_BYTES
    N, K = w.shape
    wf = w.float()
    if block:
        nb, kb = -(-N // block), K // block
        pad = nb * block - N
        wp = F.pad(wf, (0, 0, 0, pad)) if pad else wf
        blocks = wp.reshape(nb, block, kb, block)
        amax = blocks.abs().amax(dim=(1, 3))
        s = torch.where(amax > 0, amax / ref.FP8_MAX, torch.ones_like(amax))
        q = (blocks / s[:, None, :, None]).clamp(-ref.FP8_MAX, ref.FP8_MAX).to(torch.float8_e4m3fn)
        q = q.reshape(nb * block, K)[:N].contiguous()
        out = Fp8Weight(q, s.contiguous(), block)
    else:
        amax = wf.abs().amax(-1)
        s = torch.where(amax > 0, amax / ref.FP8_MAX, torch.ones_like(amax))
        q = (wf / s[:, None]).clamp(-ref.FP8_MAX, ref.FP8_MAX).to(torch.float8_e4m3fn).contiguous()
        out = Fp8Weight(q, s.contiguous(), 0)
    m = fp8_bf16_max_m(N, K, tp) if w.is_cuda else 0
    if m:
        # the fp8 weights' own values (dequantised), so both paths compute the same projection
        out.bf16, out.bf16_max_m = out.dequant(torch.bfloat16).contiguous(), m
        _BF16_COPY_BYTES += out.bf16.numel() * 2
    return out


# rows up to which plain bf16 projections run on the GEMV stream kernel (0 disables)
_GEMV_ROWS = int(os.environ.get("OME_GEMV_ROWS", "4"))


def _sk_operands_ok(x, w, bias, out) -> bool:
    return (x.stride(1) == 1 and x.stride(0) % 8 == 0 and x.data_ptr() % 16 == 0 and w.is_contiguous()
            and w.data_ptr() % 16 == 0 and (bias is None or bias.dtype == torch.bfloat16)
            and (out is None or (out.stride(1) == 1 and out.stride(0) % 4 == 0 and out.data_ptr() % 8 == 0)))


def linear(x: torch.Tensor, w, bias: torch.Tensor | None = None, out: torch.Tensor | None = None) -> torch.Tensor:
    """Dispatch: bf16 weight at a row count where the stream-K MFMA kernel was measured faster
    (``ops.gemm_sk_plan``) -> ``ops.gemm_sk``; single-row decode -> the GEMV stream kernel
    (``ops.gemv``, ``OME_GEMV_ROWS``); the weight-streaming MFMA GEMM for decode shapes where it
    was measured faster (``ops.decode_gemm_plan``, opt-in); other plain tensors -> hipBLASLt;
    Fp8Weight -> W8A16 (fp8 weight, bf16 activation) at the decode rows where ``ops.w8a16_plan``
    measured it faster, else the W8A8 MFMA path.  ``out``: write the result there (e.g. the TP all-reduce's IPC
    staging buffer)."""
    if (x.dim() == 2 and x.is_cuda and x.shape[0] > _GEMV_ROWS and type(w) is torch.Tensor
            and w.dtype == torch.bfloat16 and x.dtype == torch.bfloat16):
        plan = ops.gemm_sk_plan(x.shape[0], w.shape[0], w.shape[1], 0)
        if plan is not None and _sk_operands_ok(x, w, bias, out):
            return ops.gemm_sk(x, w, bias, out=out, bn=plan[0], nwg=plan[1], bm=plan[2])
    if out is not None:
        if x.is_cuda and x.shape[0] <= _GEMV_ROWS and ops.gemv_ok(x, w, bias, out):
            return ops.gemv(x, w, bias, out=out)
        if isinstance(w, torch.Tensor) and x.dim() == 2 and x.is_cuda:
            if bias is None:
                return torch.matmul(x, w.t(), out=out)
            return torch.addmm(bias, x, w.t(), out=out)
        out.copy_(linear(x, w, bias))
        return out
    if isinstance(w, Fp8Weight):
        if x.dim() == 2 and x.dtype == torch.bfloat16:
            M = x.shape[0]
            copy = w.bf16 is not None and M <= w.bf16_max_m
            if x.is_cuda and not (copy and M > 8):
                # decode rows: fp8 weight streamed + widened in registers, bf16 activation
                # (csrc/kernels/w8a16.hip) where measured faster than W8A8
                sp = ops.w8a16_plan(M, w.q.shape[0], w.q.shape[1], w.block)
                if sp is not None and ops.w8a16_ok(x, w.q, w.scale, w.block):
                    return ops.w8a16_gemm(x, w.q, w.scale, w.block, bias, splits=sp)
            if copy:
                return linear(x, w.bf16, bias)
        return ops.fp8_linear(x, w.q, w.scale, w.block, bias)
    if x.dim() == 2 and x.shape[0] <= 256 and x.is_cuda:
        if x.shape[0] <= _GEMV_ROWS and ops.gemv_ok(x, w, bias):
            return ops.gemv(x, w, bias)
        plan = ops.decode_gemm_plan(x, w, bias)
        if plan is not None:
            return ops.stream_gemm(x, w, bias, nf=plan[0], splits=plan[1])
    return F.linear(x, w, bias)


def fp8_block_size(cfg) -> int:
    qc = (cfg.extra or {}).get("quantization_config") or {}
    wbs = qc.get("weight_block_size")
    if wbs:
        if list(wbs) != [128, 128]:
            raise ValueError(f"unsupported fp8 weight_block_size {wbs} (128x128 only)")
        return 128
    return 0


def dequant_fp8_stream(weights, block: int, dtype=torch.bfloat16):
    """Pass (name, tensor) through, turning FP8 checkpoint weights + their ``weight_scale`` /
    ``weight_scale_inv`` companions into dequantised tensors (order-independent)."""
    pending_w: dict[str, torch.Tensor] = {}
    pending_s: dict[str, tuple[torch.Tensor, bool]] = {}

    def emit(base: str, q: torch.Tensor, s: torch.Tensor, blockwise: bool):
        s = s.float().to(q.device)
        if s.numel() == 1:
            w = q.float() * s.reshape(())
        elif blockwise:  # ``weight_scale_inv``: one scale per block x block tile
            w = ref.fp8_dequant_weight(q, s.reshape(-(-q.shape[0] // (block or 128)), -1), block or 128)
        else:            # ``weight_scale``: per output channel
            w = q.float() * s.reshape(-1, 1)
        return base + ".weight", w.to(dtype)

    for name, t in weights:
        if name.endswith(".input_scale") or name.endswith(".activation_scale"):
            continue
        if name.endswith(".weight_scale") or name.endswith(".weight_scale_inv"):
            base = name.rsplit(".", 1)[0]
            blockwise = name.endswith("_inv")
            if base in pending_w:
                yield emit(base, pending_w.pop(base), t, blockwise)
            else:
                pending_s[base] = (t, blockwise)
            continue
        if name.endswith(".weight") and t.dtype in (torch.float8_e4m3fn, torch.float8_e5m2):
            base = name[: -len(".weight")]
            if base in pending_s:
                yield emit(base, t, *pending_s.pop(base))
            else:
                pending_w[base] = t
            continue
        yield name, t
    if pending_w:
        raise ValueError(f"fp8 weights without scales: {sorted(pending_w)[:4]}")
