"""Hot-path ops.  CUDA(HIP) tensors -> hand-written gfx950 kernels (``_native``); CPU tensors ->
the fp32 reference implementations (``reference``).  No silent GPU fallback exists: if the
native library is missing on a GPU the call raises.
"""
from __future__ import annotations

import contextlib
import os

import torch
import torch.nn.functional as F

from . import reference as ref
from ._native import NativeError, available, call, ptr, stream_ptr  # noqa: F401


def _gpu(t: torch.Tensor) -> bool:
    return t.is_cuda


def _i32(t: torch.Tensor) -> torch.Tensor:
    assert t.dtype == torch.int32 and t.is_contiguous(), "metadata tensors must be contiguous int32"
    return t


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, out: torch.Tensor | None = None) -> torch.Tensor:
    if not _gpu(x):
        r = ref.rmsnorm(x, w, eps)
        if out is not None:
            out.copy_(r)
            return out
        return r
    H = x.shape[-1]
    x2 = x.reshape(-1, H)
    assert x2.stride(-1) == 1 and x.dtype == torch.bfloat16
    out = torch.empty_like(x2) if out is None else out.reshape(-1, H)
    call("ome_rmsnorm", x2.data_ptr(), x2.stride(0), w.data_ptr(), out.data_ptr(), out.stride(0), x2.shape[0], H,
         float(eps), stream_ptr())
    return out.view(x.shape)


def fused_add_rmsnorm(x: torch.Tensor, res: torch.Tensor, w: torch.Tensor, eps: float) -> None:
    """In place: res <- x + res; x <- rmsnorm(res) * w."""
    if not _gpu(x):
        return ref.fused_add_rmsnorm(x, res, w, eps)
    H = x.shape[-1]
    x2, r2 = x.view(-1, H), res.view(-1, H)
    call("ome_fused_add_rmsnorm", x2.data_ptr(), x2.stride(0), r2.data_ptr(), r2.stride(0), w.data_ptr(),
         x2.shape[0], H, float(eps), stream_ptr())


def layernorm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None, eps: float,
              out: torch.Tensor | None = None) -> torch.Tensor:
    """LayerNorm with optional bias (Starcoder2 / GPT-NeoX); ``out``: a row-strided [rows, H]
    destination (e.g. one sample's rows of a packed batch)."""
    if not _gpu(x):
        r = ref.layernorm(x, w, b, eps)
        if out is not None:
            out.copy_(r.view(out.shape))
            return out
        return r
    H = x.shape[-1]
    x2 = x.reshape(-1, H)
    assert x2.stride(-1) == 1 and x.dtype == torch.bfloat16
    if out is not None:
        assert out.stride(-1) == 1 and out.shape[-1] == H
        call("ome_layernorm", x2.data_ptr(), x2.stride(0), None, 0, w.data_ptr(), ptr(b), out.data_ptr(),
             out.stride(0), x2.shape[0], H, float(eps), stream_ptr())
        return out
    out = torch.empty_like(x2)
    call("ome_layernorm", x2.data_ptr(), x2.stride(0), None, 0, w.data_ptr(), ptr(b), out.data_ptr(), out.stride(0),
         x2.shape[0], H, float(eps), stream_ptr())
    return out.view(x.shape)


def qk_norm_rope(x: torch.Tensor, H: int, hd: int, w: torch.Tensor | None, cs: torch.Tensor | None, eps: float,
                 out: torch.Tensor, dst: torch.Tensor | None = None) -> torch.Tensor:
    """Per-head RMSNorm (``w`` [hd], None: none) + complex-pair RoPE (``cs`` fp32 [T, hd/2, 2] =
    (cos, sin), None: none) of x [T, >= H*hd] (row-strided), written to rows ``dst`` [T] int32
    (None: 0..T-1) of ``out`` [rows, H*hd] (Qwen-Image joint attention operands)."""
    T = x.shape[0]
    if not _gpu(x):
        return ref.qk_norm_rope(x, H, hd, w, cs, eps, out, dst)
    assert x.stride(1) == 1 and out.stride(-1) == 1 and x.dtype == out.dtype == torch.bfloat16
    assert cs is None or (cs.dtype == torch.float32 and cs.is_contiguous() and cs.shape[0] == T)
    o2 = out.view(out.shape[0], -1)
    call("ome_qk_norm_rope", x.data_ptr(), x.stride(0), ptr(w), ptr(cs), T, H, hd, float(eps), o2.data_ptr(),
         o2.stride(0), None if dst is None else _i32(dst).data_ptr(), stream_ptr())
    return out


def fused_add_layernorm(x: torch.Tensor, res: torch.Tensor, w: torch.Tensor, b: torch.Tensor | None,
                        eps: float) -> None:
    """In place: res <- x + res; x <- layernorm(res) * w + b."""
    if not _gpu(x):
        return ref.fused_add_layernorm(x, res, w, b, eps)
    H = x.shape[-1]
    x2, r2 = x.view(-1, H), res.view(-1, H)
    call("ome_layernorm", x2.data_ptr(), x2.stride(0), r2.data_ptr(), r2.stride(0), w.data_ptr(), ptr(b), None, 0,
         x2.shape[0], H, float(eps), stream_ptr())


def act(x: torch.Tensor, kind: int) -> torch.Tensor:
    """In place non-gated activation: 0 SiLU, 1 GELU-tanh, 3 GELU (erf), 4 ReLU^2."""
    if not _gpu(x):
        return ref.act(x, kind)
    assert x.is_contiguous() and x.dtype == torch.bfloat16
    call("ome_act", x.data_ptr(), x.numel(), int(kind), stream_ptr())
    return x


_act_inplace = act   # for callers whose ``act`` argument shadows the op


def ssm_conv1d(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None, state: torch.Tensor, cu, slot, reset,
               out: torch.Tensor | None = None) -> torch.Tensor:
    """Mamba causal depthwise conv1d + SiLU over varlen sequences (rows ``cu[s]:cu[s+1]``), continuing
    from and updating ``state`` [slots, C, K-1]; ``reset[s]`` = 1 starts sequence ``s`` from zeros."""
    T, C = x.shape
    out = torch.empty(T, C, dtype=x.dtype, device=x.device) if out is None else out
    if not _gpu(x):
        return ref.ssm_conv1d(x, w, bias, state, cu, slot, reset, out)
    assert x.stride(1) == 1 and out.stride(1) == 1 and w.is_contiguous() and state.is_contiguous()
    call("ome_ssm_conv1d", x.data_ptr(), x.stride(0), w.data_ptr(), ptr(bias), out.data_ptr(), out.stride(0),
         state.data_ptr(), _i32(cu).data_ptr(), _i32(slot).data_ptr(), _i32(reset).data_ptr(), slot.shape[0], C,
         w.shape[1], stream_ptr())
    return out


def dyn_conv1d(x: torch.Tensor, kern: torch.Tensor, state: torch.Tensor, cu, slot, reset, cpk: int = 1,
               out: torch.Tensor | None = None) -> torch.Tensor:
    """Causal depthwise conv + SiLU with per-row taps (Jet-Nemotron's dynamic convolution):
    x [T, C], kern [T, (C / cpk) * K] (row r's taps; ``cpk`` channels share one kernel), state
    [slots, C, K-1] continued / updated per sequence as in :func:`ssm_conv1d`."""
    T, C = x.shape
    K = state.shape[-1] + 1
    out = torch.empty(T, C, dtype=x.dtype, device=x.device) if out is None else out
    if not _gpu(x):
        return ref.dyn_conv1d(x, kern, state, cu, slot, reset, cpk, out)
    assert x.stride(1) == 1 and out.stride(1) == 1 and kern.stride(1) == 1 and state.is_contiguous()
    assert kern.shape[1] == (C // cpk) * K and C % cpk == 0
    call("ome_dyn_conv1d", x.data_ptr(), x.stride(0), kern.data_ptr(), kern.stride(0), cpk, out.data_ptr(),
         out.stride(0), state.data_ptr(), _i32(cu).data_ptr(), _i32(slot).data_ptr(), _i32(reset).data_ptr(),
         slot.shape[0], C, K, stream_ptr())
    return out


def ssm_scan(x, dt, B, C, A, D, dt_bias, dt_min: float, state, cu, slot, reset, H: int, P: int, N: int, G: int,
             out: torch.Tensor | None = None) -> torch.Tensor:
    """Mamba-2 selective scan, recurrent over each sequence's rows: x [T, H*P], dt [T, H], B/C
    [T, G*N] (row-strided views are fine), A/D/dt_bias fp32 [H], state fp32 [slots, H, P, N]."""
    T = x.shape[0]
    out = torch.empty(T, H * P, dtype=x.dtype, device=x.device) if out is None else out
    if not _gpu(x):
        return ref.ssm_scan(x, dt, B, C, A, D, dt_bias, dt_min, state, cu, slot, reset, H, P, N, G, out)
    assert B.stride(0) == C.stride(0) and B.stride(1) == 1 and x.stride(1) == 1 and dt.stride(1) == 1
    call("ome_ssm_scan", x.data_ptr(), x.stride(0), dt.data_ptr(), dt.stride(0), B.data_ptr(), C.data_ptr(),
         B.stride(0), A.data_ptr(), D.data_ptr(), dt_bias.data_ptr(), float(dt_min), state.data_ptr(),
         out.data_ptr(), out.stride(0), _i32(cu).data_ptr(), _i32(slot).data_ptr(), _i32(reset).data_ptr(),
         slot.shape[0], H, P, N, G, stream_ptr())
    return out


def gdn_scan(q, k, v, a, b, A_log, dt_bias, state, cu, slot, reset, Hv: int, Hk: int,
             out: torch.Tensor | None = None, v1: bool = False) -> torch.Tensor:
    """Gated DeltaNet recurrence (Qwen3-Next), per sequence rows ``cu[s]:cu[s+1]``: q / k [T, Hk*dk]
    and v [T, Hv*dv] are row-strided views of one buffer, a / b [T, Hv] views of another, A_log /
    dt_bias fp32 [Hv], state fp32 [slots, Hv, dv, dk] (S transposed: columns contiguous).  q / k
    are L2-normalised in the kernel (prep pass + DPP-row scan; ``v1`` selects the
    one-lane-per-column kernel)."""
    T = q.shape[0]
    dv, dk = state.shape[2], state.shape[3]
    out = torch.empty(T, Hv * dv, dtype=v.dtype, device=v.device) if out is None else out
    if not _gpu(q):
        return ref.gdn_scan(q, k, v, a, b, A_log, dt_bias, state, cu, slot, reset, Hv, Hk, out)
    assert q.stride(0) == k.stride(0) == v.stride(0) and a.stride(0) == b.stride(0)
    assert q.stride(1) == k.stride(1) == v.stride(1) == a.stride(1) == 1 and out.stride(1) == 1
    assert state.is_contiguous() and state.dtype == torch.float32 and q.dtype == torch.bfloat16
    ws = None if v1 else torch.empty(T * (2 * Hk * dk + Hk + 2 * Hv), dtype=torch.float32, device=q.device)
    call("ome_gdn_scan", q.data_ptr(), k.data_ptr(), v.data_ptr(), q.stride(0), a.data_ptr(), b.data_ptr(),
         a.stride(0), A_log.data_ptr(), dt_bias.data_ptr(), state.data_ptr(), out.data_ptr(), out.stride(0),
         _i32(cu).data_ptr(), _i32(slot).data_ptr(), _i32(reset).data_ptr(), slot.shape[0], T, Hv, Hk, dk, dv,
         ptr(ws), stream_ptr())
    return out


def gated_rmsnorm(y: torch.Tensor, z: torch.Tensor, w: torch.Tensor, group: int, eps: float,
                  norm_first: bool = False) -> torch.Tensor:
    """w * groupRMSNorm(y * silu(z)) (Mamba-2 output norm, groups of ``group`` channels);
    ``norm_first``: w[:group] * groupRMSNorm(y) * silu(z) (Qwen3-Next, ``w`` shared by the groups)."""
    if not _gpu(y):
        return ref.gated_rmsnorm(y, z, w, group, eps, norm_first)
    T, I = y.shape
    out = torch.empty(T, I, dtype=y.dtype, device=y.device)
    call("ome_gated_rmsnorm", y.data_ptr(), y.stride(0), z.data_ptr(), z.stride(0), w.data_ptr(), out.data_ptr(),
         out.stride(0), T, I, group, float(eps), int(norm_first), stream_ptr())
    return out


#: paged KV-cache element formats understood by the kernels (csrc/kernels/common.h KVFmt)
KV_FORMATS = {torch.bfloat16: 0, torch.float8_e4m3fn: 1, torch.float8_e5m2: 2}


def kv_format(cache: torch.Tensor) -> int:
    f = KV_FORMATS.get(cache.dtype)
    if f is None:
        raise TypeError(f"unsupported KV-cache dtype {cache.dtype} (bf16 / float8_e4m3fn / float8_e5m2)")
    return f


def rope_qkv_cache(qkv, positions, cos_sin, rot_dim, q_out, k_cache, v_cache, slots, Hq, Hkv, D, apply_rope=True,
                   q_norm_w=None, k_norm_w=None, qk_eps=1e-6, k_scale: float = 1.0, v_scale: float = 1.0) -> None:
    """``k_scale`` / ``v_scale``: dequantisation scales of an fp8 cache (entries hold x / scale)."""
    P = k_cache.shape[2]
    if not _gpu(qkv):
        return ref.rope_qkv_cache(qkv, positions, cos_sin, rot_dim, q_out, k_cache, v_cache, slots, Hq, Hkv, D, P,
                                  apply_rope, q_norm_w, k_norm_w, qk_eps, k_scale, v_scale)
    call("ome_rope_qkv_cache", qkv.data_ptr(), qkv.stride(0), _i32(positions).data_ptr(), cos_sin.data_ptr(),
         rot_dim, q_out.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(), _i32(slots).data_ptr(), qkv.shape[0], Hq,
         Hkv, D, P, int(apply_rope), ptr(q_norm_w), ptr(k_norm_w), float(qk_eps), kv_format(k_cache),
         float(k_scale), float(v_scale), stream_ptr())


def kv_cache_write(k, v, k_cache, v_cache, slots, k_scale: float = 1.0, v_scale: float = 1.0) -> None:
    P = k_cache.shape[2]
    if not _gpu(k):
        return ref.kv_cache_write(k, v, k_cache, v_cache, slots, P, k_scale, v_scale)
    T, Hkv, D = k.shape
    assert k.stride() == v.stride()
    call("ome_kv_cache_write", k.data_ptr(), v.data_ptr(), k.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
         _i32(slots).data_ptr(), T, Hkv, D, P, kv_format(k_cache), float(k_scale), float(v_scale), stream_ptr())


def act_and_mul(x: torch.Tensor, act: int = 0, out: torch.Tensor | None = None,
                interleaved: bool = False) -> torch.Tensor:
    """act 0 = SiLU (SwiGLU), 1 = GELU-tanh (GeGLU), 2 = GPT-OSS clamped SwiGLU, 3 = Phi-3-small
    GeGELU (quick-GELU gate, limit 20, ``up + 1``).  x [.., 2I] -> [.., I].  ``interleaved``:
    gate / up columns alternate in 16-column blocks (:func:`interleave_gate_up` weights)."""
    if not _gpu(x):
        if interleaved:
            g, u = deinterleave_gate_up(x.reshape(-1, x.shape[-1]))
            x = torch.cat([g, u], -1).view(*x.shape)
        return ref.act_and_mul(x, act)
    I = x.shape[-1] // 2
    rows = x.numel() // x.shape[-1]
    out = torch.empty(*x.shape[:-1], I, dtype=x.dtype, device=x.device) if out is None else out
    call("ome_act_and_mul", x.data_ptr(), out.data_ptr(), rows, I, act | (16 if interleaved else 0), stream_ptr())
    return out


def embedding(ids: torch.Tensor, table: torch.Tensor, vocab_start: int = 0, vocab_end: int | None = None,
              out: torch.Tensor | None = None) -> torch.Tensor:
    vocab_end = table.shape[0] + vocab_start if vocab_end is None else vocab_end
    if not _gpu(ids):
        return ref.embedding(ids, table, vocab_start, vocab_end)
    T, H = ids.shape[0], table.shape[1]
    out = torch.empty(T, H, dtype=table.dtype, device=table.device) if out is None else out
    call("ome_embedding", _i32(ids).data_ptr(), table.data_ptr(), out.data_ptr(), T, H, vocab_start, vocab_end,
         stream_ptr())
    return out


def fill_pending(ids: torch.Tensor, src: torch.Tensor, prev: torch.Tensor) -> None:
    """ids[i] = prev[src[i]] where src[i] >= 0 (int32, in place) — overlapped scheduling."""
    n = ids.shape[0]
    if n == 0:
        return
    if not _gpu(ids):
        m = src >= 0
        ids[m] = prev[src[m].long()].to(ids.dtype)
        return
    assert ids.dtype == src.dtype == prev.dtype == torch.int32
    call("ome_fill_pending", ids.data_ptr(), src.data_ptr(), prev.data_ptr(), n, stream_ptr())


def apply_penalties(logits, counts, slot, rep, freq, pres) -> None:
    """Repetition / frequency / presence penalties on logits [B, V] in place (neutral rows skip)."""
    if not _gpu(logits):
        return ref.apply_penalties(logits, counts, slot, rep, freq, pres)
    B, V = logits.shape
    call("ome_apply_penalties", logits.data_ptr(), int(logits.dtype == torch.bfloat16), logits.stride(0), B, V,
         counts.data_ptr(), counts.stride(0), _i32(slot).data_ptr(), rep.data_ptr(), freq.data_ptr(), pres.data_ptr(),
         stream_ptr())


def update_counts(counts, slot, ids, rep, freq, pres) -> None:
    if not _gpu(counts):
        return ref.update_counts(counts, slot, ids, rep, freq, pres)
    call("ome_update_counts", counts.data_ptr(), counts.stride(0), _i32(slot).data_ptr(), _i32(ids).data_ptr(),
         rep.data_ptr(), freq.data_ptr(), pres.data_ptr(), ids.shape[0], stream_ptr())


def fp8_quant(x: torch.Tensor, group: int = 0):
    """Dynamic activation quantisation to OCP e4m3: x [M, K] bf16 -> (q [M, K], scale f32 [M, KB]).
    ``group`` 0 = one scale per row, 128 = one per 128-wide K group (block-scaled checkpoints)."""
    if not _gpu(x):
        return ref.fp8_quant(x, group)
    M, K = x.shape
    assert x.dtype == torch.bfloat16 and x.stride(1) == 1
    q = torch.empty(M, K, dtype=torch.float8_e4m3fn, device=x.device)
    s = torch.empty(M, K // group if group else 1, dtype=torch.float32, device=x.device)
    call("ome_fp8_quant", x.data_ptr(), x.stride(0), M, K, q.data_ptr(), s.data_ptr(), group, stream_ptr())
    return q, s


def fp8_gemm(qa, sa, qw, sw, block: int = 0, bias=None, out: torch.Tensor | None = None) -> torch.Tensor:
    """out[M, N] bf16 = dequant(qa) . dequant(qw)^T (+ bias); qw [N, K] e4m3 with per-channel (block=0,
    sw [N]) or 128x128 block scales (block=128, sw [N/128, K/128])."""
    if not _gpu(qa):
        r = ref.fp8_gemm(qa, sa, qw, sw, block, bias)
        if out is not None:
            out.copy_(r)
            return out
        return r
    M, K = qa.shape
    N = qw.shape[0]
    assert qw.shape[1] == K and qa.is_contiguous() and qw.is_contiguous()
    if out is None:
        out = torch.empty(M, N, dtype=torch.bfloat16, device=qa.device)
    if M <= FP8_SK_MAX_ROWS and gemm_sk_fp8_ok(M, N, K, 128) and _sk_fp8_operands_ok(sa, sw, qw):
        # decode rows: stream-K fp8 (csrc/kernels/gemm_sk.hip, Q = 1 / 2) -- every CU busy at any M
        return gemm_sk_fp8(qa, sa, qw, sw, block, bias, out)
    if N % 256 == 0 and K % 128 == 0 and M >= FP8_MX_MIN_ROWS and -(-M // 256) * (N // 256) >= FP8_MX_MIN_TILES:
        # 256 x 256 MX-scaled MFMA tile (csrc/kernels/gemm.hip): twice the bf16 MFMA rate
        call("ome_fp8_gemm_mx", qa.data_ptr(), qa.stride(0), sa.data_ptr(), qw.data_ptr(), qw.stride(0),
             sw.data_ptr(), M, N, K, block, out.data_ptr(), out.stride(0), ptr(bias), stream_ptr())
        return out
    call("ome_fp8_gemm", qa.data_ptr(), qa.stride(0), sa.data_ptr(), qw.data_ptr(), sw.data_ptr(), M, N, K, block,
         out.data_ptr(), out.stride(0), ptr(bias), stream_ptr())
    return out


# rows up to which the dense fp8 GEMM runs on the stream-K kernel (128 x 128 tiles)
FP8_SK_MAX_ROWS = int(os.environ.get("OME_FP8_SK_MAX_ROWS", "512"))
# rows from which the dense fp8 GEMM uses the 256 x 256 MX tile (smaller M: the 64 x 64 kernel)
FP8_MX_MIN_ROWS = int(os.environ.get("OME_FP8_MX_MIN_ROWS", "65"))
# ...and from this many 256 x 256 output tiles (profiles/r03_fp8_gemm_bench.txt: below ~128 tiles
# the grid under-fills the 256 CUs and the 64 x 64 kernel is the better choice)
FP8_MX_MIN_TILES = int(os.environ.get("OME_FP8_MX_MIN_TILES", "112"))


_w8_ws: dict = {}   # W8A16 split-K partial tiles + tile counters per (device, stream)


def w8a16_ok(x: torch.Tensor, qw: torch.Tensor, sw: torch.Tensor, block: int = 0) -> bool:
    """Shape / operand conditions of ``ome_w8a16_gemm`` (csrc/kernels/w8a16.hip)."""
    if x.dim() != 2 or x.dtype != torch.bfloat16 or qw.dtype != torch.float8_e4m3fn:
        return False
    M, K = x.shape
    N = qw.shape[0]
    if not 0 < M <= 256 or block not in (0, 128) or (block and K % 128) or qw.shape[1] != K:
        return False
    if x.stride(1) != 1 or x.stride(0) % 8 or x.data_ptr() % 16 or qw.stride(1) != 1 or qw.stride(0) % 16 or \
            qw.data_ptr() % 16 or sw.dtype != torch.float32 or not sw.is_contiguous():
        return False
    return K % 16 == 0 if M <= 8 else (N % 64 == 0 and K % 64 == 0)


_W8_TABLE: dict | None = None
_W8_TABLE_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_tuned",
                              "w8a16_gfx950.json")
# rows up to which W8A16 serves fp8 projections of unmeasured shapes (every measured shape wins at
# M <= 2: the GEMV streams the fp8 weight at 2.5-4.2 TB/s, W8A8 pays an activation-quant launch)
W8A16_DEFAULT_ROWS = int(os.environ.get("OME_W8A16_ROWS", "2"))


def _w8_table() -> dict:
    global _W8_TABLE
    if _W8_TABLE is None:
        import json

        try:
            with open(os.environ.get("OME_W8A16_TABLE", _W8_TABLE_PATH)) as f:
                raw = json.load(f)
            _W8_TABLE = {k: sorted((int(m), v) for m, v in d.items()) for k, d in raw.get("shapes", {}).items()}
        except (OSError, ValueError):
            _W8_TABLE = {}
    return _W8_TABLE


def w8a16_plan(M: int, N: int, K: int, block: int) -> int | None:
    """Split-K factor when the W8A16 kernel was measured faster than W8A8 for this fp8 weight
    shape at the nearest measured row count (``ome_amd/_tuned/w8a16_gfx950.json``, written from
    ``scripts/w8a16_bench.py``), else None.  Unmeasured shapes: W8A16 at M <= W8A16_DEFAULT_ROWS."""
    if os.environ.get("OME_W8A16", "1") == "0" or M > 256:
        return None
    rows = _w8_table().get(f"{N},{K},{block}")
    if not rows:
        return 1 if M <= W8A16_DEFAULT_ROWS else None
    m_near, e = min(rows, key=lambda r: abs(r[0] - M) / max(r[0], M))
    if max(m_near, M) > 1.34 * min(m_near, M) or (m_near <= 8) != (M <= 8):
        return None
    return int(e["splits"]) if e["us"] < 0.97 * e["w8a8_us"] else None


def w8a16_mgemv_splits(M: int, N: int, K: int, target_wg: int | None = None) -> list[int]:
    """Valid K-split counts of the MFMA GEMV (``ome_w8a16_mgemv``) for this shape, the default
    (about ``target_wg`` workgroups, 2 per CU) first: each split is 256 / 512 / 1024 deep and its
    activation slice fits 64 KiB of LDS.  [] when the shape is not supported."""
    # M <= 32 only: at 64 rows the activation slice limits a split to 256 deep and the slab
    # reduction outgrows the weight stream (profiles/r06_w8a16_bench.txt, v5) -- the skinny tile wins
    if not 8 < M <= 32 or K % 256 or N % 16:
        return []
    mp = 16 if M <= 16 else 32
    tiles = -(-N // 256)
    # the kernel is instantiated for K slices of 256 / 512 / 1024 (a compile-time K loop)
    ok = [K // ks for ks in (256, 512, 1024) if K % ks == 0 and mp * (2 * ks + 16) <= 65536]
    tgt = target_wg or int(os.environ.get("OME_W8_MGEMV_WG", "512"))
    return sorted(ok, key=lambda d: (abs(tiles * d - tgt), d))


def w8a16_gemm(x: torch.Tensor, qw: torch.Tensor, sw: torch.Tensor, block: int = 0, bias=None,
               out: torch.Tensor | None = None, splits: int | None = None) -> torch.Tensor:
    """out[M, N] bf16 = x[M, K] bf16 . dequant(qw)^T (+ bias) for decode rows (M <= 256): the fp8
    weight is streamed and widened in registers, the activation stays bf16 (no quant pass).
    qw [N, K] e4m3; sw [N] per channel (block 0) or [ceil(N/128), K/128] (block 128)."""
    M, K = x.shape
    N = qw.shape[0]
    if not _gpu(x):
        w = ref.fp8_dequant_weight(qw, sw, block).float()
        r = torch.nn.functional.linear(x.float(), w, None if bias is None else bias.float()).to(torch.bfloat16)
        if out is not None:
            out.copy_(r)
            return out
        return r
    assert w8a16_ok(x, qw, sw, block), "w8a16_gemm: unsupported operands"
    out = torch.empty(M, N, dtype=torch.bfloat16, device=x.device) if out is None else out
    mg = w8a16_mgemv_splits(M, N, K)
    if mg and out.stride(1) == 1 and out.stride(0) % 4 == 0 and os.environ.get("OME_W8_MGEMV", "1") == "1":
        # 8 < M <= 64: the MFMA GEMV (weight straight to registers, activation slice in LDS)
        s = splits if splits in mg else mg[0]
        ws = cnt = None
        mp = 16 if M <= 16 else 32 if M <= 32 else 64
        if s > 1:
            key = _ws_key(x.device)
            st = _w8_ws.get(key)
            if st is None:
                st = _w8_ws[key] = _SkinnyWorkspace(x.device)
            ws, cnt = st.get(-(-N // 256) * s * 256 * 64), st.cnt   # sized for MP = 64: never regrown per M
            assert -(-N // 256) <= cnt.numel()
        call("ome_w8a16_mgemv", x.data_ptr(), x.stride(0), qw.data_ptr(), qw.stride(0), sw.data_ptr(), block,
             ptr(bias), out.data_ptr(), out.stride(0), M, N, K, K // s, ptr(ws), ptr(cnt), stream_ptr())
        return out
    s = 1 if M <= 8 else (splits or skinny_splits(M, N, K))
    ws = cnt = None
    if s > 1:
        key = _ws_key(x.device)
        st = _w8_ws.get(key)
        if st is None:
            st = _w8_ws[key] = _SkinnyWorkspace(x.device)
        ws, cnt = st.get((N // 64) * s * 256 * 64), st.cnt   # sized for Mp = 256: never regrown per M
        assert N // 64 <= cnt.numel()
    call("ome_w8a16_gemm", x.data_ptr(), x.stride(0), qw.data_ptr(), qw.stride(0), sw.data_ptr(), block, ptr(bias),
         out.data_ptr(), out.stride(0), M, N, K, s, ptr(ws), ptr(cnt), stream_ptr())
    return out


def fp8_linear(x: torch.Tensor, qw: torch.Tensor, sw: torch.Tensor, block: int = 0, bias=None) -> torch.Tensor:
    """W8A8 linear: dynamic per-token (or per-1x128-group) activation quant + FP8 MFMA GEMM."""
    shape = x.shape
    x2 = x.reshape(-1, shape[-1])
    qa, sa = fp8_quant(x2, block)
    y = fp8_gemm(qa, sa, qw, sw, block, bias)
    if y.dtype != x.dtype:  # CPU reference models may run in fp32
        y = y.to(x.dtype)
    return y.reshape(*shape[:-1], qw.shape[0])


def moe_route(logits: torch.Tensor, k: int, renorm: bool = True, scoring: str = "softmax",
              out_w: torch.Tensor | None = None, out_ids: torch.Tensor | None = None, bias: torch.Tensor | None = None,
              n_group: int = 1, topk_group: int = 1, group_mode: int = 0):
    """Router: logits [T, E] -> (weights f32 [T, k], expert ids int32 [T, k]).  ``group_mode`` 1/2 =
    DeepSeek-V2 group_limited_greedy / DeepSeek-V3 noaux_tc (with ``bias``)."""
    if not _gpu(logits):
        w, ids = ref.moe_route(logits, k, renorm, scoring, bias, n_group, topk_group, group_mode)
        if out_w is not None:
            out_w.copy_(w)
            out_ids.copy_(ids)
            return out_w, out_ids
        return w, ids
    T, E = logits.shape
    out_w = torch.empty(T, k, dtype=torch.float32, device=logits.device) if out_w is None else out_w
    out_ids = torch.empty(T, k, dtype=torch.int32, device=logits.device) if out_ids is None else out_ids
    if bias is not None:
        assert bias.dtype == torch.float32 and bias.is_contiguous()
    call("ome_moe_route", logits.data_ptr(), int(logits.dtype == torch.bfloat16), logits.stride(0), T, E, k,
         int(renorm), 0 if scoring == "softmax" else 1, ptr(bias), n_group, topk_group, group_mode,
         out_w.data_ptr(), out_ids.data_ptr(), stream_ptr())
    return out_w, out_ids


def moe_tile_m(rows: int, E: int, N: int) -> int:
    """Row tile of the grouped GEMM (static in the shapes, so graph-safe): 128x128 when experts
    get many rows (prefill: MFMA-bound), or in the decode regime when the wide-N GEMM still gives
    >= 1024 workgroups of 128 (more W bytes per barrier); else the 64x64 weight-streaming tile.
    Measured on gfx950: ``scripts/moe_gemm_bench.py`` (profiles/r01_moe_gemm_bench.txt).
    ``OME_MOE_TILE`` overrides."""
    env = os.environ.get("OME_MOE_TILE")
    if env:
        return int(env)
    avg = rows / max(1, E)
    if avg >= 128 or (avg >= 48 and -(-N // 128) * E >= 1024):
        return 128
    return 64


def moe_fp8_tile_m(rows: int, E: int) -> int:
    """Row tile of the fp8 grouped GEMM: 64 (64x128 tiles, 3-stage LDS ring) at every size, or
    128 (128x128, 2 stages) via ``OME_MOE_FP8_TILE=128``.  Measured (``scripts/fp8_moe_tile_bench.py``,
    profiles/r05_fp8_moe_tiles.md): the 64-row tile wins 1.25-1.5x at decode and ties or wins at
    prefill (256 rows / expert: 6.90 vs 6.97 ms)."""
    env = os.environ.get("OME_MOE_FP8_TILE")
    if env:
        return int(env)
    return 64


def fused_moe(x: torch.Tensor, topk_w: torch.Tensor, topk_ids: torch.Tensor, w13: torch.Tensor, w2: torch.Tensor,
              act: int = 0, scale: float = 1.0, b13: torch.Tensor | None = None,
              b2: torch.Tensor | None = None, gated: bool = True, add: torch.Tensor | None = None) -> torch.Tensor:
    """Sparse MoE MLP on MFMA: align (counting sort by expert, on device) -> grouped GEMM gate_up
    with gathered A rows -> SiLU*mul -> grouped GEMM down -> weighted combine.  Shapes are
    static given T (graph-capturable); per-expert counts never leave the GPU.  ``gated=False``:
    w13 holds only up rows [E, I, H] and the activation is applied in place (NemotronH ReLU^2).
    ``add`` [T, H] (an always-on shared expert's output): returned as add + MoE, summed inside
    the combine kernel (written into ``add`` itself)."""
    if hasattr(w13, "scale") and hasattr(w13, "q"):   # Fp8Experts (models/quant.py)
        return fused_moe_fp8(x, topk_w, topk_ids, w13, w2, act, scale, add=add)
    if not _gpu(x):
        y = ref.fused_moe(x, topk_w, topk_ids, w13, w2, act, scale, b13, b2, gated)
        return y if add is None else add.copy_((add.float() + y.float()).to(add.dtype))
    T, H = x.shape
    E, I2, _ = w13.shape
    I = I2 // 2 if gated else I2
    k = topk_ids.shape[1]
    n = T * k
    dev = x.device
    offsets = torch.empty(E + 1, dtype=torch.int32, device=dev)
    sorted_ids = torch.empty(n, dtype=torch.int32, device=dev)
    inv = torch.empty(n, dtype=torch.int32, device=dev)
    call("ome_moe_align", topk_ids.data_ptr(), n, E, offsets.data_ptr(), sorted_ids.data_ptr(), inv.data_ptr(),
         stream_ptr())
    tm = moe_tile_m(n, E, I2)
    gu = torch.empty(n, I2, dtype=x.dtype, device=dev)
    call("ome_moe_gemm", x.data_ptr(), x.stride(0), sorted_ids.data_ptr(), k, w13.data_ptr(), offsets.data_ptr(),
         E, I2, H, -(-n // tm) + E, gu.data_ptr(), gu.stride(0), ptr(b13), tm, stream_ptr())
    h = act_and_mul(gu, act) if gated else _act_inplace(gu, act)
    y = torch.empty(n, H, dtype=x.dtype, device=dev)
    tm = moe_tile_m(n, E, H)
    call("ome_moe_gemm", h.data_ptr(), h.stride(0), None, 0, w2.data_ptr(), offsets.data_ptr(), E, H, I,
         -(-n // tm) + E, y.data_ptr(), y.stride(0), ptr(b2), tm, stream_ptr())
    return _combine(y, topk_w, inv, T, k, H, scale, add)


def _combine(y, topk_w, inv, T, k, H, scale, add):
    if add is not None:
        assert add.shape == (T, H) and add.is_contiguous() and add.dtype == y.dtype
    out = add if add is not None else torch.empty(T, H, dtype=y.dtype, device=y.device)
    call("ome_moe_combine_add", y.data_ptr(), topk_w.data_ptr(), inv.data_ptr(), T, k, H, out.data_ptr(), ptr(add),
         float(scale), stream_ptr())
    return out


def fused_moe_fp8(x: torch.Tensor, topk_w: torch.Tensor, topk_ids: torch.Tensor, w13, w2, act: int = 0,
                  scale: float = 1.0, add: torch.Tensor | None = None) -> torch.Tensor:
    """FP8 experts (``Fp8Experts``: e4m3 + 128x128 block scales): the token rows are quantised once
    (1x128 groups) and gathered by the grouped GEMM, the SiLU*mul output re-quantised for the down
    projection; both grouped GEMMs are ``ome_moe_gemm_fp8`` (experts never leave fp8)."""
    if not _gpu(x):
        y = ref.fused_moe_fp8(x, topk_w, topk_ids, w13.q, w13.scale, w2.q, w2.scale, act, scale, w13.block)
        return y if add is None else add.copy_((add.float() + y.float()).to(add.dtype))
    T, H = x.shape
    E, I2, _ = w13.q.shape
    I = I2 // 2
    k = topk_ids.shape[1]
    n = T * k
    dev = x.device
    offsets = torch.empty(E + 1, dtype=torch.int32, device=dev)
    sorted_ids = torch.empty(n, dtype=torch.int32, device=dev)
    inv = torch.empty(n, dtype=torch.int32, device=dev)
    call("ome_moe_align", topk_ids.data_ptr(), n, E, offsets.data_ptr(), sorted_ids.data_ptr(), inv.data_ptr(),
         stream_ptr())
    qx, sx = fp8_quant(x, 128)
    tm = moe_fp8_tile_m(n, E)
    tiles = -(-n // tm) + E
    gu = torch.empty(n, I2, dtype=x.dtype, device=dev)
    call("ome_moe_gemm_fp8_tile", qx.data_ptr(), qx.stride(0), sx.data_ptr(), sorted_ids.data_ptr(), k,
         w13.q.data_ptr(), w13.scale.data_ptr(), offsets.data_ptr(), E, I2, H, tiles, tm, gu.data_ptr(), gu.stride(0),
         stream_ptr())
    h = act_and_mul(gu, act)
    qh, sh = fp8_quant(h, 128)
    y = torch.empty(n, H, dtype=x.dtype, device=dev)
    call("ome_moe_gemm_fp8_tile", qh.data_ptr(), qh.stride(0), sh.data_ptr(), None, 0, w2.q.data_ptr(),
         w2.scale.data_ptr(), offsets.data_ptr(), E, H, I, tiles, tm, y.data_ptr(), y.stride(0), stream_ptr())
    return _combine(y, topk_w, inv, T, k, H, scale, add)


def moe_experts_sorted(rows: torch.Tensor, ids: torch.Tensor, w13, w2, act: int, n_experts: int):
    """Expert MLP over already-dispatched rows (expert parallelism): ``rows`` [n, H], ``ids`` [n]
    local expert per row, ``n_experts`` = a null id for empty slots (never computed).  Returns
    (y [n, H] in the grouped GEMM's sorted order, inv [n] = the sorted position of row i).
    bf16 experts or Fp8Experts; nothing leaves the device (graph-capturable)."""
    n, H = rows.shape
    dev = rows.device
    E1 = n_experts + 1
    offsets = torch.empty(E1 + 1, dtype=torch.int32, device=dev)
    sorted_ids = torch.empty(n, dtype=torch.int32, device=dev)
    inv = torch.empty(n, dtype=torch.int32, device=dev)
    call("ome_moe_align", ids.data_ptr(), n, E1, offsets.data_ptr(), sorted_ids.data_ptr(), inv.data_ptr(),
         stream_ptr())
    y = torch.empty(n, H, dtype=rows.dtype, device=dev)
    if hasattr(w13, "scale") and hasattr(w13, "q"):
        I2 = w13.q.shape[1]
        tm = moe_fp8_tile_m(n, n_experts)
        tiles = -(-n // tm) + n_experts
        qx, sx = fp8_quant(rows, 128)
        gu = torch.empty(n, I2, dtype=rows.dtype, device=dev)
        call("ome_moe_gemm_fp8_tile", qx.data_ptr(), qx.stride(0), sx.data_ptr(), sorted_ids.data_ptr(), 1,
             w13.q.data_ptr(), w13.scale.data_ptr(), offsets.data_ptr(), n_experts, I2, H, tiles, tm, gu.data_ptr(),
             gu.stride(0), stream_ptr())
        h = act_and_mul(gu, act)
        qh, sh = fp8_quant(h, 128)
        call("ome_moe_gemm_fp8_tile", qh.data_ptr(), qh.stride(0), sh.data_ptr(), None, 0, w2.q.data_ptr(),
             w2.scale.data_ptr(), offsets.data_ptr(), n_experts, H, I2 // 2, tiles, tm, y.data_ptr(), y.stride(0),
             stream_ptr())
        return y, inv
    I2 = w13.shape[1]
    tm = moe_tile_m(n, n_experts, I2)
    gu = torch.empty(n, I2, dtype=rows.dtype, device=dev)
    call("ome_moe_gemm", rows.data_ptr(), rows.stride(0), sorted_ids.data_ptr(), 1, w13.data_ptr(),
         offsets.data_ptr(), n_experts, I2, H, -(-n // tm) + n_experts, gu.data_ptr(), gu.stride(0), None, tm,
         stream_ptr())
    h = act_and_mul(gu, act)
    tm = moe_tile_m(n, n_experts, H)
    call("ome_moe_gemm", h.data_ptr(), h.stride(0), None, 0, w2.data_ptr(), offsets.data_ptr(), n_experts, H,
         I2 // 2, -(-n // tm) + n_experts, y.data_ptr(), y.stride(0), None, tm, stream_ptr())
    return y, inv


class DecodeWorkspace:
    """Split-K partial buffers for paged decode, sized once (graph-capture safe)."""

    def __init__(self, max_batch: int, Hq: int, D: int, max_context: int, part_size: int = 512, device="cuda",
                 parts: int | None = None):
        """``part_size`` > 0: fixed 128-multiple key spans; ``part_size`` == 0: every sequence is split
        into ``parts`` spans of its own length (128-key granules), so short contexts use every
        partition."""
        self.part_size = part_size
        if part_size == 0:
            assert parts and parts >= 1
            self.max_parts = parts
        else:
            self.max_parts = max(1, -(-max_context // part_size))
        self.part_o = torch.empty(max_batch * Hq * self.max_parts * D, dtype=torch.float32, device=device)
        self.part_ml = torch.empty(max_batch * Hq * self.max_parts * 2, dtype=torch.float32, device=device)


def blocksparse_pack(bs) -> int:
    """(block, local_blocks, vert_stride, head_step, head0) -> the packed int64 of the attention
    kernels (attention.hip ``set_blocksparse``); None -> 0 (dense)."""
    if bs is None:
        return 0
    block, local, vert, step, h0 = (int(v) for v in bs)
    shift = block.bit_length() - 1
    if block != 1 << shift or not 0 < shift < 16 or not 0 < local < 1 << 16 or not 0 < vert < 1 << 12 or \
            not 0 <= step < 256 or not 0 <= h0 < 4096:
        raise ValueError(f"unsupported block-sparse parameters {bs}")
    return shift | local << 4 | vert << 20 | step << 32 | h0 << 40


def paged_decode(q, k_cache, v_cache, block_tables, seq_lens, scale, ws: DecodeWorkspace | None = None,
                 window: int = -1, out=None, order: torch.Tensor | None = None, k_scale: float = 1.0,
                 v_scale: float = 1.0, softcap: float = 0.0, sinks: torch.Tensor | None = None,
                 alibi: torch.Tensor | None = None, row_lo: torch.Tensor | None = None,
                 blocksparse: tuple | None = None) -> torch.Tensor:
    """q [B, Hq, D] -> [B, Hq, D].  ``alibi``: fp32 [Hq] ALiBi slopes (logit += slope * (key - query
    position)), or None.  ``row_lo``: int32 [B], row b attends keys [row_lo[b], seq_lens[b]) only
    (Mllama cross attention over a range of a request's vision-token cache).  ``order`` (int32 [B], optional): sequence visit order for the
    workgroup dispatcher (longest first balances the tail).  The cache may be bf16 or fp8
    (``k_scale`` / ``v_scale`` dequantise it).  ``blocksparse``: (block, local_blocks, vert_stride,
    head_step, head0) block-sparse causal mask (Phi-3-small), None = dense."""
    if not _gpu(q):
        r = ref.paged_decode(q, k_cache, v_cache, block_tables, seq_lens, scale, window, k_scale, v_scale, softcap,
                             sinks, alibi, row_lo, blocksparse)
        if out is not None:
            out.copy_(r)
            return out
        return r
    B, Hq, D = q.shape
    Hkv, P = k_cache.shape[1], k_cache.shape[2]
    if ws is None:
        ws = DecodeWorkspace(B, Hq, D, block_tables.shape[1] * P, device=q.device)
    out = torch.empty_like(q) if out is None else out
    call("ome_paged_decode", q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
         _i32(block_tables).data_ptr(), block_tables.stride(0), _i32(seq_lens).data_ptr(), out.data_ptr(),
         out.stride(0), ws.part_o.data_ptr(), ws.part_ml.data_ptr(), B, Hq, Hkv, D, P, ws.part_size, ws.max_parts,
         float(scale), int(window), _i32(order).data_ptr() if order is not None else None, kv_format(k_cache),
         float(k_scale), float(v_scale), float(softcap), _sinks(sinks), _sinks(alibi),
         _i32(row_lo).data_ptr() if row_lo is not None else None, blocksparse_pack(blocksparse), stream_ptr())
    return out


def _sinks(s: torch.Tensor | None):
    """Per-head fp32 [Hq] device vector (GPT-OSS attention-sink logits, ALiBi slopes), or None."""
    if s is None:
        return None
    assert s.dtype == torch.float32 and s.is_contiguous()
    return s.data_ptr()


class MLAWorkspace:
    """Split-K partials for :func:`mla_attn` (``ws_o`` [rows, 512] f32, ``ws_ml`` [rows, 2]; rows =
    tokens x heads x partitions, bounded by ``ROWS``).

    Two kernels (``mla.hip``): the all-heads kernel (DK 576 with 64 | H: one workgroup streams a
    token's latent KV once for 64 / 128 heads, one workgroup per CU) and the 16-head kernel (MiniCPM3
    shapes, TP-sharded head counts).  Partitions lift the grid towards ~1 workgroup per CU (all-heads)
    or ~1024 workgroups (16-head), and never beyond what the f32 partials' HBM round trip repays:
    large decode batches (T x H / 128 >= 256) run unsplit."""

    TARGET_WGS = 1024
    TARGET_WGS_ALL = 256
    MAX_PARTS = 16
    MAX_PARTS_ALL = 64
    ROWS = 1 << 15

    def __init__(self, device="cuda"):
        self.ws_o = torch.empty(self.ROWS * 512, dtype=torch.float32, device=device)
        self.ws_ml = torch.empty(self.ROWS * 2, dtype=torch.float32, device=device)

    @staticmethod
    def all_heads(H: int, DK: int = 576, T: int = 1 << 30) -> bool:
        """Mirror of mla.hip's kernel choice (same env knobs): all-heads only above
        ``OME_MLA_ALL_MIN_T`` (default 2) tokens -- T = 1 / 2 keep the 16-head kernel."""
        return (DK == 576 and H % 64 == 0 and os.environ.get("OME_MLA_ALL", "1") != "0"
                and T > int(os.environ.get("OME_MLA_ALL_MIN_T", "2")))

    @classmethod
    def parts(cls, T: int, H: int, DK: int = 576) -> int:
        if cls.all_heads(H, DK, T):
            wgs = T * (H // (128 if H % 128 == 0 else 64))
            p = max(1, min(cls.MAX_PARTS_ALL, cls.TARGET_WGS_ALL // max(wgs, 1)))
        else:
            wgs = T * -(-H // 16)
            p = 1 if wgs >= cls.TARGET_WGS else max(1, min(cls.MAX_PARTS, cls.TARGET_WGS // max(wgs, 1)))
        return max(1, min(p, cls.ROWS // max(T * H, 1)))


def mla_attn(q, cache, block_tables, tok_row, kv_lens, scale: float, ws: MLAWorkspace | None = None,
             out: torch.Tensor | None = None, dv: int = 512) -> torch.Tensor:
    """Absorbed multi-head latent attention (MLA) over the paged latent cache: q [T, H, DK]
    (latent-projected nope part | roped pe part), cache [pages, 16, DK] -> out [T, H, dv] (values
    = the first dv latent dims); (DK, dv) = (576, 512) DeepSeek / Kimi-K2 or (288, 256) MiniCPM3.
    Token t sees keys [0, kv_lens[t]) of block-table row tok_row[t]."""
    if not _gpu(q):
        r = ref.mla_attn(q, cache, block_tables, tok_row, kv_lens, scale, dv)
        if out is not None:
            out.copy_(r)
            return out
        return r
    T, H, DK = q.shape
    assert (DK, dv) in ((576, 512), (288, 256)), (DK, dv)
    assert q.stride(2) == 1 and q.stride(1) == DK and cache.shape[-1] == DK
    if out is None:
        out = torch.empty(T, H, dv, dtype=q.dtype, device=q.device)
    parts = MLAWorkspace.parts(T, H, DK)
    if parts > 1 and ws is None:
        ws = MLAWorkspace(q.device)
    call("ome_mla_attn", q.data_ptr(), q.stride(0), cache.data_ptr(), _i32(block_tables).data_ptr(),
         block_tables.stride(0), _i32(tok_row).data_ptr(), _i32(kv_lens).data_ptr(), T, H, DK, dv, float(scale),
         parts, out.data_ptr(), out.stride(0), ws.ws_o.data_ptr() if parts > 1 else None,
         ws.ws_ml.data_ptr() if parts > 1 else None, stream_ptr())
    return out


class _SkinnyWorkspace:
    """Split-K partial tiles + per-tile counters of :func:`skinny_gemm` (one per device; launches on
    one stream are ordered, so calls share it).  The counters are re-armed by the kernel."""

    def __init__(self, device):
        self.ws = torch.empty(0, dtype=torch.float32, device=device)
        self.cnt = torch.zeros(1 << 14, dtype=torch.int32, device=device)

    def get(self, floats: int) -> torch.Tensor:
        if self.ws.numel() < floats:
            self.ws = torch.empty(floats, dtype=torch.float32, device=self.cnt.device)
        return self.ws


_skinny_ws: dict = {}


def skinny_splits(M: int, N: int, K: int) -> int:
    """Split-K factor: 1 when the weight has >= 256 64-row tiles, else enough to reach ~2 workgroups
    per CU (capped; every split streams >= 512 K)."""
    env = os.environ.get("OME_SKINNY_SPLITS")
    tiles = N // 64
    if env:
        return max(1, min(int(env), K // 64))
    if tiles >= 256:
        return 1
    return max(1, min(-(-512 // tiles), 8, K // 512))


def skinny_gemm(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None,
                out: torch.Tensor | None = None, splits: int | None = None) -> torch.Tensor:
    """out[M, N] = x[M, K] . w[N, K]^T (+ bias) for decode-shaped M <= 256 (``skinny_gemm.hip``:
    every weight byte streamed once, split-K when N has few 64-row tiles)."""
    M, K = x.shape
    N = w.shape[0]
    if not _gpu(x):
        r = torch.nn.functional.linear(x.float(), w.float(), None if bias is None else bias.float()).to(x.dtype)
        if out is not None:
            out.copy_(r)
            return out
        return r
    assert x.stride(1) == 1 and w.is_contiguous() and x.dtype == w.dtype == torch.bfloat16
    out = torch.empty(M, N, dtype=x.dtype, device=x.device) if out is None else out
    s = splits or skinny_splits(M, N, K)
    ws = cnt = None
    if s > 1:
        st = _skinny_ws.get(x.device)
        if st is None:
            st = _skinny_ws[x.device] = _SkinnyWorkspace(x.device)
        mp = 64 if M <= 64 else 128 if M <= 128 else 256
        ws, cnt = st.get((N // 64) * s * mp * 64), st.cnt
        assert N // 64 <= cnt.numel()
    call("ome_skinny_gemm", x.data_ptr(), x.stride(0), w.data_ptr(), ptr(bias), out.data_ptr(), out.stride(0), M, N,
         K, s, ptr(ws), ptr(cnt), stream_ptr())
    return out


_stream_ws: dict = {}    # split-K partial sums per (device, stream): TBO halves never alias
_stream_cnt: dict = {}   # tile arrival counters of the single-launch split-K, per (device, stream)


def _ws_key(device) -> tuple:
    device = torch.device(device)
    return (device.index, torch.cuda.current_stream(device).cuda_stream)


def stream_gemm_plan(M: int, N: int, K: int) -> tuple[int, int]:
    """(nf, splits) of :func:`stream_gemm`: 256-row weight tiles (nf = 2) only at M <= 128 (VGPR
    budget), and split-K up to ~256 workgroups when the weight has few tiles (every split keeps
    >= 4 K steps).  ``OME_STREAM_SPLITS`` overrides the split count."""
    nf = 2 if M <= 128 and N % 256 == 0 and N // 256 >= 256 else 1
    tiles = N // (128 * nf)
    env = os.environ.get("OME_STREAM_SPLITS")
    if env:
        return nf, max(1, min(int(env), K // 64))
    if tiles >= 192:
        return nf, 1
    return nf, max(1, min(-(-256 // tiles), K // 256))


def stream_gemm_ok(M: int, N: int, K: int) -> bool:
    return 1 <= M <= 256 and N % 128 == 0 and K % 64 == 0


_stream_ws_retired: list = []


def stream_gemm_reserve(device, floats: int) -> None:
    """Pre-size the split-K workspace (call before HIP-graph capture so capture never allocates).
    Growing it later keeps the old buffer alive: graphs captured earlier replay into it."""
    key = _ws_key(device)
    ws = _stream_ws.get(key)
    if ws is None or ws.numel() < floats:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError(f"split-K workspace must be reserved before capture ({floats} floats needed)")
        if ws is not None:
            _stream_ws_retired.append(ws)
        _stream_ws[key] = torch.empty(floats, dtype=torch.float32, device=device)


def stream_gemm(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None,
                out: torch.Tensor | None = None, splits: int | None = None, nf: int | None = None) -> torch.Tensor:
    """out[M, N] = x[M, K] . w[N, K]^T (+ bias) for decode-shaped M <= 256 (``stream_gemm.hip``: the
    weight streams from HBM straight into MFMA operands, activations shared through LDS, split-K
    partials reduced by a second kernel)."""
    M, K = x.shape
    N = w.shape[0]
    if not _gpu(x):
        r = torch.nn.functional.linear(x.float(), w.float(), None if bias is None else bias.float()).to(x.dtype)
        if out is not None:
            out.copy_(r)
            return out
        return r
    assert x.stride(1) == 1 and w.is_contiguous() and x.dtype == w.dtype == torch.bfloat16
    assert stream_gemm_ok(M, N, K), (M, N, K)
    out = torch.empty(M, N, dtype=x.dtype, device=x.device) if out is None else out
    pnf, ps = stream_gemm_plan(M, N, K)
    nf, s = nf or pnf, splits or ps
    ws = cnt = None
    if s > 1:
        stream_gemm_reserve(x.device, s * M * N)
        ws = _stream_ws[_ws_key(x.device)]
        if os.environ.get("OME_STREAM_INKERNEL", "0") == "1":   # opt-in single launch: last split combines (measured slower)
            cnt = _stream_cnt.get(_ws_key(x.device))
            if cnt is None:
                cnt = _stream_cnt[_ws_key(x.device)] = torch.zeros(1 << 13, dtype=torch.int32, device=x.device)
            assert N // (128 * nf) <= cnt.numel()
    call("ome_stream_gemm", x.data_ptr(), x.stride(0), w.data_ptr(), ptr(bias), out.data_ptr(), out.stride(0), M, N,
         K, nf, s, ptr(ws), ptr(cnt), stream_ptr())
    return out


def gemv_ok(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None,
            out: torch.Tensor | None = None) -> bool:
    """gemv.hip reads x and w in 16-byte chunks: both must start on a 16-B boundary with 16-B
    row pitch; bias (if any) is a contiguous bf16 [N]; out rows are unit-stride."""
    return (isinstance(w, torch.Tensor) and x.dim() == 2 and 1 <= x.shape[0] <= 8 and x.shape[1] % 8 == 0
            and x.stride(1) == 1 and x.stride(0) % 8 == 0 and x.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and w.dim() == 2 and w.is_contiguous() and w.shape[1] == x.shape[1]
            and x.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0
            and (bias is None or (bias.dtype == torch.bfloat16 and bias.is_contiguous()
                                  and bias.numel() == w.shape[0]))
            and (out is None or (out.dtype == torch.bfloat16 and out.dim() == 2 and out.stride(1) == 1
                                 and tuple(out.shape) == (x.shape[0], w.shape[0]))))


def gemv(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None,
         out: torch.Tensor | None = None) -> torch.Tensor:
    """out[M, N] = x[M, K] . w[N, K]^T (+ bias) for M <= 8 (``gemv.hip``: a pure weight stream,
    R rows per wave, several K steps of 16-B loads in flight, no LDS)."""
    M, K = x.shape
    N = w.shape[0]
    if not _gpu(x):
        r = torch.nn.functional.linear(x.float(), w.float(), None if bias is None else bias.float()).to(x.dtype)
        if out is not None:
            out.copy_(r)
            return out
        return r
    assert gemv_ok(x, w, bias, out), (tuple(x.shape), x.stride(), w.shape)
    out = torch.empty(M, N, dtype=x.dtype, device=x.device) if out is None else out
    call("ome_gemv", x.data_ptr(), x.stride(0), w.data_ptr(), ptr(bias), out.data_ptr(), out.stride(0), M, N, K,
         stream_ptr())
    return out


def gemv_act(gu: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """out = (SiLU(gu[:, :I]) * gu[:, I:]) . w^T for M <= 8 rows: the decode down projection with
    the SwiGLU folded into the GEMV's operand load (no act_and_mul launch, no intermediate)."""
    M, I2 = gu.shape
    I = I2 // 2
    N = w.shape[0]
    if not _gpu(gu):
        return torch.nn.functional.linear(ref.act_and_mul(gu, 0).float(), w.float()).to(gu.dtype)
    assert gu.stride(1) == 1 and gu.stride(0) % 8 == 0 and w.is_contiguous() and w.shape[1] == I and I % 8 == 0
    assert gu.dtype == w.dtype == torch.bfloat16 and gu.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0
    out = torch.empty(M, N, dtype=gu.dtype, device=gu.device) if out is None else out
    call("ome_gemv_act", gu.data_ptr(), gu.stride(0), w.data_ptr(), None, out.data_ptr(), out.stride(0), M, N, I,
         stream_ptr())
    return out


# ---- decode GEMM routing: ome_stream_gemm where it measured faster than hipBLASLt --------------
# Filled during the engine's eager pre-capture pass (``decode_gemm_tuning``): every (M, N, K, bias)
# a decode bucket issues is timed once against the library GEMM and the winner recorded; graphs
# captured afterwards bake the choice in.  hipBLASLt keeps every shape it wins (at M = 256 all of
# them on an 8B model: profiles/r02_stream_gemm_bench.txt).
_gemm_route: dict = {}
_gemm_tuning = [False]
_STREAM_STATIC = os.environ.get("OME_STREAM_GEMM", "0") == "static"


class decode_gemm_tuning:
    """Context manager: record stream-vs-library choices for the GEMMs issued inside."""

    def __enter__(self):
        self.prev = _gemm_tuning[0]
        _gemm_tuning[0] = os.environ.get("OME_STREAM_GEMM", "0") == "1"
        return self

    def __exit__(self, *exc):
        _gemm_tuning[0] = self.prev
        return False


def _time_us(fn, iters: int = 20) -> float:
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1000.0 / iters


def decode_gemm_plan(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None):
    """(nf, splits) when ``stream_gemm`` is the recorded winner for this shape, else None."""
    M, K = x.shape
    N = w.shape[0]
    key = (M, N, K, bias is not None, x.device)
    if key in _gemm_route:
        return _gemm_route[key]
    if _STREAM_STATIC and 5 <= M <= 16 and K <= 4096 and stream_gemm_ok(M, N, K) and _gpu(x):
        # rule from the cold-weight microbenchmark (profiles/r02_stream_gemm_bench_cold.txt): wide
        # weights (gate_up-like) at split 4, square o-like weights at split 8, the rest on hipBLASLt
        plan = (1, 4) if N >= 16384 else (1, 8) if N <= 4096 else None
        _gemm_route[key] = plan
        return plan
    if not _gemm_tuning[0]:
        return None
    plan = None
    if (stream_gemm_ok(M, N, K) and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.stride(1) == 1
            and x.stride(0) % 8 == 0 and w.is_contiguous() and _gpu(x)):
        out = torch.empty(M, N, dtype=x.dtype, device=x.device)
        t_lib = _time_us(lambda: torch.nn.functional.linear(x, w, bias))
        nf0, s0 = stream_gemm_plan(M, N, K)
        cands = {(nf0, s0), (1, 1)}
        cands |= {(1, s) for s in (2, 4, 8) if s <= K // 256}
        if M <= 128 and N % 256 == 0:
            cands |= {(2, 1), (2, 2)}
        cands = {(nf, sp) for nf, sp in cands if sp <= K // 64 and N % (128 * nf) == 0 and (nf == 1 or M <= 128)}
        best = None
        for nf, sp in sorted(cands):
            t = _time_us(lambda: stream_gemm(x, w, bias, out=out, splits=sp, nf=nf))
            if best is None or t < best[0]:
                best = (t, nf, sp)
        if best is not None and best[0] < 0.95 * t_lib:
            plan = (best[1], best[2])
    _gemm_route[key] = plan
    return plan


def prefill_work_items(q_lens: list[int], kv_lens: list[int], tile: int = 32) -> list[tuple[int, int]]:
    """(seq, row_start) work items, heaviest (longest key range) first."""
    items = []
    for s, (ql, kl) in enumerate(zip(q_lens, kv_lens)):
        pre = kl - ql
        for r in range(0, ql, tile):
            items.append((pre + min(r + tile, ql), s, r))
    items.sort(key=lambda x: -x[0])
    return [(s, r) for _, s, r in items]


def gemm(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor | None = None, epi: int = 0, splits: int = 1,
         ws: torch.Tensor | None = None) -> torch.Tensor:
    """``csrc/kernels/gemm.hip``: out = x @ w.T (bf16, fp32 accumulate) on a 256 x 256 MFMA tile.
    ``epi=2``: w holds gate/up rows interleaved in 16-row blocks (:func:`interleave_gate_up`) and
    out = SiLU(gate) * up ([M, N/2]).  ``splits`` > 1 splits K over workgroups (fp32 slabs in
    ``ws`` + a reduce launch).  Requires N % 256 == 0, K % (64 * splits) == 0."""
    M, K = x.shape
    N = w.shape[0]
    if not _gpu(x):
        y = x.float() @ w.float().t()
        if epi == 2:
            g, u = deinterleave_gate_up(y)
            y = F.silu(g) * u
        y = y.to(x.dtype)
        if out is not None:
            out.copy_(y)
            return out
        return y
    if out is None:
        out = torch.empty(M, N // 2 if epi == 2 else N, dtype=x.dtype, device=x.device)
    if splits > 1 and ws is None:
        ws = torch.empty(splits * M * N, dtype=torch.float32, device=x.device)
    call("ome_gemm", x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), out.data_ptr(), out.stride(0), M, N, K,
         epi, splits, None if ws is None else ws.data_ptr(), stream_ptr())
    return out


def interleave_gate_up(w_gu: torch.Tensor, block: int = 16) -> torch.Tensor:
    """[2I, H] (gate rows, then up rows) -> rows in blocks of ``block`` gate / ``block`` up, the
    layout of gemm(..., epi=2)."""
    two_i, H = w_gu.shape
    i = two_i // 2
    g, u = w_gu[:i].view(i // block, block, H), w_gu[i:].view(i // block, block, H)
    return torch.stack([g, u], 1).reshape(two_i, H).contiguous()


def deinterleave_gate_up(y: torch.Tensor, block: int = 16):
    """Columns of a product with an interleaved gate/up weight -> (gate, up)."""
    M, N = y.shape
    v = y.view(M, N // (2 * block), 2, block)
    return v[:, :, 0].reshape(M, N // 2), v[:, :, 1].reshape(M, N // 2)


# ---------------------------------------------------------------------------------------------
# Stream-K MFMA GEMM (csrc/kernels/gemm_sk.hip): persistent per-XCD stream-K over bm x bn
# output tiles, fp32 partial slabs reduced in-launch by each tile's last arriver.  One workspace
# (slabs + tickets) per (device, stream): launches on one stream are ordered, so they may share
# slabs and tickets; two streams running GEMMs concurrently (a side-stream overlap, TBO halves,
# a vision tower) each get their own, so their partial sums and tickets never alias.  Graph
# replays reuse the workspace of the stream they were captured on.
_SK_MAX_WG = 256
_SK_CNT = 1 << 16
_SK_WS: dict = {}


def _sk_workspace(device: torch.device):
    key = (device.index, torch.cuda.current_stream(device).cuda_stream)
    w = _SK_WS.get(key)
    if w is None:
        ws = torch.empty(_SK_MAX_WG * 2 * 256 * 256, dtype=torch.float32, device=device)
        cnt = torch.zeros(_SK_CNT, dtype=torch.int32, device=device)   # the kernel re-arms every ticket it takes
        w = _SK_WS[key] = (ws, cnt)
    return w


def sk_workspace_bytes() -> int:
    return _SK_MAX_WG * 2 * 256 * 256 * 4 + _SK_CNT * 4


def reserve_stream_workspaces(device, streams) -> int:
    """Allocate the stream-K workspace of every stream that will run GEMMs (the current stream,
    a TBO side stream, ...) up front, i.e. before the KV cache is sized from free memory, so a
    lazily created per-stream workspace never eats into memory the KV budget already promised.
    Returns the bytes newly allocated."""
    device = torch.device(device)
    if device.type != "cuda":
        return 0
    n0 = len(_SK_WS)
    for s in streams:
        if s is None:
            _sk_workspace(device)
        else:
            with torch.cuda.stream(s):
                _sk_workspace(device)
    return (len(_SK_WS) - n0) * sk_workspace_bytes()


def gemm_sk_tiles(M: int, N: int, bn: int, bm: int = 256) -> int:
    return -(-M // bm) * (N // bn)


def gemm_sk_ok(M: int, N: int, K: int, bn: int, nwg: int, bm: int = 256) -> bool:
    """Shape / decomposition accepted by ``ome_gemm_sk`` with the shared workspace (blocks left
    without a unit simply exit)."""
    if bn not in (128, 256) or bm not in (128, 256) or N % bn or K % 64 or K <= 0 or nwg % 8 or \
            not 8 <= nwg <= _SK_MAX_WG or M <= 0:
        return False
    return gemm_sk_tiles(M, N, bn, bm) <= _SK_CNT


_SK_TABLE: dict | None = None
_SK_MODE = os.environ.get("OME_GEMM_SK", "table")   # table | 0 (hipBLASLt only)
_SK_TABLE_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_tuned",
                              "gemm_sk_gfx950.json")


def _sk_table() -> dict:
    global _SK_TABLE
    if _SK_TABLE is None:
        import json

        try:
            with open(os.environ.get("OME_GEMM_SK_TABLE", _SK_TABLE_PATH)) as f:
                raw = json.load(f)
            _SK_TABLE = {k: sorted((int(m), v) for m, v in d.items()) for k, d in raw.get("shapes", {}).items()}
        except (OSError, ValueError):
            _SK_TABLE = {}
    return _SK_TABLE


def gemm_sk_plan(M: int, N: int, K: int, epi: int = 0) -> tuple[int, int, int] | None:
    """(bn, nwg, bm) when the stream-K kernel was measured faster than hipBLASLt (gate_up: than
    hipBLASLt + act_and_mul) for this weight shape at the nearest measured row count, else None.
    Table: ``ome_amd/_tuned/gemm_sk_gfx950.json`` written by ``scripts/gemm_sk_bench.py --table``
    (cold weights, interleaved same-box timings)."""
    if _SK_MODE == "0":
        return None
    rows = _sk_table().get(f"{N},{K},{epi}")
    if not rows:
        return None
    m_near, e = min(rows, key=lambda r: abs(r[0] - M) / max(r[0], M))
    if max(m_near, M) > 1.34 * min(m_near, M):   # nothing measured close to this M
        return None
    bm = int(e.get("bm", 256))
    if e["us"] >= 0.97 * e["lib_us"] or not gemm_sk_ok(M, N, K, e["bn"], e["nwg"], bm):
        return None
    return e["bn"], e["nwg"], bm


def gemm_sk(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None, out: torch.Tensor | None = None,
            epi: int = 0, bn: int = 256, nwg: int = 256, bm: int = 256) -> torch.Tensor:
    """out = x @ w.T (+ bias) on the stream-K MFMA kernel.  ``epi=2``: w holds gate/up rows
    interleaved in 16-row blocks (:func:`interleave_gate_up`) and out = SiLU(gate) * up [M, N/2].
    ``bm`` x ``bn`` (128 | 256 each) output tile, ``nwg`` workgroups (multiple of 8; = tiles gives
    plain data-parallel tiles, 256 full stream-K)."""
    M, K = x.shape
    N = w.shape[0]
    if not _gpu(x):
        y = x.float() @ w.float().t()
        if bias is not None:
            y = y + bias.float()
        if epi == 2:
            g, u = deinterleave_gate_up(y)
            y = F.silu(g) * u
        y = y.to(x.dtype)
        if out is not None:
            out.copy_(y)
            return out
        return y
    if out is None:
        out = torch.empty(M, N // 2 if epi == 2 else N, dtype=x.dtype, device=x.device)
    ws, cnt = _sk_workspace(x.device)
    call("ome_gemm_sk", x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), ptr(bias), out.data_ptr(),
         out.stride(0), M, N, K, bm, bn, epi, nwg, ws.data_ptr(), cnt.data_ptr(), stream_ptr())
    return out


def gemm_xl_ok(M: int, N: int, K: int, bn: int = 256, nwg: int = 256) -> bool:
    """Shapes / decompositions accepted by ``ome_gemm_xl`` with the shared stream-K workspace."""
    return bn in (128, 256) and M > 0 and N % bn == 0 and K % 32 == 0 and K > 0 and nwg % 8 == 0 and \
        8 <= nwg <= _SK_MAX_WG and gemm_sk_tiles(M, N, bn, 256) <= _SK_CNT


def gemm_xl(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None, out: torch.Tensor | None = None,
            epi: int = 0, bn: int = 256, nwg: int = 256, probe: int = 0) -> torch.Tensor:
    """out = x @ w.T (+ bias) on the large-tile stream-K MFMA GEMM (csrc/kernels/gemm_xl.hip: 256 x
    ``bn`` tiles, one wave per SIMD with 128 x bn/2 accumulators of 32x32x16 MFMAs, BK = 32 LDS-DMA
    stages).  ``epi=2``: w holds gate/up rows interleaved in 16-row blocks and out = SiLU(gate) * up.
    ``probe`` 1 / 2: diagnostic skeleton builds (no DMA / no DMA and no LDS reads; wrong results)."""
    M, K = x.shape
    N = w.shape[0]
    if not _gpu(x):
        return gemm_sk(x, w, bias, out, epi)
    assert x.stride(1) == 1 and w.stride(1) == 1 and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
    if out is None:
        out = torch.empty(M, N // 2 if epi == 2 else N, dtype=x.dtype, device=x.device)
    ws, cnt = _sk_workspace(x.device)
    call("ome_gemm_xl", x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), ptr(bias), out.data_ptr(),
         out.stride(0), M, N, K, bn, epi, nwg, ws.data_ptr(), cnt.data_ptr(), probe, stream_ptr())
    return out


def gemm_pp_ok(M: int, N: int, K: int) -> bool:
    """Shapes accepted by the ping-pong 256 x 256 GEMM (csrc/kernels/gemm_pp.hip)."""
    return M > 0 and N > 0 and N % 256 == 0 and K > 0 and K % 64 == 0


def gemm_pp(x: torch.Tensor, w: torch.Tensor, bias: torch.Tensor | None = None, out: torch.Tensor | None = None,
            epi: int = 0, res: torch.Tensor | None = None) -> torch.Tensor:
    """out = x @ w.T (+ bias) on the ping-pong MFMA GEMM (256 x 256 tiles, one per workgroup).
    ``epi=1``: out = x @ w.T (+ bias) + ``res`` (may be ``out`` itself: the residual stream updated
    in place); ``epi=2``: w holds gate/up rows interleaved in 16-row blocks and out = SiLU(gate) * up."""
    M, K = x.shape
    N = w.shape[0]
    if not _gpu(x):
        y = x.float() @ w.float().t()
        if bias is not None:
            y = y + bias.float()
        if epi == 1:
            y = y + res.float()
        if epi == 2:
            g, u = deinterleave_gate_up(y)
            y = F.silu(g) * u
        y = y.to(x.dtype)
        if out is not None:
            out.copy_(y)
            return out
        return y
    assert x.stride(1) == 1 and w.stride(1) == 1 and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16
    if out is None:
        out = torch.empty(M, N // 2 if epi == 2 else N, dtype=x.dtype, device=x.device)
    call("ome_gemm_pp", x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), ptr(bias),
         ptr(res) if epi == 1 else None, res.stride(0) if epi == 1 else 0, out.data_ptr(), out.stride(0), M, N, K,
         epi, stream_ptr())
    return out


def mla_prep(a: torch.Tensor, qlr: int, lat: int, rope: int, w: torch.Tensor, eps: float, positions: torch.Tensor,
             cos_sin: torch.Tensor, slots: torch.Tensor, cache_flat: torch.Tensor, q: torch.Tensor, nope: int,
             q_full: torch.Tensor) -> None:
    """MLA pre-attention glue in one kernel (csrc/kernels/mla.hip ``ome_mla_prep``): from the fused
    q_a / kv_a projection output ``a`` [T, qlr + lat + rope] write the token's latent cache row
    ``cache_flat[slot] = [RMSNorm(c_kv) * w | RoPE(k_pe)]`` (slot < 0 -> row 0, the scratch page)
    and the roped q_pe of every head into ``q_full[:, :, lat:]`` (q [T, H, nope + rope])."""
    T, H = q.shape[0], q.shape[1]
    if not _gpu(a):
        ckv = a[:, qlr:qlr + lat + rope]
        c = ref.rmsnorm(ckv[:, :lat], w, eps)
        cs = cos_sin.index_select(0, positions.long())
        half = rope // 2

        def rot(x, cos, sin):
            x1, x2 = x[..., :half].float(), x[..., half:].float()
            return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], -1).to(x.dtype)

        k_pe = rot(ckv[:, lat:], cs[:, :half], cs[:, half:])
        cache_flat.index_copy_(0, slots.long().clamp_min(0), torch.cat([c, k_pe], -1))
        q_full[:, :, lat:] = rot(q[..., nope:], cs[:, None, :half], cs[:, None, half:])
        return
    assert a.stride(1) == 1 and q.stride(2) == 1 and q_full.stride(2) == 1 and cache_flat.is_contiguous()
    assert cos_sin.dtype == torch.float32 and cos_sin.shape[1] == rope and cos_sin.is_contiguous()
    call("ome_mla_prep", a.data_ptr(), a.stride(0), qlr, lat, rope, w.data_ptr(), float(eps), _i32(positions).data_ptr(),
         cos_sin.data_ptr(), _i32(slots).data_ptr(), cache_flat.data_ptr(), cache_flat.stride(0), q.data_ptr(),
         q.stride(0), q.stride(1), nope, H, q_full.data_ptr(), q_full.stride(0), q_full.stride(1), T, stream_ptr())


def gemm_sk_fp8_ok(M: int, N: int, K: int, bn: int = 128, nwg: int = 256) -> bool:
    return bn in (128, 256) and N % bn == 0 and K % 128 == 0 and K > 0 and nwg % 8 == 0 and \
        8 <= nwg <= _SK_MAX_WG and M > 0 and gemm_sk_tiles(M, N, bn, 128) <= _SK_CNT


def _sk_fp8_operands_ok(sa: torch.Tensor, sw: torch.Tensor, qw: torch.Tensor) -> bool:
    """Operand conditions of ``ome_gemm_sk_fp8`` beyond the shape (fp32 contiguous scales, 16-B
    aligned per-channel scales, unit-stride weight rows): callers that fail them take the other
    fp8 kernels instead of an assertion."""
    return sa.dtype == torch.float32 and sw.dtype == torch.float32 and sa.is_contiguous() and \
        sw.is_contiguous() and sw.data_ptr() % 16 == 0 and qw.stride(1) == 1 and qw.stride(0) % 16 == 0


def gemm_sk_fp8(qa: torch.Tensor, sa: torch.Tensor, qw: torch.Tensor, sw: torch.Tensor, block: int = 0,
                bias: torch.Tensor | None = None, out: torch.Tensor | None = None, epi: int = 0, bn: int = 128,
                nwg: int = 256) -> torch.Tensor:
    """W8A8 on the stream-K kernel: qa [M, K] / qw [N, K] e4m3; block 0: sa [M] (or [M, 1]) per token,
    sw [N] per channel; block 128: sa [M, K/128], sw [N/128, K/128].  128-row tiles, ``bn`` 128 | 256
    (256: per-channel only); ``epi=2`` as :func:`gemm_sk` (qw / sw rows interleaved)."""
    M, K = qa.shape
    N = qw.shape[0]
    if not _gpu(qa):
        y = ref.fp8_gemm(qa, sa, qw, sw, block, bias).float()
        if epi == 2:
            g, u = deinterleave_gate_up(y)
            y = F.silu(g) * u
        y = y.to(torch.bfloat16)
        if out is not None:
            out.copy_(y)
            return out
        return y
    assert qa.is_contiguous() and qw.stride(1) == 1 and sa.is_contiguous() and sw.is_contiguous()
    assert sa.dtype == torch.float32 and sw.dtype == torch.float32 and (block == 0 or bn == 128)
    if out is None:
        out = torch.empty(M, N // 2 if epi == 2 else N, dtype=torch.bfloat16, device=qa.device)
    ws, cnt = _sk_workspace(qa.device)
    call("ome_gemm_sk_fp8", qa.data_ptr(), qa.stride(0), sa.data_ptr(), qw.data_ptr(), qw.stride(0), sw.data_ptr(),
         block, ptr(bias), out.data_ptr(), out.stride(0), M, N, K, 128, bn, epi, nwg, ws.data_ptr(), cnt.data_ptr(),
         stream_ptr())
    return out


class PrefillPlan:
    """Work decomposition of one prefill attention call, built host-side by
    :func:`prefill_plan` and uploaded with the step's other inputs.  ``items`` is the classic
    [n, 2] (seq, row0) list; ``split`` [n4, 4] (seq, row0, chunk start, part) and ``comb``
    [nc, 4] (seq, row0, first part, parts) are the split-KV form (empty when nothing splits)."""

    __slots__ = ("items", "split", "comb", "chunk", "parts", "rows")

    def __init__(self, items, split, comb, chunk: int, parts: int, rows: int = 32):
        self.items, self.split, self.comb, self.chunk, self.parts = items, split, comb, chunk, parts
        self.rows = rows   # query rows per classic item (64: the 8-wave GQA-4 kernel)

    @property
    def shape(self):
        return self.items.shape


PREFILL_SPLIT_TARGET = int(os.environ.get("OME_PREFILL_SPLIT_ITEMS", "128"))
# query rows per classic prefill item for the GQA-4 / D=128 kernel: 32 (4 waves) or 64 (8 waves,
# every K/V stage shared by twice the rows)
PREFILL_ROWS = int(os.environ.get("OME_PREFILL_ROWS", "32"))


def prefill_rows(Hq: int, Hkv: int, D: int, page: int = 16) -> int:
    """Rows per classic prefill work item for this attention shape (see PREFILL_ROWS)."""
    ok = D == 128 and page == 16 and Hq == 4 * Hkv and os.environ.get("OME_PREFILL_ATTN", "2") == "2"
    return PREFILL_ROWS if ok and PREFILL_ROWS in (32, 64) else 32
# an item must span more than this many keys before a small grid (< 256 workgroups) is split.
# r03 (profiles/r03_prefill_split_bench_fast.txt) set 2048: at ~900 rows classic won at 700 and
# 2000 keys (27 vs 34 us, 85 vs 93 us).  r06 tried 256: +0.5 % in-process (16.30k -> 16.39k,
# within box noise) but -7 % over HTTP (15.05k -> 14.01k, profiles/r06_step_cost_ab.txt), so 2048 stays
PREFILL_SPLIT_MIN_KEYS = int(os.environ.get("OME_PREFILL_SPLIT_MIN_KEYS", "2048"))


def prefill_plan(q_lens: list[int], kv_lens: list[int], tile: int = 32, target: int | None = None,
                 kv_heads: int = 8, force: bool = False):
    """(classic items, split items, combine items, chunk, parts) for the split-KV prefill kernel.

    A short prefill leaves most CUs idle and each workgroup latency-bound on its serial chain of
    32-key K/V tile loads (profiles/r03_*: 43 us per layer for ~700 rows x <= 480 keys).  Items
    whose key range exceeds ``chunk`` keys are cut into chunks run by separate workgroups (then
    merged); ``chunk`` (a multiple of 64, >= 128) grows with the total work so that about
    ``target`` split items exist -- long prompts already have plenty of items and stay unsplit.
    Measured (profiles/r03_prefill_split_bench.txt): splitting pays when the classic grid is
    smaller than the chip (items x kv heads < 256 workgroups) AND some item has a long key range
    (> ``PREFILL_SPLIT_MIN_KEYS`` keys), e.g. 256 new rows over a 4096-token prefix 243 -> 68 us; at ~900 rows over
    <= 480 keys the classic grid is already full and splitting costs the partial round trip."""
    target = target or PREFILL_SPLIT_TARGET
    items = prefill_work_items(q_lens, kv_lens, tile)
    # the split decision and the split items use 32-row items (the split kernel's partial layout)
    items32 = items if tile == 32 else prefill_work_items(q_lens, kv_lens, 32)
    work = 0
    ends = []
    for s, r in items32:
        e = (kv_lens[s] - q_lens[s]) + min(r + 32, q_lens[s])
        ends.append(e)
        work += e
    if not force and (len(items32) * kv_heads >= 256 or max(ends, default=0) <= PREFILL_SPLIT_MIN_KEYS):
        return items, [], [], 0, 0
    chunk = max(128, -(-(-(-work // max(1, target))) // 64) * 64)
    split, comb, parts = [], [], 0
    for (s, r), e in zip(items32, ends):
        n = -(-e // chunk)
        if n <= 1:
            split.append((s, r, 0, -1))
            continue
        comb.append((s, r, parts, n))
        split.extend((s, r, c * chunk, parts + c) for c in range(n))
        parts += n
    if not comb:
        split = []
    return items, split, comb, chunk, parts


def paged_prefill(q, k_cache, v_cache, block_tables, cu_q, kv_lens, items, scale, window: int = -1,
                  out=None, k_scale: float = 1.0, v_scale: float = 1.0, softcap: float = 0.0,
                  sinks: torch.Tensor | None = None, alibi: torch.Tensor | None = None,
                  row_hi: torch.Tensor | None = None, blocksparse: tuple | None = None) -> torch.Tensor:
    """q [Tq, Hq, D]; items int32 [n, 2] from :func:`prefill_work_items`.  ``softcap`` > 0:
    attention-logit soft-capping ``cap * tanh(score / cap)`` (Gemma-2); ``alibi``: fp32 [Hq]
    ALiBi slopes; ``row_hi``: int32 [Tq], per query row the last key position it may see
    beyond the causal one (-1: causal) -- Gemma 3's bidirectional image blocks."""
    if not _gpu(q):
        r = ref.paged_prefill(q, k_cache, v_cache, block_tables, cu_q, kv_lens, scale, window, k_scale, v_scale,
                              softcap, sinks, alibi, row_hi, blocksparse)
        if out is not None:
            out.copy_(r)
            return out
        return r
    Tq, Hq, D = q.shape
    Hkv, P = k_cache.shape[1], k_cache.shape[2]
    out = torch.empty_like(q) if out is None else out
    rows = 32
    if isinstance(items, PrefillPlan):
        plan, items = items, items.items
        rows = plan.rows
        if rows != 32 and not (rows == 64 and D == 128 and P == 16 and Hq == 4 * Hkv):
            raise ValueError(f"paged_prefill: {rows}-row items need the GQA-4 / D=128 kernel, got Hq={Hq} "
                             f"Hkv={Hkv} D={D} page={P} (build the plan with prefill_rows of this layer)")
        if (plan.parts and D == 128 and P == 16 and Hq == 4 * Hkv and row_hi is None and
                os.environ.get("OME_PREFILL_ATTN", "2") == "2"):
            po = torch.empty(plan.parts * Hkv * 4 * 32 * 128, dtype=torch.float32, device=q.device)
            pml = torch.empty(plan.parts * Hkv * 4 * 32 * 2, dtype=torch.float32, device=q.device)
            call("ome_paged_prefill_split", q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
                 _i32(block_tables).data_ptr(), block_tables.stride(0), _i32(cu_q).data_ptr(),
                 _i32(kv_lens).data_ptr(), plan.split.data_ptr(), plan.split.shape[0], plan.comb.data_ptr(),
                 plan.comb.shape[0], int(plan.chunk), po.data_ptr(), pml.data_ptr(), out.data_ptr(), out.stride(0),
                 Hq, Hkv, float(scale), int(window), kv_format(k_cache), float(k_scale), float(v_scale),
                 float(softcap), _sinks(sinks), _sinks(alibi), blocksparse_pack(blocksparse), stream_ptr())
            return out
    call("ome_paged_prefill", q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(),
         _i32(block_tables).data_ptr(), block_tables.stride(0), _i32(cu_q).data_ptr(), _i32(kv_lens).data_ptr(),
         _i32(items).data_ptr(), items.shape[0], out.data_ptr(), out.stride(0), Hq, Hkv, D, P, float(scale),
         int(window), kv_format(k_cache), float(k_scale), float(v_scale), float(softcap), _sinks(sinks),
         _sinks(alibi), None if row_hi is None else _i32(row_hi).data_ptr(), rows, blocksparse_pack(blocksparse),
         stream_ptr())
    return out


_VARLEN_GENERIC = [0]


@contextlib.contextmanager
def varlen_generic():
    """Inside this block bidirectional :func:`varlen_attention` calls run the generic kernel body
    instead of the fast one (equivalence tests of the two bodies inside one process; the
    ``OME_VARLEN_FAST`` environment switch is read once per process)."""
    _VARLEN_GENERIC[0] += 1
    try:
        yield
    finally:
        _VARLEN_GENERIC[0] -= 1


def varlen_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, lengths: list[int], scale: float,
                     causal: bool = False, out: torch.Tensor | None = None,
                     k_lengths: list[int] | None = None) -> torch.Tensor:
    """Attention over packed variable-length sequences with contiguous (non-paged) K/V: encoder
    models and vision towers.  q [T, Hq, D], k / v [Tk, Hkv, D] -- any per-token stride (views of a
    fused QKV projection are read in place), head dim contiguous; ``lengths``: the host-side
    sequence lengths (sum == T).  Bidirectional unless ``causal``.  ``k_lengths``: cross
    attention -- sequence s's queries attend to ITS OWN packed key rows (``k_lengths[s]`` of them,
    possibly 0: a zero output); None = self attention (k / v rows are the query rows)."""
    T, Hq, D = q.shape
    Hkv = k.shape[1]
    if k_lengths is not None:
        assert not causal and len(k_lengths) == len(lengths) and sum(k_lengths) == k.shape[0]
    if not _gpu(q):
        r = ref.varlen_attention(q, k, v, lengths, scale, causal, k_lengths)
        if out is not None:
            out.copy_(r)
            return out
        return r
    for t in (q, k, v):
        assert t.dtype == torch.bfloat16 and t.stride(-1) == 1 and t.stride(-2) == D, "head-contiguous bf16 rows"
    assert sum(lengths) == T, (sum(lengths), T)
    out = torch.empty(T, Hq, D, dtype=q.dtype, device=q.device) if out is None else out
    cu, items = [0], []
    for s, n in enumerate(lengths):
        cu.append(cu[-1] + n)
        items.extend((s, r) for r in range(0, n, 128))
    if not items:
        return out
    cuk = [0]
    for n in k_lengths or []:
        cuk.append(cuk[-1] + n)
    # items (int2, 8-B aligned) first, then cu_seqlens (then the key ranges)
    meta = torch.tensor([x for it in items for x in it] + cu + (cuk if k_lengths is not None else []),
                        dtype=torch.int32).to(q.device, non_blocking=True)
    ni = 2 * len(items)
    call("ome_varlen_attention", q.data_ptr(), q.stride(0), k.data_ptr(), k.stride(0), v.data_ptr(), v.stride(0),
         meta[ni:].data_ptr(), meta[ni + len(cu):].data_ptr() if k_lengths is not None else None, meta.data_ptr(),
         len(items), out.data_ptr(), out.stride(0), Hq, Hkv, D, float(scale),
         int(bool(causal)) | (2 if _VARLEN_GENERIC[0] else 0), stream_ptr())
    return out


def sample(logits: torch.Tensor, temperature=None, top_k=None, top_p=None, min_p=None, seeds=None, step: int = 0,
           out_ids=None, out_logprob=None):
    """Returns (ids int32 [B], logprobs f32 [B])."""
    if not _gpu(logits):
        ids, lps = ref.sample(logits, temperature, top_k, top_p, min_p, seeds=seeds)
        if out_ids is not None:
            out_ids.copy_(ids)
            ids = out_ids
        if out_logprob is not None:
            out_logprob.copy_(lps)
            lps = out_logprob
        return ids, lps
    B, V = logits.shape
    out_ids = torch.empty(B, dtype=torch.int32, device=logits.device) if out_ids is None else out_ids
    out_logprob = torch.empty(B, dtype=torch.float32, device=logits.device) if out_logprob is None else out_logprob
    call("ome_sample", logits.data_ptr(), int(logits.dtype == torch.bfloat16), logits.stride(0), B, V,
         ptr(temperature), ptr(top_k), ptr(top_p), ptr(min_p), ptr(seeds), int(step) & (2**64 - 1),
         out_ids.data_ptr(), out_logprob.data_ptr(), stream_ptr())
    return out_ids, out_logprob


def pool(hidden: torch.Tensor, cu_lens: torch.Tensor, mode: int = 0, normalize: bool = True) -> torch.Tensor:
    if not _gpu(hidden):
        return ref.pool(hidden, cu_lens, mode, normalize)
    S, H = cu_lens.shape[0] - 1, hidden.shape[-1]
    out = torch.empty(S, H, dtype=torch.float32, device=hidden.device)
    call("ome_pool", hidden.data_ptr(), _i32(cu_lens).data_ptr(), out.data_ptr(), S, H, mode, int(normalize),
         stream_ptr())
    return out
