"""Plain-PyTorch fp32 reference implementations of every native op.

They define the semantics the HIP kernels must reproduce (the GPU numerics tests compare the
two), and they are the CPU execution path used by the CPU-only test-suite.  Cache layouts
match the kernels exactly: K cache ``[pages, Hkv, P, D]``, V cache ``[pages, Hkv, D, P]``.
"""
from __future__ import annotations

import math

import torch


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    rs = torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (xf * rs * w.float()).to(x.dtype)


def fused_add_rmsnorm(x: torch.Tensor, res: torch.Tensor, w: torch.Tensor, eps: float) -> None:
    s = (x.float() + res.float()).to(res.dtype)
    res.copy_(s)
    x.copy_(rmsnorm(s, w, eps))


def layernorm(x: torch.Tensor, w: torch.Tensor, b, eps: float) -> torch.Tensor:
    return torch.nn.functional.layer_norm(x.float(), (x.shape[-1],), w.float(), None if b is None else b.float(),
                                          eps).to(x.dtype)


def fused_add_layernorm(x: torch.Tensor, res: torch.Tensor, w: torch.Tensor, b, eps: float) -> None:
    s = (x.float() + res.float()).to(res.dtype)
    res.copy_(s)
    x.copy_(layernorm(s, w, b, eps))


def act(x: torch.Tensor, kind: int) -> torch.Tensor:
    f = x.float()
    if kind == 0:
        y = torch.nn.functional.silu(f)
    elif kind == 1:
        y = torch.nn.functional.gelu(f, approximate="tanh")
    elif kind == 4:
        y = torch.relu(f).square()
    elif kind == 5:
        y = torch.relu(f)
    else:
        y = torch.nn.functional.gelu(f)
    x.copy_(y.to(x.dtype))
    return x


_act_inplace = act   # for callers whose ``act`` argument shadows the op


def ssm_conv1d(x, w, bias, state, cu, slot, reset, out):
    """Causal depthwise conv + SiLU per sequence, continuing from / updating ``state`` [slots, C, K-1]."""
    K = w.shape[1]
    for s in range(len(slot)):
        r0, r1 = int(cu[s]), int(cu[s + 1])
        if r1 <= r0:
            continue
        st = state[int(slot[s])]
        prev = torch.zeros_like(st) if int(reset[s]) else st
        seq = torch.cat([prev.float().t(), x[r0:r1].float()], 0)          # [K-1+L, C]
        o = torch.nn.functional.conv1d(seq.t()[None], w.float()[:, None, :], None if bias is None else bias.float(),
                                       groups=w.shape[0])[0].t()          # [L, C]
        out[r0:r1] = torch.nn.functional.silu(o).to(out.dtype)
        st.copy_(seq[-(K - 1):].t().to(st.dtype))
    return out


def qk_norm_rope(x, H, hd, w, cs, eps, out, dst):
    T = x.shape[0]
    v = x[:, :H * hd].float().view(T, H, hd)
    if w is not None:
        v = (v * torch.rsqrt(v.pow(2).mean(-1, keepdim=True) + eps)).to(x.dtype).float() * w.float()
        v = v.to(x.dtype).float()
    if cs is not None:
        c, s = cs[:, None, :, 0], cs[:, None, :, 1]
        re, im = v[..., 0::2], v[..., 1::2]
        v = torch.stack([re * c - im * s, re * s + im * c], -1).flatten(-2)
    o2 = out.view(out.shape[0], H * hd)
    rows = torch.arange(T) if dst is None else dst.long().cpu()
    o2[rows.to(o2.device)] = v.reshape(T, H * hd).to(out.dtype)
    return out


def dyn_conv1d(x, kern, state, cu, slot, reset, cpk, out):
    """Per-row-tap causal depthwise conv + SiLU; tap K-1 multiplies the current row."""
    C = x.shape[1]
    K = state.shape[-1] + 1
    for s in range(len(slot)):
        r0, r1 = int(cu[s]), int(cu[s + 1])
        if r1 <= r0:
            continue
        st = state[int(slot[s])]
        prev = torch.zeros_like(st) if int(reset[s]) else st
        seq = torch.cat([prev.float().t(), x[r0:r1].float()], 0)          # [K-1+L, C]
        taps = kern[r0:r1].float().view(r1 - r0, C // cpk, 1, K).expand(-1, -1, cpk, -1).reshape(r1 - r0, C, K)
        win = seq.unfold(0, K, 1)                                         # [L, C, K]
        out[r0:r1] = torch.nn.functional.silu((win * taps).sum(-1)).to(out.dtype)
        st.copy_(seq[-(K - 1):].t().to(st.dtype))
    return out


def ssm_scan(x, dt, B, C, A, D, dt_bias, dt_min, state, cu, slot, reset, H, P, N, G, out):
    """Selective scan (Mamba-2), recurrent per sequence; ``state`` [slots, H, P, N] fp32."""
    rep = H // G
    for s in range(len(slot)):
        r0, r1 = int(cu[s]), int(cu[s + 1])
        if r1 <= r0:
            continue
        st = state[int(slot[s])]
        h = torch.zeros_like(st) if int(reset[s]) else st.clone()
        for r in range(r0, r1):
            d = torch.nn.functional.softplus(dt[r].float() + dt_bias).clamp(min=dt_min)        # [H]
            xv = x[r].float().view(H, P)
            b = B[r].float().view(G, N).repeat_interleave(rep, 0)                               # [H, N]
            c = C[r].float().view(G, N).repeat_interleave(rep, 0)
            h = h * torch.exp(d * A)[:, None, None] + (d[:, None] * xv)[..., None] * b[:, None, :]
            y = (h * c[:, None, :]).sum(-1) + D[:, None] * xv
            out[r] = y.reshape(-1).to(out.dtype)
        st.copy_(h)
    return out


def gdn_scan(q, k, v, a, b, A_log, dt_bias, state, cu, slot, reset, Hv, Hk, out):
    """Gated delta rule, recurrent per sequence; ``state`` [slots, Hv, dv, dk] fp32 (S transposed)."""
    dv, dk = state.shape[2], state.shape[3]
    rep = Hv // Hk
    for s in range(len(slot)):
        r0, r1 = int(cu[s]), int(cu[s + 1])
        if r1 <= r0:
            continue
        st = state[int(slot[s])]
        S = torch.zeros(Hv, dk, dv) if int(reset[s]) else st.transpose(1, 2).clone()             # [Hv, dk, dv]
        S = S.to(st.device)
        for r in range(r0, r1):
            kr = k[r].float().view(Hk, dk)
            kr = kr * torch.rsqrt(kr.pow(2).sum(-1, keepdim=True) + 1e-6)
            qr = q[r].float().view(Hk, dk)
            qr = qr * torch.rsqrt(qr.pow(2).sum(-1, keepdim=True) + 1e-6) * dk ** -0.5
            qr, kr = qr.repeat_interleave(rep, 0), kr.repeat_interleave(rep, 0)                 # [Hv, dk]
            g = -torch.exp(A_log) * torch.nn.functional.softplus(a[r].float() + dt_bias)
            beta = torch.sigmoid(b[r].float())
            S = S * torch.exp(g)[:, None, None]
            kv = (S * kr[..., None]).sum(1)                                                     # [Hv, dv]
            delta = (v[r].float().view(Hv, dv) - kv) * beta[:, None]
            S = S + kr[..., None] * delta[:, None, :]
            out[r] = (S * qr[..., None]).sum(1).reshape(-1).to(out.dtype)
        st.copy_(S.transpose(1, 2))
    return out


def gated_rmsnorm(y, z, w, group, eps, norm_first=False):
    T, I = y.shape
    if norm_first:
        g = y.float().view(T, I // group, group)
        g = (g * torch.rsqrt(g.pow(2).mean(-1, keepdim=True) + eps)).to(y.dtype)
        return ((w * g).float() * torch.nn.functional.silu(z.float().view(T, I // group, group))).view(T, I).to(y.dtype)
    v = y.float() * torch.nn.functional.silu(z.float())
    g = v.view(T, I // group, group)
    g = g * torch.rsqrt(g.pow(2).mean(-1, keepdim=True) + eps)
    return w * g.view(T, I).to(y.dtype)


def apply_rope(x: torch.Tensor, cs: torch.Tensor, rot_dim: int) -> torch.Tensor:
    """x [T, H, D] float, cs [T, rot_dim] (cos | sin)."""
    half = rot_dim // 2
    cos, sin = cs[:, None, :half], cs[:, None, half:rot_dim]
    x1, x2 = x[..., :half], x[..., half:rot_dim]
    out = x.clone()
    out[..., :half] = x1 * cos - x2 * sin
    out[..., half:rot_dim] = x2 * cos + x1 * sin
    return out


#: finite range of the fp8 KV-cache formats (values are saturated, never NaN)
FP8_RANGE = {torch.float8_e4m3fn: 448.0, torch.float8_e5m2: 57344.0}


def to_cache(x: torch.Tensor, dtype, scale: float = 1.0) -> torch.Tensor:
    """Cache entry for ``x``: bf16 as-is, fp8 = saturate(bf16(x) / scale) (round to nearest even)."""
    if dtype not in FP8_RANGE:
        return x.to(dtype)
    m = FP8_RANGE[dtype]
    return (x.to(torch.bfloat16).float() / scale).clamp(-m, m).to(dtype)


def rope_qkv_cache(qkv, positions, cos_sin, rot_dim, q_out, k_cache, v_cache, slots, Hq, Hkv, D, P, apply=True,
                   q_norm_w=None, k_norm_w=None, qk_eps=1e-6, k_scale=1.0, v_scale=1.0) -> None:
    T = qkv.shape[0]
    if T == 0:
        return
    q = qkv[:, : Hq * D].float().view(T, Hq, D)
    k = qkv[:, Hq * D:(Hq + Hkv) * D].float().view(T, Hkv, D)
    v = qkv[:, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D].view(T, Hkv, D)
    if q_norm_w is not None:
        q = rmsnorm(q.to(qkv.dtype), q_norm_w, qk_eps).float()
    if k_norm_w is not None:
        k = rmsnorm(k.to(qkv.dtype), k_norm_w, qk_eps).float()
    if apply:
        cs = cos_sin[positions.long()]
        q = apply_rope(q, cs, rot_dim)
        k = apply_rope(k, cs, rot_dim)
    q_out.view(T, Hq, D).copy_(q.to(q_out.dtype))
    kdt = k_cache.dtype if k_cache.dtype not in FP8_RANGE else torch.bfloat16
    kv_cache_write(k.to(kdt), v, k_cache, v_cache, slots, P, k_scale, v_scale)


def kv_cache_write(k, v, k_cache, v_cache, slots, P, k_scale=1.0, v_scale=1.0) -> None:
    sl = slots.long()
    ok = sl >= 0
    if not bool(ok.any()):
        return
    sl, k, v = sl[ok], k[ok], v[ok]
    page, off = sl // P, sl % P
    k_cache[page, :, off, :] = to_cache(k, k_cache.dtype, k_scale)
    v_cache[page, :, :, off] = to_cache(v, v_cache.dtype, v_scale)


def act_and_mul(x: torch.Tensor, act: int = 0) -> torch.Tensor:
    I = x.shape[-1] // 2
    g, u = x[..., :I].float(), x[..., I:].float()
    if act in (2, 3):  # clamped SwiGLU / GeGELU: GPT-OSS (limit 7), Phi-3-small (limit 20)
        lim = 7.0 if act == 2 else 20.0
        g = g.clamp(max=lim)
        u = u.clamp(-lim, lim)
        return ((u + 1) * g * torch.sigmoid(1.702 * g)).to(x.dtype)
    a = torch.nn.functional.silu(g) if act == 0 else torch.nn.functional.gelu(g, approximate="tanh")
    return (a * u).to(x.dtype)


def embedding(ids: torch.Tensor, table: torch.Tensor, vocab_start: int = 0, vocab_end: int | None = None):
    vocab_end = table.shape[0] + vocab_start if vocab_end is None else vocab_end
    own = (ids >= vocab_start) & (ids < vocab_end)
    local = torch.where(own, ids - vocab_start, torch.zeros_like(ids)).long()
    out = table[local]
    return out * own[:, None].to(out.dtype)


def gather_kv(k_cache, v_cache, block_table, n: int, kvh: int, P: int, k_scale=1.0, v_scale=1.0):
    """Contiguous (dequantised) K [n, D] and V [n, D] for one sequence / kv head."""
    idx = torch.arange(n, device=k_cache.device)
    pages = block_table[(idx // P).long()].long()
    off = idx % P
    k = k_cache[pages, kvh, off, :]
    v = v_cache[pages, kvh, :, off]
    return k.float() * k_scale, v.float() * v_scale


def _cap(s: torch.Tensor, softcap: float) -> torch.Tensor:
    return softcap * torch.tanh(s / softcap) if softcap and softcap > 0 else s


def _softmax_sink(s: torch.Tensor, sink) -> torch.Tensor:
    """softmax over [scores, sink] with the sink column dropped (GPT-OSS attention sinks)."""
    if sink is None:
        return torch.softmax(s, -1)
    col = sink.float().reshape(*([1] * (s.dim() - 1)), 1).expand(*s.shape[:-1], 1) if sink.dim() == 0 else sink
    full = torch.cat([s, col], -1)
    return torch.softmax(full, -1)[..., :-1]


def attn_lo(qpos, window: int):
    """First visible key for query position(s) ``qpos`` (see attention.hip ``attn_lo``): sliding
    window (``window`` > 0), chunked attention with chunks of ``-window`` (``window`` < -1), else 0."""
    if window > 0:
        return (qpos - window + 1).clamp(min=0)
    if window < -1:
        return qpos - qpos % (-window)
    return qpos * 0


def blocksparse_visible(qpos: torch.Tensor, kpos: torch.Tensor, heads: torch.Tensor, bs) -> torch.Tensor:
    """Block-sparse causal visibility (attention.hip ``Scaler::bs_visible``; Phi-3-small):
    ``bs`` = (block, local_blocks, vert_stride, head_step, head0); broadcasts qpos / kpos / heads.
    The causal limit itself is applied by the caller."""
    block, local, vert, step, h0 = bs
    qb, kb = torch.div(qpos, block, rounding_mode="floor"), torch.div(kpos, block, rounding_mode="floor")
    return ((qb - kb) < local) | (((kb + h0 + heads * step + 1) % vert) == 0)


def paged_decode(q, k_cache, v_cache, block_tables, seq_lens, scale, window=-1, k_scale=1.0,
                 v_scale=1.0, softcap=0.0, sinks=None, alibi=None, row_lo=None, blocksparse=None) -> torch.Tensor:
    B, Hq, D = q.shape
    Hkv, P = k_cache.shape[1], k_cache.shape[2]
    G = Hq // Hkv
    out = torch.zeros_like(q)
    for b in range(B):
        L = int(seq_lens[b])
        if L <= 0:
            continue
        lo = int(attn_lo(torch.tensor(L - 1), window))
        if row_lo is not None:
            lo = max(lo, int(row_lo[b]))
        for h in range(Hkv):
            k, v = gather_kv(k_cache, v_cache, block_tables[b], L, h, P, k_scale, v_scale)
            k, v = k[lo:], v[lo:]
            qh = q[b, h * G:(h + 1) * G].float()
            s = _cap((qh @ k.T) * scale, softcap)
            if alibi is not None:  # slope * (key - query position)
                kp = torch.arange(lo, L, device=q.device, dtype=torch.float32) - (L - 1)
                s = s + alibi[h * G:(h + 1) * G].float().view(G, 1).to(s.device) * kp[None]
            if blocksparse is not None:
                kp = torch.arange(lo, L, device=q.device)[None]
                hs = torch.arange(h * G, (h + 1) * G, device=q.device)[:, None]
                s = s.masked_fill(~blocksparse_visible(torch.tensor(L - 1, device=q.device), kp, hs, blocksparse),
                                  float("-inf"))
            sk = None if sinks is None else sinks[h * G:(h + 1) * G].float().view(G, 1)
            out[b, h * G:(h + 1) * G] = (_softmax_sink(s, sk) @ v).to(q.dtype)
    return out


def paged_prefill(q, k_cache, v_cache, block_tables, cu_q, kv_lens, scale, window=-1, k_scale=1.0,
                  v_scale=1.0, softcap=0.0, sinks=None, alibi=None, row_hi=None, blocksparse=None) -> torch.Tensor:
    Tq, Hq, D = q.shape
    Hkv, P = k_cache.shape[1], k_cache.shape[2]
    G = Hq // Hkv
    out = torch.zeros_like(q)
    S = len(kv_lens)
    for s in range(S):
        q0, q1 = int(cu_q[s]), int(cu_q[s + 1])
        ql, L = q1 - q0, int(kv_lens[s])
        if ql == 0:
            continue
        qpos = torch.arange(L - ql, L, device=q.device)[:, None]
        kpos = torch.arange(L, device=q.device)[None, :]
        qlim = qpos if row_hi is None else torch.maximum(qpos, row_hi[q0:q1].to(q.device).long()[:, None])
        mask = kpos <= qlim
        mask &= kpos >= attn_lo(qpos, window)
        for h in range(Hkv):
            k, v = gather_kv(k_cache, v_cache, block_tables[s], L, h, P, k_scale, v_scale)
            qh = q[q0:q1, h * G:(h + 1) * G].float().transpose(0, 1)  # [G, ql, D]
            sc = _cap((qh @ k.T) * scale, softcap)
            if alibi is not None:
                sl = alibi[h * G:(h + 1) * G].float().view(G, 1, 1).to(sc.device)
                sc = sc + sl * (kpos - qpos).float()[None]
            m = mask[None]
            if blocksparse is not None:
                hs = torch.arange(h * G, (h + 1) * G, device=q.device).view(G, 1, 1)
                m = m & blocksparse_visible(qpos[None], kpos[None], hs, blocksparse)
            sc = sc.masked_fill(~m, float("-inf"))
            sk = None if sinks is None else sinks[h * G:(h + 1) * G].float().view(G, 1, 1).expand(G, sc.shape[1], 1)
            o = _softmax_sink(sc, sk) @ v
            out[q0:q1, h * G:(h + 1) * G] = o.transpose(0, 1).to(q.dtype)
    return out


def sample(logits, temperature=None, top_k=None, top_p=None, min_p=None, generator=None, seeds=None):
    """Returns (ids int32 [B], logprob f32 [B]).  Greedy where temperature <= 0.  ``seeds``
    (int64 [B]) makes each row's draw a pure function of its counter-based seed (the CPU
    analogue of the kernel's per-row splitmix64 stream; the draws themselves differ)."""
    lf = logits.float()
    B, V = lf.shape
    ids = torch.empty(B, dtype=torch.int32, device=logits.device)
    lps = torch.empty(B, dtype=torch.float32, device=logits.device)
    for b in range(B):
        t = float(temperature[b]) if temperature is not None else 0.0
        row = lf[b]
        if t <= 0:
            i = int(torch.argmax(row))
            ids[b] = i
            lps[b] = torch.log_softmax(row, -1)[i]
            continue
        z = (row - row.max()) / t
        logp = torch.log_softmax(z, -1)
        keep = torch.ones(V, dtype=torch.bool, device=row.device)
        k = int(top_k[b]) if top_k is not None else -1
        if 0 < k < V:
            kth = torch.topk(z, k).values[-1]
            keep &= z >= kth
        p = float(top_p[b]) if top_p is not None else 1.0
        if p < 1.0:
            sz, order = torch.sort(z, descending=True)
            probs = torch.softmax(sz, -1)
            cum = torch.cumsum(probs, -1)
            n_keep = int((cum < p).sum()) + 1
            thr = sz[min(n_keep, V) - 1]
            keep &= z >= thr
        mp = float(min_p[b]) if min_p is not None else 0.0
        if mp > 0:
            keep &= z >= math.log(mp)
        probs = torch.softmax(z.masked_fill(~keep, float("-inf")), -1)
        g = generator
        if seeds is not None:
            g = torch.Generator(device=row.device)
            g.manual_seed(int(seeds[b]) & ((1 << 63) - 1))
        i = int(torch.multinomial(probs, 1, generator=g))
        ids[b] = i
        lps[b] = logp[i]
    return ids, lps


def varlen_attention(q, k, v, lengths, scale, causal=False, k_lengths=None) -> torch.Tensor:
    T, Hq, D = q.shape
    G = Hq // k.shape[1]
    out = torch.empty(T, Hq, D, dtype=q.dtype, device=q.device)
    t0 = k0 = 0
    for i, n in enumerate(lengths):
        nk = n if k_lengths is None else k_lengths[i]
        if nk == 0:
            out[t0:t0 + n] = 0
            t0 += n
            continue
        qs = q[t0:t0 + n].float().transpose(0, 1)
        ks = k[k0:k0 + nk].float().repeat_interleave(G, 1).transpose(0, 1)
        vs = v[k0:k0 + nk].float().repeat_interleave(G, 1).transpose(0, 1)
        s = (qs @ ks.transpose(1, 2)) * scale
        if causal:
            s = s.masked_fill(torch.ones(n, n, dtype=torch.bool, device=q.device).triu(1), float("-inf"))
        out[t0:t0 + n] = (s.softmax(-1) @ vs).transpose(0, 1).to(q.dtype)
        t0 += n
        k0 += nk
    return out


def pool(hidden, cu_lens, mode: int = 0, normalize: bool = True) -> torch.Tensor:
    S = len(cu_lens) - 1
    outs = []
    for s in range(S):
        b, e = int(cu_lens[s]), int(cu_lens[s + 1])
        h = hidden[e - 1].float() if mode == 0 else hidden[b].float() if mode == 2 else hidden[b:e].float().mean(0)
        outs.append(h)
    out = torch.stack(outs)
    if normalize:
        out = torch.nn.functional.normalize(out, dim=-1)
    return out


# ------------------------------------------------------------------ MoE
def moe_route(logits, k: int, renorm: bool, scoring: str = "softmax", bias=None, n_group: int = 1,
              topk_group: int = 1, group_mode: int = 0):
    """HF semantics (Mixtral/Qwen softmax top-k; DeepSeek-V2 group_limited_greedy = mode 1,
    DeepSeek-V3 noaux_tc = mode 2 with e_score_correction_bias)."""
    lf = logits.float()
    p = torch.softmax(lf, -1) if scoring == "softmax" else torch.sigmoid(lf)
    key = p + bias.float() if bias is not None else p.clone()
    if group_mode and n_group > 1:
        T, E = key.shape
        grp = key.view(T, n_group, E // n_group)
        gs = grp.max(-1).values if group_mode == 1 else grp.topk(min(2, E // n_group), -1).values.sum(-1)
        gidx = gs.topk(topk_group, -1).indices
        gmask = torch.zeros_like(gs, dtype=torch.bool).scatter_(1, gidx, True)
        key = key.masked_fill(~gmask.repeat_interleave(E // n_group, 1), 0.0)
    _, ids = torch.topk(key, k, dim=-1)  # ties: torch.topk order is implementation-defined
    w = p.gather(1, ids)
    if renorm:
        w = w / (w.sum(-1, keepdim=True) + 1e-20)
    return w.float(), ids.to(torch.int32)


def fused_moe(x, topk_w, topk_ids, w13, w2, act: int = 0, scale: float = 1.0, b13=None, b2=None, gated=True):
    """x [T, H]; w13 [E, 2I, H] (gate rows then up rows); w2 [E, H, I]; optional per-expert
    biases b13 [E, 2I], b2 [E, H] (GPT-OSS)."""
    T, H = x.shape
    out = torch.zeros(T, H, dtype=torch.float32, device=x.device)
    xf = x.float()
    for e in torch.unique(topk_ids).tolist():
        tok, slot = (topk_ids == e).nonzero(as_tuple=True)
        gu = xf[tok] @ w13[e].float().t()
        if b13 is not None:
            gu = gu + b13[e].float()
        h = (act_and_mul(gu.to(x.dtype), act) if gated else _act_inplace(gu.to(x.dtype), act)).float()
        y = h.to(x.dtype).float() @ w2[e].float().t()
        if b2 is not None:
            y = y + b2[e].float()
        y = y.to(x.dtype).float()
        out.index_add_(0, tok, y * topk_w[tok, slot].float()[:, None])
    return (out * scale).to(x.dtype)


def fused_moe_fp8(x, topk_w, topk_ids, w13q, w13s, w2q, w2s, act: int = 0, scale: float = 1.0, block: int = 128):
    """The fp8 MoE path exactly as the GPU computes it: x and the activation h are quantised to
    e4m3 with 1x128 group scales, experts are e4m3 with 128x128 block scales, products in fp32."""
    T, H = x.shape
    out = torch.zeros(T, H, dtype=torch.float32, device=x.device)
    qx, sx = fp8_quant(x, block)
    xd = qx.float() * sx.repeat_interleave(block, 1)
    for e in torch.unique(topk_ids).tolist():
        tok, slot = (topk_ids == e).nonzero(as_tuple=True)
        gu = (xd[tok] @ fp8_dequant_weight(w13q[e], w13s[e], block).t()).to(x.dtype)
        h = act_and_mul(gu, act)
        qh, sh = fp8_quant(h, block)
        hd = qh.float() * sh.repeat_interleave(block, 1)
        y = (hd @ fp8_dequant_weight(w2q[e], w2s[e], block).t()).to(x.dtype).float()
        out.index_add_(0, tok, y * topk_w[tok, slot].float()[:, None])
    return (out * scale).to(x.dtype)


SEEN_BIT = 1 << 24


def apply_penalties(logits, counts, slot, rep, freq, pres):
    """In place; see csrc/kernels/sampling.hip."""
    for b in range(logits.shape[0]):
        rp, fp, pp = float(rep[b]), float(freq[b]), float(pres[b])
        if rp == 1.0 and fp == 0.0 and pp == 0.0:
            continue
        c = counts[int(slot[b])]
        nz = (c != 0).nonzero(as_tuple=True)[0]
        if nz.numel() == 0:
            continue
        x = logits[b, nz].float()
        cc = c[nz]
        seen = (cc & SEEN_BIT) != 0
        if rp != 1.0:
            x = torch.where(seen, torch.where(x > 0, x / rp, x * rp), x)
        oc = (cc & (SEEN_BIT - 1)).float()
        x = x - fp * oc - pp * (oc > 0).float()
        logits[b, nz] = x.to(logits.dtype)


def update_counts(counts, slot, ids, rep, freq, pres):
    for b in range(ids.shape[0]):
        if float(rep[b]) == 1.0 and float(freq[b]) == 0.0 and float(pres[b]) == 0.0:
            continue
        s, t = int(slot[b]), int(ids[b])
        counts[s, t] = (counts[s, t] + 1) | SEEN_BIT


# ------------------------------------------------------------------ FP8 (OCP e4m3fn) W8A8
FP8_MAX = 448.0


def fp8_quant(x: torch.Tensor, group: int = 0):
    """x [M, K] -> (q float8_e4m3fn [M, K], scale f32 [M, K/group or 1])."""
    M, K = x.shape
    g = K if group == 0 else group
    xg = x.float().reshape(M, K // g, g)
    amax = xg.abs().amax(-1)
    s = torch.where(amax > 0, amax / FP8_MAX, torch.ones_like(amax))
    q = (xg * (1.0 / s)[..., None]).clamp(-FP8_MAX, FP8_MAX).to(torch.float8_e4m3fn).reshape(M, K)
    return q, s


def fp8_dequant_weight(q: torch.Tensor, scale: torch.Tensor, block: int) -> torch.Tensor:
    w = q.float()
    if block:
        s = scale.float().repeat_interleave(block, 0)[: w.shape[0]].repeat_interleave(block, 1)[:, : w.shape[1]]
        return w * s
    return w * scale.float().reshape(-1, 1)


def fp8_gemm(qa, sa, qw, sw, block: int, bias=None, out_dtype=torch.bfloat16):
    a = qa.float()
    a = a * (sa.float().repeat_interleave(block, 1) if block else sa.float().reshape(-1, 1))
    out = a @ fp8_dequant_weight(qw, sw, block).t()
    if bias is not None:
        out = out + bias.float()
    return out.to(out_dtype)


def mla_attn(q, cache, block_tables, tok_row, kv_lens, scale, dv=512):
    """Absorbed MLA: q [T, H, DK], cache [pages, 16, DK] -> out [T, H, dv] (values = the first dv
    latent dims)."""
    T, H, DK = q.shape
    P = cache.shape[-2]
    out = torch.empty(T, H, dv, dtype=q.dtype, device=q.device)
    flat = cache.reshape(-1, P, DK)
    for t in range(T):
        L = int(kv_lens[t])
        pages = block_tables[int(tok_row[t])][: -(-L // P)].long()
        kv = flat[pages].reshape(-1, DK)[:L].float()
        s = (q[t].float() @ kv.t()) * scale
        out[t] = (torch.softmax(s, -1) @ kv[:, :dv]).to(q.dtype)
    return out
