"""Numerics of every hand-written gfx950 kernel vs the plain-PyTorch fp32 reference of the same op."""
import math
import os
import random

import pytest
import torch

from ome_amd import ops
from ome_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(a, b, atol=2e-2, rtol=2e-2):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    assert torch.allclose(a, b, atol=atol, rtol=rtol), f"max abs err {err}"


@pytest.fixture(autouse=True)
def _seed():
    torch.manual_seed(0)
    random.seed(0)


def test_native_library_loaded():
    assert ops.available(), "libome_kernels.so must be built and loadable on the GPU box"


@pytest.mark.parametrize("rows,H", [(1, 4096), (7, 4096), (600, 4096), (3, 8192), (5, 7168), (2, 256)])
def test_rmsnorm(rows, H):
    x = torch.randn(rows, H, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(H, device=DEV, dtype=torch.bfloat16)
    _close(ops.rmsnorm(x, w, 1e-5), ref.rmsnorm(x, w, 1e-5))


@pytest.mark.parametrize("rows,H", [(1, 4096), (600, 4096), (5, 7168)])
def test_fused_add_rmsnorm(rows, H):
    x = torch.randn(rows, H, device=DEV, dtype=torch.bfloat16)
    r = torch.randn(rows, H, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(H, device=DEV, dtype=torch.bfloat16)
    x2, r2 = x.clone(), r.clone()
    ops.fused_add_rmsnorm(x, r, w, 1e-5)
    ref.fused_add_rmsnorm(x2, r2, w, 1e-5)
    _close(r, r2, atol=1e-2)
    _close(x, x2)


def _cache(pages, Hkv, D, P=16):
    k = torch.randn(pages, Hkv, P, D, device=DEV, dtype=torch.bfloat16)
    v = torch.randn(pages, Hkv, D, P, device=DEV, dtype=torch.bfloat16)
    return k, v


@pytest.mark.parametrize("qk_norm", [False, True])
@pytest.mark.parametrize("Hq,Hkv,rot", [(32, 8, 128), (8, 1, 128), (4, 2, 64)])
def test_rope_qkv_cache(Hq, Hkv, rot, qk_norm):
    from ome_amd.models.config import preset, rope_cos_sin

    D, T, P = 128, 37, 16
    cfg = preset("llama-3.1-8b")
    cfg.head_dim, cfg.partial_rotary_factor = D, rot / D
    cs = rope_cos_sin(cfg, 4096, device=DEV)
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
    pos = torch.randint(0, 4000, (T,), device=DEV, dtype=torch.int32)
    slots = torch.randperm(40 * P, device=DEV)[:T].to(torch.int32)
    slots[3] = -1
    qn = torch.randn(D, device=DEV, dtype=torch.bfloat16) if qk_norm else None
    kn = torch.randn(D, device=DEV, dtype=torch.bfloat16) if qk_norm else None
    k1, v1 = _cache(40, Hkv, D)
    k2, v2 = k1.clone(), v1.clone()
    q1 = torch.empty(T, Hq, D, device=DEV, dtype=torch.bfloat16)
    q2 = torch.empty_like(q1)
    ops.rope_qkv_cache(qkv, pos, cs, rot, q1, k1, v1, slots, Hq, Hkv, D, True, qn, kn, 1e-6)
    ref.rope_qkv_cache(qkv, pos, cs, rot, q2, k2, v2, slots, Hq, Hkv, D, P, True, qn, kn, 1e-6)
    _close(q1, q2, atol=3e-2)
    _close(k1, k2, atol=3e-2)
    assert torch.equal(v1, v2)


def test_act_and_mul():
    x = torch.randn(33, 2 * 14336, device=DEV, dtype=torch.bfloat16)
    _close(ops.act_and_mul(x, 0), ref.act_and_mul(x, 0))
    _close(ops.act_and_mul(x, 1), ref.act_and_mul(x, 1))


def test_embedding_vocab_parallel():
    table = torch.randn(1000, 512, device=DEV, dtype=torch.bfloat16)
    ids = torch.randint(0, 3000, (77,), device=DEV, dtype=torch.int32)
    assert torch.equal(ops.embedding(ids, table, 1000, 2000), ref.embedding(ids, table, 1000, 2000))


def _block_tables(seq_lens, P, num_pages):
    perm = torch.randperm(num_pages - 1)[: sum(-(-L // P) for L in seq_lens) + 1] + 1
    mx = max(-(-L // P) for L in seq_lens) + 1
    bt = torch.zeros(len(seq_lens), mx, dtype=torch.int32)
    o = 0
    for i, L in enumerate(seq_lens):
        n = -(-L // P)
        bt[i, :n] = perm[o:o + n]
        o += n
    return bt.to(DEV)


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 1), (64, 8), (16, 16)])
@pytest.mark.parametrize("seq_lens", [[1], [15, 16, 17, 33], [100, 1000, 3, 517], [5000, 7]])
@pytest.mark.parametrize("part_size", [256, 8192])
@pytest.mark.parametrize("variant", ["1", "2", "3", "4"])
def test_paged_decode(Hq, Hkv, seq_lens, part_size, variant, monkeypatch):
    monkeypatch.setenv("OME_DECODE_ATTN", variant)
    D, P = 128, 16
    npages = sum(-(-L // P) for L in seq_lens) + 8
    kc, vc = _cache(npages, Hkv, D)
    bt = _block_tables(seq_lens, P, npages)
    sl = torch.tensor(seq_lens, dtype=torch.int32, device=DEV)
    q = torch.randn(len(seq_lens), Hq, D, device=DEV, dtype=torch.bfloat16)
    ws = ops.DecodeWorkspace(len(seq_lens), Hq, D, 8192, part_size, DEV)
    scale = 1 / math.sqrt(D)
    out = ops.paged_decode(q, kc, vc, bt, sl, scale, ws)
    expect = ref.paged_decode(q, kc, vc, bt, sl, scale)
    _close(out, expect, atol=2e-2)
    if variant != "1":  # longest-first visit order must not change the result
        order = torch.argsort(sl, descending=True).to(torch.int32)
        _close(ops.paged_decode(q, kc, vc, bt, sl, scale, ws, order=order), expect, atol=2e-2)


@pytest.mark.parametrize("window", [128, -256, -64])  # sliding; chunked (Llama 4) as window < -1
@pytest.mark.parametrize("variant", ["1", "2", "3", "4"])
def test_paged_decode_window(variant, window, monkeypatch):
    monkeypatch.setenv("OME_DECODE_ATTN", variant)
    D, P, Hq, Hkv = 128, 16, 32, 8
    seq_lens = [700, 40]
    kc, vc = _cache(64, Hkv, D)
    bt = _block_tables(seq_lens, P, 64)
    sl = torch.tensor(seq_lens, dtype=torch.int32, device=DEV)
    q = torch.randn(2, Hq, D, device=DEV, dtype=torch.bfloat16)
    ws = ops.DecodeWorkspace(2, Hq, D, 1024, 256, DEV)
    out = ops.paged_decode(q, kc, vc, bt, sl, 0.088, ws, window=window)
    _close(out, ref.paged_decode(q, kc, vc, bt, sl, 0.088, window=window))


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (64, 8), (8, 1), (16, 4)])
@pytest.mark.parametrize("q_lens,kv_lens", [([5], [5]), ([37, 64, 1, 100], [37, 80, 300, 100]),
                                            ([300], [1000]), ([1, 1, 1], [20, 33, 16]), ([1000], [1000])])
@pytest.mark.parametrize("variant", ["1", "2"])
def test_paged_prefill(Hq, Hkv, q_lens, kv_lens, variant, monkeypatch):
    monkeypatch.setenv("OME_PREFILL_ATTN", variant)
    D, P = 128, 16
    npages = sum(-(-L // P) for L in kv_lens) + 8
    kc, vc = _cache(npages, Hkv, D)
    bt = _block_tables(kv_lens, P, npages)
    cu = torch.tensor([0] + list(torch.tensor(q_lens).cumsum(0)), dtype=torch.int32, device=DEV)
    kl = torch.tensor(kv_lens, dtype=torch.int32, device=DEV)
    items = torch.tensor(ops.prefill_work_items(q_lens, kv_lens), dtype=torch.int32, device=DEV)
    q = torch.randn(sum(q_lens), Hq, D, device=DEV, dtype=torch.bfloat16)
    out = ops.paged_prefill(q, kc, vc, bt, cu, kl, items, 0.0884)
    _close(out, ref.paged_prefill(q, kc, vc, bt, cu, kl, 0.0884), atol=2e-2)


def _plan(q_lens, kv_lens, target):
    items, split, comb, chunk, parts = ops.prefill_plan(q_lens, kv_lens, target=target, force=True)
    t = lambda a, c: torch.tensor(a, dtype=torch.int32, device=DEV).view(-1, c)  # noqa: E731
    return ops.PrefillPlan(t(items, 2), t(split, 4) if split else None, t(comb, 4) if comb else None, chunk, parts)


@pytest.mark.parametrize("window", [-1, 100])
@pytest.mark.parametrize("sinks", [False, True])
@pytest.mark.parametrize("target", [32, 128, 4096])
def test_paged_prefill_split_kv(window, sinks, target):
    """Split-KV prefill (chunks of the key range on separate workgroups, merged by the combine
    kernel) == the fp32 reference, with prefixes, short and long rows, windows and sinks."""
    D, P, Hq, Hkv = 128, 16, 32, 8
    q_lens, kv_lens = [480, 37, 1, 300, 700], [480, 600, 900, 300, 1400]
    npages = sum(-(-L // P) for L in kv_lens) + 8
    kc, vc = _cache(npages, Hkv, D)
    bt = _block_tables(kv_lens, P, npages)
    cu = torch.tensor([0] + list(torch.tensor(q_lens).cumsum(0)), dtype=torch.int32, device=DEV)
    kl = torch.tensor(kv_lens, dtype=torch.int32, device=DEV)
    plan = _plan(q_lens, kv_lens, target)
    if target >= 128:
        assert plan.parts > 0, "expected a split plan"
    q = torch.randn(sum(q_lens), Hq, D, device=DEV, dtype=torch.bfloat16)
    sk = torch.randn(Hq, device=DEV) if sinks else None
    out = ops.paged_prefill(q, kc, vc, bt, cu, kl, plan, 0.0884, window=window, sinks=sk)
    _close(out, ref.paged_prefill(q, kc, vc, bt, cu, kl, 0.0884, window, 1.0, 1.0, 0.0, sk), atol=2e-2)


@pytest.mark.parametrize("window", [100, -128, -48])
@pytest.mark.parametrize("variant", ["1", "2"])
def test_paged_prefill_window(window, variant, monkeypatch):
    monkeypatch.setenv("OME_PREFILL_ATTN", variant)
    D, P, Hq, Hkv = 128, 16, 32, 8
    q_lens, kv_lens = [200, 50], [500, 50]
    kc, vc = _cache(64, Hkv, D)
    bt = _block_tables(kv_lens, P, 64)
    cu = torch.tensor([0, 200, 250], dtype=torch.int32, device=DEV)
    kl = torch.tensor(kv_lens, dtype=torch.int32, device=DEV)
    items = torch.tensor(ops.prefill_work_items(q_lens, kv_lens), dtype=torch.int32, device=DEV)
    q = torch.randn(250, Hq, D, device=DEV, dtype=torch.bfloat16)
    out = ops.paged_prefill(q, kc, vc, bt, cu, kl, items, 0.0884, window=window)
    _close(out, ref.paged_prefill(q, kc, vc, bt, cu, kl, 0.0884, window=window))


def test_sample_greedy_and_filters():
    B, V = 9, 128256
    logits = torch.randn(B, V, device=DEV, dtype=torch.bfloat16) * 3
    am = logits.float().argmax(-1)
    ids, lp = ops.sample(logits)
    assert torch.equal(ids.long().cpu(), am.cpu())
    t = torch.ones(B, device=DEV)
    k1 = torch.ones(B, dtype=torch.int32, device=DEV)
    mx = logits.float().max(-1).values
    ids, _ = ops.sample(logits, t, k1, None, None, torch.arange(B, device=DEV, dtype=torch.int64))
    # top-k=1 == greedy (up to exact bf16 ties at the max)
    assert torch.equal(logits.float().gather(1, ids.long()[:, None])[:, 0], mx)
    tp = torch.full((B,), 1e-6, device=DEV)
    ids, _ = ops.sample(logits, t, None, tp, None, torch.arange(B, device=DEV, dtype=torch.int64))
    assert torch.equal(logits.float().gather(1, ids.long()[:, None])[:, 0], mx)  # tiny top-p == greedy
    ref_lp = torch.log_softmax(logits.float(), -1).gather(1, am[:, None])[:, 0]
    _, lp = ops.sample(logits)
    _close(lp, ref_lp, atol=1e-2)


def test_sample_distribution():
    V = 16
    logits = torch.log(torch.tensor([0.5, 0.25, 0.125, 0.125] + [1e-9] * (V - 4), device=DEV)).repeat(4096, 1)
    t = torch.ones(4096, device=DEV)
    seeds = torch.arange(4096, device=DEV, dtype=torch.int64) * 7919
    ids, _ = ops.sample(logits.float(), t, None, None, None, seeds)
    freq = torch.bincount(ids.long().cpu(), minlength=V).float() / 4096
    assert abs(freq[0] - 0.5) < 0.05 and abs(freq[1] - 0.25) < 0.05
    tk = torch.full((4096,), 2, dtype=torch.int32, device=DEV)
    ids, _ = ops.sample(logits.float(), t, tk, None, None, seeds)
    assert int(ids.max()) <= 1


def test_sample_topk_topp_kept_set():
    """The histogram threshold select keeps exactly the top-k / top-p sets (ties at the boundary
    value included): every draw lands in the exact set computed by sorting on the host, and the
    draws cover it."""
    B, V = 1024, 128256
    g = torch.Generator().manual_seed(3)
    row = (torch.randn(V, generator=g) * 3).to(torch.bfloat16)
    logits = row.to(DEV).repeat(B, 1)
    seeds = torch.arange(B, device=DEV, dtype=torch.int64) * 7919 + 1
    t = torch.full((B,), 0.7, device=DEV)
    z = row.float() / 0.7
    srt, order = torch.sort(z, descending=True)
    # top-k = 20: the kept set is every token >= the 20th largest value
    tk = torch.full((B,), 20, dtype=torch.int32, device=DEV)
    ids, _ = ops.sample(logits, t, tk, None, None, seeds)
    kth = srt[19]
    got = z[ids.long().cpu()]
    assert bool((got >= kth).all())
    assert len(set(ids.tolist())) >= 15
    # top-p = 0.6: smallest prefix of the sorted distribution holding >= 60 % of the mass
    p = torch.softmax(z.double(), 0)[order]
    cut = int(torch.searchsorted(torch.cumsum(p, 0), torch.tensor(0.6, dtype=torch.float64))) 
    boundary = srt[cut]
    tp = torch.full((B,), 0.6, device=DEV)
    ids, _ = ops.sample(logits, t, None, tp, None, seeds)
    got = z[ids.long().cpu()]
    assert bool((got >= boundary - 1e-4).all())
    assert len(set(ids.tolist())) >= min(cut + 1, 50) // 2


def test_pool():
    h = torch.randn(50, 256, device=DEV, dtype=torch.bfloat16)
    cu = torch.tensor([0, 10, 50], dtype=torch.int32, device=DEV)
    _close(ops.pool(h, cu, 0, True), ref.pool(h, cu, 0, True), atol=1e-3)
    _close(ops.pool(h, cu, 1, True), ref.pool(h, cu, 1, True), atol=1e-3)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_penalties(dtype):
    B, V, S = 6, 128256, 9
    logits = (torch.randn(B, V, device=DEV) * 3).to(dtype)
    counts = torch.zeros(S, V, dtype=torch.int32, device=DEV)
    g = torch.Generator().manual_seed(0)
    for s in range(S):
        idx = torch.randint(0, V, (300,), generator=g)
        counts[s, idx[:200].to(DEV)] = ref.SEEN_BIT
        counts[s, idx[200:].to(DEV)] = ref.SEEN_BIT | torch.randint(1, 5, (100,), generator=g, dtype=torch.int32).to(DEV)
    slot = torch.tensor([3, 0, 8, 1, 5, 2], dtype=torch.int32, device=DEV)
    rep = torch.tensor([1.0, 1.3, 2.0, 1.0, 1.1, 1.0], device=DEV)
    freq = torch.tensor([0.0, 0.5, 0.0, 1.0, 0.2, 0.0], device=DEV)
    pres = torch.tensor([0.0, 0.25, 0.0, 0.0, 1.5, 0.0], device=DEV)
    want = logits.clone().cpu()
    ref.apply_penalties(want, counts.cpu(), slot.cpu(), rep.cpu(), freq.cpu(), pres.cpu())
    got = logits.clone()
    ops.apply_penalties(got, counts, slot, rep, freq, pres)
    _close(got, want, atol=1e-2 if dtype == torch.bfloat16 else 1e-5, rtol=1e-2)
    ids = torch.randint(0, V, (B,), dtype=torch.int32, device=DEV)
    cw = counts.cpu().clone()
    ref.update_counts(cw, slot.cpu(), ids.cpu(), rep.cpu(), freq.cpu(), pres.cpu())
    ops.update_counts(counts, slot, ids, rep, freq, pres)
    assert torch.equal(counts.cpu(), cw)


@pytest.mark.parametrize("D", [64, 256])
@pytest.mark.parametrize("softcap", [0.0, 50.0])
@pytest.mark.parametrize("variant", ["3", "4"])
def test_paged_decode_head_dims_softcap(D, softcap, variant, monkeypatch):
    """Head dims 64 (GPT-OSS class) / 256 (Gemma-2/3) and Gemma-2 attention-logit soft-capping."""
    monkeypatch.setenv("OME_DECODE_ATTN", variant)
    Hq, Hkv, P = 8, 4, 16
    seq_lens = [1, 37, 300, 1000]
    npages = sum(-(-L // P) for L in seq_lens) + 8
    kc, vc = _cache(npages, Hkv, D)
    kc, vc = kc * 3, vc
    bt = _block_tables(seq_lens, P, npages)
    sl = torch.tensor(seq_lens, dtype=torch.int32, device=DEV)
    q = torch.randn(len(seq_lens), Hq, D, device=DEV, dtype=torch.bfloat16) * 3
    ws = ops.DecodeWorkspace(len(seq_lens), Hq, D, 2048, 256, DEV)
    scale = D ** -0.5
    out = ops.paged_decode(q, kc, vc, bt, sl, scale, ws, softcap=softcap)
    _close(out, ref.paged_decode(q, kc, vc, bt, sl, scale, -1, 1.0, 1.0, softcap), atol=3e-2)
    out_w = ops.paged_decode(q, kc, vc, bt, sl, scale, ws, window=100, softcap=softcap)
    _close(out_w, ref.paged_decode(q, kc, vc, bt, sl, scale, 100, 1.0, 1.0, softcap), atol=3e-2)


@pytest.mark.parametrize("D", [64, 128, 256])
@pytest.mark.parametrize("softcap", [0.0, 30.0])
def test_paged_prefill_head_dims_softcap(D, softcap):
    Hq, Hkv, P = 8, 2, 16
    q_lens, kv_lens = [37, 64, 1, 100], [37, 80, 300, 100]
    npages = sum(-(-L // P) for L in kv_lens) + 8
    kc, vc = _cache(npages, Hkv, D)
    kc = kc * 3
    bt = _block_tables(kv_lens, P, npages)
    cu = torch.tensor([0] + list(torch.tensor(q_lens).cumsum(0)), dtype=torch.int32, device=DEV)
    kl = torch.tensor(kv_lens, dtype=torch.int32, device=DEV)
    items = torch.tensor(ops.prefill_work_items(q_lens, kv_lens), dtype=torch.int32, device=DEV)
    q = torch.randn(sum(q_lens), Hq, D, device=DEV, dtype=torch.bfloat16) * 3
    out = ops.paged_prefill(q, kc, vc, bt, cu, kl, items, D ** -0.5, window=64, softcap=softcap)
    _close(out, ref.paged_prefill(q, kc, vc, bt, cu, kl, D ** -0.5, 64, 1.0, 1.0, softcap), atol=3e-2)


@pytest.mark.parametrize("D", [64, 256])
def test_rope_qkv_cache_head_dims(D):
    from ome_amd.models.config import preset, rope_cos_sin

    Hq, Hkv, T, P = 8, 4, 19, 16
    cfg = preset("llama-3.1-8b")
    cfg.head_dim, cfg.partial_rotary_factor = D, 1.0
    cs = rope_cos_sin(cfg, 4096, device=DEV)
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
    pos = torch.randint(0, 4000, (T,), device=DEV, dtype=torch.int32)
    slots = torch.randperm(20 * P, device=DEV)[:T].to(torch.int32)
    k1, v1 = _cache(20, Hkv, D)
    k2, v2 = k1.clone(), v1.clone()
    q1 = torch.empty(T, Hq, D, device=DEV, dtype=torch.bfloat16)
    q2 = torch.empty_like(q1)
    ops.rope_qkv_cache(qkv, pos, cs, D, q1, k1, v1, slots, Hq, Hkv, D)
    ref.rope_qkv_cache(qkv, pos, cs, D, q2, k2, v2, slots, Hq, Hkv, D, P)
    _close(q1, q2, atol=3e-2)
    _close(k1, k2, atol=3e-2)
    assert torch.equal(v1, v2)


@pytest.mark.parametrize("D", [64, 128])
@pytest.mark.parametrize("parts", [4096, 256])
def test_paged_attention_sinks(D, parts):
    """GPT-OSS attention sinks in decode (incl. split-K reduce) and prefill."""
    Hq, Hkv, P = 16, 2, 16
    seq_lens = [1, 37, 300, 1000]
    npages = sum(-(-L // P) for L in seq_lens) + 8
    kc, vc = _cache(npages, Hkv, D)
    bt = _block_tables(seq_lens, P, npages)
    sl = torch.tensor(seq_lens, dtype=torch.int32, device=DEV)
    sinks = torch.randn(Hq, device=DEV, dtype=torch.float32) * 2
    q = torch.randn(len(seq_lens), Hq, D, device=DEV, dtype=torch.bfloat16)
    ws = ops.DecodeWorkspace(len(seq_lens), Hq, D, 2048, parts, DEV)
    out = ops.paged_decode(q, kc, vc, bt, sl, D ** -0.5, ws, window=128, sinks=sinks)
    _close(out, ref.paged_decode(q, kc, vc, bt, sl, D ** -0.5, 128, 1.0, 1.0, 0.0, sinks), atol=2e-2)
    q_lens = [37, 64, 1, 100]
    kv_lens = [37, 80, 300, 100]
    cu = torch.tensor([0] + list(torch.tensor(q_lens).cumsum(0)), dtype=torch.int32, device=DEV)
    kl = torch.tensor(kv_lens, dtype=torch.int32, device=DEV)
    items = torch.tensor(ops.prefill_work_items(q_lens, kv_lens), dtype=torch.int32, device=DEV)
    bt2 = _block_tables(kv_lens, P, npages)
    qp = torch.randn(sum(q_lens), Hq, D, device=DEV, dtype=torch.bfloat16)
    outp = ops.paged_prefill(qp, kc, vc, bt2, cu, kl, items, D ** -0.5, sinks=sinks)
    _close(outp, ref.paged_prefill(qp, kc, vc, bt2, cu, kl, D ** -0.5, -1, 1.0, 1.0, 0.0, sinks), atol=2e-2)


def test_fused_moe_bias_and_gptoss_act():
    T, H, I, E, k = 37, 256, 128, 8, 4
    x = torch.randn(T, H, device=DEV, dtype=torch.bfloat16)
    w13 = torch.randn(E, 2 * I, H, device=DEV, dtype=torch.bfloat16) * 0.1
    w2 = torch.randn(E, H, I, device=DEV, dtype=torch.bfloat16) * 0.1
    b13 = torch.randn(E, 2 * I, device=DEV, dtype=torch.bfloat16)
    b2 = torch.randn(E, H, device=DEV, dtype=torch.bfloat16)
    logits = torch.randn(T, E, device=DEV, dtype=torch.bfloat16)
    tw, tid = ops.moe_route(logits, k, True)
    out = ops.fused_moe(x, tw, tid, w13, w2, 2, 1.0, b13, b2)
    _close(out, ref.fused_moe(x, tw, tid, w13, w2, 2, 1.0, b13, b2), atol=5e-2, rtol=5e-2)


@pytest.mark.parametrize("D,Hq,Hkv", [(64, 16, 2), (128, 32, 8), (128, 5, 5), (256, 8, 1)])
@pytest.mark.parametrize("parts", [4096, 256])
def test_paged_attention_alibi(D, Hq, Hkv, parts):
    """ALiBi slopes (Bloom / MPT) in every decode variant (incl. split-K) and both prefill kernels
    (v2 for GQA-4 at D=128, v1 otherwise), against the fp32 reference."""
    from ome_amd.models.decoder import alibi_slopes

    P = 16
    seq_lens = [1, 37, 300, 1000]
    npages = sum(-(-L // P) for L in seq_lens) + 8
    kc, vc = _cache(npages, Hkv, D)
    bt = _block_tables(seq_lens, P, npages)
    sl = torch.tensor(seq_lens, dtype=torch.int32, device=DEV)
    al = alibi_slopes(Hq, "bloom").to(DEV)
    q = torch.randn(len(seq_lens), Hq, D, device=DEV, dtype=torch.bfloat16)
    ws = ops.DecodeWorkspace(len(seq_lens), Hq, D, 2048, parts, DEV)
    want = ref.paged_decode(q, kc, vc, bt, sl, D ** -0.5, -1, 1.0, 1.0, 0.0, None, al)
    for variant in ("1", "2", "3", "4"):
        os.environ["OME_DECODE_ATTN"] = variant
        try:
            out = ops.paged_decode(q, kc, vc, bt, sl, D ** -0.5, ws, alibi=al)
        finally:
            os.environ.pop("OME_DECODE_ATTN")
        _close(out, want, atol=2e-2)
    q_lens = [37, 64, 1, 100]
    kv_lens = [37, 80, 300, 100]
    cu = torch.tensor([0] + list(torch.tensor(q_lens).cumsum(0)), dtype=torch.int32, device=DEV)
    kl = torch.tensor(kv_lens, dtype=torch.int32, device=DEV)
    items = torch.tensor(ops.prefill_work_items(q_lens, kv_lens), dtype=torch.int32, device=DEV)
    bt2 = _block_tables(kv_lens, P, npages)
    qp = torch.randn(sum(q_lens), Hq, D, device=DEV, dtype=torch.bfloat16)
    outp = ops.paged_prefill(qp, kc, vc, bt2, cu, kl, items, D ** -0.5, alibi=al)
    _close(outp, ref.paged_prefill(qp, kc, vc, bt2, cu, kl, D ** -0.5, -1, 1.0, 1.0, 0.0, None, al), atol=2e-2)


@pytest.mark.parametrize("parts", [2, 5, 8])
@pytest.mark.parametrize("window", [-1, 128])
def test_paged_decode_dynamic_partitions(parts, window):
    """part_size 0: every sequence split into ``parts`` spans of its own length (the decode graphs'
    small-batch workspace), incl. sinks / sliding window and lengths below one 128-key granule."""
    Hq, Hkv, D, P = 32, 8, 128, 16
    seq_lens = [1, 17, 127, 128, 129, 630, 1000, 2049]
    npages = sum(-(-L // P) for L in seq_lens) + 4
    kc, vc = _cache(npages, Hkv, D)
    bt = _block_tables(seq_lens, P, npages)
    sl = torch.tensor(seq_lens, dtype=torch.int32, device=DEV)
    q = torch.randn(len(seq_lens), Hq, D, device=DEV, dtype=torch.bfloat16)
    ws = ops.DecodeWorkspace(len(seq_lens), Hq, D, 4096, 0, DEV, parts=parts)
    sinks = torch.randn(Hq, device=DEV, dtype=torch.float32)
    for sk in (None, sinks):
        out = ops.paged_decode(q, kc, vc, bt, sl, D ** -0.5, ws, window=window, sinks=sk)
        _close(out, ref.paged_decode(q, kc, vc, bt, sl, D ** -0.5, window, 1.0, 1.0, 0.0, sk), atol=2e-2)


@pytest.mark.parametrize("q_lens,kv_lens", [([5], [5]), ([37, 64, 1, 100], [37, 80, 300, 100]),
                                            ([300], [1000]), ([1000], [1000]), ([100, 64], [164, 64])])
@pytest.mark.parametrize("window", [-1, 100])
def test_paged_prefill_64_row_items(q_lens, kv_lens, window):
    """8-wave GQA-4 prefill over 64-row items (ops.PrefillPlan rows=64) == the fp32 reference."""
    D, P, Hq, Hkv = 128, 16, 32, 8
    npages = sum(-(-L // P) for L in kv_lens) + 8
    kc, vc = _cache(npages, Hkv, D)
    bt = _block_tables(kv_lens, P, npages)
    cu = torch.tensor([0] + list(torch.tensor(q_lens).cumsum(0)), dtype=torch.int32, device=DEV)
    kl = torch.tensor(kv_lens, dtype=torch.int32, device=DEV)
    items = torch.tensor(ops.prefill_work_items(q_lens, kv_lens, 64), dtype=torch.int32, device=DEV)
    plan = ops.PrefillPlan(items, items[:0], items[:0], 0, 0, 64)
    q = torch.randn(sum(q_lens), Hq, D, device=DEV, dtype=torch.bfloat16)
    out = ops.paged_prefill(q, kc, vc, bt, cu, kl, plan, 0.0884, window=window)
    _close(out, ref.paged_prefill(q, kc, vc, bt, cu, kl, 0.0884, window), atol=2e-2)


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 1)])   # GQA-4 (the v2 prefill kernel) and G = 8 (generic)
@pytest.mark.parametrize("bs", [(64, 16, 8, 1, 0), (64, 4, 8, 1, 32), (16, 2, 3, 0, 0), (128, 3, 4, 1, 5)])
def test_blocksparse_prefill_decode(Hq, Hkv, bs):
    """Phi-3-small block-sparse causal attention (local band + per-head vertical stripes) in the
    paged prefill (classic, 64-row and split-KV plans: the FAST body skipping invisible stages for
    blocks >= 64 keys, the generic masked body below) and decode kernels == the fp32 reference."""
    D, P = 128, 16
    q_lens, kv_lens = [1500, 37, 300], [1500, 1200, 2100]
    npages = sum(-(-L // P) for L in kv_lens) + 8
    kc, vc = _cache(npages, Hkv, D)
    bt = _block_tables(kv_lens, P, npages)
    cu = torch.tensor([0] + list(torch.tensor(q_lens).cumsum(0)), dtype=torch.int32, device=DEV)
    kl = torch.tensor(kv_lens, dtype=torch.int32, device=DEV)
    q = torch.randn(sum(q_lens), Hq, D, device=DEV, dtype=torch.bfloat16)
    want = ref.paged_prefill(q, kc, vc, bt, cu, kl, 0.0884, blocksparse=bs)
    items = torch.tensor(ops.prefill_work_items(q_lens, kv_lens), dtype=torch.int32, device=DEV)
    _close(ops.paged_prefill(q, kc, vc, bt, cu, kl, items, 0.0884, blocksparse=bs), want, atol=2e-2)
    if Hq == 4 * Hkv:
        _close(ops.paged_prefill(q, kc, vc, bt, cu, kl, _plan(q_lens, kv_lens, 128), 0.0884, blocksparse=bs), want,
               atol=2e-2)
        it64 = torch.tensor(ops.prefill_work_items(q_lens, kv_lens, 64), dtype=torch.int32, device=DEV)
        plan64 = ops.PrefillPlan(it64, it64[:0], it64[:0], 0, 0, 64)
        _close(ops.paged_prefill(q, kc, vc, bt, cu, kl, plan64, 0.0884, blocksparse=bs), want, atol=2e-2)
    assert not torch.allclose(want, ref.paged_prefill(q, kc, vc, bt, cu, kl, 0.0884), atol=1e-2)   # mask bites
    qd = torch.randn(len(kv_lens), Hq, D, device=DEV, dtype=torch.bfloat16)
    ws = ops.DecodeWorkspace(len(kv_lens), Hq, D, 4096, 256, DEV)
    _close(ops.paged_decode(qd, kc, vc, bt, kl, 0.0884, ws, blocksparse=bs),
           ref.paged_decode(qd, kc, vc, bt, kl, 0.0884, blocksparse=bs), atol=2e-2)
