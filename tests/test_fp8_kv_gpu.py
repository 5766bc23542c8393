"""FP8 KV cache on gfx950: the write kernels must produce the reference's fp8 bytes, and every
attention kernel reading an fp8 cache must match the fp32 reference over the same bytes."""
import math

import pytest
import torch

from ome_amd import ops
from ome_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
FP8 = [torch.float8_e4m3fn, torch.float8_e5m2]


def _close(a, b, atol=2e-2, rtol=2e-2):
    a, b = a.float().cpu(), b.float().cpu()
    assert torch.allclose(a, b, atol=atol, rtol=rtol), f"max abs err {(a - b).abs().max().item()}"


def _fp8_cache(pages, Hkv, D, dt, P=16):
    k = (torch.randn(pages, Hkv, P, D, device=DEV) * 2).to(dt)
    v = (torch.randn(pages, Hkv, D, P, device=DEV) * 2).to(dt)
    return k, v


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


@pytest.fixture(autouse=True)
def _seed():
    torch.manual_seed(0)


@pytest.mark.parametrize("dt", FP8)
def test_rope_qkv_cache_fp8(dt):
    from ome_amd.models.config import preset, rope_cos_sin

    Hq, Hkv, D, T, P = 32, 8, 128, 29, 16
    cfg = preset("llama-3.1-8b")
    cs = rope_cos_sin(cfg, 4096, device=DEV)
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=DEV, dtype=torch.bfloat16)
    pos = torch.randint(0, 4000, (T,), device=DEV, dtype=torch.int32)
    slots = torch.randperm(40 * P, device=DEV)[:T].to(torch.int32)
    slots[2] = -1
    k1 = torch.zeros(40, Hkv, P, D, device=DEV, dtype=dt)
    v1 = torch.zeros(40, Hkv, D, P, device=DEV, dtype=dt)
    k2, v2 = k1.clone(), v1.clone()
    q1 = torch.empty(T, Hq, D, device=DEV, dtype=torch.bfloat16)
    q2 = torch.empty_like(q1)
    ops.rope_qkv_cache(qkv, pos, cs, D, q1, k1, v1, slots, Hq, Hkv, D, True, None, None, 1e-6, 0.5, 0.75)
    ref.rope_qkv_cache(qkv, pos, cs, D, q2, k2, v2, slots, Hq, Hkv, D, P, True, None, None, 1e-6, 0.5, 0.75)
    _close(q1, q2, atol=3e-2)
    # V is a pure quantisation of the same bf16 values (x * (1/s) vs x / s may flip a rounding tie)
    _close(v1.float(), v2.float(), atol=0.02, rtol=0.26)
    # K went through RoPE in fp32 on both sides; allow one fp8 ulp on a few entries
    _close(k1.float(), k2.float(), atol=0.02, rtol=0.26)


@pytest.mark.parametrize("dt", FP8)
def test_kv_cache_write_fp8(dt):
    T, Hkv, D, P = 50, 8, 128, 16
    k = torch.randn(T, Hkv, D, device=DEV, dtype=torch.bfloat16) * 3
    v = torch.randn(T, Hkv, D, device=DEV, dtype=torch.bfloat16) * 3
    slots = torch.randperm(8 * P, device=DEV)[:T].to(torch.int32)
    a = [torch.zeros(8, Hkv, P, D, device=DEV, dtype=dt), torch.zeros(8, Hkv, D, P, device=DEV, dtype=dt)]
    b = [x.clone() for x in a]
    ops.kv_cache_write(k, v, a[0], a[1], slots, 0.25, 2.0)
    ref.kv_cache_write(k, v, b[0], b[1], slots, P, 0.25, 2.0)
    # multiply-by-inverse vs divide can flip a round-to-nearest tie: compare values, not bytes
    _close(a[0].float(), b[0].float(), atol=0.02, rtol=0.26)
    _close(a[1].float(), b[1].float(), atol=0.02, rtol=0.26)


@pytest.mark.parametrize("dt", FP8)
@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 1), (64, 8)])
@pytest.mark.parametrize("seq_lens", [[1], [15, 16, 17, 33], [100, 1000, 3, 517]])
@pytest.mark.parametrize("variant", ["2", "3", "4"])
def test_paged_decode_fp8(dt, Hq, Hkv, seq_lens, variant, monkeypatch):
    monkeypatch.setenv("OME_DECODE_ATTN", variant)
    D, P = 128, 16
    npages = sum(-(-L // P) for L in seq_lens) + 8
    kc, vc = _fp8_cache(npages, Hkv, D, dt)
    bt = _block_tables(seq_lens, P, npages)
    sl = torch.tensor(seq_lens, dtype=torch.int32, device=DEV)
    q = torch.randn(len(seq_lens), Hq, D, device=DEV, dtype=torch.bfloat16)
    ws = ops.DecodeWorkspace(len(seq_lens), Hq, D, 2048, 256, DEV)
    scale = 1 / math.sqrt(D)
    out = ops.paged_decode(q, kc, vc, bt, sl, scale, ws, k_scale=0.3, v_scale=0.7)
    _close(out, ref.paged_decode(q, kc, vc, bt, sl, scale, -1, 0.3, 0.7), atol=2e-2)


@pytest.mark.parametrize("dt", FP8)
@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (8, 1)])
@pytest.mark.parametrize("q_lens,kv_lens", [([37, 64, 1, 100], [37, 80, 300, 100]), ([300], [1000])])
@pytest.mark.parametrize("variant", ["1", "2"])
def test_paged_prefill_fp8(dt, Hq, Hkv, q_lens, kv_lens, variant, monkeypatch):
    monkeypatch.setenv("OME_PREFILL_ATTN", variant)
    D, P = 128, 16
    npages = sum(-(-L // P) for L in kv_lens) + 8
    kc, vc = _fp8_cache(npages, Hkv, D, dt)
    bt = _block_tables(kv_lens, P, npages)
    cu = torch.tensor([0] + list(torch.tensor(q_lens).cumsum(0)), dtype=torch.int32, device=DEV)
    kl = torch.tensor(kv_lens, dtype=torch.int32, device=DEV)
    items = torch.tensor(ops.prefill_work_items(q_lens, kv_lens), dtype=torch.int32, device=DEV)
    q = torch.randn(sum(q_lens), Hq, D, device=DEV, dtype=torch.bfloat16)
    out = ops.paged_prefill(q, kc, vc, bt, cu, kl, items, 0.0884, k_scale=0.3, v_scale=0.7)
    _close(out, ref.paged_prefill(q, kc, vc, bt, cu, kl, 0.0884, -1, 0.3, 0.7), atol=2e-2)


def test_engine_fp8_kv_cache_graphs():
    from ome_amd.runtime.engine import Engine, EngineArgs
    from ome_amd.runtime.request import SamplingParams

    eng = Engine(EngineArgs(model="tiny-llama", device="cuda", max_running_requests=8, context_length=512,
                            kv_cache_dtype="fp8_e4m3"))
    assert eng.runner.kv.dtype == torch.float8_e4m3fn and eng.runner.use_graph
    reqs = eng.generate([[5, 6, 7, 8], list(range(10, 90))], SamplingParams(max_new_tokens=10, ignore_eos=True))
    assert all(len(r.output_ids) == 10 for r in reqs)
