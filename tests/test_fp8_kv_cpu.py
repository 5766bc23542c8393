"""FP8 KV cache (K15, ``--kv-cache-dtype fp8 / fp8_e4m3 / fp8_e5m2``): reference semantics and the
CPU engine path.  The reference (``ome_amd.ops.reference``) defines what the HIP kernels must
reproduce: cache entry = saturate(bf16(x) / scale) in OCP fp8, attention reads entry * scale.
Parity with SGLang's fp8 KV cache is unpinned (no engine in the image); the checks below pin
the semantics against the bf16 cache instead."""
import math

import pytest
import torch

from ome_amd import ops
from ome_amd.models.common import PagedKVCache, kv_cache_dtype
from ome_amd.ops import reference as ref
from ome_amd.runtime.engine import Engine, EngineArgs
from ome_amd.runtime.request import SamplingParams

FP8 = [torch.float8_e4m3fn, torch.float8_e5m2]


def test_kv_cache_dtype_names():
    assert kv_cache_dtype("auto") is torch.bfloat16
    assert kv_cache_dtype("fp8") is torch.float8_e4m3fn
    assert kv_cache_dtype("fp8_e4m3") is torch.float8_e4m3fn
    assert kv_cache_dtype("fp8_e5m2") is torch.float8_e5m2
    with pytest.raises(ValueError):
        kv_cache_dtype("int4")
    assert ops.kv_format(torch.zeros(1, dtype=torch.float8_e5m2)) == 2


@pytest.mark.parametrize("dt", FP8)
def test_to_cache_saturates_and_scales(dt):
    x = torch.tensor([0.0, 1.0, -3.5, 1e6, -1e6, 0.1])
    q = ref.to_cache(x, dt, scale=2.0)
    m = ref.FP8_RANGE[dt]
    back = q.float()
    assert torch.isfinite(back).all()
    assert back[3] == m and back[4] == -m
    assert abs(back[1] - 0.5) < 1e-6 and abs(back[2] + 1.75) < 1e-6


@pytest.mark.parametrize("dt", FP8)
def test_fp8_cache_write_and_decode_match_dequantised_bf16(dt):
    torch.manual_seed(0)
    T, Hkv, Hq, D, P = 40, 2, 8, 128, 16
    k = torch.randn(T, Hkv, D).to(torch.bfloat16)
    v = torch.randn(T, Hkv, D).to(torch.bfloat16)
    slots = torch.arange(T, dtype=torch.int32)
    kc8 = torch.zeros(4, Hkv, P, D, dtype=dt)
    vc8 = torch.zeros(4, Hkv, D, P, dtype=dt)
    ks, vs = 0.5, 0.25
    ops.kv_cache_write(k, v, kc8, vc8, slots, ks, vs)
    # a bf16 cache holding exactly the dequantised fp8 entries
    kcb, vcb = (kc8.float() * ks).to(torch.bfloat16), (vc8.float() * vs).to(torch.bfloat16)
    bt = torch.arange(4, dtype=torch.int32).view(1, 4).repeat(2, 1)
    sl = torch.tensor([T, 17], dtype=torch.int32)
    q = torch.randn(2, Hq, D).to(torch.bfloat16)
    scale = 1 / math.sqrt(D)
    a = ops.paged_decode(q, kc8, vc8, bt, sl, scale, k_scale=ks, v_scale=vs)
    b = ops.paged_decode(q, kcb, vcb, bt, sl, scale)
    assert torch.allclose(a.float(), b.float(), atol=2e-2)
    # and the fp8 result tracks the unquantised cache within fp8 noise
    kc, vc = torch.zeros(4, Hkv, P, D, dtype=torch.bfloat16), torch.zeros(4, Hkv, D, P, dtype=torch.bfloat16)
    ops.kv_cache_write(k, v, kc, vc, slots)
    c = ops.paged_decode(q, kc, vc, bt, sl, scale)
    tol = 0.08 if dt == torch.float8_e4m3fn else 0.2
    assert (a.float() - c.float()).abs().max() < tol


def test_paged_cache_bytes_and_scales():
    c = PagedKVCache(2, 8, 2, 128, 16, torch.float8_e4m3fn, "cpu")
    assert c.is_fp8 and c.k[0].element_size() == 1
    assert PagedKVCache.bytes_per_page(2, 2, 128, 16, torch.float8_e4m3fn) * 2 == \
        PagedKVCache.bytes_per_page(2, 2, 128, 16, torch.bfloat16)
    c.set_scales({1: (0.5, 2.0)})
    assert c.scales(0) == (1.0, 1.0) and c.scales(1) == (0.5, 2.0)


@pytest.mark.parametrize("name", ["fp8_e4m3", "fp8_e5m2"])
def test_engine_with_fp8_kv_cache(name):
    kw = dict(model="tiny-llama", device="cpu", max_running_requests=4, context_length=256, seed=0,
              chunked_prefill_size=32)
    e8 = Engine(EngineArgs(kv_cache_dtype=name, **kw))
    assert e8.runner.kv.dtype == kv_cache_dtype(name)
    prompts = [list(range(3, 40)), [5, 6, 7]]
    sp = SamplingParams(max_new_tokens=6, ignore_eos=True)
    r8 = e8.generate(prompts, sp)
    assert all(len(r.output_ids) == 6 for r in r8)
    eb = Engine(EngineArgs(**kw))
    rb = eb.generate(prompts, sp)
    # the first token only depends on the prefill (attention over the freshly quantised prompt)
    agree = sum(int(a.output_ids[0] == b.output_ids[0]) for a, b in zip(r8, rb))
    assert agree >= 1
