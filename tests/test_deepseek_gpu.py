"""MLA attention kernel (csrc/kernels/mla.hip), grouped routing, and the DeepSeek model on the GPU."""
import random

import pytest
import torch

from ome_amd import ops
from ome_amd.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup(lens, seed=0, dk=576):
    g = torch.Generator().manual_seed(seed)
    pages_per_row = -(-max(lens) // 16) + 1
    num_pages = len(lens) * pages_per_row + 1
    cache = (torch.randn(num_pages, 16, dk, generator=g) * 0.5).to(torch.bfloat16)
    rows = len(lens)
    perm = torch.randperm(num_pages - 1, generator=g)[: rows * pages_per_row] + 1
    bt = perm.view(rows, pages_per_row).to(torch.int32)
    return cache.to(DEV), bt.to(DEV)


@pytest.mark.parametrize("H", [16, 32, 128])
@pytest.mark.parametrize("lens", [[1], [17, 33, 1000, 5], [64] * 40, [1280, 31]])
def test_mla_decode(H, lens):
    cache, bt = _setup(lens)
    T = len(lens)
    q = (torch.randn(T, H, 576, device=DEV) * 0.3).to(torch.bfloat16)
    rows = torch.arange(T, dtype=torch.int32, device=DEV)
    kl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    out = ops.mla_attn(q, cache, bt, rows, kl, 0.0723)
    want = ref.mla_attn(q.cpu(), cache.cpu(), bt.cpu(), rows.cpu(), kl.cpu(), 0.0723)
    err = (out.float().cpu() - want.float()).abs().max().item()
    assert err < 2e-2, err


@pytest.mark.parametrize("H", [16, 64])
def test_mla_prefill_causal(H):
    # two sequences, chunked: seq 0 has 100 cached tokens + 150 new, seq 1 is a fresh 90-token prompt
    cache, bt = _setup([250, 90])
    q_lens, starts = [150, 90], [100, 0]
    tok_row, kv = [], []
    for s, (n, st) in enumerate(zip(q_lens, starts)):
        tok_row += [s] * n
        kv += [st + j + 1 for j in range(n)]
    T = len(tok_row)
    q = (torch.randn(T, H, 576, device=DEV) * 0.3).to(torch.bfloat16)
    rows = torch.tensor(tok_row, dtype=torch.int32, device=DEV)
    kl = torch.tensor(kv, dtype=torch.int32, device=DEV)
    out = ops.mla_attn(q, cache, bt, rows, kl, 0.0723)
    want = ref.mla_attn(q.cpu(), cache.cpu(), bt.cpu(), rows.cpu(), kl.cpu(), 0.0723)
    assert (out.float().cpu() - want.float()).abs().max().item() < 2e-2


@pytest.mark.parametrize("H", [40, 16, 8])
@pytest.mark.parametrize("lens", [[1], [17, 33, 1000, 5], [64] * 40])
def test_mla_minicpm3_shape(H, lens):
    """(kv_lora_rank 256 | rope 32) latent rows, head counts that are not a multiple of 16."""
    cache, bt = _setup(lens, dk=288)
    T = len(lens)
    q = (torch.randn(T, H, 288, device=DEV) * 0.3).to(torch.bfloat16)
    rows = torch.arange(T, dtype=torch.int32, device=DEV)
    kl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    out = ops.mla_attn(q, cache, bt, rows, kl, 0.0723, dv=256)
    want = ref.mla_attn(q.cpu(), cache.cpu(), bt.cpu(), rows.cpu(), kl.cpu(), 0.0723, 256)
    assert out.shape == (T, H, 256)
    assert (out.float().cpu() - want.float()).abs().max().item() < 2e-2


@pytest.mark.parametrize("mode,scoring", [(0, "softmax"), (1, "softmax"), (2, "sigmoid")])
def test_grouped_route(mode, scoring):
    torch.manual_seed(3)
    T, E = 300, 256
    logits = torch.randn(T, E, device=DEV) * 2
    bias = (torch.randn(E, device=DEV) * 0.05) if mode == 2 else None
    w, ids = ops.moe_route(logits, 8, True, scoring, bias=bias, n_group=8, topk_group=4, group_mode=mode)
    rw, rids = ref.moe_route(logits.cpu(), 8, True, scoring, bias.cpu() if bias is not None else None, 8, 4, mode)
    a = torch.sort(ids.cpu().long(), -1).values
    b = torch.sort(rids.long(), -1).values
    assert (a == b).float().mean().item() > 0.995
    assert torch.allclose(torch.sort(w.cpu(), -1).values, torch.sort(rw, -1).values, atol=1e-4)


def test_deepseek_engine_gpu():
    from ome_amd.runtime.engine import Engine, EngineArgs
    from ome_amd.runtime.request import SamplingParams

    eng = Engine(EngineArgs(model="tiny-deepseek", max_running_requests=8, context_length=512))
    rng = random.Random(0)
    prompts = [[rng.randrange(3, 1000) for _ in range(rng.randrange(3, 200))] for _ in range(6)]
    prompts.append(prompts[0])
    reqs = eng.generate(prompts, SamplingParams(max_new_tokens=16, temperature=0.0, ignore_eos=True))
    eng.flush()
    assert all(len(r.output_ids) == 16 for r in reqs)
    assert reqs[0].output_ids == reqs[-1].output_ids


def test_deepseek_gpu_vs_cpu_logits():
    from ome_amd.models import build_model
    from ome_amd.models.config import preset
    from tests.test_deepseek_cpu import _kv, _meta_prefill

    cfg = preset("tiny-deepseek")
    a = build_model(cfg, "cpu", torch.float32, load_format="dummy", seed=2)
    b = build_model(cfg, DEV, torch.bfloat16, load_format="dummy", seed=2)
    # same random weights on both devices (generators differ per device): copy CPU -> GPU
    for name, v in vars(a).items():
        if isinstance(v, list) and v and any(isinstance(t, torch.Tensor) for t in v):
            setattr(b, name, [t.to(DEV, torch.float32 if t.dtype == torch.float32 and name == "b_router"
                                   else torch.bfloat16) if isinstance(t, torch.Tensor) else t for t in v])
    for name in ("embed", "norm", "lm_head"):
        setattr(b, name, getattr(a, name).to(DEV, torch.bfloat16))
    ids = list(range(3, 40))
    la = a.compute_logits(a.forward(torch.tensor(ids, dtype=torch.int32), _meta_prefill(len(ids)), _kv(a)))
    meta = _meta_prefill(len(ids))
    for f in ("positions", "slots", "block_tables", "cu_q", "kv_lens", "items"):
        setattr(meta, f, getattr(meta, f).to(DEV))
    hk, dk, dv = b.kv_layout
    from ome_amd.models.common import PagedKVCache

    kvb = PagedKVCache(cfg.num_layers, 8, hk, dk, 16, torch.bfloat16, DEV, dv)
    lb = b.compute_logits(b.forward(torch.tensor(ids, dtype=torch.int32, device=DEV), meta, kvb)).float().cpu()
    cos = torch.nn.functional.cosine_similarity(la, lb, dim=-1)
    assert cos.min().item() > 0.99, cos.min()


@pytest.mark.parametrize("qlr,lat,rope,H,nope", [(1536, 512, 64, 16, 128), (768, 256, 32, 8, 64), (0, 512, 64, 4, 128)])
def test_mla_prep_matches_reference(qlr, lat, rope, H, nope):
    """Fused kv_a_layernorm + RoPE(k_pe) cache write + RoPE(q_pe) (``ome_mla_prep``) against the
    eager fp32 reference path, including a padding row (slot -1 -> scratch row 0)."""
    torch.manual_seed(qlr + lat)
    T, npos = 37, 4096
    a = torch.randn(T, qlr + lat + rope, dtype=torch.bfloat16)
    w = (1 + 0.1 * torch.randn(lat)).to(torch.bfloat16)
    q = torch.randn(T, H, nope + rope, dtype=torch.bfloat16)
    pos = torch.randint(0, npos, (T,), dtype=torch.int32)
    ang = torch.arange(npos)[:, None].float() * (1.0 / 10000 ** (torch.arange(0, rope, 2).float() / rope))[None]
    cs = torch.cat([ang.cos(), ang.sin()], -1).contiguous()
    slots = torch.randperm(200)[:T].to(torch.int32) + 1
    slots[5] = -1
    outs = []
    for dev in ("cpu", "cuda"):
        flat = torch.zeros(256, lat + rope, dtype=torch.bfloat16, device=dev)
        qf = torch.zeros(T, H, lat + rope, dtype=torch.bfloat16, device=dev)
        ops.mla_prep(a.to(dev), qlr, lat, rope, w.to(dev), 1e-6, pos.to(dev), cs.to(dev), slots.to(dev), flat,
                     q.to(dev), nope, qf)
        outs.append((flat.float().cpu(), qf.float().cpu()))
    (f0, q0), (f1, q1) = outs
    assert (f1 - f0).abs().max().item() <= 2e-2 * max(1.0, f0.abs().max().item())
    assert (q1[:, :, lat:] - q0[:, :, lat:]).abs().max().item() <= 2e-2 * max(1.0, q0.abs().max().item())
    assert f1[0].abs().sum() > 0   # the padding row landed in the scratch row
