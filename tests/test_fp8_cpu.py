"""FP8 W8A8 (K8): quantisers, checkpoint streaming (per-tensor / per-channel / 128x128 block
scales) and end-to-end model numerics on CPU against the bf16 model."""
import json

import pytest
import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.io.safetensors import save_file
from ome_amd.models import build_model
from ome_amd.models.config import PRESETS, ModelConfig
from ome_amd.models.quant import Fp8Weight, dequant_fp8_stream, linear, quantize_weight
from ome_amd.ops import reference as ref
from tests.test_moe_cpu import _forward


def test_quantize_weight_per_channel_error():
    w = torch.randn(256, 384) * torch.linspace(0.01, 3, 256)[:, None]
    qw = quantize_weight(w)
    assert qw.q.dtype == torch.float8_e4m3fn and qw.scale.shape == (256,)
    rel = (qw.dequant(torch.float32) - w).abs() / w.abs().amax(-1, keepdim=True)
    assert rel.max() <= 2 ** -4 + 1e-6  # half an e4m3 ulp at the top binade


def test_block_quant_round_trip_is_exact():
    w = torch.randn(320, 256)
    a = quantize_weight(w, 128)
    assert a.scale.shape == (3, 2)
    b = quantize_weight(a.dequant(torch.float32), 128)
    assert torch.equal(a.q.view(torch.uint8), b.q.view(torch.uint8)) and torch.allclose(a.scale, b.scale)


@pytest.mark.parametrize("block", [0, 128])
def test_fp8_linear_matches_bf16(block):
    x = torch.randn(37, 512)
    w = torch.randn(192, 512) * 0.05
    y = linear(x, quantize_weight(w, block))
    want = F.linear(x, w)
    assert (y.float() - want).norm() / want.norm() < 0.06


def test_activation_group_quant():
    x = torch.randn(5, 256)
    x[:, 200] = 50.0  # an outlier only affects its own 128-group under group quant
    q, s = ref.fp8_quant(x, 128)
    assert s.shape == (5, 2) and (s[:, 1] > 10 * s[:, 0]).all()
    q1, s1 = ops.fp8_quant(x, 0)
    assert s1.shape == (5, 1)


def test_dequant_stream_scale_kinds():
    w = torch.randn(256, 128)
    pc = quantize_weight(w)
    blk = quantize_weight(w, 128)
    per_tensor_s = w.abs().max() / 448
    pt_q = (w / per_tensor_s).to(torch.float8_e4m3fn)
    stream = [("a.weight_scale", pc.scale), ("a.weight", pc.q), ("b.weight", blk.q), ("b.weight_scale_inv", blk.scale),
              ("c.weight", pt_q), ("c.weight_scale", per_tensor_s.reshape(1)), ("c.input_scale", torch.ones(1)),
              ("n.weight", torch.ones(3))]
    out = dict(dequant_fp8_stream(iter(stream), 128, torch.float32))
    assert set(out) == {"a.weight", "b.weight", "c.weight", "n.weight"}
    for k in ("a.weight", "b.weight", "c.weight"):
        assert (out[k] - w).abs().max() < 0.07 * w.abs().max()
    with pytest.raises(ValueError):
        list(dequant_fp8_stream(iter([("x.weight", pc.q)]), 0))


def _cfg(quant=None, block=False):
    hf = dict(PRESETS["tiny-llama"])
    if quant:
        hf["quantization_config"] = {"quant_method": "fp8", "activation_scheme": "dynamic",
                                     **({"weight_block_size": [128, 128]} if block else {})}
    return hf


def test_fp8_model_close_to_bf16():
    ids = [3, 14, 15, 92, 65, 35, 89, 79]
    a = build_model(ModelConfig.from_hf(_cfg()), "cpu", torch.bfloat16, load_format="dummy", seed=5)
    b = build_model(ModelConfig.from_hf(_cfg("fp8")), "cpu", torch.bfloat16, load_format="dummy", seed=5)
    assert all(isinstance(b.w_qkv[i], Fp8Weight) and isinstance(b.w_d[i], Fp8Weight) for i in b.layers)
    assert b.weight_bytes() < a.weight_bytes()
    la, lb = _forward(a, ids).float(), _forward(b, ids).float()
    cos = F.cosine_similarity(la, lb, dim=-1)
    assert cos.min() > 0.98


def test_block_fp8_checkpoint_load(tmp_path):
    """A DeepSeek-style checkpoint (fp8 weights + 128x128 weight_scale_inv) loads to the same
    W8A8 model as online block quantisation of the bf16 weights."""
    src = build_model(ModelConfig.from_hf(_cfg()), "cpu", torch.bfloat16, load_format="dummy", seed=7)
    D, tp = src.D, src.tp
    t = {"model.embed_tokens.weight": src.embed, "model.norm.weight": src.norm, "lm_head.weight": src.lm_head}

    def put_fp8(name, w):
        qw = quantize_weight(w, 128)
        t[name + ".weight"] = qw.q
        t[name + ".weight_scale_inv"] = qw.scale

    for i in src.layers:
        p = f"model.layers.{i}."
        q, k, v = torch.split(src.w_qkv[i], [tp.hq * D, tp.hkv * D, tp.hkv * D])
        put_fp8(p + "self_attn.q_proj", q)
        put_fp8(p + "self_attn.k_proj", k)
        put_fp8(p + "self_attn.v_proj", v)
        put_fp8(p + "self_attn.o_proj", src.w_o[i])
        g, u = src.w_gu[i].chunk(2)
        put_fp8(p + "mlp.gate_proj", g)
        put_fp8(p + "mlp.up_proj", u)
        put_fp8(p + "mlp.down_proj", src.w_d[i])
        t[p + "input_layernorm.weight"], t[p + "post_attention_layernorm.weight"] = src.ln1[i], src.ln2[i]
    save_file({k: v.contiguous() for k, v in t.items()}, tmp_path / "model.safetensors")
    (tmp_path / "config.json").write_text(json.dumps(_cfg("fp8", block=True)))
    loaded = build_model(ModelConfig.from_path(tmp_path), "cpu", torch.bfloat16, model_path=str(tmp_path))
    assert loaded.fp8_block == 128 and isinstance(loaded.w_gu[0], Fp8Weight)
    online = build_model(ModelConfig.from_hf(_cfg("fp8", block=True)), "cpu", torch.bfloat16, load_format="dummy",
                         seed=7)
    for i in src.layers:
        for name in ("w_qkv", "w_o", "w_gu", "w_d"):
            x, y = getattr(loaded, name)[i], getattr(online, name)[i]
            assert torch.equal(x.q.view(torch.uint8), y.q.view(torch.uint8)), name
            assert torch.allclose(x.scale, y.scale)
    ids = [1, 2, 3, 4, 5]
    assert torch.equal(_forward(loaded, ids), _forward(online, ids))


def test_engine_fp8_generates():
    from ome_amd.runtime.engine import Engine, EngineArgs
    from ome_amd.runtime.request import SamplingParams

    eng = Engine(EngineArgs(model="tiny-llama", device="cpu", max_running_requests=4, context_length=128,
                            quantization="fp8"))
    assert isinstance(eng.runner.model.w_o[0], Fp8Weight)
    reqs = eng.generate([[5, 6, 7, 8], [9, 10]], SamplingParams(max_new_tokens=6, temperature=0.0, ignore_eos=True))
    assert all(len(r.output_ids) == 6 for r in reqs)


def test_fp8_moe_experts_quantized_and_reference_path():
    """quantization: fp8 on an MoE model keeps the experts fp8 (Fp8Experts, 128x128 blocks) and
    the CPU reference path of fused_moe runs the quantised emulation."""
    import torch

    from ome_amd import ops
    from ome_amd.models import build_model
    from ome_amd.models.config import preset
    from ome_amd.models.quant import Fp8Experts, quantize_experts

    cfg = preset("tiny-moe")
    cfg.quantization = "fp8"
    m = build_model(cfg, "cpu", torch.float32, load_format="dummy", seed=1)
    i = sorted(m.moe_layers)[0]
    assert isinstance(m.w13[i], Fp8Experts) and m.w13[i].q.dtype == torch.float8_e4m3fn
    w = torch.randn(4, 256, 384) * 0.05
    q = quantize_experts(w)
    assert q.scale.shape == (4, 2, 3)
    assert (q.dequant(torch.float32) - w).abs().max() < 0.06 * w.abs().max()
    x = torch.randn(5, 256)
    tw, tid = ops.moe_route(torch.randn(5, 8), 2)
    y = ops.fused_moe(x, tw, tid, m.w13[i], m.w2[i], 0, 1.0)
    assert y.shape == (5, 256) and torch.isfinite(y).all()


def test_w8a16_mgemv_split_choice():
    """The MFMA GEMV's K splits: 256-deep multiples that divide K, the activation slice within
    64 KiB of LDS, the split count nearest ~512 workgroups first (csrc/kernels/w8a16.hip)."""
    from ome_amd import ops

    assert ops.w8a16_mgemv_splits(8, 4096, 4096) == []       # GEMV rows
    assert ops.w8a16_mgemv_splits(33, 4096, 4096) == []      # skinny tile rows
    assert ops.w8a16_mgemv_splits(16, 4096, 4000) == []      # K not a multiple of 256
    for M, N, K in [(16, 6144, 4096), (32, 4096, 14336), (32, 28672, 4096), (20, 576, 7168)]:
        sp = ops.w8a16_mgemv_splits(M, N, K)
        mp = 16 if M <= 16 else 32 if M <= 32 else 64
        assert sp and all(K % d == 0 and K // d in (256, 512, 1024) and mp * (2 * (K // d) + 16) <= 65536
                          for d in sp)
        tiles = -(-N // 256)
        assert abs(tiles * sp[0] - 512) == min(abs(tiles * d - 512) for d in sp)
