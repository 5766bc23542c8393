"""MoE (Mixtral / Qwen3-MoE naming) on CPU: HF checkpoint loading round-trip and routing ref."""
import json

import pytest
import torch

from ome_amd.io.safetensors import save_file
from ome_amd.models import build_model
from ome_amd.models.common import AttnMeta, PagedKVCache
from ome_amd.models.config import PRESETS, ModelConfig
from ome_amd.ops import reference as ref


def _export_hf(m, path, style):
    cfg = m.cfg
    D, tp = m.D, m.tp
    t = {"model.embed_tokens.weight": m.embed, "model.norm.weight": m.norm, "lm_head.weight": m.lm_head}
    I = m.moe_inter
    for i in m.layers:
        p = f"model.layers.{i}."
        q, k, v = torch.split(m.w_qkv[i], [tp.hq * D, tp.hkv * D, tp.hkv * D])
        t[p + "self_attn.q_proj.weight"], t[p + "self_attn.k_proj.weight"], t[p + "self_attn.v_proj.weight"] = q, k, v
        t[p + "self_attn.o_proj.weight"] = m.w_o[i]
        t[p + "input_layernorm.weight"], t[p + "post_attention_layernorm.weight"] = m.ln1[i], m.ln2[i]
        if m.qn[i] is not None:
            t[p + "self_attn.q_norm.weight"], t[p + "self_attn.k_norm.weight"] = m.qn[i], m.kn[i]
        blk = "block_sparse_moe" if style == "mixtral" else "mlp"
        t[p + f"{blk}.gate.weight"] = m.w_router[i]
        for e in range(m.E):
            g, u = m.w13[i][e, :I], m.w13[i][e, I:]
            names = ("w1", "w3", "w2") if style == "mixtral" else ("gate_proj", "up_proj", "down_proj")
            t[p + f"{blk}.experts.{e}.{names[0]}.weight"] = g
            t[p + f"{blk}.experts.{e}.{names[1]}.weight"] = u
            t[p + f"{blk}.experts.{e}.{names[2]}.weight"] = m.w2[i][e]
    save_file({k: v.contiguous() for k, v in t.items()}, path / "model.safetensors")


def _forward(m, ids):
    T = len(ids)
    kv = PagedKVCache(m.cfg.num_layers, 8, m.tp.hkv, m.D, 16, m.dtype, "cpu")
    bt = torch.tensor([[1, 2, 3, 4]], dtype=torch.int32)
    meta = AttnMeta("prefill", torch.arange(T, dtype=torch.int32), torch.arange(16, 16 + T, dtype=torch.int32), bt,
                    cu_q=torch.tensor([0, T], dtype=torch.int32), kv_lens=torch.tensor([T], dtype=torch.int32),
                    items=torch.tensor([[0, 0]], dtype=torch.int32))
    return m.compute_logits(m.forward(torch.tensor(ids, dtype=torch.int32), meta, kv))


@pytest.mark.parametrize("style", ["mixtral", "qwen3"])
def test_moe_hf_roundtrip(tmp_path, style):
    hf = dict(PRESETS["tiny-moe"])
    if style == "mixtral":
        hf.update(architectures=["MixtralForCausalLM"], model_type="mixtral", num_local_experts=8,
                  intermediate_size=128)
        hf.pop("num_experts", None)
        hf.pop("moe_intermediate_size", None)
    cfg = ModelConfig.from_hf(hf)
    a = build_model(cfg, "cpu", torch.float32, load_format="dummy", seed=3)
    _export_hf(a, tmp_path, style)
    (tmp_path / "config.json").write_text(json.dumps(hf))
    b = build_model(ModelConfig.from_path(tmp_path), "cpu", torch.float32, model_path=str(tmp_path))
    ids = [3, 14, 15, 92, 65, 35]
    assert torch.allclose(_forward(a, ids), _forward(b, ids), atol=1e-5)


def test_moe_route_reference():
    logits = torch.randn(5, 8)
    w, ids = ref.moe_route(logits, 2, True)
    assert torch.allclose(w.sum(-1), torch.ones(5))
    assert (ids[:, 0] == logits.argmax(-1)).all()
