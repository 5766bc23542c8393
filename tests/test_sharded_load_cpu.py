"""Rank-aware checkpoint loading (LlamaForCausalLM.shard_plan + libomeio strided reads): under
TP each rank reads only its shard of every weight -- column-parallel q/k/v/gate/up and the
vocab-parallel embedding / LM head by rows, row-parallel o/down by per-row column slices -- and
pipeline stages skip other stages' layers.  Shards must equal the narrow of a full load, and the
bytes pread per rank must be about 1/TP of the sharded tensors."""
import json

import pytest
import torch

from ome_amd.io import native as nio
from ome_amd.io.safetensors import save_file
from ome_amd.models import build_model
from ome_amd.models.config import PRESETS, ModelConfig
from ome_amd.parallel import state as pstate

pytestmark = pytest.mark.skipif(not nio.available(), reason="libomeio not built")


def _hf_checkpoint(path, cfg: ModelConfig, seed: int = 0):
    g = torch.Generator().manual_seed(seed)
    H, D, I, V = cfg.hidden_size, cfg.head_dim, cfg.intermediate_size, cfg.vocab_size
    w = {"model.embed_tokens.weight": torch.randn(V, H, generator=g), "model.norm.weight": torch.rand(H, generator=g),
         "lm_head.weight": torch.randn(V, H, generator=g)}
    for i in range(cfg.num_layers):
        p = f"model.layers.{i}."
        w[p + "self_attn.q_proj.weight"] = torch.randn(cfg.num_heads * D, H, generator=g)
        w[p + "self_attn.k_proj.weight"] = torch.randn(cfg.num_kv_heads * D, H, generator=g)
        w[p + "self_attn.v_proj.weight"] = torch.randn(cfg.num_kv_heads * D, H, generator=g)
        w[p + "self_attn.o_proj.weight"] = torch.randn(H, cfg.num_heads * D, generator=g)
        w[p + "mlp.gate_proj.weight"] = torch.randn(I, H, generator=g)
        w[p + "mlp.up_proj.weight"] = torch.randn(I, H, generator=g)
        w[p + "mlp.down_proj.weight"] = torch.randn(H, I, generator=g)
        w[p + "input_layernorm.weight"] = torch.rand(H, generator=g)
        w[p + "post_attention_layernorm.weight"] = torch.rand(H, generator=g)
    save_file({k: v.to(torch.bfloat16).contiguous() for k, v in w.items()}, path / "model.safetensors")
    return w


def _load(path, cfg, tp, rank, pp=1, pp_rank=0):
    prev = pstate.get()
    pstate.set_state(pstate.ParallelState(tp_size=tp, tp_rank=rank, pp_size=pp, pp_rank=pp_rank,
                                          world_size=tp * pp, rank=pp_rank * tp + rank))
    try:
        b0 = nio.bytes_read()
        m = build_model(cfg, "cpu", torch.bfloat16, model_path=str(path), load_format="safetensors")
        return m, nio.bytes_read() - b0
    finally:
        pstate.set_state(prev)


@pytest.mark.parametrize("tp", [2, 4])
def test_tp_ranks_read_only_their_shards(tmp_path, tp):
    hf = dict(PRESETS["tiny-llama"])
    hf.update(num_key_value_heads=4, num_attention_heads=4)
    cfg = ModelConfig.from_hf(hf)
    (tmp_path / "config.json").write_text(json.dumps(hf))
    _hf_checkpoint(tmp_path, cfg)
    full, full_bytes = _load(tmp_path, cfg, 1, 0)
    assert not full._presliced
    for r in range(tp):
        m, nbytes = _load(tmp_path, cfg, tp, r)
        assert m._presliced
        D, hq, hkv = cfg.head_dim, cfg.num_heads // tp, cfg.num_kv_heads // tp
        for i in range(cfg.num_layers):
            q, k, v = full.w_qkv[i].split([cfg.num_heads * D, cfg.num_kv_heads * D, cfg.num_kv_heads * D], 0)
            want = torch.cat([q[r * hq * D:(r + 1) * hq * D], k[r * hkv * D:(r + 1) * hkv * D],
                              v[r * hkv * D:(r + 1) * hkv * D]], 0)
            assert torch.equal(m.w_qkv[i], want)
            assert torch.equal(m.w_o[i], full.w_o[i][:, r * hq * D:(r + 1) * hq * D])
            I = cfg.intermediate_size // tp
            g, u = full.w_gu[i].split([cfg.intermediate_size] * 2, 0)
            assert torch.equal(m.w_gu[i], torch.cat([g[r * I:(r + 1) * I], u[r * I:(r + 1) * I]], 0))
            assert torch.equal(m.w_d[i], full.w_d[i][:, r * I:(r + 1) * I])
        V = cfg.vocab_size // tp
        assert torch.equal(m.embed, full.embed[r * V:(r + 1) * V])
        assert torch.equal(m.lm_head, full.lm_head[r * V:(r + 1) * V])
        # every sharded tensor contributes 1/tp of its bytes; norms are read whole (tiny)
        assert nbytes < full_bytes / tp * 1.05, (nbytes, full_bytes)


def test_pipeline_stage_skips_other_layers(tmp_path):
    hf = dict(PRESETS["tiny-llama"])
    hf.update(num_hidden_layers=4)
    cfg = ModelConfig.from_hf(hf)
    _hf_checkpoint(tmp_path, cfg, seed=3)
    full, full_bytes = _load(tmp_path, cfg, 1, 0)
    m, nbytes = _load(tmp_path, cfg, 1, 0, pp=2, pp_rank=1)
    assert m._presliced and m.layers == [2, 3]
    for i in (2, 3):
        assert torch.equal(m.w_qkv[i], full.w_qkv[i]) and torch.equal(m.w_d[i], full.w_d[i])
    layer_bytes = sum(t.numel() * 2 for t in (full.w_qkv[0], full.w_o[0], full.w_gu[0], full.w_d[0]))
    assert nbytes < full_bytes - 2 * layer_bytes * 0.99


def test_shard_geometry():
    assert nio.shard_ranges([8, 4], 2, None)[1:] == ("flat", 0, 1, 64, 64)
    assert nio.shard_ranges([8, 4], 2, ("rows", 2, 3)) == ([3, 4], "flat", 16, 1, 24, 24)
    assert nio.shard_ranges([8, 4], 2, ("cols", 1, 2)) == ([8, 2], "strided", 2, 8, 4, 8)
