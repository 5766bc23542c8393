"""DeepSeek-V2/V3 (MLA + grouped-top-k MoE) on CPU.

The model runs MLA in the absorbed form over a 576-wide latent cache with rope dims
de-interleaved at load time; the reference below is a plain transcription of the HF
``modeling_deepseek`` semantics (decompressed per-head K/V, interleaved rope, HF MoEGate) over a
checkpoint exported in HF naming, so the test pins absorption, the rope permutation, the
routing and the loader together.  Parity with the HF implementation itself is unpinned
(transformers' DeepSeek code is not run here)."""
import json
import math

import pytest
import torch
import torch.nn.functional as F

from ome_amd.io.safetensors import save_file
from ome_amd.models import build_model
from ome_amd.models.common import AttnMeta, PagedKVCache
from ome_amd.models.config import PRESETS, ModelConfig, rope_cos_sin
from ome_amd.ops import reference as ref


def _hf_weights(cfg: ModelConfig, seed=0):
    g = torch.Generator().manual_seed(seed)

    def rn(*s, std=0.05):
        return torch.randn(*s, generator=g) * std

    H, nh = cfg.hidden_size, cfg.num_heads
    qk = cfg.qk_nope_head_dim + cfg.qk_rope_head_dim
    w = {"model.embed_tokens.weight": rn(cfg.vocab_size, H, std=1.0), "model.norm.weight": 1 + rn(H),
         "lm_head.weight": rn(cfg.vocab_size, H)}
    for i in range(cfg.num_layers):
        p = f"model.layers.{i}."
        w[p + "input_layernorm.weight"] = 1 + rn(H)
        w[p + "post_attention_layernorm.weight"] = 1 + rn(H)
        if cfg.q_lora_rank:
            w[p + "self_attn.q_a_proj.weight"] = rn(cfg.q_lora_rank, H)
            w[p + "self_attn.q_a_layernorm.weight"] = 1 + rn(cfg.q_lora_rank)
            w[p + "self_attn.q_b_proj.weight"] = rn(nh * qk, cfg.q_lora_rank)
        else:
            w[p + "self_attn.q_proj.weight"] = rn(nh * qk, H)
        w[p + "self_attn.kv_a_proj_with_mqa.weight"] = rn(cfg.kv_lora_rank + cfg.qk_rope_head_dim, H)
        w[p + "self_attn.kv_a_layernorm.weight"] = 1 + rn(cfg.kv_lora_rank)
        w[p + "self_attn.kv_b_proj.weight"] = rn(nh * (cfg.qk_nope_head_dim + cfg.v_head_dim), cfg.kv_lora_rank)
        w[p + "self_attn.o_proj.weight"] = rn(H, nh * cfg.v_head_dim)
        if i >= cfg.first_k_dense_replace:
            I, E = cfg.moe_intermediate_size, cfg.num_experts
            w[p + "mlp.gate.weight"] = rn(E, H, std=0.5)
            if cfg.model_type == "deepseek_v3":
                w[p + "mlp.gate.e_score_correction_bias"] = rn(E, std=0.1)
            for e in range(E):
                w[p + f"mlp.experts.{e}.gate_proj.weight"] = rn(I, H)
                w[p + f"mlp.experts.{e}.up_proj.weight"] = rn(I, H)
                w[p + f"mlp.experts.{e}.down_proj.weight"] = rn(H, I)
            SI = cfg.num_shared_experts * I
            w[p + "mlp.shared_experts.gate_proj.weight"] = rn(SI, H)
            w[p + "mlp.shared_experts.up_proj.weight"] = rn(SI, H)
            w[p + "mlp.shared_experts.down_proj.weight"] = rn(H, SI)
        else:
            w[p + "mlp.gate_proj.weight"] = rn(cfg.intermediate_size, H)
            w[p + "mlp.up_proj.weight"] = rn(cfg.intermediate_size, H)
            w[p + "mlp.down_proj.weight"] = rn(H, cfg.intermediate_size)
    return w


def _rms(x, w, eps):
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w


def _hf_forward(cfg: ModelConfig, w: dict, ids: list[int], h0: torch.Tensor | None = None) -> torch.Tensor:
    """HF modeling_deepseek semantics, fp32, single causal sequence (``h0``: input embeddings)."""
    T, nh = len(ids), cfg.num_heads
    nope, rope, vd = cfg.qk_nope_head_dim, cfg.qk_rope_head_dim, cfg.v_head_dim
    eps = cfg.rms_norm_eps
    rc = ModelConfig(**{**cfg.__dict__, "head_dim": rope, "partial_rotary_factor": 1.0})
    cs = rope_cos_sin(rc, T)
    cos = torch.cat([cs[:, : rope // 2]] * 2, -1)
    sin = torch.cat([cs[:, rope // 2:]] * 2, -1)

    def rot_half(x):
        return torch.cat([-x[..., rope // 2:], x[..., : rope // 2]], -1)

    def hf_rope(x):  # x [..., T, rope] interleaved pairs -> de-interleave view -> rotate_half
        s = x.shape
        x = x.reshape(*s[:-1], rope // 2, 2).transpose(-1, -2).reshape(s)
        return x * cos + rot_half(x) * sin

    scale = (nope + rope) ** -0.5
    sc = cfg.rope_scaling or {}
    if sc.get("mscale_all_dim"):
        m = 0.1 * sc["mscale_all_dim"] * math.log(sc["factor"]) + 1.0
        scale *= m * m
    h = w["model.embed_tokens.weight"][ids] if h0 is None else h0
    mask = torch.full((T, T), float("-inf")).triu(1)
    for i in range(cfg.num_layers):
        p = f"model.layers.{i}."
        x = _rms(h, w[p + "input_layernorm.weight"], eps)
        if cfg.q_lora_rank:
            q = _rms(x @ w[p + "self_attn.q_a_proj.weight"].t(), w[p + "self_attn.q_a_layernorm.weight"], eps)
            q = q @ w[p + "self_attn.q_b_proj.weight"].t()
        else:
            q = x @ w[p + "self_attn.q_proj.weight"].t()
        q = q.view(T, nh, nope + rope).transpose(0, 1)
        ckv = x @ w[p + "self_attn.kv_a_proj_with_mqa.weight"].t()
        c, k_pe = ckv[:, : cfg.kv_lora_rank], ckv[:, cfg.kv_lora_rank:]
        kv = (_rms(c, w[p + "self_attn.kv_a_layernorm.weight"], eps) @ w[p + "self_attn.kv_b_proj.weight"].t())
        kv = kv.view(T, nh, nope + vd).transpose(0, 1)
        k_nope, v = kv[..., :nope], kv[..., nope:]
        q_pe = hf_rope(q[..., nope:])
        k_pe = hf_rope(k_pe)[None].expand(nh, T, rope)
        qq = torch.cat([q[..., :nope], q_pe], -1)
        kk = torch.cat([k_nope, k_pe], -1)
        att = torch.softmax(qq @ kk.transpose(1, 2) * scale + mask, -1) @ v
        h = h + att.transpose(0, 1).reshape(T, nh * vd) @ w[p + "self_attn.o_proj.weight"].t()
        x = _rms(h, w[p + "post_attention_layernorm.weight"], eps)
        if i >= cfg.first_k_dense_replace:
            logits = x @ w[p + "mlp.gate.weight"].t()
            scores = torch.sigmoid(logits) if cfg.scoring_func == "sigmoid" else torch.softmax(logits, -1)
            choice = scores + w.get(p + "mlp.gate.e_score_correction_bias", torch.zeros(cfg.num_experts))
            G = cfg.n_group
            grp = choice.view(T, G, -1)
            gsc = grp.topk(2, -1).values.sum(-1) if cfg.model_type == "deepseek_v3" else grp.max(-1).values
            gm = torch.zeros_like(gsc).scatter_(1, gsc.topk(cfg.topk_group, -1).indices, 1.0)
            tmp = choice.masked_fill(gm.repeat_interleave(cfg.num_experts // G, 1) == 0, 0.0)
            idx = tmp.topk(cfg.num_experts_per_tok, -1).indices
            wt = scores.gather(1, idx)
            if cfg.norm_topk_prob:
                wt = wt / (wt.sum(-1, keepdim=True) + 1e-20)
            if cfg.model_type == "deepseek_v3" or not cfg.norm_topk_prob:
                wt = wt * cfg.routed_scaling_factor
            y = torch.zeros_like(x)
            for t in range(T):
                for j in range(idx.shape[1]):
                    e = int(idx[t, j])
                    q_ = f"{p}mlp.experts.{e}."
                    a = F.silu(x[t] @ w[q_ + "gate_proj.weight"].t()) * (x[t] @ w[q_ + "up_proj.weight"].t())
                    y[t] += wt[t, j] * (a @ w[q_ + "down_proj.weight"].t())
            s_ = p + "mlp.shared_experts."
            y += (F.silu(x @ w[s_ + "gate_proj.weight"].t()) * (x @ w[s_ + "up_proj.weight"].t())) @ \
                w[s_ + "down_proj.weight"].t()
        else:
            y = (F.silu(x @ w[p + "mlp.gate_proj.weight"].t()) * (x @ w[p + "mlp.up_proj.weight"].t())) @ \
                w[p + "mlp.down_proj.weight"].t()
        h = h + y
    return _rms(h, w["model.norm.weight"], eps) @ w["lm_head.weight"].t()


def _meta_prefill(T, start=0):
    pos = torch.arange(start, start + T, dtype=torch.int32)
    bt = torch.tensor([[1, 2, 3, 4]], dtype=torch.int32)
    slots = bt[0, (pos // 16).long()] * 16 + pos % 16
    return AttnMeta("prefill", pos, slots.to(torch.int32), bt, cu_q=torch.tensor([0, T], dtype=torch.int32),
                    kv_lens=torch.tensor([start + T], dtype=torch.int32), items=torch.tensor([[0, 0]], dtype=torch.int32))


def _kv(m):
    hk, dk, dv = m.kv_layout
    return PagedKVCache(m.cfg.num_layers, 8, hk, dk, 16, m.dtype, "cpu", dv)


@pytest.mark.parametrize("name", ["tiny-deepseek", "tiny-deepseek-v2"])
def test_deepseek_matches_hf_semantics(tmp_path, name):
    hf = dict(PRESETS[name])
    cfg = ModelConfig.from_hf(hf)
    w = _hf_weights(cfg, seed=1)
    save_file({k: v.contiguous() for k, v in w.items()}, tmp_path / "model.safetensors")
    (tmp_path / "config.json").write_text(json.dumps(hf))
    m = build_model(ModelConfig.from_path(tmp_path), "cpu", torch.float32, model_path=str(tmp_path))
    assert type(m).__name__ == "DeepseekForCausalLM" and m.kv_layout == (1, 576, 0)
    ids = [3, 14, 15, 92, 65, 35, 89, 79, 32, 38, 46, 26, 43, 38, 32, 79, 50, 28, 84]
    want = _hf_forward(cfg, w, ids)
    kv = _kv(m)
    got = m.compute_logits(m.forward(torch.tensor(ids, dtype=torch.int32), _meta_prefill(len(ids)), kv))
    assert torch.allclose(got, want, atol=2e-3, rtol=2e-3), (got - want).abs().max()
    # chunked prefill over the latent cache: the last 5 tokens attend to the cached first 14
    kv2 = _kv(m)
    m.forward(torch.tensor(ids[:14], dtype=torch.int32), _meta_prefill(14), kv2)
    got2 = m.compute_logits(m.forward(torch.tensor(ids[14:], dtype=torch.int32), _meta_prefill(5, 14), kv2))
    assert torch.allclose(got2, want[14:], atol=2e-3, rtol=2e-3)


def test_grouped_routing_reference():
    torch.manual_seed(0)
    logits = torch.randn(6, 16)
    bias = torch.randn(16) * 0.1
    w, ids = ref.moe_route(logits, 4, True, "sigmoid", bias, n_group=4, topk_group=2, group_mode=2)
    key = torch.sigmoid(logits) + bias
    gs = key.view(6, 4, 4).topk(2, -1).values.sum(-1)
    top_groups = gs.topk(2, -1).indices
    for t in range(6):
        assert set((ids[t] // 4).tolist()) <= set(top_groups[t].tolist())
    assert torch.allclose(w.sum(-1), torch.ones(6))


def test_deepseek_engine_generates():
    from ome_amd.runtime.engine import Engine, EngineArgs
    from ome_amd.runtime.request import SamplingParams

    eng = Engine(EngineArgs(model="tiny-deepseek", device="cpu", max_running_requests=4, context_length=128,
                            enable_mixed_chunk=True))
    prompts = [[5, 6, 7, 8, 9] * 4, [9, 10, 11], [5, 6, 7, 8, 9] * 4]
    reqs = eng.generate(prompts, SamplingParams(max_new_tokens=8, temperature=0.0, ignore_eos=True))
    assert all(len(r.output_ids) == 8 for r in reqs)
    assert reqs[0].output_ids == reqs[2].output_ids
