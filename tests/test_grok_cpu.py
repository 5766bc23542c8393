"""Grok-1 / Grok-2 on CPU: checkpoints in both weight layouts (hpcai-tech Grok-1 names, xai-org /
SGLang Grok-2 names) load into ``models/grok.py`` and its prefill logits match an independent
plain-PyTorch fp32 forward of the published Grok architecture (sandwich norms, embedding / output
multipliers, attention-logit soft-capping, GELU-gated experts with un-renormalised softmax top-2,
Grok-2 router / final soft-capping and the residual dense MLP).  transformers has no Grok model,
so parity with the original implementation is unpinned beyond this reference."""
import json
import math

import pytest
import torch
import torch.nn.functional as F

from ome_amd.io.safetensors import save_file
from ome_amd.models import build_model, model_class, supported
from ome_amd.models.common import AttnMeta, PagedKVCache
from ome_amd.models.config import PRESETS, ModelConfig


def _rand_ckpt(hf: dict, layout: str, seed: int = 0) -> dict[str, torch.Tensor]:
    g = torch.Generator().manual_seed(seed)
    r = lambda *s, std=0.05: torch.randn(*s, generator=g) * std  # noqa: E731
    H, L, V = hf["hidden_size"], hf["num_hidden_layers"], hf["vocab_size"]
    nh, nkv = hf["num_attention_heads"], hf["num_key_value_heads"]
    D = hf.get("head_dim") or H // nh
    E = hf.get("num_experts") or hf["num_local_experts"]
    I = hf.get("moe_intermediate_size") or hf["intermediate_size"]
    t = {"model.embed_tokens.weight": r(V, H, std=0.02), "model.norm.weight": 1 + r(H, std=0.1)}
    if not hf.get("tie_word_embeddings"):
        t["lm_head.weight"] = r(V, H, std=0.02)
    for i in range(L):
        p = f"model.layers.{i}."
        at = "attn" if layout == "hpcai" else "self_attn"
        for n, rows in (("q_proj", nh * D), ("k_proj", nkv * D), ("v_proj", nkv * D)):
            t[p + f"{at}.{n}.weight"] = r(rows, H)
        t[p + f"{at}.o_proj.weight"] = r(H, nh * D)
        for n in ("pre_attn_norm", "post_attn_norm", "pre_moe_norm", "post_moe_norm"):
            t[p + f"{n}.weight"] = 1 + r(H, std=0.1)
        blk = "moe_block" if layout == "hpcai" else "block_sparse_moe"
        t[p + f"{blk}.gate.weight"] = r(E, H, std=0.3)
        names = ("linear", "linear_v", "linear_1") if layout == "hpcai" else ("w1", "w3", "w2")
        for e in range(E):
            t[p + f"{blk}.experts.{e}.{names[0]}.weight"] = r(I, H)
            t[p + f"{blk}.experts.{e}.{names[1]}.weight"] = r(I, H)
            t[p + f"{blk}.experts.{e}.{names[2]}.weight"] = r(H, I)
        if hf.get("residual_moe"):
            Id = hf["intermediate_size"]
            t[p + "mlp.gate_proj.weight"], t[p + "mlp.up_proj.weight"] = r(Id, H), r(Id, H)
            t[p + "mlp.down_proj.weight"] = r(H, Id)
    return t


def _rms(x, w, eps):
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w


def _rope(x, pos, theta):
    d = x.shape[-1]
    inv = 1.0 / theta ** (torch.arange(0, d, 2, dtype=torch.float64) / d)
    f = pos[:, None].double() * inv[None]
    cos, sin = torch.cat([f.cos(), f.cos()], -1).float(), torch.cat([f.sin(), f.sin()], -1).float()
    x1, x2 = x[..., : d // 2], x[..., d // 2:]
    return x * cos[:, None] + torch.cat([-x2, x1], -1) * sin[:, None]


def _reference_logits(hf: dict, w: dict, ids: list[int], layout: str) -> torch.Tensor:
    """Plain fp32 Grok forward (one causal sequence)."""
    H, L = hf["hidden_size"], hf["num_hidden_layers"]
    nh, nkv = hf["num_attention_heads"], hf["num_key_value_heads"]
    D = hf.get("head_dim") or H // nh
    E = hf.get("num_experts") or hf["num_local_experts"]
    k = hf["num_experts_per_tok"]
    eps = hf["rms_norm_eps"]
    cap = hf.get("attn_logit_softcapping") or hf.get("max_attn_value") or 0.0
    scale = hf.get("attn_output_multiplier") or D ** -0.5
    T = len(ids)
    pos = torch.arange(T)
    x = w["model.embed_tokens.weight"][torch.tensor(ids)] * hf["embedding_multiplier_scale"]
    at = "attn" if layout == "hpcai" else "self_attn"
    blk = "moe_block" if layout == "hpcai" else "block_sparse_moe"
    names = ("linear", "linear_v", "linear_1") if layout == "hpcai" else ("w1", "w3", "w2")
    mask = torch.ones(T, T).tril().bool()
    for i in range(L):
        p = f"model.layers.{i}."
        h = _rms(x, w[p + "pre_attn_norm.weight"], eps)
        q = (h @ w[p + f"{at}.q_proj.weight"].T).view(T, nh, D)
        kk = (h @ w[p + f"{at}.k_proj.weight"].T).view(T, nkv, D)
        v = (h @ w[p + f"{at}.v_proj.weight"].T).view(T, nkv, D)
        q, kk = _rope(q, pos, hf["rope_theta"]), _rope(kk, pos, hf["rope_theta"])
        rep = nh // nkv
        kk, v = kk.repeat_interleave(rep, 1), v.repeat_interleave(rep, 1)
        s = torch.einsum("qhd,khd->hqk", q, kk) * scale
        if cap:
            s = cap * torch.tanh(s / cap)
        s = s.masked_fill(~mask, float("-inf")).softmax(-1)
        a = torch.einsum("hqk,khd->qhd", s, v).reshape(T, nh * D)
        a = a @ w[p + f"{at}.o_proj.weight"].T
        x = x + _rms(a, w[p + "post_attn_norm.weight"], eps)
        h = _rms(x, w[p + "pre_moe_norm.weight"], eps)
        logits = h @ w[p + f"{blk}.gate.weight"].T
        if hf.get("router_logit_softcapping"):
            c = hf["router_logit_softcapping"]
            logits = c * torch.tanh(logits / c)
        probs = logits.softmax(-1)
        tw, ti = probs.topk(k, -1)
        moe = torch.zeros_like(h)
        for e in range(E):
            sel = (ti == e)
            rows = sel.any(-1)
            if not rows.any():
                continue
            we = (tw * sel).sum(-1)[rows]
            he = h[rows]
            g = F.gelu(he @ w[p + f"{blk}.experts.{e}.{names[0]}.weight"].T, approximate="tanh")
            u = he @ w[p + f"{blk}.experts.{e}.{names[1]}.weight"].T
            moe[rows] += we[:, None] * ((g * u) @ w[p + f"{blk}.experts.{e}.{names[2]}.weight"].T)
        if hf.get("residual_moe"):
            g = F.gelu(h @ w[p + "mlp.gate_proj.weight"].T, approximate="tanh")
            dense = (g * (h @ w[p + "mlp.up_proj.weight"].T)) @ w[p + "mlp.down_proj.weight"].T
            moe = (moe + dense) / math.sqrt(2)
        x = x + _rms(moe, w[p + "post_moe_norm.weight"], eps)
    x = _rms(x, w["model.norm.weight"], eps)
    head = w.get("lm_head.weight", w["model.embed_tokens.weight"])
    out = (x @ head.T) * hf["output_multiplier_scale"]
    if hf.get("final_logit_softcapping"):
        c = hf["final_logit_softcapping"]
        out = c * torch.tanh(out / c)
    return out


def _forward(m, ids):
    T = len(ids)
    kv = PagedKVCache(m.cfg.num_layers, 8, m.tp.hkv, m.D, 16, m.dtype, "cpu")
    bt = torch.tensor([[1, 2, 3, 4]], dtype=torch.int32)
    meta = AttnMeta("prefill", torch.arange(T, dtype=torch.int32), torch.arange(16, 16 + T, dtype=torch.int32), bt,
                    cu_q=torch.tensor([0, T], dtype=torch.int32), kv_lens=torch.tensor([T], dtype=torch.int32),
                    items=torch.tensor([[0, 0]], dtype=torch.int32))
    return m.compute_logits(m.forward(torch.tensor(ids, dtype=torch.int32), meta, kv))


@pytest.mark.parametrize("preset,layout", [("tiny-grok1", "hpcai"), ("tiny-grok2", "sglang"),
                                           ("tiny-grok1", "sglang")])
def test_grok_logits_match_reference(tmp_path, preset, layout):
    hf = dict(PRESETS[preset])
    w = _rand_ckpt(hf, layout)
    save_file({k: v.contiguous() for k, v in w.items()}, tmp_path / "model.safetensors")
    (tmp_path / "config.json").write_text(json.dumps(hf))
    cfg = ModelConfig.from_path(tmp_path)
    assert supported(cfg.architecture) and model_class(cfg).__name__ == "GrokForCausalLM"
    m = build_model(cfg, "cpu", torch.float32, model_path=str(tmp_path))
    ids = [3, 14, 15, 92, 65, 35, 89, 79, 323]
    ours = _forward(m, ids)
    ref = _reference_logits(hf, w, ids, layout)
    assert ours.shape == ref.shape
    assert torch.allclose(ours, ref, atol=2e-4, rtol=1e-3), (ours - ref).abs().max()


def test_grok_random_init_and_sizes():
    for name in ("tiny-grok1", "tiny-grok2"):
        cfg = ModelConfig.from_hf(PRESETS[name])
        m = build_model(cfg, "cpu", torch.float32, load_format="dummy")
        assert torch.isfinite(_forward(m, [1, 2, 3])).all()
        assert m.renorm is False and m.act == 1
    g1 = ModelConfig.from_hf(PRESETS["grok-1"])
    assert 300e9 < g1.num_params() < 330e9   # the catalog's 300B-320B model size range
