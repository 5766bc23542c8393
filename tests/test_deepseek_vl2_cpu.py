"""DeepSeek-VL2 (``models/deepseek_vl2.py``) on CPU: a tiny random checkpoint in the published layout
(``vision.*`` timm SigLIP, ``projector.layers.*``, ``image_newline`` / ``view_seperator``,
``language.*`` DeepSeek-V2 MLA + MoE).  The image features are checked against an independent
fp32 restatement (ViT with exact GELU and final LayerNorm, zero-pad + ``F.unfold`` 2x2 projector,
global-then-tiles layout with row newlines), and greedy generation through the engine against the
HF-semantics DeepSeek reference of ``test_deepseek_cpu.py`` fed the same embeddings.  No
DeepSeek-VL2 class is importable here: parity with the remote code is unpinned."""
import json

import numpy as np
import pytest
import torch
import torch.nn.functional as F

PIL = pytest.importorskip("PIL")

from test_deepseek_cpu import _hf_forward, _hf_weights  # noqa: E402

from ome_amd.io.safetensors import save_file  # noqa: E402
from ome_amd.models.config import PRESETS, ModelConfig  # noqa: E402
from ome_amd.models.deepseek_vl2 import best_resolution, num_image_tokens, preprocess_deepseek_vl2  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402

E, HEADS, DEPTH, PS, SIZE = 64, 2, 2, 14, 56   # 4 x 4 patches per tile -> 2 x 2 tokens after the unfold
IMG = 1000
CANDS = [[56, 56], [56, 112], [112, 56]]


def _vision(g):
    r = lambda *s, std=0.05: torch.randn(*s, generator=g) * std  # noqa: E731
    side = SIZE // PS
    w = {"patch_embed.proj.weight": r(E, 3, PS, PS), "patch_embed.proj.bias": r(E), "pos_embed": r(1, side * side, E),
         "norm.weight": 1 + r(E), "norm.bias": r(E), "attn_pool.latent": r(1, 1, E)}
    for b in range(DEPTH):
        p = f"blocks.{b}."
        w.update({p + "norm1.weight": 1 + r(E), p + "norm1.bias": r(E), p + "attn.qkv.weight": r(3 * E, E, std=0.1),
                  p + "attn.qkv.bias": r(3 * E), p + "attn.proj.weight": r(E, E), p + "attn.proj.bias": r(E),
                  p + "norm2.weight": 1 + r(E), p + "norm2.bias": r(E), p + "mlp.fc1.weight": r(3 * E, E),
                  p + "mlp.fc1.bias": r(3 * E), p + "mlp.fc2.weight": r(E, 3 * E), p + "mlp.fc2.bias": r(E)})
    return w


def _vit_ref(w, px):
    n = px.shape[0]
    x = F.conv2d(px, w["patch_embed.proj.weight"], w["patch_embed.proj.bias"], stride=PS).flatten(2).transpose(1, 2)
    x = x + w["pos_embed"]
    for b in range(DEPTH):
        p = f"blocks.{b}."
        h = F.layer_norm(x, (E,), w[p + "norm1.weight"], w[p + "norm1.bias"], 1e-6)
        q, k, v = (h @ w[p + "attn.qkv.weight"].T + w[p + "attn.qkv.bias"]).view(n, -1, 3, HEADS, E // HEADS).unbind(2)
        a = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2))
        x = x + a.transpose(1, 2).reshape(n, -1, E) @ w[p + "attn.proj.weight"].T + w[p + "attn.proj.bias"]
        h = F.layer_norm(x, (E,), w[p + "norm2.weight"], w[p + "norm2.bias"], 1e-6)
        x = x + F.gelu(h @ w[p + "mlp.fc1.weight"].T + w[p + "mlp.fc1.bias"]) @ w[p + "mlp.fc2.weight"].T + \
            w[p + "mlp.fc2.bias"]
    return F.layer_norm(x, (E,), w["norm.weight"], w["norm.bias"], 1e-6)


def _features_ref(vw, pw, px, grid):
    f = _vit_ref(vw, px)                                        # [n, 16, E]
    n, hw, _ = f.shape
    side = int(hw ** 0.5)
    x = f.reshape(n, side, side, E).permute(0, 3, 1, 2)
    x = F.unfold(x, kernel_size=2, stride=2).permute(0, 2, 1)   # [n, 4, 4E]
    x = F.gelu(x @ pw["layers.0.weight"].T + pw["layers.0.bias"]) @ pw["layers.2.weight"].T + pw["layers.2.bias"]
    s, H = side // 2, x.shape[-1]
    _, th, tw = grid
    rows = []
    g = x[0].view(s, s, H)
    for r in range(s):
        rows += [g[r], pw["image_newline"][None]]
    rows.append(pw["view_seperator"][None])
    tiles = x[1:].view(th, tw, s, s, H)
    for tr in range(th):
        for r in range(s):
            rows += [tiles[tr, tc, r] for tc in range(tw)] + [pw["image_newline"][None]]
    return torch.cat(rows, 0)


def _build(tmp_path):
    hf = dict(PRESETS["tiny-deepseek-v2"])
    cfg = ModelConfig.from_hf(hf)
    lw = _hf_weights(cfg, seed=4)
    g = torch.Generator().manual_seed(5)
    vw = _vision(g)
    H = cfg.hidden_size
    pw = {"layers.0.weight": torch.randn(H, 4 * E, generator=g) * 0.05, "layers.0.bias": torch.randn(H, generator=g) * 0.02,
          "layers.2.weight": torch.randn(H, H, generator=g) * 0.05, "layers.2.bias": torch.randn(H, generator=g) * 0.02,
          "image_newline": torch.randn(H, generator=g), "view_seperator": torch.randn(H, generator=g)}
    sd = {"language." + k: v.contiguous() for k, v in lw.items()}
    sd.update({"vision." + k: v.contiguous() for k, v in vw.items()})
    sd.update({"projector." + k: v.contiguous() for k, v in pw.items() if k.startswith("layers.")})
    sd["image_newline"], sd["view_seperator"] = pw["image_newline"], pw["view_seperator"]
    save_file(sd, tmp_path / "model.safetensors")
    full = {"architectures": ["DeepseekVLV2ForCausalLM"], "model_type": "deepseek_vl_v2", "language_config": hf,
            "vision_config": {"layers": DEPTH, "width": E, "heads": HEADS, "mlp_ratio": 3, "patch_size": PS,
                              "image_size": SIZE, "select_layer": -1},
            "projector_config": {"projector_type": "downsample_mlp_gelu", "downsample_ratio": 2, "depth": 2,
                                 "mlp_ratio": 1, "input_dim": E, "n_embed": H},
            "tile_tag": "2D", "global_view_pos": "head", "candidate_resolutions": CANDS, "image_token_id": IMG}
    (tmp_path / "config.json").write_text(json.dumps(full))
    return cfg, lw, vw, pw


def test_best_resolution():
    assert best_resolution(100, 40, CANDS) == (112, 56)
    assert best_resolution(40, 100, CANDS) == (56, 112)
    assert best_resolution(50, 50, CANDS) == (56, 56)
    assert num_image_tokens(1, 2, 14) == 14 * 15 + 1 + 14 * 29


def test_deepseek_vl2_matches_reference(tmp_path):
    from PIL import Image

    cfg, lw, vw, pw = _build(tmp_path)
    img = Image.fromarray(np.random.default_rng(1).integers(0, 255, (40, 100, 3), dtype=np.uint8))
    px, grid = preprocess_deepseek_vl2(img, SIZE, True, CANDS)
    assert grid == (1, 1, 2) and px.shape == (3, 3, SIZE, SIZE)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=2,
                            context_length=512))
    m = eng.runner.model
    assert type(m).__name__ == "DeepseekVLV2ForCausalLM"
    want = _features_ref(vw, pw, px, grid)
    got = m.encode_images(px, [grid])
    assert got.shape == want.shape == (num_image_tokens(1, 2, 2), cfg.hidden_size)
    assert (got - want).abs().max().item() < 1e-3, (got - want).abs().max()
    prompt = [5, 9, IMG, 12, 7]
    req = eng.make_mm_request(prompt, [img], SamplingParams(max_new_tokens=3, ignore_eos=True))
    assert req.mm.spans == [(2, 17)]
    eng.add_request(req)
    while not req.finished:
        eng.step()
    ids = list(req.prompt_ids)
    emb = lw["model.embed_tokens.weight"][ids].clone()
    emb[2:19] = want
    toks = []
    for _ in range(3):
        nxt = int(_hf_forward(cfg, lw, ids, emb)[-1].argmax())
        toks.append(nxt)
        ids.append(nxt)
        emb = torch.cat([emb, lw["model.embed_tokens.weight"][[nxt]]], 0)
    assert req.output_ids == toks
