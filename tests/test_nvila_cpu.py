"""NVILA (``models/nvila.py``) on CPU: a tiny checkpoint in the VILA layout (``llm/`` = transformers
Qwen2, ``vision_tower/`` = transformers SiglipVisionModel, ``mm_projector/`` = the
``mlp_downsample_3x3_fix`` stack) against an fp32 restatement of the Dynamic-S2 + chessboard +
3x3-fold projector pipeline written here with explicit loops on top of transformers' SigLIP,
and greedy generation through the engine against transformers' Qwen2 fed the same embeddings.
The VILA remote code is not importable offline: parity with it is unpinned."""
import json

import numpy as np
import pytest
import torch
import torch.nn.functional as F

transformers = pytest.importorskip("transformers")
pytest.importorskip("PIL")

from ome_amd.io.safetensors import save_file  # noqa: E402
from ome_amd.models.nvila import closest_grid, preprocess_nvila  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402

IMG = 500
SCALES = [84, 168, 252]


def _init(m, g):
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "norm" in n:
                p.copy_(1 + torch.randn(p.shape, generator=g) * 0.1 if n.endswith("weight") else
                        torch.randn(p.shape, generator=g) * 0.05)
            else:
                p.copy_(torch.randn(p.shape, generator=g) * 0.08)


def _checkpoint(tmp_path):
    T = transformers
    g = torch.Generator().manual_seed(0)
    llm = T.Qwen2ForCausalLM(T.Qwen2Config(vocab_size=512, hidden_size=128, intermediate_size=256,
                                           num_hidden_layers=2, num_attention_heads=2, num_key_value_heads=1,
                                           max_position_embeddings=4096, tie_word_embeddings=False))
    vt = T.SiglipVisionModel(T.SiglipVisionConfig(hidden_size=64, intermediate_size=128, num_hidden_layers=3,
                                                  num_attention_heads=4, image_size=84, patch_size=14,
                                                  vision_use_head=False))
    _init(llm, g)
    _init(vt, g)
    llm, vt = llm.float().eval(), vt.float().eval()
    for m in (llm, vt):
        m.config._attn_implementation = "eager"
    llm.save_pretrained(tmp_path / "llm", safe_serialization=True)
    vt.save_pretrained(tmp_path / "vision_tower", safe_serialization=True)
    C, H = 64 * 3, 128
    r = lambda *s, std=0.05: torch.randn(*s, generator=g) * std  # noqa: E731
    proj = {"layers.1.weight": 1 + r(9 * C), "layers.1.bias": r(9 * C), "layers.2.weight": r(3 * C, 9 * C),
            "layers.2.bias": r(3 * C), "layers.4.weight": 1 + r(3 * C), "layers.4.bias": r(3 * C),
            "layers.5.weight": r(H, 3 * C, std=0.1), "layers.5.bias": r(H), "layers.7.weight": r(H, H, std=0.1),
            "layers.7.bias": r(H)}
    (tmp_path / "mm_projector").mkdir()
    save_file(proj, str(tmp_path / "mm_projector" / "model.safetensors"))
    (tmp_path / "mm_projector" / "config.json").write_text(json.dumps({"mm_projector_type": "mlp_downsample_3x3_fix"}))
    (tmp_path / "config.json").write_text(json.dumps({
        "architectures": ["LlavaLlamaModel"], "model_type": "llava_llama", "mm_vision_select_layer": -2,
        "image_aspect_ratio": "dynamic_s2", "s2_scales": ",".join(map(str, SCALES)), "s2_max_split_size": 84,
        "max_tiles": 12, "image_token_id": IMG}))
    return llm, vt, proj


def _image(h=70, w=130):
    from PIL import Image

    return Image.fromarray(np.random.default_rng(2).integers(0, 255, (h, w, 3), dtype=np.uint8))


def _features_ref(vt, proj, px, rows, cols):
    """Dynamic-S2 merge + chessboard + 3x3 fold + projector, restated with loops."""
    with torch.no_grad():
        hs = vt(pixel_values=px, output_hidden_states=True).hidden_states[-2]     # [tiles, 36, 64]
    s, E = 6, 64
    maps, off = [], 0
    for k, sc in enumerate(SCALES):
        r, c = (rows, cols) if k == len(SCALES) - 1 else (sc // 84, sc // 84)
        mp = torch.zeros(E, r * s, c * s)
        for i in range(r):
            for j in range(c):
                mp[:, i * s:(i + 1) * s, j * s:(j + 1) * s] = hs[off + i * c + j].view(s, s, E).permute(2, 0, 1)
        off += r * c
        maps.append(mp)
    size = maps[-1].shape[1:]
    merged = torch.cat([F.adaptive_avg_pool2d(mp[None], size)[0] for mp in maps], 0)     # [3E, R, C]
    Cm = merged.shape[0]
    toks = torch.zeros(rows * 2, cols * 2, 128)
    for i in range(rows):
        for j in range(cols):
            blk = torch.zeros(Cm, 9, 9)          # 6 x 6 block, zero padded to 9 x 9 for the 3 x 3 fold
            blk[:, :6, :6] = merged[:, i * s:(i + 1) * s, j * s:(j + 1) * s]
            for a in range(2):
                for b in range(2):
                    v = torch.cat([blk[:, 3 * a + di, 3 * b + dj] for di in range(3) for dj in range(3)])
                    h = F.layer_norm(v, (9 * Cm,), proj["layers.1.weight"], proj["layers.1.bias"], 1e-5)
                    h = F.gelu(F.linear(h, proj["layers.2.weight"], proj["layers.2.bias"]))
                    h = F.layer_norm(h, (3 * Cm,), proj["layers.4.weight"], proj["layers.4.bias"], 1e-5)
                    h = F.gelu(F.linear(h, proj["layers.5.weight"], proj["layers.5.bias"]))
                    toks[2 * i + a, 2 * j + b] = F.linear(h, proj["layers.7.weight"], proj["layers.7.bias"])
    return toks.reshape(-1, 128)


def test_closest_grid():
    assert closest_grid(130, 70, 9, 12, 84) in ((4, 2), (4, 3))
    assert closest_grid(100, 100, 9, 12, 84) == (3, 3)
    c, r = closest_grid(50, 200, 9, 12, 84)
    assert r > c and 9 <= r * c <= 12


def test_nvila_features_and_generate(tmp_path):
    llm, vt, proj = _checkpoint(tmp_path)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=2,
                            context_length=1024))
    m = eng.runner.model
    assert type(m).__name__ == "NVILAForCausalLM" and m.scales == SCALES and m.k == 3 and m.side == 6
    img = _image()
    px, (rows, cols) = preprocess_nvila(img, SCALES, 84, 12)
    assert px.shape[0] == 1 + 4 + rows * cols and (cols, rows) == closest_grid(130, 70, 9, 12, 84)
    want = _features_ref(vt, proj, px, rows, cols)
    got = m.encode_images(px, [(rows, cols)])
    assert got.shape == want.shape == (rows * 2 * cols * 2, 128)
    assert (got - want).abs().max().item() < 2e-3 * max(1.0, want.abs().max().item())
    prompt = [1, 9, IMG, 12, 7, 40]
    req = eng.make_mm_request(prompt, [img], SamplingParams(max_new_tokens=5, ignore_eos=True))
    n = want.shape[0]
    assert req.mm.spans == [(2, n)] and len(req.prompt_ids) == len(prompt) - 1 + n
    eng.add_request(req)
    while not req.finished:
        eng.step()
    ids = torch.tensor(req.prompt_ids)
    with torch.no_grad():
        emb = llm.get_input_embeddings()(ids)
        emb[2:2 + n] = want
        toks = []
        for _ in range(5):
            nxt = int(llm(inputs_embeds=emb[None]).logits[0, -1].argmax())
            toks.append(nxt)
            emb = torch.cat([emb, llm.get_input_embeddings()(torch.tensor([nxt]))], 0)
    assert req.output_ids == toks


def test_nvila_random_init_preset():
    from ome_amd.models import build_model
    from ome_amd.models.config import preset

    m = build_model(preset("tiny-nvila"), "cpu", torch.float32)
    px, (rows, cols) = preprocess_nvila(_image(), m.scales, m.base, m.max_tiles)
    f = m.encode_images(px, [(rows, cols)])
    assert f.shape == (m._n_tokens(rows, cols), m.cfg.hidden_size) and torch.isfinite(f).all()
