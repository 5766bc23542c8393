"""Qwen-VL (``models/qwen_vl.py``) on CPU: a tiny Qwen (v1) checkpoint (converted from a random HF
Llama, as in tests/test_decoder_remote_families_cpu.py) plus a tiny ViT + Resampler in the remote
code's ``transformer.visual.*`` layout.  The image embeddings are checked against an independent
fp32 restatement of the remote ``visual.py`` (per-head [q|k|v] in_proj, bicubic position resize,
2-D sin-cos Resampler positions, ln_post @ proj); greedy generation with an image through the
engine against HF Llama fed the same embeddings.  The remote code is not importable here: parity
with it is unpinned."""
import json
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

transformers = pytest.importorskip("transformers")
pytest.importorskip("PIL")

from ome_amd.io.safetensors import save_file  # noqa: E402
from ome_amd.models.qwen_vl import preprocess_qwen_vl, resize_pos, sincos_2d  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402

START, END, PAD = 500, 501, 502
VC = dict(image_size=56, patch_size=14, width=64, layers=2, heads=2, mlp_ratio=2.0, output_dim=256, n_queries=4,
          image_start_id=START)


def _visual(g):
    r = lambda *s, std=0.08: torch.randn(*s, generator=g) * std  # noqa: E731
    E, O, M = VC["width"], VC["output_dim"], int(VC["width"] * VC["mlp_ratio"])
    w = {"conv1.weight": r(E, 3, 14, 14), "positional_embedding": r(256, E, std=0.3),
         "ln_pre.weight": 1 + r(E, std=0.1), "ln_pre.bias": r(E), "ln_post.weight": 1 + r(O, std=0.1),
         "ln_post.bias": r(O), "proj": r(O, O), "attn_pool.query": r(VC["n_queries"], O, std=0.5),
         "attn_pool.pos_embed": torch.from_numpy(sincos_2d(O, 2)).float(), "attn_pool.kv_proj.weight": r(O, E),
         "attn_pool.attn.in_proj_weight": r(3 * O, O), "attn_pool.attn.in_proj_bias": r(3 * O),
         "attn_pool.attn.out_proj.weight": r(O, O), "attn_pool.attn.out_proj.bias": r(O),
         "attn_pool.ln_q.weight": 1 + r(O, std=0.1), "attn_pool.ln_q.bias": r(O),
         "attn_pool.ln_kv.weight": 1 + r(O, std=0.1), "attn_pool.ln_kv.bias": r(O)}
    for i in range(VC["layers"]):
        p = f"transformer.resblocks.{i}."
        w.update({p + "ln_1.weight": 1 + r(E, std=0.1), p + "ln_1.bias": r(E), p + "ln_2.weight": 1 + r(E, std=0.1),
                  p + "ln_2.bias": r(E), p + "attn.in_proj.weight": r(3 * E, E), p + "attn.in_proj.bias": r(3 * E),
                  p + "attn.out_proj.weight": r(E, E), p + "attn.out_proj.bias": r(E),
                  p + "mlp.c_fc.weight": r(M, E), p + "mlp.c_fc.bias": r(M), p + "mlp.c_proj.weight": r(E, M),
                  p + "mlp.c_proj.bias": r(E)})
    return w


def _visual_ref(w, px):
    """fp32 restatement of visual.py's VisionTransformer.forward (batch-first)."""
    E, heads, O = VC["width"], VC["heads"], VC["output_dim"]
    hd = E // heads
    x = F.conv2d(px.float(), w["conv1.weight"], stride=14)
    n, _, s, _ = x.shape
    x = x.reshape(n, E, -1).permute(0, 2, 1)
    T = s * s
    # get_abs_pos: 16 x 16 table -> s x s, bicubic
    pe = F.interpolate(w["positional_embedding"].reshape(1, 16, 16, E).permute(0, 3, 1, 2), size=(s, s),
                       mode="bicubic", align_corners=False).permute(0, 2, 3, 1).reshape(T, E)
    x = F.layer_norm(x + pe, (E,), w["ln_pre.weight"], w["ln_pre.bias"], 1e-6)
    for i in range(VC["layers"]):
        p = f"transformer.resblocks.{i}."
        h = F.layer_norm(x, (E,), w[p + "ln_1.weight"], w[p + "ln_1.bias"], 1e-6)
        mixed = (h @ w[p + "attn.in_proj.weight"].T + w[p + "attn.in_proj.bias"]).view(n, T, heads, 3 * hd)
        q, k, v = mixed.split(hd, dim=-1)
        a = torch.softmax(torch.einsum("bqhd,bkhd->bhqk", q, k) / math.sqrt(hd), -1)
        o = torch.einsum("bhqk,bkhd->bqhd", a, v).reshape(n, T, E)
        x = x + o @ w[p + "attn.out_proj.weight"].T + w[p + "attn.out_proj.bias"]
        h = F.layer_norm(x, (E,), w[p + "ln_2.weight"], w[p + "ln_2.bias"], 1e-6)
        x = x + F.gelu(h @ w[p + "mlp.c_fc.weight"].T + w[p + "mlp.c_fc.bias"]) @ w[p + "mlp.c_proj.weight"].T + \
            w[p + "mlp.c_proj.bias"]
    # Resampler
    pos = w["attn_pool.pos_embed"]
    pos_k = F.interpolate(pos.reshape(1, 2, 2, O).permute(0, 3, 1, 2), size=(s, s), mode="bicubic",
                          align_corners=False).permute(0, 2, 3, 1).reshape(T, O)
    kv = F.layer_norm(x @ w["attn_pool.kv_proj.weight"].T, (O,), w["attn_pool.ln_kv.weight"],
                      w["attn_pool.ln_kv.bias"], 1e-6)
    q = F.layer_norm(w["attn_pool.query"], (O,), w["attn_pool.ln_q.weight"], w["attn_pool.ln_q.bias"], 1e-6)
    mha = torch.nn.MultiheadAttention(O, O // 128, batch_first=True)
    with torch.no_grad():
        mha.in_proj_weight.copy_(w["attn_pool.attn.in_proj_weight"])
        mha.in_proj_bias.copy_(w["attn_pool.attn.in_proj_bias"])
        mha.out_proj.weight.copy_(w["attn_pool.attn.out_proj.weight"])
        mha.out_proj.bias.copy_(w["attn_pool.attn.out_proj.bias"])
        out = mha((q + pos)[None].expand(n, -1, -1), kv + pos_k[None], kv)[0]
    out = F.layer_norm(out, (O,), w["ln_post.weight"], w["ln_post.bias"], 1e-6) @ w["proj"]
    return out.reshape(-1, O)


def _checkpoint(tmp_path):
    from safetensors.torch import load_file

    from tests.test_decoder_remote_families_cpu import _convert

    hf = _convert("qwen1", tmp_path)
    sd = {k: v.clone() for k, v in load_file(tmp_path / "model.safetensors").items()}
    g = torch.Generator().manual_seed(3)
    vis = _visual(g)
    sd.update({"transformer.visual." + k: v for k, v in vis.items()})
    save_file({k: v.contiguous() for k, v in sd.items()}, str(tmp_path / "model.safetensors"))
    cfg = json.loads((tmp_path / "config.json").read_text())
    cfg["visual"] = VC
    (tmp_path / "config.json").write_text(json.dumps(cfg))
    return hf, vis


def _image():
    from PIL import Image

    return Image.fromarray(np.random.default_rng(1).integers(0, 255, (70, 90, 3), dtype=np.uint8))


def test_qwen_vl_image_features_and_generate(tmp_path):
    hf, vis = _checkpoint(tmp_path)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=2,
                            context_length=256))
    m = eng.runner.model
    assert type(m).__name__ == "QwenVLForCausalLM" and m.image_prompt_ids() == [START, END]
    img = _image()
    px = preprocess_qwen_vl(img, 56)
    want = _visual_ref(vis, px)
    got = m.encode_images(px)
    assert got.shape == want.shape == (4, 256)
    assert (got - want).abs().max().item() < 1e-3 * max(1.0, want.abs().max().item())
    # an image prompt: <img> [path bytes] </img> -> <img> 4 placeholder rows </img>
    prompt = [1, 9, START, 77, 78, END, 12, 7, 40]
    req = eng.make_mm_request(prompt, [img], SamplingParams(max_new_tokens=5, ignore_eos=True))
    assert req.prompt_ids[:3] == [1, 9, START] and req.prompt_ids[3:7] == [PAD] * 4 and req.prompt_ids[7] == END
    assert req.mm.spans == [(3, 4)]
    eng.add_request(req)
    while not req.finished:
        eng.step()
    ids = torch.tensor(req.prompt_ids)
    with torch.no_grad():
        emb = hf.get_input_embeddings()(ids)
        emb[3:7] = want
        toks = []
        for _ in range(5):
            nxt = int(hf(inputs_embeds=emb[None]).logits[0, -1].argmax())
            toks.append(nxt)
            emb = torch.cat([emb, hf.get_input_embeddings()(torch.tensor([nxt]))], 0)
    assert req.output_ids == toks


def test_qwen_vl_text_only_unchanged(tmp_path):
    hf, _ = _checkpoint(tmp_path)
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=2,
                            context_length=256))
    ids = [(7 * i + 3) % 480 + 3 for i in range(20)]
    with torch.no_grad():
        ref = hf.generate(torch.tensor([ids]), max_new_tokens=5, do_sample=False)[0, len(ids):].tolist()
    assert eng.generate([ids], SamplingParams(max_new_tokens=5, ignore_eos=True))[0].output_ids == ref


def test_resize_pos_identity_and_sincos_layout():
    t = torch.randn(16, 8)
    assert resize_pos(t, 16) is t
    pe = sincos_2d(8, 2)   # cells (row, col): (0,0) (0,1) (1,0) (1,1); first half = column coordinate
    assert np.allclose(pe[1, :2], np.sin([1.0, 1e-2])) and np.allclose(pe[2, :2], 0.0)
    assert np.allclose(pe[2, 4:6], np.sin([1.0, 1e-2]))
