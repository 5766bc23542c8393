"""Kimi-VL (``models/kimi_vl.py``) on CPU reference ops against transformers' Kimi-K2.5
(MoonViT + DeepSeek-V3; tiny random ``Kimi_K25ForConditionalGeneration``, fp32): vision features
(bicubically resampled learned positions, 2D rotary, LayerNorm / GELU-tanh blocks, per-patch
LayerNorm + 2 x 2 merge + projector) and greedy generation with log-probs through the engine,
from the transformers checkpoint layout and from the same weights re-laid into the original
Kimi-VL layout (fused ``wqkv`` with interleaved-pair rotary rows, ``norm0`` / ``mlp.fc0`` names,
``multi_modal_projector``).  The Kimi-VL preprocessing rule is checked on its own (parity
unpinned: the transformers processor needs torchvision, absent here)."""
import json

import numpy as np
import pytest
import torch

transformers = pytest.importorskip("transformers")
PIL = pytest.importorskip("PIL")
try:
    from transformers.models.kimi_k25 import modeling_kimi_k25 as K  # noqa: F401
except Exception:  # noqa: BLE001
    pytest.skip("transformers without Kimi-K2.5", allow_module_level=True)

from safetensors.torch import load_file, save_file  # noqa: E402
from ome_amd.models.kimi_vl import kimi_resize, preprocess_kimi_vl  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402

IMG, BOI, EOI = 500, 501, 502


def _image(seed=0, h=80, w=60):
    from PIL import Image

    return Image.fromarray(np.random.default_rng(seed).integers(0, 255, (h, w, 3), dtype=np.uint8))


def _hf_model(tmp_path):
    T = transformers
    torch.manual_seed(0)
    tc = dict(model_type="deepseek_v3", vocab_size=512, hidden_size=256, intermediate_size=256, num_hidden_layers=2,
              num_attention_heads=16, num_key_value_heads=16, q_lora_rank=None, kv_lora_rank=512,
              qk_nope_head_dim=32, qk_rope_head_dim=64, v_head_dim=32, moe_intermediate_size=64,
              n_routed_experts=8, num_experts_per_tok=2, n_shared_experts=1, first_k_dense_replace=1, n_group=2,
              topk_group=1, routed_scaling_factor=2.0, norm_topk_prob=True, max_position_embeddings=2048,
              tie_word_embeddings=False)
    vc = dict(hidden_size=64, num_hidden_layers=2, num_attention_heads=4, intermediate_size=96, patch_size=14,
              pos_emb_height=6, pos_emb_width=6, merge_kernel_size=[2, 2])
    cfg = T.Kimi_K25Config(text_config=tc, vision_config=vc, image_token_id=IMG, vision_start_token_id=BOI,
                           vision_end_token_id=EOI, projection_hidden_size=64, tie_word_embeddings=False)
    m = T.Kimi_K25ForConditionalGeneration(cfg)
    with torch.no_grad():
        for n, p in m.named_parameters():
            if "norm" in n:
                p.normal_(1.0, 0.1) if n.endswith("weight") else p.normal_(0.0, 0.05)
            else:
                p.normal_(0.0, 0.08)
        for n, b in m.named_buffers():
            if n.endswith("e_score_correction_bias"):
                b.normal_(0.0, 0.05)
    m = m.float().eval()
    for c in (m.config, m.config.vision_config, m.config.text_config):
        c._attn_implementation = "eager"
    # the in-memory (transformers) names: save_pretrained's legacy-name conversion for this family
    # also rewrites the language model's names (``self_attn.q_proj`` -> ``self_wqkv``)
    tmp_path.mkdir(parents=True, exist_ok=True)
    save_file({k: v.contiguous() for k, v in m.state_dict().items()}, str(tmp_path / "model.safetensors"))
    m.config.architectures = ["Kimi_K25ForConditionalGeneration"]
    m.config.to_json_file(str(tmp_path / "config.json"))
    m.generation_config.eos_token_id = None
    return m


def _to_original(src, dst, heads, hd):
    """Re-lay a saved transformers checkpoint into the original Kimi-VL names / qkv layout."""
    import shutil

    dst.mkdir()
    w = {}
    for f in src.glob("*.safetensors"):
        w.update(load_file(str(f)))
    # rotate-half rows (j, j + hd/2) -> interleaved pairs (2j, 2j + 1)
    inv = torch.empty(hd, dtype=torch.long)
    inv[torch.cat([torch.arange(0, hd, 2), torch.arange(1, hd, 2)])] = torch.arange(hd)

    def interleave(t):
        return t.reshape(heads, hd, *t.shape[1:])[:, inv].reshape(t.shape)

    out, blocks = {}, {}
    for n, t in w.items():
        if n.startswith("model.vision_tower."):
            r = n[len("model.vision_tower."):]
            if r.startswith("layers."):
                p = r.split(".")
                b, mod, kind = int(p[1]), ".".join(p[2:-1]), p[-1]
                if mod in ("attn.q_proj", "attn.k_proj", "attn.v_proj"):
                    blocks.setdefault((b, kind), {})[mod] = t
                    continue
                mod = {"attn.proj": "wo", "norm1": "norm0", "norm2": "norm1", "mlp.fc1": "mlp.fc0",
                       "mlp.fc2": "mlp.fc1"}[mod]
                out[f"vision_tower.encoder.blocks.{b}.{mod}.{kind}"] = t
            elif r.startswith("final_layernorm."):
                out["vision_tower.encoder." + r] = t
            elif r == "patch_embed.pos_emb.position_embeddings":
                out["vision_tower.patch_embed.pos_emb.weight"] = t
            else:
                out["vision_tower." + r] = t
        elif n.startswith("model.mm_projector."):
            r = n[len("model.mm_projector."):]
            r = r.replace("in_proj", "linear_1").replace("out_proj", "linear_2")
            out["multi_modal_projector." + r] = t
        elif n.startswith("model.language_model."):
            out["language_model.model." + n[len("model.language_model."):]] = t
        elif n == "lm_head.weight":
            out["language_model.lm_head.weight"] = t
        else:
            out[n] = t
    for (b, kind), d in blocks.items():
        out[f"vision_tower.encoder.blocks.{b}.wqkv.{kind}"] = torch.cat(
            [interleave(d["attn.q_proj"]), interleave(d["attn.k_proj"]), d["attn.v_proj"]])
    save_file({k: v.contiguous() for k, v in out.items()}, str(dst / "model.safetensors"))
    cfg = json.loads((src / "config.json").read_text())
    vc = cfg.pop("vision_config")
    cfg.update(architectures=["KimiVLForConditionalGeneration"], model_type="kimi_vl",
               media_placeholder_token_id=cfg.pop("image_token_id"),
               vision_config=dict(model_type="moonvit", patch_size=vc["patch_size"],
                                  init_pos_emb_height=vc["pos_emb_height"], init_pos_emb_width=vc["pos_emb_width"],
                                  num_attention_heads=vc["num_attention_heads"],
                                  num_hidden_layers=vc["num_hidden_layers"], hidden_size=vc["hidden_size"],
                                  intermediate_size=vc["intermediate_size"], merge_kernel_size=vc["merge_kernel_size"]))
    (dst / "config.json").write_text(json.dumps(cfg))
    for f in src.glob("generation_config.json"):
        shutil.copy(f, dst / f.name)


def _flat(pv):
    return pv.reshape(pv.shape[0], -1)


def test_kimi_resize_rule():
    assert kimi_resize(80, 60) == ((80, 60), (84, 84))
    (nh, nw), (ph, pw) = kimi_resize(2000, 1000, max_patches=4096)
    assert (2000 // 14) * (1000 // 14) > 4096 and (nh // 14) * (nw // 14) <= 4096
    assert ph % 28 == 0 and pw % 28 == 0 and ph - nh < 28 and pw - nw < 28
    pv, g = preprocess_kimi_vl(_image(0, 80, 60))
    assert g == (1, 6, 6) and pv.shape == (36, 3 * 14 * 14)
    # zero padding happens before normalisation: padded pixels are (0 - 0.5) / 0.5
    assert np.allclose(pv.reshape(6, 6, 3, 14, 14)[:, 5, :, :, 4:], -1.0)


@pytest.mark.parametrize("layout", ["transformers", "original"])
def test_kimi_vl_matches_hf(tmp_path, layout):
    hf = _hf_model(tmp_path / "hf")
    path = tmp_path / "hf"
    if layout == "original":
        path = tmp_path / "orig"
        _to_original(tmp_path / "hf", path, heads=4, hd=16)
    imgs = [_image(0, 80, 60), _image(1, 60, 110)]
    eng = Engine(EngineArgs(model_path=str(path), device="cpu", dtype="float32", max_running_requests=4,
                            context_length=1024))
    m = eng.runner.model
    assert type(m).__name__ == "KimiVLForConditionalGeneration"
    pre = [preprocess_kimi_vl(im) for im in imgs]
    pv = torch.cat([torch.from_numpy(p) for p, _ in pre]).reshape(-1, 3, 14, 14)
    grid = torch.tensor([g for _, g in pre])
    with torch.no_grad():
        want = torch.cat(list(hf.model.get_image_features(pixel_values=pv, image_grid_thw=grid).pooler_output))
    got = m.encode_images(_flat(pv), [tuple(g) for g in grid.tolist()])
    assert (got - want).abs().max().item() < 1e-3, (got - want).abs().max()
    prompt = [1, 9, BOI, IMG, EOI, 33, 41, BOI, IMG, EOI, 12, 7]
    req = eng.make_mm_request(prompt, imgs, SamplingParams(max_new_tokens=6, ignore_eos=True, logprobs=True))
    ex = list(req.prompt_ids)
    for s, k in req.mm.spans:
        ex[s:s + k] = [IMG] * k
    assert ex.count(IMG) == want.shape[0]
    eng.add_request(req)
    while not req.finished:
        eng.step()
    ids = torch.tensor([ex])
    with torch.no_grad():
        out = hf.generate(ids, pixel_values=pv, image_grid_thw=grid, max_new_tokens=6, do_sample=False,
                          output_scores=True, return_dict_in_generate=True)
    ref = out.sequences[0, len(ex):].tolist()
    assert req.output_ids == ref
    ref_lp = [torch.log_softmax(s[0].float(), -1)[tk].item() for s, tk in zip(out.scores, ref)]
    assert np.allclose(req.output_logprobs, ref_lp, atol=2e-3), (req.output_logprobs, ref_lp)
