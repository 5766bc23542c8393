"""MiniCPM-V 2.6 (``models/minicpmv.py``) on CPU.  No MiniCPM-V 2.6 class is importable, so the
reference is assembled from library modules: transformers' Idefics2 NaViT embeddings (bucketised
positions over variable patch grids) + SigLIP encoder / post-LayerNorm for the vision tower, torch
``nn.MultiheadAttention`` + LayerNorms for the resampler (with an independent 2-D sin-cos table),
and transformers' Qwen2 for the language model (manual greedy over inputs_embeds).  Checks the
slicing geometry, the prompt expansion (image-id / image / slice markers, row newlines), the image
features and greedy generation through the engine (fp32, CPU reference ops)."""
import json

import numpy as np
import pytest
import torch

transformers = pytest.importorskip("transformers")
PIL = pytest.importorskip("PIL")

from ome_amd.io.safetensors import save_file  # noqa: E402
from ome_amd.models.minicpmv import preprocess_minicpmv, sliced_grid  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402

V, H, E, NQ, SCALE, PS = 600, 256, 64, 4, 56, 14
MARK = ("<image>", "</image>", "<slice>", "</slice>", "<image_id>", "</image_id>")


def _build(tmp_path):
    T = transformers
    torch.manual_seed(0)
    lc = T.Qwen2Config(vocab_size=V, hidden_size=H, intermediate_size=512, num_hidden_layers=2, num_attention_heads=4,
                       num_key_value_heads=2, max_position_embeddings=1024, tie_word_embeddings=False)
    lm = T.Qwen2ForCausalLM(lc)
    vc = T.SiglipVisionConfig(hidden_size=E, intermediate_size=128, num_hidden_layers=2, num_attention_heads=2,
                              image_size=70, patch_size=PS)
    vis = T.SiglipVisionModel(vc)
    for m in (lm, vis):
        with torch.no_grad():
            for n, p in m.named_parameters():
                if "norm" in n:
                    p.normal_(1.0, 0.1) if n.endswith("weight") else p.normal_(0.0, 0.05)
                else:
                    p.normal_(0.0, 0.08)
        m.float().eval()
        m.config._attn_implementation = "eager"
    g = torch.Generator().manual_seed(2)
    r = lambda *s, std=0.08: torch.randn(*s, generator=g) * std  # noqa: E731
    rs = {"query": r(NQ, H, std=0.5), "kv_proj.weight": r(H, E), "attn.in_proj_weight": r(3 * H, H),
          "attn.in_proj_bias": r(3 * H, std=0.02), "attn.out_proj.weight": r(H, H), "attn.out_proj.bias": r(H),
          "ln_q.weight": 1 + r(H), "ln_q.bias": r(H), "ln_kv.weight": 1 + r(H), "ln_kv.bias": r(H),
          "ln_post.weight": 1 + r(H), "ln_post.bias": r(H), "proj": r(H, H)}
    sd = {"llm." + k: v.detach().clone().contiguous() for k, v in lm.state_dict().items()}
    for k, v in vis.state_dict().items():
        k = k[len("vision_model."):] if k.startswith("vision_model.") else k
        sd["vpm." + k] = v.detach().clone().contiguous()
    sd.update({"resampler." + k: v.contiguous() for k, v in rs.items()})
    save_file(sd, tmp_path / "model.safetensors")
    cfg = {k: v for k, v in lc.to_dict().items() if k not in ("architectures", "model_type", "transformers_version")}
    cfg.update(architectures=["MiniCPMV"], model_type="minicpmv", version=2.6, query_num=NQ, slice_mode=True,
               use_image_id=True, drop_vision_last_layer=False,
               slice_config={"max_slice_nums": 4, "patch_size": PS, "scale_resolution": SCALE},
               vision_config={k: vc.to_dict()[k] for k in ("hidden_size", "intermediate_size", "num_hidden_layers",
                                                           "num_attention_heads", "image_size", "patch_size",
                                                           "hidden_act", "layer_norm_eps")})
    (tmp_path / "config.json").write_text(json.dumps(cfg))
    from tokenizers import AddedToken, Tokenizer
    from tokenizers.models import WordLevel

    vocab = {f"t{i}": i for i in range(570)}
    vocab.update({str(d): 570 + d for d in range(10)})
    vocab["Ċ"] = 580
    tok = Tokenizer(WordLevel(vocab, unk_token="t0"))
    tok.add_special_tokens([AddedToken(t, special=True) for t in MARK])   # 581 .. 586
    tok.save(str(tmp_path / "tokenizer.json"))
    return lm, vis, rs


def _sincos(dim, h, w):
    gw, gh = np.meshgrid(np.arange(w, dtype=np.float32), np.arange(h, dtype=np.float32))
    out = []
    for pos in (gw, gh):
        om = 1.0 / 10000 ** (np.arange(dim // 4, dtype=np.float32) / (dim / 4.0))
        a = pos[..., None] * om
        out += [np.sin(a), np.cos(a)]
    return torch.from_numpy(np.concatenate(out, -1)).reshape(h * w, dim)


def _ref_features(vis, rs, rows, grids):
    vc = vis.config
    ic = transformers.Idefics2VisionConfig(hidden_size=E, image_size=vc.image_size, patch_size=PS)
    emb = transformers.models.idefics2.modeling_idefics2.Idefics2VisionEmbeddings(ic)
    sdv = vis.state_dict()
    pre = "vision_model." if any(k.startswith("vision_model.") for k in sdv) else ""
    emb.load_state_dict({"patch_embedding.weight": sdv[pre + "embeddings.patch_embedding.weight"],
                         "patch_embedding.bias": sdv[pre + "embeddings.patch_embedding.bias"],
                         "position_embedding.weight": sdv[pre + "embeddings.position_embedding.weight"]})
    core = vis.vision_model if hasattr(vis, "vision_model") else vis
    mha = torch.nn.MultiheadAttention(H, H // 128, batch_first=False)
    mha.load_state_dict({"in_proj_weight": rs["attn.in_proj_weight"], "in_proj_bias": rs["attn.in_proj_bias"],
                         "out_proj.weight": rs["attn.out_proj.weight"], "out_proj.bias": rs["attn.out_proj.bias"]})
    ln = lambda x, k: torch.nn.functional.layer_norm(x, (x.shape[-1],), rs[k + ".weight"], rs[k + ".bias"], 1e-6)  # noqa
    outs, off = [], 0
    with torch.no_grad():
        for _, h, w in grids:
            x = rows[off:off + h * w]
            off += h * w
            img = x.view(h, w, 3, PS, PS).permute(2, 0, 3, 1, 4).reshape(1, 3, h * PS, w * PS)
            e = emb(img, torch.ones(1, h, w, dtype=torch.bool))
            f = core.post_layernorm(core.encoder(e).last_hidden_state)[0]
            kv = ln(f @ rs["kv_proj.weight"].T, "ln_kv")
            q = ln(rs["query"], "ln_q")
            o = mha(q[:, None], (kv + _sincos(H, h, w))[:, None], kv[:, None])[0][:, 0]
            outs.append(ln(o, "ln_post") @ rs["proj"])
    return torch.cat(outs)


def test_slice_grid_choice():
    assert sliced_grid(448, 448, 9, 448) is None                  # one slice's worth: not split
    assert sliced_grid(1344, 448, 9, 448) == (3, 1)               # 3:1 panorama -> 3 x 1
    assert sliced_grid(1000, 1000, 9, 448) in ((2, 2),)           # ceil(4.98) = 5 -> 2 x 2 is the closest square


def test_minicpmv_matches_reference(tmp_path):
    from PIL import Image

    lm, vis, rs = _build(tmp_path)
    img = Image.fromarray(np.random.default_rng(0).integers(0, 255, (60, 100, 3), dtype=np.uint8))
    rows, g, layout = preprocess_minicpmv(img, 4, SCALE, PS)
    assert layout == (2, 1) and len(g) == 3
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=2,
                            context_length=512))
    m = eng.runner.model
    grids = [(1, h, w) for h, w in g]
    want = _ref_features(vis, rs, rows, grids)
    got = m.encode_images(rows, grids)
    assert got.shape == want.shape == (3 * NQ, H)
    assert (got - want).abs().max().item() < 1e-3, (got - want).abs().max()
    IMG = m.image_id
    assert IMG == 581
    prompt = [1, 9, IMG, 12, 7]
    req = eng.make_mm_request(prompt, [img], SamplingParams(max_new_tokens=5, ignore_eos=True))
    # <image_id> 0 </image_id> <image> f*4 </image> <slice> f*4 </slice> <slice> f*4 </slice>
    ids = req.prompt_ids
    assert ids[:2] == [1, 9] and ids[2:5] == [585, 570, 586] and ids[5] == 581 and ids[10] == 582
    assert ids[11] == 583 and ids[16] == 584 and ids[17] == 583 and ids[22] == 584 and ids[23:] == [12, 7]
    assert req.mm.spans == [(6, NQ), (12, NQ), (18, NQ)]
    eng.add_request(req)
    while not req.finished:
        eng.step()
    t = torch.tensor(ids)
    with torch.no_grad():
        emb = lm.get_input_embeddings()(t)
        for k, (s, n) in enumerate(req.mm.spans):
            emb[s:s + n] = want[k * NQ:(k + 1) * NQ]
        toks = []
        for _ in range(5):
            nxt = int(lm(inputs_embeds=emb[None]).logits[0, -1].argmax())
            toks.append(nxt)
            emb = torch.cat([emb, lm.get_input_embeddings()(torch.tensor([nxt]))], 0)
    assert req.output_ids == toks
