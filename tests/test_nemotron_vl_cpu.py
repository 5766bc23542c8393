"""Nemotron Nano v2 VL (``models/nemotron_vl.py``) on CPU: a tiny random checkpoint in the remote
code's layout (``language_model.*`` = transformers' NemotronH, ``vision_model.radio_model.*`` =
RADIO ViT, ``mlp1.*``) under both architecture names.  The image features are checked against an
independent fp32 restatement of RADIO (CPE table resize + window, class / register tokens,
pre-norm blocks, final LayerNorm) + 0.5 pixel shuffle + RMSNorm / ReLU^2 projector, and greedy
generation with an image through the engine against transformers' NemotronH fed the same
embeddings.  RADIO and the remote code are not importable here: parity with them is unpinned."""
import json

import numpy as np
import pytest
import torch
import torch.nn.functional as F

transformers = pytest.importorskip("transformers")
PIL = pytest.importorskip("PIL")

from ome_amd.io.safetensors import save_file  # noqa: E402
from ome_amd.models.internvl import preprocess_internvl  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402
from ome_amd.runtime.request import SamplingParams  # noqa: E402

IMG, START, END = 500, 501, 502
E, HEADS, DEPTH, PS, SIZE, GRID, NSKIP, PH = 64, 2, 2, 16, 64, 8, 4, 256
MEAN, STD = (0.5, 0.4, 0.3), (0.2, 0.25, 0.3)


def _radio(g):
    r = lambda *s, std=0.05: torch.randn(*s, generator=g) * std  # noqa: E731
    w = {"patch_generator.embedder.weight": r(E, 3 * PS * PS), "patch_generator.pos_embed": r(1, GRID * GRID, E),
         "patch_generator.cls_token.token": r(NSKIP, E, std=0.5), "norm.weight": 1 + r(E, std=0.1),
         "norm.bias": r(E)}
    for b in range(DEPTH):
        p = f"blocks.{b}."
        w.update({p + "norm1.weight": 1 + r(E, std=0.1), p + "norm1.bias": r(E), p + "attn.qkv.weight": r(3 * E, E, std=0.1),
                  p + "attn.qkv.bias": r(3 * E), p + "attn.proj.weight": r(E, E), p + "attn.proj.bias": r(E),
                  p + "norm2.weight": 1 + r(E, std=0.1), p + "norm2.bias": r(E), p + "mlp.fc1.weight": r(4 * E, E),
                  p + "mlp.fc1.bias": r(4 * E), p + "mlp.fc2.weight": r(E, 4 * E), p + "mlp.fc2.bias": r(E)})
    return w


def _radio_ref(w, px):
    n, s = px.shape[0], SIZE // PS
    x = px.reshape(n, 3, s, PS, s, PS).permute(0, 2, 4, 1, 3, 5).reshape(n, s * s, -1)
    x = x @ w["patch_generator.embedder.weight"].T
    tab = w["patch_generator.pos_embed"].view(1, GRID, GRID, E).permute(0, 3, 1, 2)
    tab = F.interpolate(tab, size=(s, s), mode="bilinear", align_corners=True)[0, :, :s, :s]
    x = x + tab.permute(1, 2, 0).reshape(s * s, E)
    x = torch.cat([w["patch_generator.cls_token.token"].expand(n, NSKIP, E), x], 1)
    for b in range(DEPTH):
        p = f"blocks.{b}."
        h = F.layer_norm(x, (E,), w[p + "norm1.weight"], w[p + "norm1.bias"], 1e-6)
        q, k, v = (h @ w[p + "attn.qkv.weight"].T + w[p + "attn.qkv.bias"]).view(n, -1, 3, HEADS, E // HEADS).unbind(2)
        a = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2))
        x = x + a.transpose(1, 2).reshape(n, -1, E) @ w[p + "attn.proj.weight"].T + w[p + "attn.proj.bias"]
        h = F.layer_norm(x, (E,), w[p + "norm2.weight"], w[p + "norm2.bias"], 1e-6)
        x = x + F.gelu(h @ w[p + "mlp.fc1.weight"].T + w[p + "mlp.fc1.bias"]) @ w[p + "mlp.fc2.weight"].T + \
            w[p + "mlp.fc2.bias"]
    x = F.layer_norm(x, (E,), w["norm.weight"], w["norm.bias"], 1e-6)
    return x[:, NSKIP:]


def _features_ref(w, proj, px):
    """RADIO -> InternVL pixel shuffle (v2) -> RMSNorm -> Linear -> ReLU^2 -> Linear."""
    f = _radio_ref(w, px)
    n, s = f.shape[0], SIZE // PS
    x = f.reshape(n, s, s, E)
    x = x.view(n, s, s // 2, E * 2).permute(0, 2, 1, 3).reshape(n, s // 2, s // 2, E * 4)
    x = x.permute(0, 2, 1, 3).reshape(-1, E * 4)
    x = x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-5) * proj["mlp1.0.weight"]
    return F.relu(x @ proj["mlp1.1.weight"].T).pow(2) @ proj["mlp1.3.weight"].T


def _build(tmp_path, arch):
    torch.manual_seed(0)
    lc = transformers.NemotronHConfig(
        vocab_size=512, hidden_size=128, num_attention_heads=4, num_key_value_heads=2, head_dim=32,
        intermediate_size=256, mamba_num_heads=8, mamba_head_dim=16, ssm_state_size=32, n_groups=2, conv_kernel=4,
        hybrid_override_pattern="M*-M-", max_position_embeddings=512, chunk_size=16, pad_token_id=0,
        bos_token_id=1, eos_token_id=2)
    lm = transformers.NemotronHForCausalLM(lc)
    with torch.no_grad():
        for n, p in lm.named_parameters():
            if n.endswith("norm.weight") or n.endswith("norm_f.weight"):
                p.normal_(1.0, 0.1)
            elif n.endswith("A_log"):
                p.uniform_(-1.0, 1.0)
            elif n.endswith("dt_bias"):
                p.normal_(-1.0, 0.5)
            elif n.endswith(".D"):
                p.normal_(1.0, 0.2)
            else:
                p.normal_(0.0, 0.08)
    lm = lm.float().eval()
    lm.config._attn_implementation = "eager"
    g = torch.Generator().manual_seed(3)
    radio = _radio(g)
    proj = {"mlp1.0.weight": 1 + torch.randn(4 * E, generator=g) * 0.1,
            "mlp1.1.weight": torch.randn(PH, 4 * E, generator=g) * 0.05,
            "mlp1.3.weight": torch.randn(128, PH, generator=g) * 0.05}
    sd = {"language_model." + k: v.detach().clone().contiguous() for k, v in lm.state_dict().items()}
    sd.update({"vision_model.radio_model.model." + k: v.contiguous() for k, v in radio.items()})
    sd["vision_model.radio_model.input_conditioner.norm_mean"] = torch.tensor(MEAN).view(3, 1, 1)
    sd["vision_model.radio_model.input_conditioner.norm_std"] = torch.tensor(STD).view(3, 1, 1)
    sd.update({k: v.contiguous() for k, v in proj.items()})
    save_file(sd, tmp_path / "model.safetensors")
    llm = lc.to_dict()
    llm["architectures"] = ["NemotronHForCausalLM"]
    cfg = {"architectures": [arch], "model_type": "NemotronH_Nano_VL_V2", "llm_config": llm,
           "vision_config": {"hidden_size": E, "num_attention_heads": HEADS, "num_hidden_layers": DEPTH,
                             "patch_size": PS, "cpe_max_size": GRID * PS, "model_type": "radio"},
           "force_image_size": SIZE, "patch_size": PS, "downsample_ratio": 0.5, "img_context_token_id": IMG,
           "max_dynamic_patch": 4, "use_thumbnail": True, "projector_hidden_size": PH, "vit_hidden_size": E,
           "norm_mean": list(MEAN), "norm_std": list(STD)}
    (tmp_path / "config.json").write_text(json.dumps(cfg))
    # the <img> / </img> ids come from the tokenizer's added tokens
    from tokenizers import AddedToken, Tokenizer
    from tokenizers.models import WordLevel

    tok = Tokenizer(WordLevel({f"t{i}": i for i in range(IMG)}, unk_token="t0"))
    tok.add_special_tokens([AddedToken(t, special=True) for t in ("<image>", "<img>", "</img>")])   # 500, 501, 502
    tok.save(str(tmp_path / "tokenizer.json"))
    return lm, radio, proj


@pytest.mark.parametrize("arch", ["NemotronH_Nano_VL_V2", "NemotronVLForConditionalGeneration"])
def test_nemotron_vl_matches_reference(tmp_path, arch):
    from PIL import Image

    lm, radio, proj = _build(tmp_path, arch)
    img = Image.fromarray(np.random.default_rng(0).integers(0, 255, (70, 130, 3), dtype=np.uint8))
    px = preprocess_internvl(img, SIZE, 4, True, MEAN, STD)
    assert px.shape[0] == 3   # 2 x 1 tiles + thumbnail
    eng = Engine(EngineArgs(model_path=str(tmp_path), device="cpu", dtype="float32", max_running_requests=2,
                            context_length=512))
    m = eng.runner.model
    assert m.image_prompt_ids() == [START, IMG, END]
    want = _features_ref(radio, proj, px)
    got = m.encode_images(px)
    assert got.shape == want.shape == (3 * 4, 128)
    assert (got - want).abs().max().item() < 1e-3, (got - want).abs().max()
    prompt = [1, 9, START, IMG, END, 12, 7, 40]
    req = eng.make_mm_request(prompt, [img], SamplingParams(max_new_tokens=5, ignore_eos=True))
    assert req.mm.spans == [(3, 12)]
    eng.add_request(req)
    while not req.finished:
        eng.step()
    ids = torch.tensor(req.prompt_ids)
    with torch.no_grad():
        emb = lm.get_input_embeddings()(ids.clamp(max=511))
        emb[3:15] = want
        toks = []
        for _ in range(5):   # greedy without a cache: NemotronH.generate takes no inputs_embeds
            nxt = int(lm(inputs_embeds=emb[None], use_cache=False).logits[0, -1].argmax())
            toks.append(nxt)
            emb = torch.cat([emb, lm.get_input_embeddings()(torch.tensor([nxt]))], 0)
    assert req.output_ids == toks
