"""Qwen-Image diffusion path (``ome_amd/diffusion``) on CPU.  diffusers is not importable here, so
every piece is checked against an independent fp32 restatement of the published diffusers
semantics (parity with diffusers itself unpinned):

* sampler: the exponential dynamic shift + terminal stretch schedule in closed form;
* MMDiT: per-sample joint attention with complex (``torch.polar``) 3-axis RoPE, (shift, scale,
  gate) modulation, AdaLayerNormContinuous (scale, shift) -- against the packed two-sample
  (prompt / negative prompt of different lengths) forward;
* VAE: the causal 3-D convolutions run as ``F.conv3d`` over [0, 0, frame] (two zero frames of
  causal padding) with the full 5-D kernels, against the 2-D last-tap form;
* pipelines: text-to-image determinism and CFG, edit with an input image, the OpenAI images
  HTTP endpoint."""
import base64
import io
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from ome_amd.diffusion.pipeline import QwenImagePipeline, pack, unpack
from ome_amd.diffusion.qwen_image_dit import QwenImageDiT
from ome_amd.diffusion.scheduler import FlowMatchConfig, sigmas_for
from ome_amd.diffusion.vae import QwenImageVAE

CFG = dict(num_layers=2, num_attention_heads=2, attention_head_dim=64, joint_attention_dim=96, in_channels=64,
           out_channels=16, patch_size=2, axes_dims_rope=[16, 24, 24])


def test_schedule_closed_form():
    c = FlowMatchConfig()
    s = sigmas_for(10, 4096, c)
    mu = 4096 * (0.9 - 0.5) / (8192 - 256) + 0.5 - (0.9 - 0.5) / (8192 - 256) * 256
    t = np.linspace(1.0, 0.1, 10)
    sh = math.exp(mu) / (math.exp(mu) + (1 / t - 1))
    st = 1 - (1 - sh) / ((1 - sh[-1]) / (1 - 0.02))
    assert np.allclose(s[:-1], st) and s[-1] == 0.0
    assert abs(s[-2] - 0.02) < 1e-12 and s[0] == pytest.approx(1.0)
    assert np.all(np.diff(s) < 0)


# ------------------------------------------------------------------ MMDiT reference
def _ref_dit(w, cfg, img, txts, t, shapes):
    H, hd = cfg["num_attention_heads"], cfg["attention_head_dim"]
    D = H * hd
    a0, a1, a2 = cfg["axes_dims_rope"]

    def rope_params(index, dim):
        f = torch.outer(index.double(), 1.0 / torch.pow(10000, torch.arange(0, dim, 2).double().div(dim)))
        return torch.polar(torch.ones_like(f), f)

    pos = torch.arange(4096)
    neg = torch.arange(4096).flip(0) * -1 - 1
    pf = torch.cat([rope_params(pos, a0), rope_params(pos, a1), rope_params(pos, a2)], 1)
    nf = torch.cat([rope_params(neg, a0), rope_params(neg, a1), rope_params(neg, a2)], 1)
    sp = [a0 // 2, a1 // 2, a2 // 2]
    fp, fn = pf.split(sp, 1), nf.split(sp, 1)
    vid, top = [], 0
    for idx, (f, h, ww) in enumerate(shapes):
        fr = fp[0][idx:idx + f].view(f, 1, 1, -1).expand(f, h, ww, -1)
        fh = torch.cat([fn[1][-(h - h // 2):], fp[1][:h // 2]], 0).view(1, h, 1, -1).expand(f, h, ww, -1)
        fw = torch.cat([fn[2][-(ww - ww // 2):], fp[2][:ww // 2]], 0).view(1, 1, ww, -1).expand(f, h, ww, -1)
        vid.append(torch.cat([fr, fh, fw], -1).reshape(f * h * ww, -1))
        top = max(top, h // 2, ww // 2)
    vid = torch.cat(vid)

    def rot(x, fr):   # x [S, H, hd]
        xc = torch.view_as_complex(x.double().reshape(*x.shape[:-1], -1, 2))
        return torch.view_as_real(xc * fr[:, None]).flatten(-2).float()

    def lin(x, n):
        return x @ w[n + ".weight"].float().T + w[n + ".bias"].float()

    def rms(x, n):
        return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + 1e-6) * w[n].float()

    def ln(x):
        return F.layer_norm(x, (x.shape[-1],), eps=1e-6)

    half = 128
    ex = torch.exp(-math.log(10000) * torch.arange(half).float() / half)
    outs = []
    for b in range(len(txts)):
        a = 1000 * t[b] * ex
        e = torch.cat([a.cos(), a.sin()])
        temb = lin(F.silu(lin(e, "time_text_embed.timestep_embedder.linear_1")), "time_text_embed.timestep_embedder.linear_2")
        x = lin(img[b].float(), "img_in")
        c = lin(rms(txts[b].float(), "txt_norm.weight"), "txt_in")
        tf = pf[top:top + c.shape[0]]
        for i in range(cfg["num_layers"]):
            p = f"transformer_blocks.{i}."
            im = lin(F.silu(temb), p + "img_mod.1")
            tm = lin(F.silu(temb), p + "txt_mod.1")
            (i1, i2), (t1, t2) = im.chunk(2), tm.chunk(2)

            def modulate(z, mp):
                sh, sc, g = mp.chunk(3)
                return z * (1 + sc) + sh, g

            xi, gi = modulate(ln(x), i1)
            xt, gt = modulate(ln(c), t1)
            q = rms(lin(xi, p + "attn.to_q").view(-1, H, hd), p + "attn.norm_q.weight")
            k = rms(lin(xi, p + "attn.to_k").view(-1, H, hd), p + "attn.norm_k.weight")
            v = lin(xi, p + "attn.to_v").view(-1, H, hd)
            q2 = rms(lin(xt, p + "attn.add_q_proj").view(-1, H, hd), p + "attn.norm_added_q.weight")
            k2 = rms(lin(xt, p + "attn.add_k_proj").view(-1, H, hd), p + "attn.norm_added_k.weight")
            v2 = lin(xt, p + "attn.add_v_proj").view(-1, H, hd)
            q, k, q2, k2 = rot(q, vid), rot(k, vid), rot(q2, tf), rot(k2, tf)
            jq, jk, jv = (torch.cat([u2, u]).transpose(0, 1) for u2, u in ((q2, q), (k2, k), (v2, v)))
            o = F.scaled_dot_product_attention(jq, jk, jv).transpose(0, 1).reshape(-1, D)
            L = c.shape[0]
            x = x + gi * lin(o[L:], p + "attn.to_out.0")
            c = c + gt * lin(o[:L], p + "attn.to_add_out")
            hx, g2 = modulate(ln(x), i2)
            x = x + g2 * lin(F.gelu(lin(hx, p + "img_mlp.net.0.proj"), approximate="tanh"), p + "img_mlp.net.2")
            hc, g3 = modulate(ln(c), t2)
            c = c + g3 * lin(F.gelu(lin(hc, p + "txt_mlp.net.0.proj"), approximate="tanh"), p + "txt_mlp.net.2")
        sc, sh = lin(F.silu(temb), "norm_out.linear").chunk(2)
        outs.append(lin(ln(x) * (1 + sc) + sh, "proj_out"))
    return torch.stack(outs)


def test_dit_matches_reference():
    dit = QwenImageDiT(CFG, "cpu", torch.float32).init_random(3, std=0.08)
    shapes = [(1, 4, 6), (1, 2, 4)]   # generated latents + one conditioning image (edit layout)
    N = sum(f * h * w for f, h, w in shapes)
    g = torch.Generator().manual_seed(0)
    img = torch.randn(1, N, 64, generator=g).expand(2, N, 64).contiguous()
    txts = [torch.randn(7, 96, generator=g), torch.randn(4, 96, generator=g)]
    t = torch.tensor([0.7, 0.7])
    got = dit.forward(img, txts, t, shapes)
    want = _ref_dit(dit.state_dict(), CFG, img, txts, t, shapes)
    assert got.shape == want.shape == (2, N, 64)
    assert (got - want).abs().max().item() < 2e-3 * want.abs().max().item(), (got - want).abs().max()


# ------------------------------------------------------------------ VAE reference
VCFG = dict(base_dim=8, z_dim=4, dim_mult=[1, 2, 2], num_res_blocks=1,
            latents_mean=[0.1, -0.2, 0.0, 0.3], latents_std=[1.5, 0.8, 1.0, 2.0])


def _vae_weights(vae, seed=0):
    g = torch.Generator().manual_seed(seed)
    out = {}
    for k, s in vae.shapes().items():
        if k.endswith(".gamma"):
            out[k] = 1 + 0.1 * torch.randn(*s, generator=g)
        elif k.endswith(".bias"):
            out[k] = 0.05 * torch.randn(*s, generator=g)
        else:
            out[k] = torch.randn(*s, generator=g) * (s[1] * s[-1] * s[-2]) ** -0.5
    return out


def _ref_vae(w, cfg, z=None, img=None):
    """Literal causal-3D semantics on a single frame (T = 1): pad two zero frames in front."""
    def conv(x, n, stride=1):
        k = w[n + ".weight"]
        if k.dim() == 5:
            kt, kh = k.shape[2], k.shape[3]
            x5 = F.pad(x[:, :, None], (kh // 2, kh // 2, kh // 2, kh // 2, kt - 1, 0))
            return F.conv3d(x5, k, w[n + ".bias"])[:, :, 0]
        return F.conv2d(x, k, w[n + ".bias"], stride=stride, padding=k.shape[-1] // 2 if stride == 1 else 0)

    def norm(x, n):
        return F.normalize(x, dim=1) * x.shape[1] ** 0.5 * w[n + ".gamma"].reshape(1, -1, 1, 1)

    def res(x, n):
        h = conv(x, n + ".conv_shortcut") if n + ".conv_shortcut.weight" in w else x
        y = conv(F.silu(norm(x, n + ".norm1")), n + ".conv1")
        return conv(F.silu(norm(y, n + ".norm2")), n + ".conv2") + h

    def attn(x, n):
        B, C, Hh, W = x.shape
        qkv = F.conv2d(norm(x, n + ".norm"), w[n + ".to_qkv.weight"], w[n + ".to_qkv.bias"])
        q, k, v = qkv.reshape(B, 1, 3 * C, -1).permute(0, 1, 3, 2).chunk(3, -1)
        o = F.scaled_dot_product_attention(q, k, v).squeeze(1).permute(0, 2, 1).reshape(B, C, Hh, W)
        return x + F.conv2d(o, w[n + ".proj.weight"], w[n + ".proj.bias"])

    mean = torch.tensor(cfg["latents_mean"]).view(1, -1, 1, 1)
    std = torch.tensor(cfg["latents_std"]).view(1, -1, 1, 1)
    nl = len(cfg["dim_mult"])
    if z is not None:
        x = conv(z * std + mean, "post_quant_conv")
        x = conv(x, "decoder.conv_in")
        x = res(attn(res(x, "decoder.mid_block.resnets.0"), "decoder.mid_block.attentions.0"), "decoder.mid_block.resnets.1")
        for i in range(nl):
            for r in range(cfg["num_res_blocks"] + 1):
                x = res(x, f"decoder.up_blocks.{i}.resnets.{r}")
            if i != nl - 1:
                x = F.conv2d(F.interpolate(x, scale_factor=2.0, mode="nearest-exact"),
                             w[f"decoder.up_blocks.{i}.upsamplers.0.resample.1.weight"],
                             w[f"decoder.up_blocks.{i}.upsamplers.0.resample.1.bias"], padding=1)
        return conv(F.silu(norm(x, "decoder.norm_out")), "decoder.conv_out").clamp(-1, 1)
    x = conv(img, "encoder.conv_in")
    k = 0
    for i in range(nl):
        for _ in range(cfg["num_res_blocks"]):
            x = res(x, f"encoder.down_blocks.{k}")
            k += 1
        if i != nl - 1:
            x = F.conv2d(F.pad(x, (0, 1, 0, 1)), w[f"encoder.down_blocks.{k}.resample.1.weight"],
                         w[f"encoder.down_blocks.{k}.resample.1.bias"], stride=2)
            k += 1
    x = res(attn(res(x, "encoder.mid_block.resnets.0"), "encoder.mid_block.attentions.0"), "encoder.mid_block.resnets.1")
    x = conv(F.silu(norm(x, "encoder.norm_out")), "encoder.conv_out")
    mu = conv(x, "quant_conv")[:, :cfg["z_dim"]]
    return (mu - mean) / std


def test_vae_single_frame_equals_causal_3d():
    vae = QwenImageVAE(VCFG, "cpu", torch.float32)
    w = _vae_weights(vae)
    vae.load(w.items())
    g = torch.Generator().manual_seed(1)
    z = torch.randn(1, 4, 5, 6, generator=g)
    out = vae.decode(z)
    assert out.shape == (1, 3, 20, 24)
    assert torch.allclose(out, _ref_vae(w, VCFG, z=z), atol=1e-4)
    img = torch.rand(1, 3, 32, 24, generator=g) * 2 - 1
    lat = vae.encode(img)
    assert lat.shape == (1, 4, 8, 6)
    assert torch.allclose(lat, _ref_vae(w, VCFG, img=img), atol=1e-4)


def test_pack_roundtrip():
    x = torch.randn(1, 16, 6, 8)
    p = pack(x)
    assert p.shape == (1, 12, 64) and torch.equal(unpack(p, 6, 8), x)
    assert torch.equal(p[0, 0, :4], x[0, 0, :2, :2].reshape(-1))   # channel-major 2x2 patch


@pytest.fixture(scope="module")
def pipe():
    return QwenImagePipeline.random("tiny-qwen-image", "t2i", device="cpu", dtype=torch.float32)


def test_t2i_deterministic_and_cfg(pipe):
    a = pipe("a red cube on a table", width=64, height=48, steps=3, seed=5)
    b = pipe("a red cube on a table", width=64, height=48, steps=3, seed=5)
    assert a.shape == (48, 64, 3) and a.dtype == np.uint8 and np.array_equal(a, b)
    c = pipe("a red cube on a table", negative_prompt=" ", width=64, height=48, steps=3, seed=5, true_cfg_scale=4.0)
    assert c.shape == a.shape and not np.array_equal(a, c)
    assert pipe.stats["images"] == 3


def test_edit_pipeline_runs():
    from PIL import Image

    p = QwenImagePipeline.random("tiny-qwen-image", "edit", device="cpu", dtype=torch.float32)
    src = Image.fromarray(np.random.default_rng(0).integers(0, 255, (40, 56, 3), dtype=np.uint8))
    out = p("make it blue", width=64, height=64, steps=2, seed=1, images=[src])
    assert out.shape == (64, 64, 3)


def test_images_http_endpoint(pipe):
    from fastapi.testclient import TestClient

    from ome_amd.diffusion.server import build_app

    client = TestClient(build_app(pipe, "Qwen/Qwen-Image"))
    assert client.get("/health").status_code == 200
    assert client.get("/v1/models").json()["data"][0]["id"] == "Qwen/Qwen-Image"
    r = client.post("/v1/images/generations", json={"prompt": "a cat", "size": "64x32", "n": 1,
                                                   "num_inference_steps": 2, "seed": 3})
    assert r.status_code == 200, r.text
    from PIL import Image

    im = Image.open(io.BytesIO(base64.b64decode(r.json()["data"][0]["b64_json"])))
    assert im.size == (64, 32)
    assert "ome_images_generated_total" in client.get("/metrics").text
