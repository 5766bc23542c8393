"""Qwen-Image VAE (diffusers ``AutoencoderKLQwenImage``, the Wan-2.1 causal video VAE) for still
images.

A still image is one latent frame; every causal 3-D convolution of the video VAE then sees its
own frame plus two zero frames of causal padding, so it IS the 2-D convolution with the kernel's
last temporal tap -- and the temporal up / down-sampling convolutions are skipped on the first
chunk.  So the image path runs as plain 2-D convolutions (MIOpen through PyTorch-ROCm, channels
in bf16) with the checkpoint's 5-D weights sliced once at load:

* norm: channel RMS normalisation ``normalize(x, dim=1) * sqrt(C) * gamma``;
* residual blocks: norm -> SiLU -> conv3x3 -> norm -> SiLU -> conv3x3 (+ 1x1 shortcut);
* mid block: res -> single-head spatial self-attention (1x1 qkv / proj) -> res;
* decoder: conv_in, mid, up blocks (3 res blocks, then nearest 2x + conv3x3 to half the
  channels), norm, SiLU, conv_out -> clamp [-1, 1]; encoder: conv_in, down blocks (2 res blocks,
  then zero-pad (0, 1, 0, 1) + stride-2 conv3x3), mid, norm, SiLU, conv_out -> (mu, logvar);
* latents are normalised by the config's per-channel ``latents_mean`` / ``latents_std``.
Weights keep the diffusers names (``decoder.up_blocks.0.resnets.1.conv2.weight`` ...).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


class QwenImageVAE:
    def __init__(self, cfg: dict, device="cuda", dtype=torch.bfloat16):
        self.cfg = dict(cfg)
        self.device, self.dtype = torch.device(device), dtype
        self.base = int(cfg.get("base_dim", 96))
        self.z = int(cfg.get("z_dim", 16))
        self.mult = [int(m) for m in cfg.get("dim_mult", (1, 2, 4, 4))]
        self.nres = int(cfg.get("num_res_blocks", 2))
        if cfg.get("attn_scales"):
            raise NotImplementedError("VAE attention at down / up scales")
        self.mean = torch.tensor(cfg.get("latents_mean") or [0.0] * self.z, dtype=torch.float32)
        self.std = torch.tensor(cfg.get("latents_std") or [1.0] * self.z, dtype=torch.float32)
        self.w: dict[str, torch.Tensor] = {}

    # ------------------------------------------------------------------ structure
    def _enc_dims(self):
        d = [self.base * m for m in [1] + self.mult]
        return list(zip(d[:-1], d[1:]))

    def _dec_dims(self):
        d = [self.base * m for m in [self.mult[-1]] + self.mult[::-1]]
        out = []
        for i, (a, b) in enumerate(zip(d[:-1], d[1:])):
            out.append((a // 2 if i > 0 else a, b))
        return out

    def shapes(self) -> dict[str, tuple]:
        s: dict[str, tuple] = {}

        def conv(name, cin, cout, k=3, t=3):
            s[name + ".weight"] = (cout, cin, t, k, k)
            s[name + ".bias"] = (cout,)

        def res(name, cin, cout):
            s[name + ".norm1.gamma"] = (cin, 1, 1, 1)
            conv(name + ".conv1", cin, cout)
            s[name + ".norm2.gamma"] = (cout, 1, 1, 1)
            conv(name + ".conv2", cout, cout)
            if cin != cout:
                conv(name + ".conv_shortcut", cin, cout, 1, 1)

        def mid(name, dim):
            res(name + ".resnets.0", dim, dim)
            s[name + ".attentions.0.norm.gamma"] = (dim, 1, 1)
            s[name + ".attentions.0.to_qkv.weight"], s[name + ".attentions.0.to_qkv.bias"] = (3 * dim, dim, 1, 1), (3 * dim,)
            s[name + ".attentions.0.proj.weight"], s[name + ".attentions.0.proj.bias"] = (dim, dim, 1, 1), (dim,)
            res(name + ".resnets.1", dim, dim)

        # encoder
        ed = self._enc_dims()
        conv("encoder.conv_in", 3, ed[0][0])
        k = 0
        for i, (a, b) in enumerate(ed):
            for r in range(self.nres):
                res(f"encoder.down_blocks.{k}", a if r == 0 else b, b)
                k += 1
            if i != len(self.mult) - 1:
                s[f"encoder.down_blocks.{k}.resample.1.weight"] = (b, b, 3, 3)
                s[f"encoder.down_blocks.{k}.resample.1.bias"] = (b,)
                k += 1
        top = ed[-1][1]
        mid("encoder.mid_block", top)
        s["encoder.norm_out.gamma"] = (top, 1, 1, 1)
        conv("encoder.conv_out", top, 2 * self.z)
        conv("quant_conv", 2 * self.z, 2 * self.z, 1, 1)
        # decoder
        conv("post_quant_conv", self.z, self.z, 1, 1)
        dd = self._dec_dims()
        conv("decoder.conv_in", self.z, dd[0][0])
        mid("decoder.mid_block", dd[0][0])
        for i, (a, b) in enumerate(dd):
            for r in range(self.nres + 1):
                res(f"decoder.up_blocks.{i}.resnets.{r}", a if r == 0 else b, b)
            if i != len(self.mult) - 1:
                s[f"decoder.up_blocks.{i}.upsamplers.0.resample.1.weight"] = (b // 2, b, 3, 3)
                s[f"decoder.up_blocks.{i}.upsamplers.0.resample.1.bias"] = (b // 2,)
        s["decoder.norm_out.gamma"] = (dd[-1][1], 1, 1, 1)
        conv("decoder.conv_out", dd[-1][1], 3)
        return s

    def _put(self, name: str, t: torch.Tensor) -> None:
        if t.dim() == 5:   # causal 3-D kernel on a first (only) frame: its last temporal tap
            t = t[:, :, -1]
        elif name.endswith(".gamma"):
            t = t.reshape(-1)
        self.w[name] = t.to(device=self.device, dtype=self.dtype).contiguous()

    def init_random(self, seed: int = 0, std: float = 0.05) -> "QwenImageVAE":
        g = torch.Generator(device="cpu")
        g.manual_seed(seed)
        for k, shp in self.shapes().items():
            if k.endswith(".gamma"):
                t = 1.0 + 0.1 * torch.randn(*shp, generator=g)
            elif k.endswith(".bias"):
                t = 0.01 * torch.randn(*shp, generator=g)
            else:
                fan = shp[1] * (shp[-1] * shp[-2])
                t = torch.randn(*shp, generator=g) * (fan ** -0.5)
            self._put(k, t)
        return self

    def load(self, weights, parts: tuple[str, ...] = ("encoder", "decoder")) -> "QwenImageVAE":
        want = self.shapes()
        for name, t in weights:
            if name in want:
                self._put(name, t)
        need = [k for k in want if any(k.startswith(p) or (p == "decoder" and k.startswith("post_quant")) or
                                       (p == "encoder" and k.startswith("quant_conv")) for p in parts)]
        missing = [k for k in need if k not in self.w]
        if missing:
            raise ValueError(f"VAE checkpoint incomplete: {missing[:4]}")
        return self

    # ------------------------------------------------------------------ ops
    def _conv(self, x, name, stride=1, pad=None):
        wt = self.w[name + ".weight"]
        p = wt.shape[-1] // 2 if pad is None else pad
        return F.conv2d(x, wt, self.w.get(name + ".bias"), stride=stride, padding=p)

    def _norm(self, x, name):
        g = self.w[name + ".gamma"]
        return F.normalize(x.float(), dim=1).mul_(x.shape[1] ** 0.5).to(x.dtype) * g.view(1, -1, 1, 1)

    def _res(self, x, name):
        h = self._conv(x, name + ".conv_shortcut") if name + ".conv_shortcut.weight" in self.w else x
        y = self._conv(F.silu(self._norm(x, name + ".norm1")), name + ".conv1")
        y = self._conv(F.silu(self._norm(y, name + ".norm2")), name + ".conv2")
        return y + h

    def _attn(self, x, name):
        B, C, H, W = x.shape
        h = self._norm(x, name + ".norm")
        qkv = self._conv(h, name + ".to_qkv", pad=0).view(B, 3 * C, H * W).transpose(1, 2)
        q, k, v = qkv.chunk(3, -1)
        o = F.scaled_dot_product_attention(q[:, None], k[:, None], v[:, None])[:, 0]
        return x + self._conv(o.transpose(1, 2).reshape(B, C, H, W), name + ".proj", pad=0)

    def _mid(self, x, name):
        x = self._res(x, name + ".resnets.0")
        return self._res(self._attn(x, name + ".attentions.0"), name + ".resnets.1")

    # ------------------------------------------------------------------ decode / encode
    def decode(self, z: torch.Tensor) -> torch.Tensor:
        """normalised latents [B, z, h, w] -> image [B, 3, 8h, 8w] in [-1, 1]."""
        x = z.to(self.device, torch.float32) * self.std.to(self.device).view(1, -1, 1, 1) + \
            self.mean.to(self.device).view(1, -1, 1, 1)
        x = self._conv(x.to(self.dtype), "post_quant_conv", pad=0)
        x = self._mid(self._conv(x, "decoder.conv_in"), "decoder.mid_block")
        for i in range(len(self.mult)):
            for r in range(self.nres + 1):
                x = self._res(x, f"decoder.up_blocks.{i}.resnets.{r}")
            if i != len(self.mult) - 1:
                x = F.interpolate(x, scale_factor=2.0, mode="nearest")
                x = self._conv(x, f"decoder.up_blocks.{i}.upsamplers.0.resample.1")
        x = self._conv(F.silu(self._norm(x, "decoder.norm_out")), "decoder.conv_out")
        return x.float().clamp_(-1.0, 1.0)

    def encode(self, img: torch.Tensor) -> torch.Tensor:
        """image [B, 3, H, W] in [-1, 1] -> normalised latent mean [B, z, H/8, W/8]."""
        x = self._conv(img.to(self.device, self.dtype), "encoder.conv_in")
        k = 0
        for i in range(len(self.mult)):
            for _ in range(self.nres):
                x = self._res(x, f"encoder.down_blocks.{k}")
                k += 1
            if i != len(self.mult) - 1:
                x = self._conv(F.pad(x, (0, 1, 0, 1)), f"encoder.down_blocks.{k}.resample.1", stride=2, pad=0)
                k += 1
        x = self._mid(x, "encoder.mid_block")
        x = self._conv(F.silu(self._norm(x, "encoder.norm_out")), "encoder.conv_out")
        mu = self._conv(x, "quant_conv", pad=0)[:, :self.z].float()
        return (mu - self.mean.to(self.device).view(1, -1, 1, 1)) / self.std.to(self.device).view(1, -1, 1, 1)
