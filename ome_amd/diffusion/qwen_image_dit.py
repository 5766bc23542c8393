"""Qwen-Image MMDiT (diffusers ``QwenImageTransformer2DModel``) on the ome_amd kernels.

Reference catalog: ``config/runtimes/srt/Qwen/Qwen-Image-rt.yaml:15`` (``QwenImagePipeline``),
``Qwen-Image-Edit-rt.yaml`` and ``Qwen-Image-Edit-Plus-rt.yaml``.  60 dual-stream blocks,
3072 wide (24 x 128 heads), 20B parameters -- 41 GB of bf16 on one MI355X.

Per block, for the image stream (packed 2x2 latent patches) and the text stream (Qwen2.5-VL
hidden states) separately: AdaLN modulation from the timestep embedding (SiLU -> GEMM -> shift /
scale / gate x 2), affine-free LayerNorm, q / k / v GEMMs, per-head RMSNorm on q / k, 3-axis
complex RoPE (frame, height, width; centred for images, text after the largest image index);
then ONE joint attention over [text; image] of each sample -- the classifier-free-guidance pair
(prompt, negative prompt) rides in the same launch as two packed varlen sequences
(``ops.varlen_attention``: bidirectional MFMA flash attention, no padding) -- out projections,
gated residuals, and the GELU-tanh MLPs.  Weights keep the diffusers names.
"""
from __future__ import annotations

import math

import torch

from ome_amd import ops
from ome_amd.models.quant import linear


class QwenImageDiT:
    def __init__(self, cfg: dict, device="cuda", dtype=torch.bfloat16):
        self.cfg = dict(cfg)
        self.device, self.dtype = torch.device(device), dtype
        self.heads = int(cfg.get("num_attention_heads", 24))
        self.hd = int(cfg.get("attention_head_dim", 128))
        self.D = self.heads * self.hd
        self.L = int(cfg.get("num_layers", 60))
        self.cin = int(cfg.get("in_channels", 64))
        self.cout = int(cfg.get("out_channels", 16))
        self.patch = int(cfg.get("patch_size", 2))
        self.txt_dim = int(cfg.get("joint_attention_dim", 3584))
        self.axes = [int(a) for a in cfg.get("axes_dims_rope", (16, 56, 56))]
        if sum(self.axes) != self.hd:
            raise ValueError(f"axes_dims_rope {self.axes} must sum to the head dim {self.hd}")
        self.eps = 1e-6
        self.w: dict[str, torch.Tensor] = {}
        self._ones = torch.ones(self.D, dtype=dtype, device=self.device)
        self._zeros = torch.zeros(self.D, dtype=dtype, device=self.device)
        self._freq_cache: dict = {}

    # ------------------------------------------------------------------ weights
    def shapes(self) -> dict[str, tuple]:
        D, I, hd = self.D, 4 * self.D, self.hd
        s = {"img_in.weight": (D, self.cin), "img_in.bias": (D,), "txt_norm.weight": (self.txt_dim,),
             "txt_in.weight": (D, self.txt_dim), "txt_in.bias": (D,),
             "time_text_embed.timestep_embedder.linear_1.weight": (D, 256),
             "time_text_embed.timestep_embedder.linear_1.bias": (D,),
             "time_text_embed.timestep_embedder.linear_2.weight": (D, D),
             "time_text_embed.timestep_embedder.linear_2.bias": (D,),
             "norm_out.linear.weight": (2 * D, D), "norm_out.linear.bias": (2 * D,),
             "proj_out.weight": (self.patch ** 2 * self.cout, D), "proj_out.bias": (self.patch ** 2 * self.cout,)}
        for i in range(self.L):
            p = f"transformer_blocks.{i}."
            for st in ("img", "txt"):
                s[p + f"{st}_mod.1.weight"], s[p + f"{st}_mod.1.bias"] = (6 * D, D), (6 * D,)
                s[p + f"{st}_mlp.net.0.proj.weight"], s[p + f"{st}_mlp.net.0.proj.bias"] = (I, D), (I,)
                s[p + f"{st}_mlp.net.2.weight"], s[p + f"{st}_mlp.net.2.bias"] = (D, I), (D,)
            for n in ("to_q", "to_k", "to_v", "add_q_proj", "add_k_proj", "add_v_proj", "to_out.0", "to_add_out"):
                s[p + f"attn.{n}.weight"], s[p + f"attn.{n}.bias"] = (D, D), (D,)
            for n in ("norm_q", "norm_k", "norm_added_q", "norm_added_k"):
                s[p + f"attn.{n}.weight"] = (hd,)
        return s

    def init_random(self, seed: int = 0, std: float = 0.02) -> "QwenImageDiT":
        g = torch.Generator(device=self.device)
        g.manual_seed(seed)
        for k, shp in self.shapes().items():
            t = torch.empty(*shp, dtype=self.dtype, device=self.device)
            if k.endswith("norm.weight") or ".norm_" in k:
                t.fill_(1.0)
            elif k.endswith(".bias"):
                t.normal_(0.0, std * 0.1, generator=g)
            else:
                t.normal_(0.0, std, generator=g)
            self.w[k] = t
        return self

    def load(self, weights) -> "QwenImageDiT":
        want = self.shapes()
        for name, t in weights:
            if name in want:
                if tuple(t.shape) != want[name]:
                    raise ValueError(f"{name}: shape {tuple(t.shape)} != {want[name]}")
                self.w[name] = t.to(device=self.device, dtype=self.dtype).contiguous()
        missing = [k for k in want if k not in self.w]
        if missing:
            raise ValueError(f"transformer checkpoint incomplete: {missing[:4]}")
        return self

    def weight_bytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in self.w.values())

    # ------------------------------------------------------------------ embeddings
    def timestep_embedding(self, t: torch.Tensor) -> torch.Tensor:
        """t [B] in [0, 1] (sigma) -> [B, D]: sinusoid(256, flip to cos|sin, scale 1000) -> MLP."""
        half = 128
        ex = torch.exp(-math.log(10000.0) * torch.arange(half, dtype=torch.float32, device=t.device) / half)
        a = 1000.0 * t.float()[:, None] * ex[None]
        e = torch.cat([a.cos(), a.sin()], -1).to(self.dtype)
        p = "time_text_embed.timestep_embedder."
        h = linear(e, self.w[p + "linear_1.weight"], self.w[p + "linear_1.bias"])
        return linear(ops.act(h.contiguous(), 0), self.w[p + "linear_2.weight"], self.w[p + "linear_2.bias"])

    def _axis(self, pos: torch.Tensor, dim: int) -> torch.Tensor:
        inv = 1.0 / torch.pow(10000.0, torch.arange(0, dim, 2, dtype=torch.float64) / dim)
        return pos.double()[:, None] * inv[None]

    def rope_angles(self, img_shapes: list[tuple[int, int, int]], txt_len: int) -> tuple[torch.Tensor, torch.Tensor]:
        """(image angles [sum f*h*w, hd/2], text angles [txt_len, hd/2]) of the 3-axis RoPE: frame =
        image index, height / width centred (-(n - n//2) .. n//2 - 1), text from the largest
        half-extent on (all three axes at the same position)."""
        key = (tuple(img_shapes), txt_len)
        got = self._freq_cache.get(key)
        if got is not None:
            return got
        a0, a1, a2 = self.axes
        parts, top = [], 0
        for idx, (f, h, w) in enumerate(img_shapes):
            fr = self._axis(torch.arange(idx, idx + f), a0)
            hh = self._axis(torch.cat([torch.arange(-(h - h // 2), 0), torch.arange(h // 2)]), a1)
            ww = self._axis(torch.cat([torch.arange(-(w - w // 2), 0), torch.arange(w // 2)]), a2)
            ang = torch.cat([fr[:, None, None].expand(f, h, w, -1), hh[None, :, None].expand(f, h, w, -1),
                             ww[None, None, :].expand(f, h, w, -1)], -1).reshape(f * h * w, -1)
            parts.append(ang)
            top = max(top, h // 2, w // 2)
        tp = torch.arange(top, top + txt_len)
        txt = torch.cat([self._axis(tp, a0), self._axis(tp, a1), self._axis(tp, a2)], -1)
        got = (torch.cat(parts).float().to(self.device), txt.float().to(self.device))
        self._freq_cache[key] = got
        return got

    @staticmethod
    def _rope(x: torch.Tensor, ang: torch.Tensor) -> torch.Tensor:
        """x [T, H, hd] with (even, odd) pairs as complex numbers, rotated by ang [T, hd/2]."""
        xf = x.float().view(*x.shape[:-1], -1, 2)
        c, s = ang.cos()[:, None, :], ang.sin()[:, None, :]
        re, im = xf[..., 0], xf[..., 1]
        return torch.stack([re * c - im * s, re * s + im * c], -1).flatten(-2).to(x.dtype)

    # ------------------------------------------------------------------ forward
    def _mod_norm(self, x: torch.Tensor, shift: torch.Tensor, scale: torch.Tensor, rows: list[int]) -> torch.Tensor:
        """affine-free LayerNorm, then x * (1 + scale_b) + shift_b per sample (rows per sample)."""
        h = ops.layernorm(x.contiguous(), self._ones, self._zeros, self.eps)
        if len(rows) == 1:
            return h * (1 + scale[0]) + shift[0]
        sc = torch.repeat_interleave(1 + scale, torch.tensor(rows, device=x.device), 0)
        sh = torch.repeat_interleave(shift, torch.tensor(rows, device=x.device), 0)
        return h * sc + sh

    def _gate(self, g: torch.Tensor, rows: list[int]) -> torch.Tensor:
        return g[0] if len(rows) == 1 else torch.repeat_interleave(g, torch.tensor(rows, device=g.device), 0)

    def forward(self, img: torch.Tensor, txt: list[torch.Tensor], t: torch.Tensor,
                img_shapes: list[tuple[int, int, int]]) -> torch.Tensor:
        """img [B, N, in_channels] packed latents (every sample the same image layout), txt: B text
        hidden-state tensors [L_b, txt_dim] (lengths may differ), t [B] sigma in [0, 1] ->
        velocity [B, N, patch^2 * out_channels]."""
        w, D, H, hd = self.w, self.D, self.heads, self.hd
        B, N, _ = img.shape
        lt = [int(x.shape[0]) for x in txt]
        x = linear(img.reshape(B * N, -1).to(self.dtype), w["img_in.weight"], w["img_in.bias"])
        c = torch.cat([u.to(device=self.device, dtype=self.dtype) for u in txt], 0)
        c = linear(ops.rmsnorm(c.contiguous(), w["txt_norm.weight"], self.eps), w["txt_in.weight"], w["txt_in.bias"])
        temb = self.timestep_embedding(t.to(self.device))
        temb_act = ops.act(temb.clone(), 0)    # SiLU(temb), shared by every modulation GEMM
        img_ang, txt_ang_full = self.rope_angles(img_shapes, max(lt))
        txt_ang = torch.cat([txt_ang_full[:n] for n in lt], 0)
        img_ang_b = img_ang.repeat(B, 1)
        lens = [n + N for n in lt]
        nr, tr = [N] * B, lt
        toff = [0]
        for n in lt:
            toff.append(toff[-1] + n)
        for i in range(self.L):
            p = f"transformer_blocks.{i}."
            im = linear(temb_act, w[p + "img_mod.1.weight"], w[p + "img_mod.1.bias"]).view(B, 6, D)
            tm = linear(temb_act, w[p + "txt_mod.1.weight"], w[p + "txt_mod.1.bias"]).view(B, 6, D)
            xi = self._mod_norm(x, im[:, 0], im[:, 1], nr)
            xt = self._mod_norm(c, tm[:, 0], tm[:, 1], tr)

            def qkv(h, pre, names):
                q = linear(h, w[pre + names[0] + ".weight"], w[pre + names[0] + ".bias"]).view(-1, H, hd)
                k = linear(h, w[pre + names[1] + ".weight"], w[pre + names[1] + ".bias"]).view(-1, H, hd)
                v = linear(h, w[pre + names[2] + ".weight"], w[pre + names[2] + ".bias"]).view(-1, H, hd)
                return q, k, v

            qi, ki, vi = qkv(xi, p + "attn.", ("to_q", "to_k", "to_v"))
            qt, kt, vt = qkv(xt, p + "attn.", ("add_q_proj", "add_k_proj", "add_v_proj"))
            qi = self._rope(ops.rmsnorm(qi.reshape(-1, hd), w[p + "attn.norm_q.weight"], self.eps).view(-1, H, hd),
                            img_ang_b)
            ki = self._rope(ops.rmsnorm(ki.reshape(-1, hd), w[p + "attn.norm_k.weight"], self.eps).view(-1, H, hd),
                            img_ang_b)
            qt = self._rope(ops.rmsnorm(qt.reshape(-1, hd), w[p + "attn.norm_added_q.weight"], self.eps)
                            .view(-1, H, hd), txt_ang)
            kt = self._rope(ops.rmsnorm(kt.reshape(-1, hd), w[p + "attn.norm_added_k.weight"], self.eps)
                            .view(-1, H, hd), txt_ang)
            # joint [text_b; image_b] sequences, packed
            js = lambda a, b: torch.cat([z for bb in range(B) for z in (a[toff[bb]:toff[bb + 1]],  # noqa: E731
                                                                          b[bb * N:(bb + 1) * N])], 0)
            o = ops.varlen_attention(js(qt, qi), js(kt, ki), js(vt, vi), lens, hd ** -0.5).reshape(-1, D)
            oi = torch.cat([o[sum(lens[:bb]) + lt[bb]:sum(lens[:bb + 1])] for bb in range(B)], 0)
            ot = torch.cat([o[sum(lens[:bb]):sum(lens[:bb]) + lt[bb]] for bb in range(B)], 0)
            x = x + self._gate(im[:, 2], nr) * linear(oi.contiguous(), w[p + "attn.to_out.0.weight"],
                                                      w[p + "attn.to_out.0.bias"])
            c = c + self._gate(tm[:, 2], tr) * linear(ot.contiguous(), w[p + "attn.to_add_out.weight"],
                                                      w[p + "attn.to_add_out.bias"])
            for st, mod, rows in (("img", im, nr), ("txt", tm, tr)):
                src = x if st == "img" else c
                hn = self._mod_norm(src, mod[:, 3], mod[:, 4], rows)
                f = ops.act(linear(hn, w[p + f"{st}_mlp.net.0.proj.weight"], w[p + f"{st}_mlp.net.0.proj.bias"]), 1)
                y = linear(f, w[p + f"{st}_mlp.net.2.weight"], w[p + f"{st}_mlp.net.2.bias"])
                if st == "img":
                    x = x + self._gate(mod[:, 5], rows) * y
                else:
                    c = c + self._gate(mod[:, 5], rows) * y
        e = linear(temb_act, w["norm_out.linear.weight"], w["norm_out.linear.bias"]).view(B, 2, D)
        x = self._mod_norm(x, e[:, 1], e[:, 0], nr)   # AdaLayerNormContinuous: (scale, shift) order
        return linear(x, w["proj_out.weight"], w["proj_out.bias"]).view(B, N, -1)
