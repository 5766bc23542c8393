"""Qwen-Image MMDiT (diffusers ``QwenImageTransformer2DModel``) on the ome_amd kernels.

Reference catalog: ``config/runtimes/srt/Qwen/Qwen-Image-rt.yaml:15`` (``QwenImagePipeline``),
``Qwen-Image-Edit-rt.yaml`` and ``Qwen-Image-Edit-Plus-rt.yaml``.  60 dual-stream blocks,
3072 wide (24 x 128 heads), 20B parameters -- 41 GB of bf16 on one MI355X.

Per block, for the image stream (packed 2x2 latent patches) and the text stream (Qwen2.5-VL
hidden states) separately: AdaLN modulation from the timestep embedding (SiLU -> GEMM -> shift /
scale / gate x 2) applied as the affine of the LayerNorm kernel itself (weight 1 + scale, bias
shift: one launch per sample), ONE fused q|k|v GEMM per stream (the three diffusers projections
concatenated at load), then ``ome_qk_norm_rope``: per-head RMSNorm + 3-axis complex RoPE (frame,
height, width; centred for images, text after the largest image index) written straight into the
joint [text; image] sequence of each sample (v copied there by the same kernel) -- no per-block
gathers; ONE joint attention over all samples -- the classifier-free-guidance pair (prompt,
negative prompt) rides in the same launch as two packed varlen sequences
(``ops.varlen_attention``: bidirectional MFMA flash attention, no padding) -- out projections on
row gathers of the attention output, gated residuals (in-place addcmul per sample), and the
GELU-tanh MLPs.  Weights keep the diffusers names (q / k / v fused at load).
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
        self._fuse()
        return self

    _QKV = {"img": ("to_q", "to_k", "to_v"), "txt": ("add_q_proj", "add_k_proj", "add_v_proj")}

    def _fuse(self) -> None:
        """[q; k; v] of each stream -> one GEMM weight (the three originals are dropped)."""
        for i in range(self.L):
            p = f"transformer_blocks.{i}.attn."
            for st, names in self._QKV.items():
                if p + names[0] + ".weight" not in self.w:
                    continue
                for kind in ("weight", "bias"):
                    self.w[p + f"{st}_qkv.{kind}"] = torch.cat([self.w.pop(p + f"{n}.{kind}") for n in names], 0)

    def state_dict(self) -> dict[str, torch.Tensor]:
        """Weights under their diffusers names (fused q|k|v split back into views)."""
        out = {}
        for k, t in self.w.items():
            if k.endswith(("img_qkv.weight", "img_qkv.bias", "txt_qkv.weight", "txt_qkv.bias")):
                pre, st, kind = k[:k.rindex(".", 0, k.rindex("."))], k.split(".")[-2][:3], k.split(".")[-1]
                for n, part in zip(self._QKV[st], t.chunk(3, 0)):
                    out[f"{pre}.{n}.{kind}"] = part
            else:
                out[k] = t
        return out

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
        self._fuse()
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

    # ------------------------------------------------------------------ forward
    def _mod_norm(self, x: torch.Tensor, shift: torch.Tensor, scale: torch.Tensor, rows: list[int]) -> torch.Tensor:
        """LayerNorm(x) * (1 + scale_b) + shift_b per sample: the modulation IS the LayerNorm's affine
        (weight 1 + scale_b, bias shift_b), one launch per sample's rows."""
        out = torch.empty_like(x)
        r0 = 0
        for bb, n in enumerate(rows):
            ops.layernorm(x[r0:r0 + n], (1 + scale[bb]).contiguous(), shift[bb].contiguous(), self.eps,
                          out=out[r0:r0 + n])
            r0 += n
        return out

    @staticmethod
    def _gated_add(x: torch.Tensor, g: torch.Tensor, y: torch.Tensor, rows: list[int]) -> None:
        """x += g_b * y over each sample's rows (in place)."""
        r0 = 0
        for bb, n in enumerate(rows):
            x[r0:r0 + n].addcmul_(y[r0:r0 + n], g[bb])
            r0 += n

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
        # (cos, sin) tables once per forward, fp32 [rows, hd/2, 2]
        cs_img = torch.stack([img_ang.cos(), img_ang.sin()], -1).repeat(B, 1, 1).contiguous()
        cs_txt = torch.stack([txt_ang.cos(), txt_ang.sin()], -1).contiguous()
        lens = [n + N for n in lt]
        nr, tr = [N] * B, lt
        total = sum(lens)
        # joint packed sequence per sample = [text_b; image_b]: destination rows of both streams
        starts = [sum(lens[:bb]) for bb in range(B)]
        dst_img = torch.cat([torch.arange(st + lt[bb], st + lens[bb]) for bb, st in enumerate(starts)])
        dst_txt = torch.cat([torch.arange(st, st + lt[bb]) for bb, st in enumerate(starts)])
        dst_img, dst_txt = dst_img.to(self.device), dst_txt.to(self.device)
        di32, dt32 = dst_img.to(torch.int32), dst_txt.to(torch.int32)
        for i in range(self.L):
            p = f"transformer_blocks.{i}."
            a = p + "attn."
            im = linear(temb_act, w[p + "img_mod.1.weight"], w[p + "img_mod.1.bias"]).view(B, 6, D)
            tm = linear(temb_act, w[p + "txt_mod.1.weight"], w[p + "txt_mod.1.bias"]).view(B, 6, D)
            pi = linear(self._mod_norm(x, im[:, 0], im[:, 1], nr), w[a + "img_qkv.weight"], w[a + "img_qkv.bias"])
            pt = linear(self._mod_norm(c, tm[:, 0], tm[:, 1], tr), w[a + "txt_qkv.weight"], w[a + "txt_qkv.bias"])
            q = torch.empty(total, H, hd, dtype=self.dtype, device=self.device)
            k, v = torch.empty_like(q), torch.empty_like(q)
            # per-head RMSNorm + 3-axis RoPE written straight into the joint sequences
            for src, cs, dst, nq, nk in ((pi, cs_img, di32, "norm_q", "norm_k"),
                                         (pt, cs_txt, dt32, "norm_added_q", "norm_added_k")):
                ops.qk_norm_rope(src[:, :D], H, hd, w[a + nq + ".weight"], cs, self.eps, q, dst)
                ops.qk_norm_rope(src[:, D:2 * D], H, hd, w[a + nk + ".weight"], cs, self.eps, k, dst)
                ops.qk_norm_rope(src[:, 2 * D:], H, hd, None, None, self.eps, v, dst)
            o = ops.varlen_attention(q, k, v, lens, hd ** -0.5).reshape(total, D)
            self._gated_add(x, im[:, 2], linear(o.index_select(0, dst_img), w[a + "to_out.0.weight"],
                                                w[a + "to_out.0.bias"]), nr)
            self._gated_add(c, tm[:, 2], linear(o.index_select(0, dst_txt), w[a + "to_add_out.weight"],
                                                w[a + "to_add_out.bias"]), tr)
            for st, mod, rows in (("img", im, nr), ("txt", tm, tr)):
                src = x if st == "img" else c
                hn = self._mod_norm(src, mod[:, 3], mod[:, 4], rows)
                f = ops.act(linear(hn, w[p + f"{st}_mlp.net.0.proj.weight"], w[p + f"{st}_mlp.net.0.proj.bias"]), 1)
                self._gated_add(src, mod[:, 5], linear(f, w[p + f"{st}_mlp.net.2.weight"],
                                                       w[p + f"{st}_mlp.net.2.bias"]), rows)
        e = linear(temb_act, w["norm_out.linear.weight"], w["norm_out.linear.bias"]).view(B, 2, D)
        x = self._mod_norm(x, e[:, 1], e[:, 0], nr)   # AdaLayerNormContinuous: (scale, shift) order
        return linear(x, w["proj_out.weight"], w["proj_out.bias"]).view(B, N, -1)
