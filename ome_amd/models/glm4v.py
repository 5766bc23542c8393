"""GLM-4.5V (``Glm4vMoeForConditionalGeneration``; reference catalog
``config/runtimes/srt/zai-org/glm-4-5v-rt.yaml``) on the Qwen2-VL image path of ``qwen2_vl.py``.

* preprocessing: the GLM-4V resize rule (sides multiples of 28, upscale below 28 px, area
  bounds counted over the 2-frame temporal patch), bicubic, CLIP mean / std, Qwen2-VL patch
  order (merge-block major);
* vision tower: patch GEMM (+bias) -> RMSNorm -> learned 2D positions bicubically resampled to
  each image's patch grid (``grid_sample``, border padding) -> blocks of RMSNorm -> fused QKV
  GEMM -> 2D rotary -> varlen MFMA attention per image -> O GEMM; RMSNorm -> SwiGLU (fused
  gate|up GEMM + SiLU-and-mul kernel) -> post-RMSNorm -> 2 x 2 down-sampling convolution as one
  GEMM over each merge block -> merger (GEMM -> LayerNorm -> GELU -> SwiGLU);
* language model: GLM-4.5 MoE -- biased q / k / v, partial (1/2) NeoX rotary with M-RoPE
  sections over the rotary half, sigmoid router with the selection-only
  ``e_score_correction_bias`` and grouped top-k (``ome_moe_route`` noaux_tc), routed scaling,
  un-gated shared experts, dense first layers -- the ``moe.py`` grouped MFMA experts.
"""
from __future__ import annotations

import dataclasses
import math

import numpy as np
import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.models.config import ModelConfig
from ome_amd.models.moe import MoEForCausalLM
from ome_amd.models.quant import linear
from ome_amd.models.qwen2_vl import Qwen2VisionTower, Qwen2VLForConditionalGeneration
from ome_amd.multimodal.inputs import CLIP_MEAN, CLIP_STD, load_image, patchify
from ome_amd.parallel import state as pstate


def glm4v_smart_resize(h: int, w: int, factor: int = 28, min_pixels: int = 112 * 112,
                       max_pixels: int = 28 * 28 * 15000, frames: int = 2) -> tuple[int, int]:
    if h < factor or w < factor:
        s = max(factor / h, factor / w)
        h, w = int(h * s), int(w * s)
    if max(h, w) / min(h, w) > 200:
        raise ValueError("image aspect ratio must be < 200")
    hb, wb = round(h / factor) * factor, round(w / factor) * factor
    if frames * hb * wb > max_pixels:
        beta = math.sqrt(frames * h * w / max_pixels)
        hb, wb = max(factor, math.floor(h / beta / factor) * factor), max(factor, math.floor(w / beta / factor) * factor)
    elif frames * hb * wb < min_pixels:
        beta = math.sqrt(min_pixels / (frames * h * w))
        hb, wb = math.ceil(h * beta / factor) * factor, math.ceil(w * beta / factor) * factor
    return hb, wb


def preprocess_glm4v(image, patch: int = 14, merge: int = 2, temporal: int = 2, min_pixels: int = 112 * 112,
                     max_pixels: int = 28 * 28 * 15000, mean=CLIP_MEAN, std=CLIP_STD):
    from PIL import Image

    img = load_image(image)
    h, w = glm4v_smart_resize(img.height, img.width, patch * merge, min_pixels, max_pixels, temporal)
    a = np.asarray(img.resize((w, h), Image.BICUBIC), dtype=np.float32) / 255.0
    a = (a - np.asarray(mean, np.float32)) / np.asarray(std, np.float32)
    return patchify(a.transpose(2, 0, 1), patch, merge, temporal)


class Glm4vVisionTower(Qwen2VisionTower):
    def __init__(self, vc: dict, out_hidden: int, device, dtype):
        self.device, self.dtype = device, dtype
        self.E = int(vc.get("hidden_size", 1536))
        self.depth = int(vc.get("depth", 24))
        self.heads = int(vc.get("num_heads", 12))
        self.hd = self.E // self.heads
        self.out = int(vc.get("out_hidden_size") or out_hidden)
        self.ctx = int(vc.get("intermediate_size", 13696))   # merger SwiGLU width
        self.patch = int(vc.get("patch_size", 14))
        self.merge = int(vc.get("spatial_merge_size", 2))
        self.temporal = int(vc.get("temporal_patch_size", 2))
        self.cin = int(vc.get("in_channels", 3))
        self.side = int(vc.get("image_size", 336)) // self.patch
        self.eps = float(vc.get("rms_norm_eps", 1e-5))
        self.qkv_bias = bool(vc.get("attention_bias", False))
        if vc.get("hidden_act", "silu") != "silu":
            raise NotImplementedError(f"vision hidden_act {vc.get('hidden_act')!r}")
        self.w: dict[str, torch.Tensor] = {}
        self._pend: dict = {}   # gate / up halves waiting for their partner
        rd = self.hd // 2
        self.inv = 1.0 / (10000.0 ** (torch.arange(0, rd, 2, dtype=torch.float32) / rd))

    def init_random(self, gen: torch.Generator, std: float = 0.02) -> None:
        E, O, C, m2 = self.E, self.out, self.ctx, self.merge ** 2
        shapes = {"patch_embed.proj.weight": (E, self.cin * self.temporal * self.patch ** 2),
                  "patch_embed.proj.bias": (E,), "post_conv_layernorm.weight": (E,),
                  "embeddings.position_embedding.weight": (self.side ** 2, E), "post_layernorm.weight": (E,),
                  "downsample.weight": (O, E * m2), "downsample.bias": (O,), "merger.proj.weight": (O, O),
                  "merger.post_projection_norm.weight": (O,), "merger.post_projection_norm.bias": (O,),
                  "merger.gate_up": (2 * C, O), "merger.down_proj.weight": (O, C)}
        for b in range(self.depth):
            p = f"blocks.{b}."
            shapes.update({p + "norm1.weight": (E,), p + "norm2.weight": (E,), p + "attn.qkv.weight": (3 * E, E),
                           p + "attn.proj.weight": (E, E), p + "mlp.gate_up": (2 * O, E),
                           p + "mlp.down_proj.weight": (E, O)})
            if self.qkv_bias:
                shapes[p + "attn.qkv.bias"] = (3 * E,)
        for k, s in shapes.items():
            t = torch.empty(*s, dtype=self.dtype, device=self.device)
            if "norm" in k and k.endswith("weight"):
                t.fill_(1.0)
            elif len(s) == 1:
                t.zero_()
            else:
                t.normal_(0.0, std, generator=gen)
            self.w[k] = t

    def load(self, name: str, t: torch.Tensor, pend: dict | None = None) -> None:
        pend = self._pend if pend is None else pend
        if name in ("patch_embed.proj.weight", "downsample.weight"):
            t = t.reshape(t.shape[0], -1)
        for fused, parts in (("mlp.gate_up", ("mlp.gate_proj.weight", "mlp.up_proj.weight")),
                             ("merger.gate_up", ("merger.gate_proj.weight", "merger.up_proj.weight"))):
            for j, part in enumerate(parts):
                if name.endswith(part):
                    key = name[:-len(part)] + fused
                    got = pend.setdefault(key, {})
                    got[j] = t
                    if len(got) == 2:
                        self.w[key] = torch.cat([got[0], got[1]]).to(device=self.device, dtype=self.dtype).contiguous()
                        del pend[key]
                    return
        self.w[name] = t.to(device=self.device, dtype=self.dtype).contiguous()

    def _pos_embed(self, grids) -> torch.Tensor:
        """Learned positions resampled per patch (bicubic ``grid_sample``, align_corners=False,
        border padding), merge-block order."""
        s, m, E = self.side, self.merge, self.E
        table = self.w["embeddings.position_embedding.weight"].float().view(s, s, E).permute(2, 0, 1)[None]
        out = []
        for t, h, w in grids:
            hp = torch.arange(h).view(h, 1).expand(h, w).reshape(h // m, m, w // m, m).transpose(1, 2).reshape(-1)
            wp = torch.arange(w).view(1, w).expand(h, w).reshape(h // m, m, w // m, m).transpose(1, 2).reshape(-1)
            g = torch.stack([(wp.float() + 0.5) / w * 2 - 1, (hp.float() + 0.5) / h * 2 - 1], -1)
            g = g.to(table.device)[None, :, None, :]
            e = F.grid_sample(table, g, mode="bicubic", align_corners=False, padding_mode="border")
            out.append(e[0, :, :, 0].t().repeat(t, 1))
        return torch.cat(out).to(self.dtype)

    def forward(self, pixel_values: torch.Tensor, grids: list[tuple[int, int, int]]) -> torch.Tensor:
        dev, dt, E, Hh, D, w = self.device, self.dtype, self.E, self.heads, self.hd, self.w
        x = linear(pixel_values.to(device=dev, dtype=dt), w["patch_embed.proj.weight"], w["patch_embed.proj.bias"])
        x = ops.rmsnorm(x, w["post_conv_layernorm.weight"], self.eps)
        x = x + self._pos_embed(grids).to(dev)
        ang = self.rot_pos(grids).to(dev)
        emb = torch.cat([ang, ang], -1)
        cos, sin = emb.cos()[:, None, :], emb.sin()[:, None, :]
        lens = [h * ww for t, h, ww in grids for _ in range(t)]
        N = x.shape[0]

        def rope(t):
            tf = t.float()
            return (tf * cos + torch.cat([-tf[..., D // 2:], tf[..., :D // 2]], -1) * sin).to(dt)

        for b in range(self.depth):
            p = f"blocks.{b}."
            h = ops.rmsnorm(x, w[p + "norm1.weight"], self.eps)
            qkv = linear(h, w[p + "attn.qkv.weight"], w.get(p + "attn.qkv.bias")).view(N, 3, Hh, D)
            a = ops.varlen_attention(rope(qkv[:, 0]), rope(qkv[:, 1]), qkv[:, 2], lens, D ** -0.5).reshape(N, E)
            x = x + linear(a, w[p + "attn.proj.weight"])
            h = ops.rmsnorm(x, w[p + "norm2.weight"], self.eps)
            x = x + linear(ops.act_and_mul(linear(h, w[p + "mlp.gate_up"]), 0), w[p + "mlp.down_proj.weight"])
        x = ops.rmsnorm(x, w["post_layernorm.weight"], self.eps)
        m2 = self.merge ** 2
        # 2 x 2 conv over each merge block (channel-major, like the Conv2d weight) = one GEMM
        x = x.view(-1, self.merge, self.merge, E).permute(0, 3, 1, 2).reshape(-1, E * m2).contiguous()
        x = linear(x, w["downsample.weight"], w["downsample.bias"])
        h = linear(x, w["merger.proj.weight"])
        h = ops.layernorm(h, w["merger.post_projection_norm.weight"], w["merger.post_projection_norm.bias"], 1e-5)
        h = ops.act(h, 3)
        return linear(ops.act_and_mul(linear(h, w["merger.gate_up"]), 0), w["merger.down_proj.weight"])


def _glm_cfg(cfg: ModelConfig) -> ModelConfig:
    ex = cfg.extra or {}
    ns = int(ex.get("n_shared_experts") or 0)
    return dataclasses.replace(cfg, shared_expert_intermediate_size=ns * int(cfg.moe_intermediate_size or 0),
                               num_shared_experts=ns, scoring_func="sigmoid")


class Glm4vMoeForConditionalGeneration(Qwen2VLForConditionalGeneration, MoEForCausalLM):
    tower_cls = Glm4vVisionTower

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        if pstate.get().ep_size > 1:
            raise NotImplementedError("GLM-4.5V with expert parallelism")
        cfg = _glm_cfg(cfg)
        super().__init__(cfg, device, dtype, max_positions)
        ex = cfg.extra or {}
        self.image_token_id = int(ex.get("image_token_id", 151363))
        self.vision_start_id = int(ex.get("image_start_token_id", 151339))
        self.vision_end_id = int(ex.get("image_end_token_id", 151340))
        self.routed_scale = float(cfg.routed_scaling_factor or 1.0)
        self.b_router: list[torch.Tensor | None] = [None] * cfg.num_layers

    def init_random(self, seed: int = 0, std: float = 0.02):
        super().init_random(seed, std)
        for i in self.moe_layers:
            self.b_router[i] = torch.zeros(self.E, dtype=torch.float32, device=self.device)
        return self

    def load_hf_weights(self, weights):
        def renamed():
            for name, w in weights:
                n = name.replace("model.language_model.", "model.")
                if n.endswith(".mlp.gate.e_score_correction_bias"):
                    i = int(n.split("layers.")[1].split(".")[0])
                    self.b_router[i] = w.to(device=self.device, dtype=torch.float32).contiguous()
                    continue
                yield n.replace(".mlp.shared_experts.", ".mlp.shared_expert."), w

        super().load_hf_weights(renamed())
        for i in self.moe_layers:
            if self.b_router[i] is None:
                self.b_router[i] = torch.zeros(self.E, dtype=torch.float32, device=self.device)
        return self

    def make_mm_input(self, prompt_ids: list[int], images: list):
        """GLM-4V resize rule, otherwise the Qwen2-VL placeholder expansion and M-RoPE positions."""
        from ome_amd.multimodal import MMInput, expand_image_tokens, mrope_positions

        pvs, grids = [], []
        for im in images:
            if isinstance(im, tuple):
                pv, g = im
            else:
                pv, g = preprocess_glm4v(im, self.visual.patch, self.merge, self.visual.temporal)
            pvs.append(torch.as_tensor(pv, dtype=torch.float32))
            grids.append(tuple(int(v) for v in g))
        ids, spans = expand_image_tokens(list(prompt_ids), self.image_token_id, grids, self.merge, pvs,
                                         self.cfg.vocab_size)
        pos, delta = mrope_positions(len(ids), spans, grids, self.merge)
        return ids, MMInput(torch.cat(pvs, 0), grids, spans, pos, delta)

    def mlp(self, i: int, x: torch.Tensor) -> torch.Tensor:
        if i not in self.moe_layers:
            return super().mlp(i, x)
        cfg = self.cfg
        logits = F.linear(x.float(), self.w_router[i].float())          # the router runs in fp32
        tw, tid = ops.moe_route(logits, self.k, self.renorm, "sigmoid", bias=self.b_router[i],
                                n_group=cfg.n_group, topk_group=cfg.topk_group, group_mode=2)
        out = ops.fused_moe(x, tw, tid, self.w13[i], self.w2[i], self.act, self.routed_scale)
        if self.w_sgu[i] is not None:
            out = out + linear(ops.act_and_mul(linear(x, self.w_sgu[i]), self.act), self.w_sd[i])
        return pstate.tp_all_reduce(out)
