"""Qwen3-VL (``Qwen3VLForConditionalGeneration``, ``Qwen3VLMoeForConditionalGeneration``;
reference catalog ``config/runtimes/srt/Qwen/qwen3-vl-235b-a22b-instruct-rt.yaml``, model-config
fixtures ``pkg/hfutil/modelconfig/testdata/qwen3_vl_*.json``).

Differences from Qwen2-VL (``qwen2_vl.py``, whose placeholder / M-RoPE / HIP-graph decode path
is reused):
* language model: Qwen3 (per-head q/k RMSNorm), dense or MoE (fused ``experts.gate_up_proj`` /
  ``down_proj`` checkpoints), M-RoPE with INTERLEAVED sections (frequency j takes t / h / w by
  j mod 3 inside the h / w section lengths) -- only the per-row cos/sin table of image chunks
  changes; text and decode rows stay plain RoPE at ``position + rope_delta``;
* vision tower: 16-px patches, a learned 48 x 48 position table bilinearly resampled
  (align_corners) to every image grid, pre-LN blocks with GELU-tanh MLPs on the varlen MFMA
  attention, a final 2 x 2 merger (LayerNorm -> GEMM -> GELU -> GEMM) and DEEPSTACK mergers
  (post-shuffle LayerNorm) at ``deepstack_visual_indexes``, whose outputs are added to the image
  rows of the hidden states after decoder layers 0, 1, 2 (``meta.extra['deepstack']``);
* preprocessing: the Qwen2-VL rule with factor 32 and mean = std = 0.5.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.models.config import ModelConfig
from ome_amd.models.moe import MoEForCausalLM
from ome_amd.models.qwen2_vl import Qwen2VisionTower, Qwen2VLForConditionalGeneration
from ome_amd.models.quant import linear


class Qwen3VisionTower(Qwen2VisionTower):
    def __init__(self, vc: dict, out_hidden: int, device, dtype):
        self.device, self.dtype = device, dtype
        self.E = int(vc.get("hidden_size", 1152))
        self.depth = int(vc.get("depth", 27))
        self.heads = int(vc.get("num_heads", 16))
        self.hd = self.E // self.heads
        self.I = int(vc.get("intermediate_size", 4304))
        self.patch = int(vc.get("patch_size", 16))
        self.merge = int(vc.get("spatial_merge_size", 2))
        self.temporal = int(vc.get("temporal_patch_size", 2))
        self.cin = int(vc.get("in_channels", 3))
        self.out_hidden = int(vc.get("out_hidden_size") or out_hidden)
        self.side = int(round(int(vc.get("num_position_embeddings", 2304)) ** 0.5))
        self.deep = [int(i) for i in (vc.get("deepstack_visual_indexes") or [])]
        act = vc.get("hidden_act", "gelu_pytorch_tanh")
        self.act = {"gelu_pytorch_tanh": 1, "gelu": 3}.get(act)
        if self.act is None:
            raise NotImplementedError(f"vision hidden_act {act!r}")
        self.w: dict[str, torch.Tensor] = {}
        rd = self.hd // 2
        self.inv = 1.0 / (10000.0 ** (torch.arange(0, rd, 2, dtype=torch.float32) / rd))

    def _merger_shapes(self, p: str, post: bool) -> dict:
        E4 = self.E * self.merge ** 2
        n = E4 if post else self.E
        return {p + "norm.weight": (n,), p + "norm.bias": (n,), p + "linear_fc1.weight": (E4, E4),
                p + "linear_fc1.bias": (E4,), p + "linear_fc2.weight": (self.out_hidden, E4),
                p + "linear_fc2.bias": (self.out_hidden,)}

    def init_random(self, gen: torch.Generator, std: float = 0.02) -> None:
        E, I = self.E, self.I
        shapes = {"patch_embed.proj.weight": (E, self.cin * self.temporal * self.patch ** 2),
                  "patch_embed.proj.bias": (E,), "pos_embed.weight": (self.side ** 2, E)}
        shapes.update(self._merger_shapes("merger.", False))
        for k in range(len(self.deep)):
            shapes.update(self._merger_shapes(f"deepstack_merger_list.{k}.", True))
        for b in range(self.depth):
            p = f"blocks.{b}."
            shapes.update({p + "norm1.weight": (E,), p + "norm1.bias": (E,), p + "norm2.weight": (E,),
                           p + "norm2.bias": (E,), p + "attn.qkv.weight": (3 * E, E), p + "attn.qkv.bias": (3 * E,),
                           p + "attn.proj.weight": (E, E), p + "attn.proj.bias": (E,),
                           p + "mlp.linear_fc1.weight": (I, E), p + "mlp.linear_fc1.bias": (I,),
                           p + "mlp.linear_fc2.weight": (E, I), p + "mlp.linear_fc2.bias": (E,)})
        for k, s in shapes.items():
            t = torch.empty(*s, dtype=self.dtype, device=self.device)
            if k.endswith(("norm1.weight", "norm2.weight", "norm.weight")):
                t.fill_(1.0)
            elif len(s) == 1:
                t.zero_()
            else:
                t.normal_(0.0, std, generator=gen)
            self.w[k] = t

    def _ln(self, x, p):
        return ops.layernorm(x.contiguous(), self.w[p + ".weight"], self.w[p + ".bias"], 1e-6)

    def _pos(self, grids) -> torch.Tensor:
        """Learned positions resampled to each (h, w) grid, in merge-block order, per frame."""
        E, s, m = self.E, self.side, self.merge
        table = self.w["pos_embed.weight"].float().view(s, s, E).permute(2, 0, 1)[None]
        out = []
        for t, h, w in grids:
            g = F.interpolate(table, size=(h, w), mode="bilinear", align_corners=True)[0]   # [E, h, w]
            g = g.permute(1, 2, 0).reshape(h // m, m, w // m, m, E).permute(0, 2, 1, 3, 4).reshape(h * w, E)
            out.append(g.repeat(t, 1))
        return torch.cat(out).to(self.dtype)

    def _merge(self, x: torch.Tensor, p: str, post: bool) -> torch.Tensor:
        E4 = self.E * self.merge ** 2
        x = self._ln(x.reshape(-1, E4), p + "norm") if post else self._ln(x, p + "norm").reshape(-1, E4)
        x = ops.act(linear(x, self.w[p + "linear_fc1.weight"], self.w[p + "linear_fc1.bias"]), 3)
        return linear(x, self.w[p + "linear_fc2.weight"], self.w[p + "linear_fc2.bias"])

    def forward(self, pixel_values: torch.Tensor, grids: list[tuple[int, int, int]]):
        """-> (merged features [N/4, out], [deepstack level features, each [N/4, out]])."""
        dev, dt, E, Hh, D = self.device, self.dtype, self.E, self.heads, self.hd
        x = linear(pixel_values.to(device=dev, dtype=dt), self.w["patch_embed.proj.weight"],
                   self.w["patch_embed.proj.bias"])
        x = x + self._pos(grids).to(dev)
        ang = self.rot_pos(grids).to(dev)
        emb = torch.cat([ang, ang], -1)
        cos, sin = emb.cos()[:, None, :], emb.sin()[:, None, :]
        lens = [h * w for t, h, w in grids for _ in range(t)]
        N = x.shape[0]

        def rope(t):
            tf = t.float()
            half = D // 2
            return (tf * cos + torch.cat([-tf[..., half:], tf[..., :half]], -1) * sin).to(dt)

        deep = []
        for b in range(self.depth):
            p = f"blocks.{b}."
            h = self._ln(x, p + "norm1")
            qkv = linear(h, self.w[p + "attn.qkv.weight"], self.w[p + "attn.qkv.bias"]).view(N, 3, Hh, D)
            a = ops.varlen_attention(rope(qkv[:, 0]), rope(qkv[:, 1]), qkv[:, 2], lens, D ** -0.5).reshape(N, E)
            x = x + linear(a, self.w[p + "attn.proj.weight"], self.w[p + "attn.proj.bias"])
            h = self._ln(x, p + "norm2")
            f = ops.act(linear(h, self.w[p + "mlp.linear_fc1.weight"], self.w[p + "mlp.linear_fc1.bias"]), self.act)
            x = x + linear(f, self.w[p + "mlp.linear_fc2.weight"], self.w[p + "mlp.linear_fc2.bias"])
            if b in self.deep:
                deep.append(self._merge(x, f"deepstack_merger_list.{self.deep.index(b)}.", True))
        return self._merge(x, "merger.", False), deep


class _Qwen3VLBits:
    """Interleaved M-RoPE sections + Qwen3-VL image preprocessing on top of the Qwen2-VL path."""
    tower_cls = Qwen3VisionTower

    def _setup_qwen3(self, cfg: ModelConfig) -> None:
        ex = cfg.extra or {}
        rp = ex.get("rope_parameters") or ex.get("rope_scaling") or {}
        sec = list(rp.get("mrope_section") or [24, 20, 20])
        half = cfg.rot_dim // 2
        sel = np.zeros(half, dtype=np.int64)           # frequency j -> t (0), h (1) or w (2)
        sel[1:3 * sec[1]:3] = 1
        sel[2:3 * sec[2]:3] = 2
        self.mrope_sec = torch.from_numpy(sel)
        self.image_processor_kwargs = {"min_pixels": 65536, "max_pixels": 16777216, "mean": (0.5, 0.5, 0.5),
                                       "std": (0.5, 0.5, 0.5)}

    def encode_images(self, pixel_values: torch.Tensor, grids):
        return self.visual.forward(pixel_values, grids)

    def weight_bytes(self) -> int:
        return super().weight_bytes()


class Qwen3VLForConditionalGeneration(_Qwen3VLBits, Qwen2VLForConditionalGeneration):
    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        self._setup_qwen3(cfg)


class Qwen3VLMoeForConditionalGeneration(_Qwen3VLBits, Qwen2VLForConditionalGeneration, MoEForCausalLM):
    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        self._setup_qwen3(cfg)
