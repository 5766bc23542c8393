"""Mistral 3 vision-language models (``Mistral3ForConditionalGeneration``: Mistral-Small-3.1-24B;
reference catalog ``config/runtimes/srt/mistralai/mistral-small-3-1-24b-instruct-2503-rt.yaml``).

* preprocessing (Pixtral rule): scale the image down so its longest edge fits
  ``longest_edge`` (floor), round each side UP to a multiple of patch x merge (28 px), bicubic
  resize, rescale, CLIP mean / std; variable-size images are patchified to rows
  [n_patches, 3 * 14 * 14] (no square padding, no tiling);
* prompt: each ``[IMG]`` becomes, per row of merged 2 x 2 patch blocks, ``[IMG] * cols`` followed
  by ``[IMG_BREAK]`` -- the last row ending in ``[IMG_END]``; only the ``[IMG]`` rows (content-hash
  ids) receive features, one placeholder span per row;
* Pixtral tower: patch GEMM (no bias) -> RMSNorm -> layers of RMSNorm -> fused QKV GEMM -> 2D RoPE
  (frequency pairs alternate between the patch row and column index) -> bidirectional varlen MFMA
  attention per image -> O GEMM; RMSNorm -> fused gate|up GEMM -> SiLU-and-mul kernel -> down GEMM;
* projector: RMSNorm -> 2 x 2 patch merger (channel-major unfold order, one GEMM) -> GEMM -> GELU
  -> GEMM.
The language model is the dense decoder of ``llama.py`` (Mistral text config).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.models.config import ModelConfig
from ome_amd.models.llama import LlamaForCausalLM
from ome_amd.models.quant import linear
from ome_amd.multimodal.inputs import CLIP_MEAN, CLIP_STD, MMInput, load_image, pad_token_id
from ome_amd.parallel import state as pstate


def preprocess_pixtral(image, longest_edge: int = 1540, unit: int = 28, patch: int = 14,
                       mean=CLIP_MEAN, std=CLIP_STD) -> tuple[torch.Tensor, int, int]:
    """-> (patch rows float32 [h * w, 3 * patch * patch] in (c, kh, kw) order, h, w in patches)."""
    from PIL import Image

    img = load_image(image)
    W, H = img.size
    ratio = max(H / longest_edge, W / longest_edge)
    if ratio > 1:
        H, W = int(math.floor(H / ratio)), int(math.floor(W / ratio))
    H, W = ((H - 1) // unit + 1) * unit, ((W - 1) // unit + 1) * unit
    img = img.resize((W, H), Image.BICUBIC)
    a = np.asarray(img, dtype=np.float32) / 255.0
    a = (a - np.asarray(mean, np.float32)) / np.asarray(std, np.float32)
    h, w = H // patch, W // patch
    px = torch.from_numpy(np.ascontiguousarray(a.transpose(2, 0, 1)))          # [3, H, W]
    rows = px.reshape(3, h, patch, w, patch).permute(1, 3, 0, 2, 4).reshape(h * w, 3 * patch * patch)
    return rows, h, w


class PixtralVisionTower:
    def __init__(self, vc: dict, device, dtype, feature_layer: int = -1):
        self.device, self.dtype = device, dtype
        self.E = int(vc.get("hidden_size", 1024))
        self.heads = int(vc.get("num_attention_heads", 16))
        self.D = int(vc.get("head_dim") or self.E // self.heads)
        self.depth = int(vc.get("num_hidden_layers", 24))
        self.I = int(vc.get("intermediate_size", 4096))
        self.patch = int(vc.get("patch_size", 14))
        self.C = int(vc.get("num_channels", 3))
        self.max_side = int(vc.get("image_size", 1540)) // self.patch
        rp = vc.get("rope_parameters") or {}
        self.theta = float(rp.get("rope_theta", vc.get("rope_theta", 10000.0)))
        act = vc.get("hidden_act", "gelu")
        self.act = {"silu": 0, "gelu_pytorch_tanh": 1, "gelu": 3}.get(act)
        if self.act is None:
            raise NotImplementedError(f"pixtral hidden_act {act!r}")
        # hidden_states[k]: k = 0 after ln_pre, k = i + 1 after layer i
        self.n_layers = feature_layer if feature_layer >= 0 else self.depth + 1 + feature_layer
        self.w: dict[str, torch.Tensor] = {}

    def _t(self, t):
        return t.to(device=self.device, dtype=self.dtype).contiguous()

    def init_random(self, gen: torch.Generator, std: float = 0.02) -> None:
        E, I = self.E, self.I
        shapes = {"patch.weight": (E, self.C * self.patch ** 2), "ln_pre": (E,)}
        for b in range(self.n_layers):
            p = f"layers.{b}."
            shapes.update({p + "qkv": (3 * self.heads * self.D, E), p + "o": (E, self.heads * self.D),
                           p + "gu": (2 * I, E), p + "down": (E, I), p + "attn_norm": (E,), p + "ffn_norm": (E,)})
        for k, s in shapes.items():
            t = torch.empty(*s, dtype=self.dtype, device=self.device)
            if len(s) == 1:
                t.fill_(1.0)
            else:
                t.normal_(0.0, std, generator=gen)
            self.w[k] = t

    def load(self, name: str, t: torch.Tensor, pend: dict) -> None:
        """``name`` relative to ``vision_tower.`` (layers past the feature layer are dropped)."""
        if name == "patch_conv.weight":
            self.w["patch.weight"] = self._t(t.reshape(t.shape[0], -1))
        elif name == "ln_pre.weight":
            self.w["ln_pre"] = self._t(t)
        elif name.startswith("transformer.layers."):
            parts = name.split(".")
            b, mod = int(parts[2]), ".".join(parts[3:-1])
            if b >= self.n_layers:
                return
            p = f"layers.{b}."
            if mod in ("attention.q_proj", "attention.k_proj", "attention.v_proj"):
                got = pend.setdefault((b, "qkv"), {})
                got[mod[-6]] = t
                if len(got) == 3:
                    self.w[p + "qkv"] = self._t(torch.cat([got["q"], got["k"], got["v"]]))
                    del pend[(b, "qkv")]
            elif mod in ("feed_forward.gate_proj", "feed_forward.up_proj"):
                got = pend.setdefault((b, "gu"), {})
                got[mod.split(".")[1]] = t
                if len(got) == 2:
                    self.w[p + "gu"] = self._t(torch.cat([got["gate_proj"], got["up_proj"]]))
                    del pend[(b, "gu")]
            else:
                key = {"attention.o_proj": "o", "feed_forward.down_proj": "down", "attention_norm": "attn_norm",
                       "ffn_norm": "ffn_norm"}[mod]
                self.w[p + key] = self._t(t)

    def rope(self, grids) -> tuple[torch.Tensor, torch.Tensor]:
        """cos / sin [N, D] (rotate-half layout): frequency pairs alternate row / column index."""
        D = self.D
        freqs = 1.0 / (self.theta ** (torch.arange(0, D, 2, dtype=torch.float32) / D))
        ang = []
        for _, h, w in grids:
            hh, ww = torch.meshgrid(torch.arange(h), torch.arange(w), indexing="ij")
            ang.append(torch.cat([hh.reshape(-1, 1).float() * freqs[::2], ww.reshape(-1, 1).float() * freqs[1::2]], 1))
        a = torch.cat(ang).to(self.device)
        a = torch.cat([a, a], -1)
        return a.cos()[:, None, :], a.sin()[:, None, :]

    def forward(self, patches: torch.Tensor, grids) -> torch.Tensor:
        """patches [N, 3 * p * p] of all images -> features [N, E] of the selected layer."""
        w, E, Hh, D = self.w, self.E, self.heads, self.D
        x = linear(patches.to(device=self.device, dtype=self.dtype), w["patch.weight"])
        x = ops.rmsnorm(x, w["ln_pre"], 1e-5)
        N = x.shape[0]
        cos, sin = self.rope(grids)
        lens = [h * ww for _, h, ww in grids]

        def rot(t):
            tf = t.float()
            return (tf * cos + torch.cat([-tf[..., D // 2:], tf[..., :D // 2]], -1) * sin).to(self.dtype)

        for b in range(self.n_layers):
            p = f"layers.{b}."
            h = ops.rmsnorm(x, w[p + "attn_norm"], 1e-5)
            qkv = linear(h, w[p + "qkv"]).view(N, 3, Hh, D)
            a = ops.varlen_attention(rot(qkv[:, 0]), rot(qkv[:, 1]), qkv[:, 2], lens, D ** -0.5).reshape(N, Hh * D)
            x = x + linear(a, w[p + "o"])
            h = ops.rmsnorm(x, w[p + "ffn_norm"], 1e-5)
            gu = linear(h, w[p + "gu"])
            if self.act == 3:   # exact GELU: no fused gated kernel mode
                g, u = gu.chunk(2, -1)
                f = (F.gelu(g.float()) * u.float()).to(self.dtype)
            else:
                f = ops.act_and_mul(gu, self.act)
            x = x + linear(f, w[p + "down"])
        return x


class Mistral3ForConditionalGeneration(LlamaForCausalLM):
    is_multimodal = True

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        ex = cfg.extra or {}
        vc = ex.get("vision_config") or {}
        layer = ex.get("vision_feature_layer", -1)
        if not isinstance(layer, int):
            raise NotImplementedError("multi-layer vision features")
        if ex.get("projector_hidden_act", "gelu") != "gelu":
            raise NotImplementedError(f"projector act {ex.get('projector_hidden_act')!r}")
        self.visual = PixtralVisionTower(vc, self.device, dtype, layer)
        self.merge = int(ex.get("spatial_merge_size", 2))
        self.image_id = int(ex.get("image_token_index", ex.get("image_token_id", 10)))
        self.break_id = int(ex.get("image_break_token_id", 12))
        self.end_id = int(ex.get("image_end_token_id", 13))
        self.longest_edge = int(ex.get("longest_edge") or vc.get("image_size", 1540))
        self.proj_bias = bool(ex.get("multimodal_projector_bias", False))
        self.proj: dict[str, torch.Tensor | None] = {}

    def init_random(self, seed: int = 0, std: float = 0.02) -> "Mistral3ForConditionalGeneration":
        super().init_random(seed, std)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 4463)
        self.visual.init_random(gen, std)
        H, E, m2 = self.cfg.hidden_size, self.visual.E, self.merge ** 2
        mk = lambda *s: torch.empty(*s, dtype=self.dtype, device=self.device).normal_(0.0, std, generator=gen)  # noqa
        self.proj = {"norm": torch.ones(E, dtype=self.dtype, device=self.device), "merge": mk(E, E * m2),
                     "w1": mk(H, E), "w2": mk(H, H), "b1": None, "b2": None}
        if self.proj_bias:
            self.proj["b1"] = torch.zeros(H, dtype=self.dtype, device=self.device)
            self.proj["b2"] = torch.zeros(H, dtype=self.dtype, device=self.device)
        return self

    _PROJ = {"multi_modal_projector.norm.weight": "norm",
             "multi_modal_projector.patch_merger.merging_layer.weight": "merge",
             "multi_modal_projector.linear_1.weight": "w1", "multi_modal_projector.linear_1.bias": "b1",
             "multi_modal_projector.linear_2.weight": "w2", "multi_modal_projector.linear_2.bias": "b2"}

    def load_hf_weights(self, weights) -> "Mistral3ForConditionalGeneration":
        pend: dict = {}
        self.proj = {"b1": None, "b2": None}

        def text_only():
            for name, w in weights:
                n = name[len("model."):] if name.startswith("model.") else name
                if n.startswith("vision_tower."):
                    self.visual.load(n[len("vision_tower."):], w, pend)
                elif n in self._PROJ:
                    self.proj[self._PROJ[n]] = w.to(device=self.device, dtype=self.dtype).contiguous()
                elif n.startswith("language_model."):
                    rest = n[len("language_model."):]
                    yield ("lm_head.weight" if rest == "lm_head.weight" else
                           "model." + (rest[len("model."):] if rest.startswith("model.") else rest)), w
                else:
                    yield name, w

        super().load_hf_weights(text_only())
        if pend:
            raise ValueError(f"incomplete vision projections: {sorted(pend)}")
        return self

    def weight_bytes(self) -> int:
        n = super().weight_bytes() + sum(t.numel() * t.element_size() for t in self.visual.w.values())
        return n + sum(t.numel() * t.element_size() for t in self.proj.values() if t is not None)

    # ------------------------------------------------------------------ multimodal
    def image_prompt_ids(self) -> list[int]:
        return [self.image_id]

    def make_mm_input(self, prompt_ids: list[int], images: list):
        where = [i for i, t in enumerate(prompt_ids) if t == self.image_id]
        if len(where) != len(images):
            raise ValueError(f"prompt has {len(where)} image tokens for {len(images)} images")
        ids, rows, grids, spans, last = [], [], [], [], 0
        m = self.merge
        for i, im in zip(where, images):
            if isinstance(im, tuple):   # pre-patchified (rows, h, w)
                px, h, w = im
            else:
                px, h, w = preprocess_pixtral(im, self.longest_edge, self.visual.patch * m, self.visual.patch)
            ids += prompt_ids[last:i]
            pid = pad_token_id(px, self.cfg.vocab_size)
            nh, nw = h // m, w // m
            for r in range(nh):
                spans.append((len(ids), nw))
                ids += [pid] * nw + [self.end_id if r == nh - 1 else self.break_id]
            rows.append(px)
            grids.append((1, h, w))
            last = i + 1
        ids += prompt_ids[last:]
        return ids, MMInput(torch.cat(rows, 0), grids, spans)

    def encode_images(self, patches: torch.Tensor, grids) -> torch.Tensor:
        p, m, E = self.proj, self.merge, self.visual.E
        x = ops.rmsnorm(self.visual.forward(patches, grids), p["norm"], self.cfg.rms_norm_eps)
        merged, off = [], 0
        for _, h, w in grids:   # 2 x 2 blocks, channel-major within a block (torch unfold order)
            g = x[off:off + h * w].view(h // m, m, w // m, m, E).permute(0, 2, 4, 1, 3)
            merged.append(g.reshape(-1, E * m * m))
            off += h * w
        x = linear(torch.cat(merged, 0).contiguous(), p["merge"])
        x = ops.act(linear(x, p["w1"], p["b1"]), 3)
        return linear(x, p["w2"], p["b2"])

    def embed_with_images(self, ids: torch.Tensor, rows: torch.Tensor, feats: torch.Tensor) -> torch.Tensor:
        h = pstate.tp_all_reduce(ops.embedding(ids, self.embed, self.tp.vocab_start, self.tp.vocab_end))
        if rows.numel():
            h.index_copy_(0, rows, feats.to(h.dtype))
        return h
