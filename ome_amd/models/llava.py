"""LLaVA-1.5 style vision-language models: ``LlavaForConditionalGeneration`` (llava-hf layout) and
``LlavaLlamaForCausalLM`` (the original LLaVA repository layout; reference catalog
``config/runtimes/srt/liuhaotian/llava-v1-5-13b-rt.yaml``), and the shared CLIP vision tower.

* preprocessing: (original layout, ``image_aspect_ratio: pad``) pad to a square with the CLIP
  mean colour, then the CLIP processor: shortest edge -> ``image_size`` (bicubic), centre crop,
  rescale, CLIP mean / std;
* prompt: each image placeholder (``image_token_index``; -200 in the original layout) becomes
  one token per selected patch (576 for ViT-L/14 at 336 px) carrying a content-hash id, spliced
  with the projected features (plain 1D RoPE);
* CLIP tower: patch GEMM (no bias), class token first, learned positions, pre-LayerNorm, encoder
  layers (LayerNorm -> fused QKV GEMM (+bias) -> bidirectional varlen MFMA attention per image ->
  O GEMM; LayerNorm -> quick-GELU MLP), features from ``vision_feature_layer`` (-2), class token
  dropped (``default``); projector GEMM -> GELU -> GEMM.
The language model is the dense decoder of ``llama.py`` (Llama / Mistral / Qwen2 text configs).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.models.config import ModelConfig
from ome_amd.models.llama import LlamaForCausalLM
from ome_amd.models.quant import linear
from ome_amd.multimodal.inputs import CLIP_MEAN, CLIP_STD, MMInput, load_image, pad_token_id
from ome_amd.parallel import state as pstate

LLAVA_ARCHS = {"LlavaForConditionalGeneration", "LlavaLlamaForCausalLM"}
ORIG_IMAGE_TOKEN = -200   # IMAGE_TOKEN_INDEX of the original LLaVA code


def preprocess_clip(image, size: int = 336, pad_square: bool = False, mean=CLIP_MEAN, std=CLIP_STD) -> torch.Tensor:
    """-> float32 [1, 3, size, size]."""
    from PIL import Image

    img = load_image(image)
    if pad_square and img.width != img.height:
        s = max(img.width, img.height)
        bg = Image.new("RGB", (s, s), tuple(int(x * 255) for x in mean))
        bg.paste(img, ((s - img.width) // 2, (s - img.height) // 2))
        img = bg
    w, h = img.size
    sc = size / min(w, h)
    nw, nh = max(size, round(w * sc)), max(size, round(h * sc))
    img = img.resize((nw, nh), Image.BICUBIC)
    left, top = (nw - size) // 2, (nh - size) // 2
    img = img.crop((left, top, left + size, top + size))
    a = np.asarray(img, dtype=np.float32) / 255.0
    a = (a - np.asarray(mean, np.float32)) / np.asarray(std, np.float32)
    return torch.from_numpy(np.ascontiguousarray(a.transpose(2, 0, 1)))[None]


# CLIP ViT-L/14-336 (``openai/clip-vit-large-patch14-336``): the original layout does not embed
# the vision config
CLIP_L336 = dict(hidden_size=1024, intermediate_size=4096, num_hidden_layers=24, num_attention_heads=16,
                 image_size=336, patch_size=14, hidden_act="quick_gelu", layer_norm_eps=1e-5)


class CLIPVisionTower:
    def __init__(self, vc: dict, device, dtype, feature_layer: int = -2, strategy: str = "default"):
        self.device, self.dtype = device, dtype
        self.E = int(vc.get("hidden_size", 1024))
        self.heads = int(vc.get("num_attention_heads", 16))
        self.D = self.E // self.heads
        self.depth = int(vc.get("num_hidden_layers", 24))
        self.I = int(vc.get("intermediate_size", 4096))
        self.image = int(vc.get("image_size", 336))
        self.patch = int(vc.get("patch_size", 14))
        self.C = int(vc.get("num_channels", 3))
        self.eps = float(vc.get("layer_norm_eps", 1e-5))
        self.quick = vc.get("hidden_act", "quick_gelu") == "quick_gelu"
        self.side = self.image // self.patch
        self.n_patch = self.side ** 2
        # hidden_states[k]: k = 0 the embeddings, k = i + 1 after layer i
        self.feature_layer = feature_layer if feature_layer >= 0 else self.depth + 1 + feature_layer
        self.strategy = strategy
        self.tokens = self.n_patch + (1 if strategy == "full" else 0)
        self.w: dict[str, torch.Tensor] = {}

    def _t(self, t):
        return t.to(device=self.device, dtype=self.dtype).contiguous()

    def init_random(self, gen: torch.Generator, std: float = 0.02) -> None:
        E, I = self.E, self.I
        shapes = {"patch.weight": (E, self.C * self.patch ** 2), "cls": (E,), "pos": (self.n_patch + 1, E),
                  "pre_ln.weight": (E,), "pre_ln.bias": (E,)}
        for b in range(self.feature_layer):
            p = f"layers.{b}."
            shapes.update({p + "qkv.weight": (3 * E, E), p + "qkv.bias": (3 * E,), p + "o.weight": (E, E),
                           p + "o.bias": (E,), p + "fc1.weight": (I, E), p + "fc1.bias": (I,), p + "fc2.weight": (E, I),
                           p + "fc2.bias": (E,), p + "ln1.weight": (E,), p + "ln1.bias": (E,), p + "ln2.weight": (E,),
                           p + "ln2.bias": (E,)})
        for k, s in shapes.items():
            t = torch.empty(*s, dtype=self.dtype, device=self.device)
            if k.endswith(("ln1.weight", "ln2.weight", "pre_ln.weight")):
                t.fill_(1.0)
            elif len(s) == 1 and k != "cls":
                t.zero_()
            else:
                t.normal_(0.0, std, generator=gen)
            self.w[k] = t

    _REN = {"self_attn.out_proj": "o", "mlp.fc1": "fc1", "mlp.fc2": "fc2", "layer_norm1": "ln1", "layer_norm2": "ln2"}

    def load(self, name: str, t: torch.Tensor, pend: dict) -> None:
        """``name`` relative to ``vision_model.`` (layers past the feature layer are dropped)."""
        if name == "embeddings.patch_embedding.weight":
            self.w["patch.weight"] = self._t(t.reshape(t.shape[0], -1))
        elif name == "embeddings.class_embedding":
            self.w["cls"] = self._t(t)
        elif name == "embeddings.position_embedding.weight":
            self.w["pos"] = self._t(t)
        elif name.startswith("pre_layrnorm."):
            self.w["pre_ln." + name.split(".")[-1]] = self._t(t)
        elif name.startswith("encoder.layers."):
            parts = name.split(".")
            b, mod, kind = int(parts[2]), ".".join(parts[3:-1]), parts[-1]
            if b >= self.feature_layer:
                return
            if mod in ("self_attn.q_proj", "self_attn.k_proj", "self_attn.v_proj"):
                got = pend.setdefault((b, kind), {})
                got[mod[-6]] = t
                if len(got) == 3:
                    self.w[f"layers.{b}.qkv.{kind}"] = self._t(torch.cat([got["q"], got["k"], got["v"]]))
                    del pend[(b, kind)]
                return
            self.w[f"layers.{b}.{self._REN[mod]}.{kind}"] = self._t(t)

    def forward(self, pixels: torch.Tensor) -> torch.Tensor:
        """pixels [n, C, S, S] -> selected features [n * tokens, E]."""
        w, E, n, ps, s = self.w, self.E, pixels.shape[0], self.patch, self.side
        x = pixels.to(device=self.device, dtype=self.dtype)
        x = x.reshape(n, self.C, s, ps, s, ps).permute(0, 2, 4, 1, 3, 5).reshape(n * self.n_patch, -1)
        x = linear(x, w["patch.weight"]).view(n, self.n_patch, E)
        x = torch.cat([w["cls"].view(1, 1, E).expand(n, 1, E), x], 1) + w["pos"]
        L = self.n_patch + 1
        T = n * L
        x = ops.layernorm(x.reshape(T, E).contiguous(), w["pre_ln.weight"], w["pre_ln.bias"], self.eps)
        lens = [L] * n
        for b in range(self.feature_layer):
            p = f"layers.{b}."
            h = ops.layernorm(x, w[p + "ln1.weight"], w[p + "ln1.bias"], self.eps)
            qkv = linear(h, w[p + "qkv.weight"], w[p + "qkv.bias"]).view(T, 3, self.heads, self.D)
            a = ops.varlen_attention(qkv[:, 0], qkv[:, 1], qkv[:, 2], lens, self.D ** -0.5).reshape(T, E)
            x = x + linear(a, w[p + "o.weight"], w[p + "o.bias"])
            h = ops.layernorm(x, w[p + "ln2.weight"], w[p + "ln2.bias"], self.eps)
            f = linear(h, w[p + "fc1.weight"], w[p + "fc1.bias"])
            f = f * torch.sigmoid(1.702 * f) if self.quick else ops.act(f, 3)
            x = x + linear(f, w[p + "fc2.weight"], w[p + "fc2.bias"])
        x = x.view(n, L, E)
        if self.strategy != "full":
            x = x[:, 1:]
        return x.reshape(-1, E).contiguous()


class LlavaForConditionalGeneration(LlamaForCausalLM):
    is_multimodal = True

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        ex = cfg.extra or {}
        self.orig = cfg.architecture == "LlavaLlamaForCausalLM"
        if self.orig:
            vc = {**CLIP_L336, **(ex.get("vision_config") or {})}   # mm_vision_tower is ViT-L/14-336
            layer = int(ex.get("mm_vision_select_layer", -2))
            strategy = "full" if ex.get("mm_vision_select_feature", "patch") == "cls_patch" else "default"
            self.image_id = int(ex.get("image_token_index", ORIG_IMAGE_TOKEN))
            self.pad_square = ex.get("image_aspect_ratio", "pad") == "pad"
            if ex.get("mm_projector_type", "mlp2x_gelu") != "mlp2x_gelu":
                raise NotImplementedError(f"mm_projector_type {ex.get('mm_projector_type')!r}")
        else:
            vc = ex.get("vision_config") or dict(CLIP_L336)
            layer = ex.get("vision_feature_layer", -2)
            if not isinstance(layer, int):
                raise NotImplementedError("multi-layer vision features")
            strategy = ex.get("vision_feature_select_strategy", "default")
            self.image_id = int(ex.get("image_token_index", ex.get("image_token_id", 32000)))
            self.pad_square = False
            if ex.get("projector_hidden_act", "gelu") != "gelu":
                raise NotImplementedError(f"projector act {ex.get('projector_hidden_act')!r}")
        self.visual = CLIPVisionTower(vc, self.device, dtype, int(layer), strategy)
        self.proj: dict[str, torch.Tensor | None] = {}

    def init_random(self, seed: int = 0, std: float = 0.02) -> "LlavaForConditionalGeneration":
        super().init_random(seed, std)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 4457)
        self.visual.init_random(gen, std)
        H, E = self.cfg.hidden_size, self.visual.E
        mk = lambda *s: torch.empty(*s, dtype=self.dtype, device=self.device).normal_(0.0, std, generator=gen)  # noqa
        self.proj = {"w1": mk(H, E), "b1": torch.zeros(H, dtype=self.dtype, device=self.device), "w2": mk(H, H),
                     "b2": torch.zeros(H, dtype=self.dtype, device=self.device)}
        return self

    _PROJ = {"multi_modal_projector.linear_1.weight": "w1", "multi_modal_projector.linear_1.bias": "b1",
             "multi_modal_projector.linear_2.weight": "w2", "multi_modal_projector.linear_2.bias": "b2",
             "mm_projector.0.weight": "w1", "mm_projector.0.bias": "b1", "mm_projector.2.weight": "w2",
             "mm_projector.2.bias": "b2"}

    def load_hf_weights(self, weights) -> "LlavaForConditionalGeneration":
        pend: dict = {}

        def text_only():
            for name, w in weights:
                n = name[len("model."):] if name.startswith("model.") else name
                for pre in ("vision_tower.vision_tower.vision_model.", "vision_tower.vision_model.", "vision_tower."):
                    if n.startswith(pre):
                        self.visual.load(n[len(pre):], w, pend)
                        break
                else:
                    if n in self._PROJ:
                        self.proj[self._PROJ[n]] = w.to(device=self.device, dtype=self.dtype).contiguous()
                    elif n.startswith("language_model."):
                        rest = n[len("language_model."):]
                        yield ("lm_head.weight" if rest == "lm_head.weight" else
                               "model." + (rest[len("model."):] if rest.startswith("model.") else rest)), w
                    elif n.startswith(("vision_resampler.", "image_newline")):
                        continue
                    else:
                        yield name, w

        super().load_hf_weights(text_only())
        if pend:
            raise ValueError(f"incomplete vision q/k/v projections: {sorted(pend)}")
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
        ids, pvs, spans, last = [], [], [], 0
        n = self.visual.tokens
        for i, im in zip(where, images):
            px = im if isinstance(im, torch.Tensor) else preprocess_clip(im, self.visual.image, self.pad_square)
            ids += prompt_ids[last:i]
            spans.append((len(ids), n))
            ids += [pad_token_id(px, self.cfg.vocab_size)] * n
            pvs.append(px)
            last = i + 1
        ids += prompt_ids[last:]
        return ids, MMInput(torch.cat(pvs, 0), [(1, self.visual.side, self.visual.side)] * len(pvs), spans)

    def encode_images(self, pixel_values: torch.Tensor, grids=None) -> torch.Tensor:
        p = self.proj
        h = linear(self.visual.forward(pixel_values), p["w1"], p["b1"])
        return linear(ops.act(h, 3), p["w2"], p["b2"])

    def embed_with_images(self, ids: torch.Tensor, rows: torch.Tensor, feats: torch.Tensor) -> torch.Tensor:
        h = pstate.tp_all_reduce(ops.embedding(ids, self.embed, self.tp.vocab_start, self.tp.vocab_end))
        if rows.numel():
            h.index_copy_(0, rows, feats.to(h.dtype))
        return h
