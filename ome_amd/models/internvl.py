"""InternVL 2 / 2.5 / 3 vision-language models: the original ``InternVLChatModel`` layout (reference
catalog ``config/runtimes/srt/OpenGVLab/InternVL2_5-8B-rt.yaml``) and the transformers
``InternVLForConditionalGeneration`` layout.

* preprocessing: dynamic tiling -- the tile grid (cols x rows, 1..max_dynamic_patch tiles) whose
  aspect ratio is closest to the image's (ties -> more tiles while the image area exceeds half
  the canvas), bicubic resize to the canvas, 448-px tiles in row-major order plus a thumbnail
  when more than one tile, ImageNet mean / std;
* prompt: each image becomes ``<img>`` + ``<IMG_CONTEXT>`` x 256 per tile (content-hash ids) +
  ``</img>``;
* InternViT tower: patch GEMM (+bias), class token, learned positions, pre-norm blocks
  (LayerNorm or RMSNorm) with fused QKV GEMM, optional full-width q / k RMSNorm (InternViT-6B),
  bidirectional varlen MFMA attention per tile, layer-scale (``ls1`` / ``ls2``) residuals,
  GELU MLP; class token dropped;
* 0.5 pixel shuffle (2 x 2 neighbourhoods -> 4x channels, 1/4 tokens) -> LayerNorm -> GEMM ->
  GELU -> GEMM;
* language model: whatever ``llm_config`` / ``text_config`` names -- InternLM2 (``decoder.py``
  spec), Qwen2 / Llama (``llama.py``) -- the class is composed at load time
  (:func:`internvl_class`), so the LM keeps its own fused kernels and HIP-graph decode.
"""
from __future__ import annotations

import dataclasses

import numpy as np
import torch

from ome_amd import ops
from ome_amd.models.config import ModelConfig
from ome_amd.models.quant import linear
from ome_amd.multimodal.inputs import MMInput, load_image, pad_token_id
from ome_amd.parallel import state as pstate

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
INTERNVL_ARCHS = {"InternVLChatModel", "InternVLForConditionalGeneration"}
# <img>, </img>, <IMG_CONTEXT> of the InternVL tokenizers, by language-model family
_SPECIAL = {"InternLM2ForCausalLM": (92544, 92545, 92546), "Qwen2ForCausalLM": (151665, 151666, 151667),
            "LlamaForCausalLM": (128258, 128259, 128260)}


def tile_grid(w: int, h: int, tile: int, max_tiles: int, min_tiles: int = 1) -> tuple[int, int]:
    """(cols, rows) of the tiling canvas (InternVL ``dynamic_preprocess``)."""
    grids = sorted([(c, r) for c in range(1, max_tiles + 1) for r in range(1, max_tiles + 1)
                    if min_tiles <= c * r <= max_tiles], key=lambda g: g[0] * g[1])
    aspect, area = w / h, w * h
    best, best_diff = (1, 1), float("inf")
    for g in grids:
        d = abs(aspect - g[0] / g[1])
        if d < best_diff:
            best, best_diff = g, d
        elif d == best_diff and area > 0.5 * tile * tile * g[0] * g[1]:
            best = g
    return best


def preprocess_internvl(image, tile: int = 448, max_tiles: int = 12, thumbnail: bool = True,
                        mean=IMAGENET_MEAN, std=IMAGENET_STD) -> torch.Tensor:
    """-> float32 [n_tiles, 3, tile, tile]."""
    from PIL import Image

    img = load_image(image)
    cols, rows = tile_grid(img.width, img.height, tile, max_tiles)
    canvas = img.resize((tile * cols, tile * rows), Image.BICUBIC)
    tiles = [canvas.crop((c * tile, r * tile, (c + 1) * tile, (r + 1) * tile)) for r in range(rows)
             for c in range(cols)]
    if thumbnail and len(tiles) > 1:
        tiles.append(img.resize((tile, tile), Image.BICUBIC))
    a = np.stack([np.asarray(t, dtype=np.float32) for t in tiles]) / 255.0
    a = (a - np.asarray(mean, np.float32)) / np.asarray(std, np.float32)
    return torch.from_numpy(np.ascontiguousarray(a.transpose(0, 3, 1, 2)))


class InternViTTower:
    def __init__(self, vc: dict, device, dtype, feature_layer: int = -1):
        self.device, self.dtype = device, dtype
        self.E = int(vc.get("hidden_size", 1024))
        self.heads = int(vc.get("num_attention_heads", 16))
        self.D = self.E // self.heads
        self.depth = int(vc.get("num_hidden_layers", 24))
        self.I = int(vc.get("intermediate_size", 4096))
        im, ps = vc.get("image_size", 448), vc.get("patch_size", 14)
        self.image = int(im[0] if isinstance(im, (list, tuple)) else im)
        self.patch = int(ps[0] if isinstance(ps, (list, tuple)) else ps)
        self.side = self.image // self.patch
        self.n_patch = self.side ** 2
        self.eps = float(vc.get("layer_norm_eps", 1e-6))
        self.rms = vc.get("norm_type", "layer_norm") == "rms_norm"
        self.qk_norm = bool(vc.get("qk_normalization", vc.get("use_qk_norm", False)))
        self.qkv_bias = bool(vc.get("qkv_bias", vc.get("attention_bias", True)))
        if vc.get("hidden_act", "gelu") != "gelu":
            raise NotImplementedError(f"InternViT hidden_act {vc.get('hidden_act')!r}")
        self.n_layers = feature_layer if feature_layer >= 0 else self.depth + 1 + feature_layer
        self.w: dict[str, torch.Tensor | None] = {}

    def _t(self, t):
        return t.to(device=self.device, dtype=self.dtype).contiguous()

    def init_random(self, gen: torch.Generator, std: float = 0.02) -> None:
        E, I = self.E, self.I
        shapes = {"patch.weight": (E, 3 * self.patch ** 2), "patch.bias": (E,), "cls": (E,),
                  "pos": (self.n_patch + 1, E)}
        for b in range(self.n_layers):
            p = f"layers.{b}."
            shapes.update({p + "qkv.weight": (3 * E, E), p + "proj.weight": (E, E), p + "proj.bias": (E,),
                           p + "fc1.weight": (I, E), p + "fc1.bias": (I,), p + "fc2.weight": (E, I),
                           p + "fc2.bias": (E,), p + "norm1.weight": (E,), p + "norm2.weight": (E,),
                           p + "ls1": (E,), p + "ls2": (E,)})
            if self.qkv_bias:
                shapes[p + "qkv.bias"] = (3 * E,)
            if not self.rms:
                shapes.update({p + "norm1.bias": (E,), p + "norm2.bias": (E,)})
            if self.qk_norm:
                shapes.update({p + "q_norm": (E,), p + "k_norm": (E,)})
        for k, s in shapes.items():
            t = torch.empty(*s, dtype=self.dtype, device=self.device)
            if k.endswith(("norm1.weight", "norm2.weight", "q_norm", "k_norm")):
                t.fill_(1.0)
            elif k.endswith(("ls1", "ls2")):
                t.fill_(0.1)
            elif len(s) == 1 and k != "cls":
                t.zero_()
            else:
                t.normal_(0.0, std, generator=gen)
            self.w[k] = t

    # original InternViT names (relative to ``vision_model.``) and transformers names
    # (relative to ``vision_tower.``) -> ours
    _ORIG = {"attn.proj": "proj", "mlp.fc1": "fc1", "mlp.fc2": "fc2", "norm1": "norm1", "norm2": "norm2",
             "attn.q_norm": "q_norm", "attn.k_norm": "k_norm", "ls1": "ls1", "ls2": "ls2", "attn.qkv": "qkv"}
    _HF = {"attention.projection_layer": "proj", "mlp.fc1": "fc1", "mlp.fc2": "fc2", "layernorm_before": "norm1",
           "layernorm_after": "norm2", "attention.q_norm": "q_norm", "attention.k_norm": "k_norm",
           "lambda_1": "ls1", "lambda_2": "ls2"}

    def load(self, name: str, t: torch.Tensor, pend: dict) -> None:
        if name in ("embeddings.class_embedding", "embeddings.cls_token"):
            self.w["cls"] = self._t(t.reshape(-1))
        elif name in ("embeddings.patch_embedding.weight", "embeddings.patch_embeddings.projection.weight"):
            self.w["patch.weight"] = self._t(t.reshape(t.shape[0], -1))
        elif name in ("embeddings.patch_embedding.bias", "embeddings.patch_embeddings.projection.bias"):
            self.w["patch.bias"] = self._t(t)
        elif name in ("embeddings.position_embedding", "embeddings.position_embeddings"):
            self.w["pos"] = self._t(t.reshape(-1, t.shape[-1]))
        elif name.startswith(("encoder.layers.", "encoder.layer.")):
            parts = name.split(".")
            b = int(parts[2])
            if b >= self.n_layers:
                return
            rest = parts[3:]
            kind = rest[-1] if rest[-1] in ("weight", "bias") else ""
            mod = ".".join(rest[:-1]) if kind else ".".join(rest)
            p = f"layers.{b}."
            if mod in ("attention.q_proj", "attention.k_proj", "attention.v_proj"):
                got = pend.setdefault((b, kind), {})
                got[mod[-6]] = t
                if len(got) == 3:
                    self.w[p + "qkv." + kind] = self._t(torch.cat([got["q"], got["k"], got["v"]]))
                    del pend[(b, kind)]
                return
            key = self._ORIG.get(mod) or self._HF.get(mod)
            if key is None:
                raise KeyError(f"unexpected InternViT weight {name}")
            if key in ("ls1", "ls2", "q_norm", "k_norm"):
                self.w[p + key] = self._t(t)
            else:
                self.w[p + key + "." + kind] = self._t(t)

    def _norm(self, x, p):
        if self.rms:
            return ops.rmsnorm(x, self.w[p + ".weight"], self.eps)
        return ops.layernorm(x, self.w[p + ".weight"], self.w.get(p + ".bias"), self.eps)

    def forward(self, pixels: torch.Tensor) -> torch.Tensor:
        """pixels [n, 3, S, S] -> patch features (class token dropped) [n * side^2, E]."""
        w, E, n, ps, s = self.w, self.E, pixels.shape[0], self.patch, self.side
        x = pixels.to(device=self.device, dtype=self.dtype)
        x = x.reshape(n, 3, s, ps, s, ps).permute(0, 2, 4, 1, 3, 5).reshape(n * self.n_patch, -1)
        x = linear(x, w["patch.weight"], w["patch.bias"]).view(n, self.n_patch, E)
        x = (torch.cat([w["cls"].view(1, 1, E).expand(n, 1, E), x], 1) + w["pos"]).reshape(-1, E).contiguous()
        L = self.n_patch + 1
        T = n * L
        lens = [L] * n
        for b in range(self.n_layers):
            p = f"layers.{b}."
            h = self._norm(x, p + "norm1")
            qkv = linear(h, w[p + "qkv.weight"], w.get(p + "qkv.bias"))
            q, k, v = qkv[:, :E], qkv[:, E:2 * E], qkv[:, 2 * E:]
            if self.qk_norm:
                q = ops.rmsnorm(q, w[p + "q_norm"], self.eps)
                k = ops.rmsnorm(k, w[p + "k_norm"], self.eps)
            a = ops.varlen_attention(q.reshape(T, self.heads, self.D), k.reshape(T, self.heads, self.D),
                                     v.reshape(T, self.heads, self.D), lens, self.D ** -0.5).reshape(T, E)
            x = x + linear(a, w[p + "proj.weight"], w[p + "proj.bias"]) * w[p + "ls1"]
            h = ops.act(linear(self._norm(x, p + "norm2"), w[p + "fc1.weight"], w[p + "fc1.bias"]), 3)
            x = x + linear(h, w[p + "fc2.weight"], w[p + "fc2.bias"]) * w[p + "ls2"]
        return x.view(n, L, E)[:, 1:].reshape(-1, E)


class _InternVLMixin:
    """Vision tower + projector + multimodal hooks on top of a language-model class."""
    is_multimodal = True

    def _setup_vision(self, full: ModelConfig) -> None:
        ex = full.extra or {}
        self.orig_layout = full.architecture == "InternVLChatModel"
        vc = ex.get("vision_config") or {}
        layer = ex.get("select_layer", ex.get("vision_feature_layer", -1))
        self.visual = InternViTTower(vc, self.device, self.dtype, int(layer))
        self.ratio = float(ex.get("downsample_ratio", 0.5))
        self.ps = int(round(1 / self.ratio))
        self.tokens_per_tile = (self.visual.side // self.ps) ** 2
        self.max_tiles = int(ex.get("max_dynamic_patch", 12)) if ex.get("dynamic_image_size", True) else 1
        self.thumbnail = bool(ex.get("use_thumbnail", True))
        lm_arch = self.cfg.architecture
        st, en, ctx = _SPECIAL.get(lm_arch, _SPECIAL["Qwen2ForCausalLM"])
        self.img_start = int(ex.get("img_start_token_id", st))
        self.img_end = int(ex.get("img_end_token_id", en))
        self.image_id = int(ex.get("img_context_token_id", ex.get("image_token_id", ctx)))
        if ex.get("ps_version", "v2") != "v2":
            raise NotImplementedError("pixel shuffle v1")
        self.proj: dict[str, torch.Tensor | None] = {}

    def init_random(self, seed: int = 0, std: float = 0.02):
        super().init_random(seed, std)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 4481)
        self.visual.init_random(gen, std)
        H, C = self.cfg.hidden_size, self.visual.E * self.ps ** 2
        mk = lambda *s: torch.empty(*s, dtype=self.dtype, device=self.device).normal_(0.0, std, generator=gen)  # noqa
        z = lambda n: torch.zeros(n, dtype=self.dtype, device=self.device)  # noqa: E731
        self.proj = {"ln.weight": torch.ones(C, dtype=self.dtype, device=self.device), "ln.bias": z(C),
                     "w1": mk(H, C), "b1": z(H), "w2": mk(H, H), "b2": z(H)}
        return self

    _PROJ = {"mlp1.0.weight": "ln.weight", "mlp1.0.bias": "ln.bias", "mlp1.1.weight": "w1", "mlp1.1.bias": "b1",
             "mlp1.3.weight": "w2", "mlp1.3.bias": "b2",
             "multi_modal_projector.layer_norm.weight": "ln.weight", "multi_modal_projector.layer_norm.bias": "ln.bias",
             "multi_modal_projector.linear_1.weight": "w1", "multi_modal_projector.linear_1.bias": "b1",
             "multi_modal_projector.linear_2.weight": "w2", "multi_modal_projector.linear_2.bias": "b2"}

    def load_hf_weights(self, weights):
        pend: dict = {}

        def lm_only():
            for name, w in weights:
                n = name[len("model."):] if name.startswith("model.") and not self.orig_layout else name
                if n.startswith(("vision_model.", "vision_tower.")):
                    self.visual.load(n.split(".", 1)[1], w, pend)
                elif n in self._PROJ:
                    self.proj[self._PROJ[n]] = w.to(device=self.device, dtype=self.dtype).contiguous()
                elif n.startswith("language_model."):
                    rest = n[len("language_model."):]
                    # language_model.{model.*, output / lm_head} (original and saved transformers
                    # checkpoints) or language_model.* (transformers' in-memory names)
                    yield (rest if rest.startswith(("model.", "lm_head.", "output.")) else "model." + rest), w
                else:
                    yield name, w

        super().load_hf_weights(lm_only())
        if pend:
            raise ValueError(f"incomplete InternViT projections: {sorted(pend)}")
        return self

    def weight_bytes(self) -> int:
        n = super().weight_bytes() + sum(t.numel() * t.element_size() for t in self.visual.w.values()
                                         if t is not None)
        return n + sum(t.numel() * t.element_size() for t in self.proj.values() if t is not None)

    # ------------------------------------------------------------------ multimodal
    def image_prompt_ids(self) -> list[int]:
        return [self.img_start, self.image_id, self.img_end]

    def make_mm_input(self, prompt_ids: list[int], images: list):
        where = [i for i, t in enumerate(prompt_ids) if t == self.image_id]
        if len(where) != len(images):
            raise ValueError(f"prompt has {len(where)} image tokens for {len(images)} images")
        ids, pvs, spans, last = [], [], [], 0
        for i, im in zip(where, images):
            px = im if isinstance(im, torch.Tensor) else preprocess_internvl(im, self.visual.image, self.max_tiles,
                                                                             self.thumbnail)
            n = px.shape[0] * self.tokens_per_tile
            ids += prompt_ids[last:i]
            spans.append((len(ids), n))
            ids += [pad_token_id(px, self.cfg.vocab_size)] * n
            pvs.append(px)
            last = i + 1
        ids += prompt_ids[last:]
        px = torch.cat(pvs, 0)
        return ids, MMInput(px, [(1, self.visual.side, self.visual.side)] * px.shape[0], spans)

    def encode_images(self, pixel_values: torch.Tensor, grids=None) -> torch.Tensor:
        n, s, E, r = pixel_values.shape[0], self.visual.side, self.visual.E, self.ps
        x = self.visual.forward(pixel_values).view(n, s, s, E)
        # pixel shuffle v2 (transformers InternVLModel.pixel_shuffle): [n, s, s, E] -> [n, s/r, s/r, E r^2]
        x = x.view(n, s, s // r, E * r).permute(0, 2, 1, 3).reshape(n, s // r, s // r, E * r * r)
        x = x.permute(0, 2, 1, 3).reshape(n * (s // r) ** 2, E * r * r).contiguous()
        p = self.proj
        x = ops.layernorm(x, p["ln.weight"], p["ln.bias"], 1e-5)
        x = ops.act(linear(x, p["w1"], p["b1"]), 3)
        return linear(x, p["w2"], p["b2"])

    def embed_with_images(self, ids: torch.Tensor, rows: torch.Tensor, feats: torch.Tensor) -> torch.Tensor:
        h = self._text_embed(ids)
        if rows.numel():
            h.index_copy_(0, rows, feats.to(h.dtype))
        return h

    def _text_embed(self, ids: torch.Tensor) -> torch.Tensor:
        h = pstate.tp_all_reduce(ops.embedding(ids, self.embed, self.tp.vocab_start, self.tp.vocab_end))
        scale = getattr(getattr(self, "spec", None), "embed_scale", 1.0)
        return h * scale if scale != 1.0 else h


def _text_config(cfg: ModelConfig) -> ModelConfig:
    ex = cfg.extra or {}
    llm = ex.get("llm_config") or ex.get("text_config") or {}
    arch = (llm.get("architectures") or [None])[0]
    if arch is None:
        mt = llm.get("model_type", "qwen2")
        arch = {"qwen2": "Qwen2ForCausalLM", "llama": "LlamaForCausalLM", "internlm2": "InternLM2ForCausalLM",
                "qwen3": "Qwen3ForCausalLM", "nemotron_h": "NemotronHForCausalLM"}.get(mt, "Qwen2ForCausalLM")
    return dataclasses.replace(cfg, architecture=arch, model_type=llm.get("model_type", cfg.model_type))


_CLASSES: dict = {}


def internvl_class(cfg: ModelConfig):
    """A class = InternVL vision hooks + the language model's own class."""
    from ome_amd.models import model_class

    tcfg = _text_config(cfg)
    base = model_class(tcfg)
    cls = _CLASSES.get(base)
    if cls is None:
        def __init__(self, cfg_full: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions=None):
            base.__init__(self, _text_config(cfg_full), device, dtype, max_positions)
            self.full_cfg = cfg_full
            self._setup_vision(cfg_full)

        cls = type(f"InternVL_{base.__name__}", (_InternVLMixin, base), {"__init__": __init__})
        _CLASSES[base] = cls
    return cls
