"""Nemotron Nano 12B v2 VL (``NemotronH_Nano_VL_V2`` / ``NemotronVLForConditionalGeneration``).

Reference catalog: ``config/models/nvidia/NVIDIA-Nemotron-Nano-12B-v2-VL-{BF16,FP8}.yaml`` (the
two checkpoints name the same architecture differently).  The model is the InternVL recipe on a
NemotronH hybrid Mamba-2 / attention language model (``nemotron_h.py``):

* preprocessing: InternVL dynamic tiling (``internvl.tile_grid``) with 512-px tiles, a thumbnail
  when more than one tile, the RADIO input conditioner's mean / std (``norm_mean`` / ``norm_std``);
* RADIO v2.5 tower (:class:`RadioTower`): 16-px patch GEMM, class + register tokens, a CPE
  position table (``cpe_max_size / patch`` squared) bilinearly resized (align-corners) to the
  larger grid side and windowed to the tile grid, pre-norm ViT blocks (fused QKV + bias,
  bidirectional varlen MFMA attention per tile, GELU MLP), final LayerNorm; the class / register
  tokens are dropped;
* 0.5 pixel shuffle (InternVL v2 order) -> RMSNorm -> GEMM -> ReLU^2 -> GEMM (``mlp1``, no bias);
* prompt: ``<img>`` + ``<image>`` x 256 per tile + ``</img>``.
No reference implementation is importable here (RADIO and the remote code are not in
transformers): ``tests/test_nemotron_vl_cpu.py`` checks against an independent fp32 restatement,
so parity with the remote code is unpinned.
"""
from __future__ import annotations

import json
from pathlib import Path

import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.models.config import ModelConfig
from ome_amd.models.internvl import _InternVLMixin, _text_config, preprocess_internvl
from ome_amd.models.quant import linear
from ome_amd.multimodal.inputs import CLIP_MEAN, CLIP_STD

NEMOTRON_VL_ARCHS = {"NemotronH_Nano_VL_V2", "NemotronVLForConditionalGeneration"}


def special_token_ids(model_path: str | None, names: list[str]) -> dict[str, int]:
    """ids of added tokens by content, read from ``tokenizer.json`` (no tokenizer library)."""
    if not model_path:
        return {}
    p = Path(model_path) / "tokenizer.json"
    if not p.is_file():
        return {}
    try:
        added = json.loads(p.read_text()).get("added_tokens") or []
    except (OSError, ValueError):
        return {}
    want = set(names)
    return {t["content"]: int(t["id"]) for t in added if t.get("content") in want}


class RadioTower:
    """RADIO v2.5 ViT (``vision_model.radio_model.*``)."""

    def __init__(self, vc: dict, device, dtype, image: int = 512, patch: int = 16):
        args = vc.get("args") or {}
        self.device, self.dtype = device, dtype
        self.E = int(vc.get("hidden_size") or args.get("hidden_size") or 1280)
        self.heads = int(vc.get("num_attention_heads") or args.get("num_heads") or 16)
        self.D = self.E // self.heads
        self.depth = int(vc.get("num_hidden_layers") or args.get("depth") or 32)
        self.I = int(vc.get("intermediate_size") or 4 * self.E)
        self.patch = int(vc.get("patch_size") or patch)
        self.image = int(image)
        self.side = self.image // self.patch
        self.max_grid = int(vc.get("cpe_max_size") or args.get("cpe_max_size") or 2048) // self.patch
        self.n_skip = int(vc.get("num_skip") or (vc.get("num_cls_tokens", 1) + vc.get("num_registers", 0)) or 1)
        self.eps = float(vc.get("layer_norm_eps", 1e-6))
        self.w: dict[str, torch.Tensor] = {}
        self._pos: dict[tuple[int, int], torch.Tensor] = {}

    def _t(self, t):
        return t.to(device=self.device, dtype=self.dtype).contiguous()

    def init_random(self, gen: torch.Generator, std: float = 0.02) -> None:
        E, I = self.E, self.I
        shapes = {"patch.weight": (E, 3 * self.patch ** 2), "pos": (self.max_grid ** 2, E), "cls": (self.n_skip, E),
                  "norm.weight": (E,), "norm.bias": (E,)}
        for b in range(self.depth):
            p = f"blocks.{b}."
            shapes.update({p + "qkv.weight": (3 * E, E), p + "qkv.bias": (3 * E,), p + "proj.weight": (E, E),
                           p + "proj.bias": (E,), p + "fc1.weight": (I, E), p + "fc1.bias": (I,),
                           p + "fc2.weight": (E, I), p + "fc2.bias": (E,), p + "norm1.weight": (E,),
                           p + "norm1.bias": (E,), p + "norm2.weight": (E,), p + "norm2.bias": (E,)})
        for k, s in shapes.items():
            t = torch.empty(*s, dtype=self.dtype, device=self.device)
            if k.endswith(("norm1.weight", "norm2.weight", "norm.weight")):
                t.fill_(1.0)
            elif len(s) == 1:
                t.zero_()
            else:
                t.normal_(0.0, std, generator=gen)
            self.w[k] = t
        self._pos.clear()

    def load(self, name: str, t: torch.Tensor) -> None:
        """``name`` relative to ``radio_model.``."""
        if name.startswith("input_conditioner.") or name.endswith("summary_idxs"):
            return
        if name.startswith("model."):
            name = name[len("model."):]
        if name == "patch_generator.embedder.weight":
            self.w["patch.weight"] = self._t(t.reshape(t.shape[0], -1))
        elif name == "patch_generator.embedder.bias":
            self.w["patch.bias"] = self._t(t)
        elif name == "patch_generator.pos_embed":
            self.w["pos"] = self._t(t.reshape(-1, t.shape[-1]))
            self.max_grid = int(round(self.w["pos"].shape[0] ** 0.5))
        elif name == "patch_generator.cls_token.token":
            self.w["cls"] = self._t(t.reshape(-1, t.shape[-1]))
            self.n_skip = self.w["cls"].shape[0]
        elif name in ("norm.weight", "norm.bias"):
            self.w[name] = self._t(t)
        elif name.startswith("blocks."):
            parts = name.split(".")
            mod = ".".join(parts[2:-1])
            key = {"attn.qkv": "qkv", "attn.proj": "proj", "mlp.fc1": "fc1", "mlp.fc2": "fc2", "norm1": "norm1",
                   "norm2": "norm2"}.get(mod)
            if key is None:
                raise KeyError(f"unexpected RADIO weight {name}")
            self.w[f"blocks.{parts[1]}.{key}.{parts[-1]}"] = self._t(t)
        self._pos.clear()

    def pos_embed(self, h: int, w: int) -> torch.Tensor:
        """CPE table for an h x w patch grid: resize (bilinear, align corners) to the larger side,
        keep the top-left h x w window -> [h*w, E]."""
        got = self._pos.get((h, w))
        if got is None:
            g, E = self.max_grid, self.E
            tab = self.w["pos"].float().view(1, g, g, E).permute(0, 3, 1, 2)
            m = max(h, w)
            if m != g:
                tab = F.interpolate(tab, size=(m, m), mode="bilinear", align_corners=True)
            got = tab[0, :, :h, :w].permute(1, 2, 0).reshape(h * w, E).to(self.dtype).contiguous()
            self._pos[(h, w)] = got
        return got

    def forward(self, pixels: torch.Tensor) -> torch.Tensor:
        """pixels [n, 3, S, S] (normalised) -> patch features [n * side^2, E]."""
        w, E, n, ps, s = self.w, self.E, pixels.shape[0], self.patch, pixels.shape[-1] // self.patch
        x = pixels[..., :s * ps, :s * ps].to(device=self.device, dtype=self.dtype)   # a stride-ps conv drops the rest
        x = x.reshape(n, 3, s, ps, s, ps).permute(0, 2, 4, 1, 3, 5).reshape(n * s * s, -1)
        x = linear(x, w["patch.weight"], w.get("patch.bias")).view(n, s * s, E) + self.pos_embed(s, s)
        k = self.n_skip
        x = torch.cat([w["cls"].view(1, k, E).expand(n, k, E), x], 1).reshape(-1, E).contiguous()
        L = s * s + k
        T = n * L
        lens = [L] * n
        for b in range(self.depth):
            p = f"blocks.{b}."
            h = ops.layernorm(x, w[p + "norm1.weight"], w[p + "norm1.bias"], self.eps)
            qkv = linear(h, w[p + "qkv.weight"], w.get(p + "qkv.bias")).view(T, 3, self.heads, self.D)
            a = ops.varlen_attention(qkv[:, 0], qkv[:, 1], qkv[:, 2], lens, self.D ** -0.5).reshape(T, E)
            x = x + linear(a, w[p + "proj.weight"], w.get(p + "proj.bias"))
            h = ops.layernorm(x, w[p + "norm2.weight"], w[p + "norm2.bias"], self.eps)
            x = x + linear(ops.act(linear(h, w[p + "fc1.weight"], w.get(p + "fc1.bias")), 3), w[p + "fc2.weight"],
                           w.get(p + "fc2.bias"))
        if "norm.weight" in w:
            x = ops.layernorm(x, w["norm.weight"], w.get("norm.bias"), self.eps)
        return x.view(n, L, E)[:, k:].reshape(-1, E)


class _NemotronVLMixin(_InternVLMixin):
    def _setup_vision(self, full: ModelConfig) -> None:
        ex = full.extra or {}
        self.orig_layout = True
        size = int(ex.get("force_image_size") or ex.get("image_size") or 512)
        self.visual = RadioTower(ex.get("vision_config") or {}, self.device, self.dtype, size,
                                 int(ex.get("patch_size") or 16))
        self.ratio = float(ex.get("downsample_ratio", 0.5))
        self.ps = int(round(1 / self.ratio))
        self.tokens_per_tile = (self.visual.side // self.ps) ** 2
        self.max_tiles = int(ex.get("max_dynamic_patch") or ex.get("max_num_tiles") or 12)
        self.thumbnail = bool(ex.get("use_thumbnail", True))
        self.mean = tuple(ex.get("norm_mean") or CLIP_MEAN)
        self.std = tuple(ex.get("norm_std") or CLIP_STD)
        names = [ex.get("img_start_token", "<img>"), ex.get("img_end_token", "</img>"),
                 ex.get("img_context_token", "<image>")]
        tok = special_token_ids(ex.get("_model_path"), names)
        st, en = ex.get("img_start_token_id", tok.get(names[0])), ex.get("img_end_token_id", tok.get(names[1]))
        self.img_start = None if st is None else int(st)
        self.img_end = None if en is None else int(en)
        ctx = ex.get("img_context_token_id", tok.get(names[2]))
        if ctx is None:
            raise ValueError("Nemotron VL config has no img_context_token_id")
        self.image_id = int(ctx)
        self.proj: dict[str, torch.Tensor | None] = {}

    def init_random(self, seed: int = 0, std: float = 0.02):
        self._lm_base.init_random(self, seed, std)   # the language model's own init
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 5119)
        self.visual.init_random(gen, std)
        H, C = self.cfg.hidden_size, self.visual.E * self.ps ** 2
        P = int((self.full_cfg.extra or {}).get("projector_hidden_size") or 4 * H)
        mk = lambda *s: torch.empty(*s, dtype=self.dtype, device=self.device).normal_(0.0, std, generator=gen)  # noqa
        self.proj = {"norm": torch.ones(C, dtype=self.dtype, device=self.device), "w1": mk(P, C), "w2": mk(H, P)}
        return self

    _PROJ = {"mlp1.0.weight": "norm", "mlp1.1.weight": "w1", "mlp1.3.weight": "w2"}

    def load_hf_weights(self, weights):
        def lm_only():
            for name, w in weights:
                if name.startswith("vision_model.radio_model."):
                    self.visual.load(name[len("vision_model.radio_model."):], w)
                elif name in self._PROJ:
                    self.proj[self._PROJ[name]] = w.to(device=self.device, dtype=self.dtype).contiguous()
                elif name.startswith("language_model."):
                    yield name[len("language_model."):], w
                elif not name.startswith("vision_model."):
                    yield name, w

        self._lm_base.load_hf_weights(self, lm_only())
        return self

    def image_prompt_ids(self) -> list[int]:
        return [t for t in (self.img_start, self.image_id, self.img_end) if t is not None]

    def make_mm_input(self, prompt_ids: list[int], images: list):
        images = [im if isinstance(im, torch.Tensor) else
                  preprocess_internvl(im, self.visual.image, self.max_tiles, self.thumbnail, self.mean, self.std)
                  for im in images]
        return super().make_mm_input(prompt_ids, images)

    def encode_images(self, pixel_values: torch.Tensor, grids=None) -> torch.Tensor:
        n, s, E, r = pixel_values.shape[0], self.visual.side, self.visual.E, self.ps
        x = self.visual.forward(pixel_values).view(n, s, s, E)
        x = x.view(n, s, s // r, E * r).permute(0, 2, 1, 3).reshape(n, s // r, s // r, E * r * r)
        x = x.permute(0, 2, 1, 3).reshape(n * (s // r) ** 2, E * r * r).contiguous()
        p = self.proj
        x = ops.rmsnorm(x, p["norm"], 1e-5)
        x = ops.act(linear(x, p["w1"]), 4)   # ReLU^2
        return linear(x, p["w2"])


_CLASSES: dict = {}


def nemotron_vl_class(cfg: ModelConfig):
    """Nemotron VL hooks + the language model's own class (NemotronH)."""
    from ome_amd.models import model_class

    base = model_class(_text_config(cfg))
    cls = _CLASSES.get(base)
    if cls is None:
        def __init__(self, cfg_full: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions=None):
            base.__init__(self, _text_config(cfg_full), device, dtype, max_positions)
            self.full_cfg = cfg_full
            self._setup_vision(cfg_full)

        cls = type(f"NemotronVL_{base.__name__}", (_NemotronVLMixin, base), {"__init__": __init__, "_lm_base": base})
        _CLASSES[base] = cls
    return cls
