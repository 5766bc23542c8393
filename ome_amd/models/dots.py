"""rednote-hilab dots.ocr (``DotsOCRForConditionalGeneration``) and dots.vlm1
(``DotsVLMForConditionalGeneration``): the dots NaViT vision encoder on a Qwen2 (dots.ocr) or
DeepSeek-V3 MLA / MoE (dots.vlm1) language model.

Reference catalog: ``config/runtimes/srt/rednote-hilab/dots-ocr-rt.yaml`` and
``dots-vlm1-inst-rt.yaml``.  The vision encoder (:class:`DotsVisionTower`), MI355X-side:

* Qwen2-VL patchification (``smart_resize`` to multiples of 28, CLIP mean / std, 14-px patches in
  2x2-merge-block-major order, one temporal patch);
* patch GEMM (+bias) -> RMSNorm; 2-D rotary (row / column halves of each head, base 10000, the
  Qwen2-VL ``rot_pos`` table); pre-norm blocks: RMSNorm -> fused QKV GEMM -> bidirectional varlen
  MFMA attention per image -> proj; RMSNorm -> SwiGLU (``fc2(silu(fc1 x) * fc3 x)``); a final
  ``post_trunk_norm`` RMSNorm;
* merger: LayerNorm -> 2x2 merge (4E) -> GEMM -> GELU -> GEMM to the LM width.
The language model keeps plain 1-D positions; image features replace the ``<|imgpad|>`` rows.
The LM class is composed at load time (:func:`dots_class`): Qwen2 on ``llama.py``, DeepSeek-V3 on
``deepseek.py`` -- each keeps its own kernels and HIP-graph decode.  No dots class is importable
here: ``tests/test_dots_cpu.py`` checks against an independent fp32 restatement of the encoder and
transformers' Qwen2 (parity with the remote code unpinned).
"""
from __future__ import annotations

import dataclasses

import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.models.config import ModelConfig
from ome_amd.models.qwen2_vl import Qwen2VisionTower
from ome_amd.models.quant import linear
from ome_amd.multimodal.inputs import MMInput, pad_token_id, preprocess_image
from ome_amd.parallel import state as pstate

DOTS_ARCHS = {"DotsOCRForConditionalGeneration", "DotsVLMForConditionalGeneration"}


class DotsVisionTower(Qwen2VisionTower):
    def __init__(self, vc: dict, out_hidden: int, device, dtype):
        self.device, self.dtype = device, dtype
        self.E = int(vc.get("embed_dim") or vc.get("hidden_size") or 1536)
        self.depth = int(vc.get("num_hidden_layers", 42))
        self.heads = int(vc.get("num_attention_heads", 12))
        self.hd = self.E // self.heads
        self.inter = int(vc.get("intermediate_size", 4224))
        self.patch = int(vc.get("patch_size", 14))
        self.merge = int(vc.get("spatial_merge_size", 2))
        self.temporal = int(vc.get("temporal_patch_size", 1))
        self.cin = int(vc.get("num_channels", 3))
        self.eps = float(vc.get("rms_norm_eps", 1e-5))
        self.post_norm = bool(vc.get("post_norm", True))
        self.out_hidden = out_hidden
        self.w: dict[str, torch.Tensor] = {}
        rd = self.hd // 2
        self.inv = 1.0 / (10000.0 ** (torch.arange(0, rd, 2, dtype=torch.float32) / rd))

    def init_random(self, gen: torch.Generator, std: float = 0.02) -> None:
        E, I, mh = self.E, self.inter, self.E * self.merge ** 2
        shapes = {"patch.weight": (E, self.cin * self.temporal * self.patch ** 2), "patch.bias": (E,),
                  "patch_norm": (E,), "post_norm": (E,), "merger.ln_q.weight": (E,), "merger.ln_q.bias": (E,),
                  "merger.mlp.0.weight": (mh, mh), "merger.mlp.0.bias": (mh,),
                  "merger.mlp.2.weight": (self.out_hidden, mh), "merger.mlp.2.bias": (self.out_hidden,)}
        for b in range(self.depth):
            p = f"blocks.{b}."
            shapes.update({p + "norm1": (E,), p + "norm2": (E,), p + "qkv": (3 * E, E), p + "proj": (E, E),
                           p + "gu": (2 * I, E), p + "down": (E, I)})
        for k, s in shapes.items():
            t = torch.empty(*s, dtype=self.dtype, device=self.device)
            if k.endswith(("norm1", "norm2", "patch_norm", "post_norm", "ln_q.weight")):
                t.fill_(1.0)
            elif len(s) == 1:
                t.zero_()
            else:
                t.normal_(0.0, std, generator=gen)
            self.w[k] = t

    def load(self, name: str, t: torch.Tensor, pend: dict | None = None) -> None:
        """``name`` relative to ``vision_tower.``."""
        put = lambda k, v: self.w.__setitem__(k, v.to(device=self.device, dtype=self.dtype).contiguous())  # noqa
        if name == "patch_embed.patchifier.proj.weight":
            put("patch.weight", t.reshape(t.shape[0], -1))
        elif name == "patch_embed.patchifier.proj.bias":
            put("patch.bias", t)
        elif name == "patch_embed.patchifier.norm.weight":
            put("patch_norm", t)
        elif name == "post_trunk_norm.weight":
            put("post_norm", t)
        elif name.startswith("merger."):
            put(name, t)
        elif name.startswith("blocks."):
            parts = name.split(".")
            b, mod = int(parts[1]), ".".join(parts[2:])
            p = f"blocks.{b}."
            key = {"norm1.weight": "norm1", "norm2.weight": "norm2", "attn.qkv.weight": "qkv",
                   "attn.qkv.bias": "qkv_b", "attn.proj.weight": "proj", "attn.proj.bias": "proj_b",
                   "mlp.fc2.weight": "down", "mlp.fc2.bias": "down_b"}.get(mod)
            if key is not None:
                put(p + key, t)
            elif mod in ("mlp.fc1.weight", "mlp.fc3.weight"):
                got = (pend if pend is not None else {}).setdefault(("gu", b), {})
                got[mod[4:7]] = t
                if len(got) == 2:
                    put(p + "gu", torch.cat([got["fc1"], got["fc3"]], 0))
                    pend.pop(("gu", b), None)
            else:
                raise KeyError(f"unexpected dots vision weight {name}")

    def forward(self, pixel_values: torch.Tensor, grids: list[tuple[int, int, int]]) -> torch.Tensor:
        dev, dt, E, Hh, D, w = self.device, self.dtype, self.E, self.heads, self.hd, self.w
        x = linear(pixel_values.to(device=dev, dtype=dt), w["patch.weight"], w.get("patch.bias"))
        x = ops.rmsnorm(x, w["patch_norm"], self.eps)
        ang = self.rot_pos(grids).to(dev)
        emb = torch.cat([ang, ang], -1)
        cos, sin = emb.cos()[:, None, :], emb.sin()[:, None, :]
        lens = [h * ww for t, h, ww in grids for _ in range(t)]
        N = x.shape[0]

        def rope(t):
            tf = t.float()
            half = D // 2
            return (tf * cos + torch.cat([-tf[..., half:], tf[..., :half]], -1) * sin).to(dt)

        for b in range(self.depth):
            p = f"blocks.{b}."
            h = ops.rmsnorm(x, w[p + "norm1"], self.eps)
            qkv = linear(h, w[p + "qkv"], w.get(p + "qkv_b")).view(N, 3, Hh, D)
            a = ops.varlen_attention(rope(qkv[:, 0]), rope(qkv[:, 1]), qkv[:, 2], lens, D ** -0.5).reshape(N, E)
            x = x + linear(a, w[p + "proj"], w.get(p + "proj_b"))
            h = ops.rmsnorm(x, w[p + "norm2"], self.eps)
            x = x + linear(ops.act_and_mul(linear(h, w[p + "gu"]), 0), w[p + "down"], w.get(p + "down_b"))
        if self.post_norm:
            x = ops.rmsnorm(x, w["post_norm"], self.eps)
        h = ops.layernorm(x, w["merger.ln_q.weight"], w["merger.ln_q.bias"], 1e-6).reshape(-1, E * self.merge ** 2)
        h = ops.act(linear(h, w["merger.mlp.0.weight"], w["merger.mlp.0.bias"]), 3)
        return linear(h, w["merger.mlp.2.weight"], w["merger.mlp.2.bias"])


class _DotsMixin:
    is_multimodal = True

    def _setup_vision(self, full: ModelConfig) -> None:
        ex = full.extra or {}
        self.visual = DotsVisionTower(ex.get("vision_config") or {}, self.cfg.hidden_size, self.device, self.dtype)
        self.merge = self.visual.merge
        self.image_token_id = int(ex.get("image_token_id", 151665))
        self.min_pixels = int(ex.get("min_pixels", 3136))
        self.max_pixels = int(ex.get("max_pixels", 11289600))

    def init_random(self, seed: int = 0, std: float = 0.02):
        self._lm_base.init_random(self, seed, std)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 9091)
        self.visual.init_random(gen, std)
        return self

    def load_hf_weights(self, weights):
        pend: dict = {}

        def lm_only():
            for name, w in weights:
                if name.startswith("vision_tower."):
                    self.visual.load(name[len("vision_tower."):], w, pend)
                elif name.startswith("language_model."):
                    rest = name[len("language_model."):]
                    yield (rest if rest.startswith(("model.", "lm_head.")) else "model." + rest), w
                else:
                    yield name, w

        self._lm_base.load_hf_weights(self, lm_only())
        if pend:
            raise ValueError(f"incomplete dots vision MLPs: {sorted(pend)}")
        return self

    def weight_bytes(self) -> int:
        return self._lm_base.weight_bytes(self) + sum(t.numel() * t.element_size() for t in self.visual.w.values())

    def image_prompt_ids(self) -> list[int]:
        return [self.image_token_id]

    def make_mm_input(self, prompt_ids: list[int], images: list):
        where = [i for i, t in enumerate(prompt_ids) if t == self.image_token_id]
        if len(where) != len(images):
            raise ValueError(f"prompt has {len(where)} image tokens for {len(images)} images")
        ids, pvs, grids, spans, last = [], [], [], [], 0
        for i, im in zip(where, images):
            pv, g = im if isinstance(im, tuple) else preprocess_image(
                im, patch=self.visual.patch, merge=self.merge, temporal=self.visual.temporal,
                min_pixels=self.min_pixels, max_pixels=self.max_pixels)
            pv = torch.as_tensor(pv, dtype=torch.float32)
            g = tuple(int(v) for v in g)
            n = g[0] * g[1] * g[2] // self.merge ** 2
            ids += prompt_ids[last:i]
            spans.append((len(ids), n))
            ids += [pad_token_id(pv, self.cfg.vocab_size)] * n
            pvs.append(pv)
            grids.append(g)
            last = i + 1
        ids += prompt_ids[last:]
        return ids, MMInput(torch.cat(pvs, 0), grids, spans)

    def encode_images(self, pixel_values: torch.Tensor, grids) -> torch.Tensor:
        return self.visual.forward(pixel_values, grids)

    def embed_with_images(self, ids: torch.Tensor, rows: torch.Tensor, feats: torch.Tensor) -> torch.Tensor:
        h = pstate.tp_all_reduce(ops.embedding(ids, self.embed, self.tp.vocab_start, self.tp.vocab_end))
        if rows.numel():
            h.index_copy_(0, rows, feats.to(h.dtype))
        return h


def _text_config(cfg: ModelConfig) -> ModelConfig:
    ex = cfg.extra or {}
    nested = ex.get("text_config") or ex.get("language_config") or ex.get("llm_config")
    if nested:   # dots.vlm1: the DeepSeek-V3 language model's own config
        arch = (nested.get("architectures") or ["DeepseekV3ForCausalLM"])[0]
        return dataclasses.replace(cfg, architecture=arch, model_type=nested.get("model_type", "deepseek_v3"))
    # dots.ocr: a flat Qwen2 config (biased q / k / v)
    return dataclasses.replace(cfg, architecture="Qwen2ForCausalLM", model_type="qwen2", attention_bias=True)


_CLASSES: dict = {}


def dots_class(cfg: ModelConfig):
    from ome_amd.models import model_class

    base = model_class(_text_config(cfg))
    cls = _CLASSES.get(base)
    if cls is None:
        def __init__(self, cfg_full: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions=None):
            base.__init__(self, _text_config(cfg_full), device, dtype, max_positions)
            self.full_cfg = cfg_full
            self._setup_vision(cfg_full)

        cls = type(f"Dots_{base.__name__}", (_DotsMixin, base), {"__init__": __init__, "_lm_base": base})
        _CLASSES[base] = cls
    return cls
