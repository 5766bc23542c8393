"""LLaVA-NeXT / LLaVA-1.6 with a Llama-family LM: the transformers
``LlavaNextForConditionalGeneration`` and the original ``LlavaLlamaForCausalLM`` layout when its
config asks for ``image_aspect_ratio: anyres`` (reference catalog ``config/models/**/llava-v1-6-*``,
``llava-next-8b``; served there by the ``LlavaLlamaForCausalLM`` runtime).

The pipeline is LLaVA-OneVision's (``llava_onevision.py``: best-resolution pinpoint, aspect-kept
resize + zero padding, whole image squashed to one tile first, grid features re-assembled,
padding cut away, an ``image_newline`` column per row) with the LLaVA-1.5 parts swapped in: the
CLIP ViT-L/14-336 tower of ``llava.py`` (feature layer -2, class token dropped), CLIP mean / std,
336-px tiles, no ``anyres_max`` down-sampling, and every image of a prompt gets the anyres
treatment.  The language model is ``llama.py``.
"""
from __future__ import annotations

import torch

from ome_amd import ops
from ome_amd.models.config import ModelConfig
from ome_amd.models.llama import LlamaForCausalLM
from ome_amd.models.llava import CLIP_L336, ORIG_IMAGE_TOKEN, CLIPVisionTower
from ome_amd.models.llava_onevision import LlavaOnevisionForConditionalGeneration, preprocess_onevision
from ome_amd.models.quant import linear
from ome_amd.multimodal.inputs import CLIP_MEAN, CLIP_STD, MMInput, pad_token_id


def is_anyres_llava(cfg: ModelConfig) -> bool:
    """An original-layout LLaVA checkpoint of the 1.6 / NeXT generation."""
    return "anyres" in str((cfg.extra or {}).get("image_aspect_ratio", ""))


class LlavaNextForConditionalGeneration(LlavaOnevisionForConditionalGeneration):
    is_multimodal = True

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        LlamaForCausalLM.__init__(self, cfg, device, dtype, max_positions)   # (not OneVision's SigLIP set-up)
        ex = cfg.extra or {}
        self.orig = cfg.architecture == "LlavaLlamaForCausalLM"
        if self.orig:
            vc = {**CLIP_L336, **(ex.get("vision_config") or {})}
            layer = int(ex.get("mm_vision_select_layer", -2))
            strategy = "full" if ex.get("mm_vision_select_feature", "patch") == "cls_patch" else "default"
            self.image_id = int(ex.get("image_token_index", ORIG_IMAGE_TOKEN))
            if ex.get("mm_projector_type", "mlp2x_gelu") != "mlp2x_gelu":
                raise NotImplementedError(f"mm_projector_type {ex.get('mm_projector_type')!r}")
            if "unpad" not in ex.get("mm_patch_merge_type", "spatial_unpad"):
                raise NotImplementedError(f"mm_patch_merge_type {ex.get('mm_patch_merge_type')!r}")
        else:
            vc = ex.get("vision_config") or dict(CLIP_L336)
            layer = ex.get("vision_feature_layer", -2)
            if not isinstance(layer, int):
                raise NotImplementedError("multi-layer vision features")
            strategy = ex.get("vision_feature_select_strategy", "default")
            self.image_id = int(ex.get("image_token_index", ex.get("image_token_id", 32000)))
            if ex.get("projector_hidden_act", "gelu") != "gelu":
                raise NotImplementedError(f"projector act {ex.get('projector_hidden_act')!r}")
        if strategy != "default":
            raise NotImplementedError("class-token features with anyres packing")
        self.pinpoints = [tuple(p) for p in ex.get("image_grid_pinpoints") or [[336, 672], [672, 336], [672, 672],
                                                                                [1008, 336], [336, 1008]]]
        self.max_tiles = 10 ** 9   # (LLaVA-NeXT packs the whole unpadded grid)
        self.visual = CLIPVisionTower(vc, self.device, dtype, int(layer), strategy)
        self.side = self.visual.side
        self.proj: dict[str, torch.Tensor | None] = {}
        self.newline: torch.Tensor | None = None

    def init_random(self, seed: int = 0, std: float = 0.02) -> "LlavaNextForConditionalGeneration":
        LlamaForCausalLM.init_random(self, seed, std)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 4519)
        self.visual.init_random(gen, std)
        H, E = self.cfg.hidden_size, self.visual.E
        mk = lambda *s: torch.empty(*s, dtype=self.dtype, device=self.device).normal_(0.0, std, generator=gen)  # noqa
        z = torch.zeros(H, dtype=self.dtype, device=self.device)
        self.proj = {"w1": mk(H, E), "b1": z, "w2": mk(H, H), "b2": z.clone()}
        self.newline = mk(H)
        return self

    def _n_tokens(self, n_tiles: int, h: int, w: int) -> int:
        from ome_amd.models.llava_onevision import anyres_layout

        _, _, H2, W2 = anyres_layout(h, w, self.pinpoints, self.visual.image, self.side, self.max_tiles)
        return self.side ** 2 + H2 * (W2 + 1)

    def make_mm_input(self, prompt_ids: list[int], images: list):
        where = [i for i, t in enumerate(prompt_ids) if t == self.image_id]
        if len(where) != len(images):
            raise ValueError(f"prompt has {len(where)} image tokens for {len(images)} images")
        ids, pvs, grids, spans, last = [], [], [], [], 0
        for i, im in zip(where, images):
            px, h, w = im if isinstance(im, tuple) else preprocess_onevision(
                im, self.pinpoints, self.visual.image, True, mean=CLIP_MEAN, std=CLIP_STD)
            n = self._n_tokens(px.shape[0], h, w)
            ids += prompt_ids[last:i]
            spans.append((len(ids), n))
            ids += [pad_token_id(px, self.cfg.vocab_size)] * n
            pvs.append(px)
            grids.append((px.shape[0], h, w))
            last = i + 1
        ids += prompt_ids[last:]
        return ids, MMInput(torch.cat(pvs, 0), grids, spans)

    def _tile_features(self, pixel_values: torch.Tensor) -> torch.Tensor:
        p, s = self.proj, self.side
        f = self.visual.forward(pixel_values)   # [n * side^2, E]: layer -2, class token dropped
        return linear(ops.act(linear(f, p["w1"], p["b1"]), 3), p["w2"], p["b2"]).view(pixel_values.shape[0], s * s, -1)
