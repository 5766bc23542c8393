"""LLaVA-OneVision / LLaVA-NeXT with a Qwen2 LM: the original ``LlavaQwenForCausalLM`` layout
(reference catalog ``config/runtimes/srt/lmms-lab/llava-onevision-qwen2-7b-ov-rt.yaml``,
``llava-next-72b-rt.yaml``) and the transformers ``LlavaOnevisionForConditionalGeneration``.

* preprocessing ("anyres"): the grid pinpoint that keeps the most image resolution (least waste
  on ties) -> aspect-preserving bicubic resize into it, zero padding, 384-px tiles; the whole
  image resized to 384 x 384 goes first.  Several images in one prompt: each is padded to a square
  (mean colour) and sent as a single tile;
* SigLIP-SO400M tower (the shared SigLIP tower, varlen MFMA attention) -> hidden state of the
  feature layer (no post-LayerNorm) -> GEMM -> GELU -> GEMM;
* "spatial_unpad" packing: grid features re-assembled into one feature map, the padding rows /
  columns cut away, bilinear down-sampling when larger than ``anyres_max_N`` tiles (x1.1 slack),
  an ``image_newline`` column appended, then flattened after the base tile's 729 features.  The
  token count is a pure function of (image size, pinpoints), so the prompt is expanded on the
  host before the tower runs.
The language model is ``llama.py`` (Qwen2 config).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.models.config import ModelConfig
from ome_amd.models.gemma3_vision import SiglipVisionTower
from ome_amd.models.llama import LlamaForCausalLM
from ome_amd.models.quant import linear
from ome_amd.multimodal.inputs import MMInput, load_image, pad_token_id
from ome_amd.parallel import state as pstate

ORIG_IMAGE_TOKEN = -200
SIGLIP_SO400M_384 = dict(hidden_size=1152, intermediate_size=4304, num_hidden_layers=27, num_attention_heads=16,
                         image_size=384, patch_size=14, hidden_act="gelu_pytorch_tanh", layer_norm_eps=1e-6)


def best_resolution(h: int, w: int, pinpoints) -> tuple[int, int]:
    """(height, width) pinpoint keeping the most effective resolution, least waste on ties."""
    best, best_eff, best_waste = None, 0, float("inf")
    for ph, pw in pinpoints:
        s = min(pw / w, ph / h)
        eff = min(int(w * s) * int(h * s), w * h)
        waste = ph * pw - eff
        if eff > best_eff or (eff == best_eff and waste < best_waste):
            best, best_eff, best_waste = (ph, pw), eff, waste
    return best


def anyres_layout(h: int, w: int, pinpoints, tile: int, side: int, max_tiles: int):
    """-> (grid rows, grid cols, feature-map height, width after unpad / down-sampling)."""
    bh, bw = best_resolution(h, w, pinpoints)
    nph, npw = bh // tile, bw // tile
    H, W = nph * side, npw * side
    if w / h > W / H:
        pad = (H - int(round(h * (W / w), 7))) // 2
        H2, W2 = H - 2 * pad, W
    else:
        pad = (W - int(round(w * (H / h), 7))) // 2
        H2, W2 = H, W - 2 * pad
    ratio = math.sqrt(H2 * W2 / (max_tiles * side * side))
    if ratio > 1.1:
        H2, W2 = int(H2 // ratio), int(W2 // ratio)
    return nph, npw, H2, W2


def _norm(a: np.ndarray, mean, std) -> np.ndarray:
    return ((a / 255.0 - np.asarray(mean, np.float32)) / np.asarray(std, np.float32)).transpose(2, 0, 1)


def preprocess_onevision(image, pinpoints, tile: int = 384, anyres: bool = True, mean=(0.5, 0.5, 0.5),
                         std=(0.5, 0.5, 0.5)) -> tuple[torch.Tensor, int, int]:
    """-> (float32 [n_tiles, 3, tile, tile], original height, width)."""
    from PIL import Image

    img = load_image(image)
    w, h = img.size
    if not anyres:
        s = max(w, h)
        bg = Image.new("RGB", (s, s), tuple(int(x * 255) for x in mean))
        bg.paste(img, ((s - w) // 2, (s - h) // 2))
        a = np.asarray(bg.resize((tile, tile), Image.BICUBIC), dtype=np.float32)
        return torch.from_numpy(np.ascontiguousarray(_norm(a, mean, std)))[None], h, w
    bh, bw = best_resolution(h, w, pinpoints)
    sw, sh = bw / w, bh / h
    if sw < sh:
        nw, nh = bw, min(math.ceil(h * sw), bh)
    else:
        nh, nw = bh, min(math.ceil(w * sh), bw)
    canvas = np.zeros((bh, bw, 3), dtype=np.float32)
    top, left = (bh - nh) // 2, (bw - nw) // 2
    canvas[top:top + nh, left:left + nw] = np.asarray(img.resize((nw, nh), Image.BICUBIC), dtype=np.float32)
    tiles = [np.asarray(img.resize((tile, tile), Image.BICUBIC), dtype=np.float32)]
    tiles += [canvas[r:r + tile, c:c + tile] for r in range(0, bh, tile) for c in range(0, bw, tile)]
    return torch.from_numpy(np.ascontiguousarray(np.stack([_norm(t, mean, std) for t in tiles]))), h, w


class LlavaOnevisionForConditionalGeneration(LlamaForCausalLM):
    is_multimodal = True

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        ex = cfg.extra or {}
        self.orig = cfg.architecture == "LlavaQwenForCausalLM"
        if self.orig:
            vc = {**SIGLIP_SO400M_384, **(ex.get("vision_config") or {})}
            layer = int(ex.get("mm_vision_select_layer", -2))
            self.image_id = int(ex.get("image_token_index", ORIG_IMAGE_TOKEN))
            aspect = ex.get("image_aspect_ratio", "anyres_max_9")
            if ex.get("mm_projector_type", "mlp2x_gelu") != "mlp2x_gelu":
                raise NotImplementedError(f"mm_projector_type {ex.get('mm_projector_type')!r}")
            if "unpad" not in ex.get("mm_patch_merge_type", "spatial_unpad"):
                raise NotImplementedError(f"mm_patch_merge_type {ex.get('mm_patch_merge_type')!r}")
        else:
            vc = dict(ex.get("vision_config") or SIGLIP_SO400M_384)
            layer = ex.get("vision_feature_layer", -1)
            if not isinstance(layer, int):
                raise NotImplementedError("multi-layer vision features")
            if ex.get("vision_feature_select_strategy", "full") != "full":
                raise NotImplementedError("class-token towers")
            self.image_id = int(ex.get("image_token_index", ex.get("image_token_id", 151646)))
            aspect = ex.get("vision_aspect_ratio", "anyres_max_9")
        self.max_tiles = int(aspect.split("anyres_max_")[1]) if "anyres_max_" in aspect else 10 ** 9
        self.pinpoints = [tuple(p) for p in ex.get("image_grid_pinpoints") or [[384, 384]]]
        self.visual = SiglipVisionTower(vc, self.device, dtype)
        depth = self.visual.depth
        self.n_layers = layer if layer >= 0 else depth + 1 + layer   # hidden_states[k]: after k layers
        self.side = self.visual.side
        self.proj: dict[str, torch.Tensor | None] = {}
        self.newline: torch.Tensor | None = None

    def init_random(self, seed: int = 0, std: float = 0.02) -> "LlavaOnevisionForConditionalGeneration":
        super().init_random(seed, std)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 4507)
        self.visual.init_random(gen, std)
        H, E = self.cfg.hidden_size, self.visual.E
        mk = lambda *s: torch.empty(*s, dtype=self.dtype, device=self.device).normal_(0.0, std, generator=gen)  # noqa
        z = torch.zeros(H, dtype=self.dtype, device=self.device)
        self.proj = {"w1": mk(H, E), "b1": z, "w2": mk(H, H), "b2": z}
        self.newline = mk(H)
        return self

    _PROJ = {"multi_modal_projector.linear_1.weight": "w1", "multi_modal_projector.linear_1.bias": "b1",
             "multi_modal_projector.linear_2.weight": "w2", "multi_modal_projector.linear_2.bias": "b2",
             "mm_projector.0.weight": "w1", "mm_projector.0.bias": "b1", "mm_projector.2.weight": "w2",
             "mm_projector.2.bias": "b2"}

    def load_hf_weights(self, weights) -> "LlavaOnevisionForConditionalGeneration":
        pend: dict = {}
        self.proj = {"b1": None, "b2": None}

        def lm_only():
            for name, w in weights:
                n = name[len("model."):] if name.startswith("model.") else name
                for pre in ("vision_tower.vision_tower.vision_model.", "vision_tower.vision_model.", "vision_tower."):
                    if n.startswith(pre):
                        self.visual.load(n[len(pre):], w, pend)
                        break
                else:
                    if n in self._PROJ:
                        self.proj[self._PROJ[n]] = w.to(device=self.device, dtype=self.dtype).contiguous()
                    elif n == "image_newline":
                        self.newline = w.to(device=self.device, dtype=self.dtype).contiguous()
                    elif n.startswith("language_model."):
                        rest = n[len("language_model."):]
                        yield (rest if rest.startswith(("model.", "lm_head.")) else "model." + rest), w
                    elif n.startswith(("vision_resampler.",)):
                        continue
                    else:
                        yield name, w

        super().load_hf_weights(lm_only())
        if pend:
            raise ValueError(f"incomplete vision projections: {sorted(pend)}")
        return self

    def weight_bytes(self) -> int:
        n = super().weight_bytes() + sum(t.numel() * t.element_size() for t in self.visual.w.values())
        return n + sum(t.numel() * t.element_size() for t in self.proj.values() if t is not None)

    # ------------------------------------------------------------------ multimodal
    def image_prompt_ids(self) -> list[int]:
        return [self.image_id]

    def _n_tokens(self, n_tiles: int, h: int, w: int) -> int:
        if n_tiles == 1:
            return self.side ** 2 + 1
        _, _, H2, W2 = anyres_layout(h, w, self.pinpoints, self.visual.image, self.side, self.max_tiles)
        return self.side ** 2 + H2 * (W2 + 1)

    def make_mm_input(self, prompt_ids: list[int], images: list):
        where = [i for i, t in enumerate(prompt_ids) if t == self.image_id]
        if len(where) != len(images):
            raise ValueError(f"prompt has {len(where)} image tokens for {len(images)} images")
        anyres = len(images) == 1   # several images in one prompt: one padded tile each
        ids, pvs, grids, spans, last = [], [], [], [], 0
        for i, im in zip(where, images):
            px, h, w = im if isinstance(im, tuple) else preprocess_onevision(im, self.pinpoints, self.visual.image,
                                                                             anyres)
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
        """[n_tiles, side * side, hidden]: tower -> GEMM -> GELU -> GEMM per tile."""
        p, s = self.proj, self.side
        f = self.visual.forward(pixel_values, self.n_layers, post_norm=False).reshape(-1, self.visual.E)
        return linear(ops.act(linear(f, p["w1"], p["b1"]), 3), p["w2"], p["b2"]).view(pixel_values.shape[0], s * s, -1)

    def encode_images(self, pixel_values: torch.Tensor, grids) -> torch.Tensor:
        s = self.side
        f = self._tile_features(pixel_values)
        out, off = [], 0
        nl = self.newline
        for n, h, w in grids:
            feats = f[off:off + n]
            off += n
            if n == 1:
                out += [feats[0], nl[None]]
                continue
            nph, npw, H2, W2 = anyres_layout(h, w, self.pinpoints, self.visual.image, s, self.max_tiles)
            g = feats[1:].view(nph, npw, s, s, -1).permute(4, 0, 2, 1, 3).reshape(-1, nph * s, npw * s)
            H, W = nph * s, npw * s
            if w / h > W / H:
                pad = (H - int(round(h * (W / w), 7))) // 2
                g = g[:, pad:H - pad]
            else:
                pad = (W - int(round(w * (H / h), 7))) // 2
                g = g[:, :, pad:W - pad]
            if (g.shape[1], g.shape[2]) != (H2, W2):
                g = F.interpolate(g[None].float(), [H2, W2], mode="bilinear")[0].to(g.dtype)
            g = torch.cat([g, nl[:, None, None].expand(-1, H2, 1)], -1)
            out += [feats[0], g.flatten(1, 2).t()]
        return torch.cat(out, 0).contiguous()

    def embed_with_images(self, ids: torch.Tensor, rows: torch.Tensor, feats: torch.Tensor) -> torch.Tensor:
        h = pstate.tp_all_reduce(ops.embedding(ids, self.embed, self.tp.vocab_start, self.tp.vocab_end))
        if rows.numel():
            h.index_copy_(0, rows, feats.to(h.dtype))
        return h
