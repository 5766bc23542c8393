"""Llama-3.2-Vision (Mllama) image inputs: tiled preprocessing and the text -> image visibility
segments of cross attention.

Preprocessing follows the Mllama image-processor contract (the reference catalog serves
``MllamaForConditionalGeneration`` through SGLang, e.g.
``config/runtimes/srt/meta/llama-3-2-11b-vision-instruct-rt.yaml``): pick the tile canvas (<= 4
tiles of ``tile`` px) that needs the least up-scaling (else the least down-scaling, ties -> the
smallest area), resize preserving the aspect ratio (bilinear), zero-pad to the canvas, rescale
to [0, 1], normalise with the CLIP mean / std, cut into tiles (row-major) and pad the tile axis to
``max_tiles``.  ``aspect_ratio_id`` is 1 + the index of (tiles_h, tiles_w) among the supported
arrangements.

Cross-attention visibility (the processor's ``get_cross_attention_token_mask`` + the model's
``_prepare_cross_attention_mask``): text tokens from an ``<|image|>`` token up to the next image
token see that image's real tiles (consecutive image tokens form one group that sees all of its
images; the last group extends to the end of the sequence, generated tokens included); tokens
before the first image have no visible image, for which the model attends to *every* vision
token (padding tiles too) and zeroes the cross layer's MLP contribution.  The vision-token cache
of a request stores the real tiles of all its images first, in image order, then all padding
tiles, so every one of these sets is one contiguous key range ``[lo, hi)``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import torch

from ome_amd.multimodal.inputs import load_image

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


def supported_arrangements(max_tiles: int) -> list[tuple[int, int]]:
    return [(a, b) for a in range(1, max_tiles + 1) for b in range(1, max_tiles + 1) if a * b <= max_tiles]


def optimal_canvas(h: int, w: int, max_tiles: int, tile: int) -> tuple[int, int]:
    best, best_key = None, None
    cands = [(a * tile, b * tile) for a, b in supported_arrangements(max_tiles)]
    scales = [min(ch / h, cw / w) for ch, cw in cands]
    up = [s for s in scales if s >= 1]
    target = min(up) if up else max(scales)
    for (ch, cw), s in zip(cands, scales):
        if s == target:
            key = ch * cw
            if best is None or key < best_key:
                best, best_key = (ch, cw), key
    return best


def fit_to_canvas(h: int, w: int, ch: int, cw: int, tile: int) -> tuple[int, int]:
    tw = min(max(w, tile), cw)
    th = min(max(h, tile), ch)
    sh, sw = th / h, tw / w
    if sw < sh:
        return min(math.floor(h * sw) or 1, th), tw
    return th, min(math.floor(w * sh) or 1, tw)


def preprocess_image(image, tile: int = 560, max_tiles: int = 4, mean=CLIP_MEAN, std=CLIP_STD):
    """-> (pixel_values float32 [max_tiles, 3, tile, tile], aspect_ratio_id, num_tiles).  ``mean`` /
    ``std``: the checkpoint's ``preprocessor_config.json`` values (Llama-3.2-Vision: CLIP's)."""
    from PIL import Image

    img = load_image(image)
    if img.mode != "RGB":
        img = img.convert("RGB")
    W, H = img.size
    ch, cw = optimal_canvas(H, W, max_tiles, tile)
    nh, nw = fit_to_canvas(H, W, ch, cw, tile)
    img = img.resize((nw, nh), Image.BILINEAR)
    a = np.asarray(img, dtype=np.float32).transpose(2, 0, 1)  # [3, nh, nw]
    canvas = np.zeros((3, ch, cw), dtype=np.float32)
    canvas[:, :nh, :nw] = a
    canvas = canvas / 255.0
    canvas = (canvas - np.asarray(mean, np.float32)[:, None, None]) / np.asarray(std, np.float32)[:, None, None]
    th, tw = ch // tile, cw // tile
    tiles = canvas.reshape(3, th, tile, tw, tile).transpose(1, 3, 0, 2, 4).reshape(th * tw, 3, tile, tile)
    out = np.zeros((max_tiles, 3, tile, tile), dtype=np.float32)
    out[: th * tw] = tiles
    ar_id = supported_arrangements(max_tiles).index((th, tw)) + 1
    return torch.from_numpy(out), ar_id, th * tw


@dataclass
class CrossMMInput:
    """A request's images for a cross-attention (Mllama) model."""

    pixel_values: torch.Tensor          # [n_img, max_tiles, 3, tile, tile]
    ar_ids: list[int]                   # aspect ratio id per image
    num_tiles: list[int]                # real tiles per image
    image_pos: list[int]                # prompt index of each <|image|> token
    cross_only: bool = True             # marker: attention-side multimodal input (no embedding rows)
    rope_delta: int = 0                 # plain 1D RoPE (no M-RoPE offset for generated tokens)
    release: object = None              # frees the model-side vision-token cache (set by the model)

    def cache_key(self) -> tuple[bytes, int]:
        """Cross-attention feeds the image into every text row: salt the whole prompt."""
        from ome_amd.multimodal.inputs import mm_cache_key

        return mm_cache_key(self, 0)

    def segments(self, tokens_per_tile: int, max_tiles: int) -> list[tuple[int, int, int, int]]:
        """``(text_start, lo, hi, mlp_on)`` per visibility segment, in text order: rows at
        positions >= text_start (up to the next segment) attend keys [lo, hi) of the request's
        vision-token cache (real tiles of all images first, then padding tiles)."""
        n = len(self.image_pos)
        total = n * max_tiles * tokens_per_tile
        vstart = np.concatenate([[0], np.cumsum([t * tokens_per_tile for t in self.num_tiles])]).tolist()
        segs = [(0, 0, total, 0)]
        g0 = 0
        for k in range(n):  # image k's mask runs from its token to its group's end: a row at
            # position p sees the images of its group whose token is at or before p
            if k > 0 and self.image_pos[k] != self.image_pos[k - 1] + 1:
                g0 = k
            segs.append((self.image_pos[k], vstart[g0], vstart[k + 1], 1))
        return segs
