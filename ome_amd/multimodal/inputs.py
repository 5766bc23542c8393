"""Image preprocessing (Qwen2-VL patchification), placeholder expansion and M-RoPE positions.

Preprocessing follows the Qwen2-VL image processor contract (``smart_resize`` to multiples of
``patch * merge`` inside [min_pixels, max_pixels], rescale 1/255, CLIP mean/std normalisation,
the frame repeated to ``temporal_patch_size``, patches flattened as (C, T, ps, ps) in
merge-block-major order) so ``pixel_values`` match what the HF processor feeds the vision tower.
"""
from __future__ import annotations

import base64
import hashlib
import io
import math
from dataclasses import dataclass, field

import numpy as np
import torch

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


@dataclass(eq=False)
class MMInput:
    """Per-request multimodal state (lives on :class:`ome_amd.runtime.request.Request.mm`)."""

    pixel_values: torch.Tensor                 # [sum patches, C*T*ps*ps] float32 (host)
    grid_thw: list[tuple[int, int, int]]       # per image, in patches (before merging)
    spans: list[tuple[int, int]]               # per image: (first prompt index, number of tokens)
    mrope_pos: np.ndarray | None = None        # [3, prompt_len] int64 (None: plain 1D positions)
    rope_delta: int = 0                        # decode position offset (max mrope pos + 1 - len)
    features: torch.Tensor | None = field(default=None, repr=False)  # [sum tokens, H] on device
    atomic: bool = False                       # spans attend bidirectionally: never split a span across chunks

    @property
    def num_tokens(self) -> int:
        return sum(n for _, n in self.spans)

    def cache_key(self) -> tuple[bytes, int]:
        """(salt, first prompt index it applies from) for the prefix cache: see :func:`mm_cache_key`."""
        return mm_cache_key(self, min((s for s, _ in self.spans), default=0))


def mm_cache_key(mm, salt_from: int) -> tuple[bytes, int]:
    """128-bit BLAKE2b digest of EVERYTHING the request's KV depends on besides its token ids
    (pixel values, grids, spans, image positions), cached on ``mm``.  The prefix cache mixes it
    into the hash chain of every page from ``salt_from`` on, so two requests with identical text
    but different images can never share KV pages -- the placeholder ids alone are a hash reduced
    modulo the vocabulary (:func:`pad_token_id`) and collide at ~1/vocab per image pair."""
    got = getattr(mm, "_cache_key", None)
    if got is None:
        h = hashlib.blake2b(digest_size=16)
        for name, v in sorted(vars(mm).items()):
            if name.startswith("_") or name in ("features", "release") or callable(v):
                continue
            if isinstance(v, torch.Tensor):
                h.update(v.detach().cpu().contiguous().view(torch.uint8).numpy().tobytes())
            elif isinstance(v, np.ndarray):
                h.update(np.ascontiguousarray(v).tobytes())
            else:
                h.update(repr(v).encode())
            h.update(name.encode())
        got = (h.digest(), salt_from)
        mm._cache_key = got
    return got


def load_image(src):
    """PIL image from a ``data:`` URL, raw base64, a local path, bytes or a PIL image (no network:
    ``http(s)`` URLs are refused offline)."""
    from PIL import Image

    if hasattr(src, "convert"):
        return src.convert("RGB")
    if isinstance(src, (bytes, bytearray)):
        return Image.open(io.BytesIO(src)).convert("RGB")
    if not isinstance(src, str):
        raise ValueError("image must be a data URL, base64 string, path or bytes")
    if src.startswith("data:"):
        src = src.split(",", 1)[1]
        return Image.open(io.BytesIO(base64.b64decode(src))).convert("RGB")
    if src.startswith(("http://", "https://")):
        raise ValueError("remote image URLs are not fetched by this runtime; send a data: URL")
    if src.startswith("file://"):
        src = src[len("file://"):]
    try:
        return Image.open(src).convert("RGB")
    except (FileNotFoundError, OSError):
        return Image.open(io.BytesIO(base64.b64decode(src))).convert("RGB")


def smart_resize(h: int, w: int, factor: int = 28, min_pixels: int = 56 * 56,
                 max_pixels: int = 14 * 14 * 4 * 1280) -> tuple[int, int]:
    """Qwen2-VL resize rule: both sides multiples of ``factor``, area in [min, max], aspect kept."""
    if max(h, w) / min(h, w) > 200:
        raise ValueError("image aspect ratio must be < 200")
    hb, wb = round(h / factor) * factor, round(w / factor) * factor
    if hb * wb > max_pixels:
        beta = math.sqrt(h * w / max_pixels)
        hb, wb = math.floor(h / beta / factor) * factor, math.floor(w / beta / factor) * factor
    elif hb * wb < min_pixels:
        beta = math.sqrt(min_pixels / (h * w))
        hb, wb = math.ceil(h * beta / factor) * factor, math.ceil(w * beta / factor) * factor
    return max(hb, factor), max(wb, factor)


def patchify(img: np.ndarray, patch: int = 14, merge: int = 2, temporal: int = 2):
    """``img`` [C, H, W] float32 (normalised, H/W multiples of patch*merge) ->
    (pixel_values [gh*gw, C*temporal*patch*patch], (1, gh, gw))."""
    C, H, W = img.shape
    gh, gw = H // patch, W // patch
    x = np.broadcast_to(img[None], (temporal, C, H, W))
    x = x.reshape(1, temporal, C, gh // merge, merge, patch, gw // merge, merge, patch)
    # -> [t, gh/m, gw/m, m, m, C, T, ps, ps]
    x = x.transpose(0, 3, 6, 4, 7, 2, 1, 5, 8)
    return np.ascontiguousarray(x.reshape(gh * gw, C * temporal * patch * patch)), (1, gh, gw)


def preprocess_image(image, patch: int = 14, merge: int = 2, temporal: int = 2, min_pixels: int = 56 * 56,
                     max_pixels: int = 14 * 14 * 4 * 1280, mean=CLIP_MEAN, std=CLIP_STD):
    from PIL import Image

    img = load_image(image)
    h, w = smart_resize(img.height, img.width, patch * merge, min_pixels, max_pixels)
    img = img.resize((w, h), Image.BICUBIC)
    a = np.asarray(img, dtype=np.float32) / 255.0
    a = (a - np.asarray(mean, np.float32)) / np.asarray(std, np.float32)
    return patchify(a.transpose(2, 0, 1), patch, merge, temporal)


def pad_token_id(pixels: np.ndarray | torch.Tensor, vocab: int) -> int:
    """Content-derived stand-in id for an image's placeholder tokens: identical images share
    prefix-cache pages, different images never match (the rows are overwritten by the vision
    features, so the id itself is never embedded)."""
    b = pixels.numpy().tobytes() if isinstance(pixels, torch.Tensor) else np.asarray(pixels).tobytes()
    return int.from_bytes(hashlib.blake2b(b, digest_size=8).digest(), "little") % vocab


def expand_image_tokens(ids: list[int], image_token_id: int, grids: list[tuple[int, int, int]], merge: int,
                        pixels: list | None = None, vocab: int | None = None):
    """Each ``image_token_id`` in ``ids`` (one per image, in order) becomes t*h*w/merge^2 tokens.
    Returns (new ids, spans).  With ``pixels``/``vocab`` the expanded run uses a content hash id."""
    out, spans, k = [], [], 0
    for t in ids:
        if t != image_token_id:
            out.append(t)
            continue
        if k >= len(grids):
            raise ValueError("more image placeholders than images")
        gt, gh, gw = grids[k]
        n = gt * gh * gw // (merge * merge)
        tok = pad_token_id(pixels[k], vocab) if pixels is not None and vocab else image_token_id
        spans.append((len(out), n))
        out.extend([tok] * n)
        k += 1
    if k != len(grids):
        raise ValueError(f"{len(grids)} images but {k} placeholders in the prompt")
    return out, spans


def mrope_positions(L: int, spans: list[tuple[int, int]], grids: list[tuple[int, int, int]], merge: int):
    """Qwen2-VL 3D RoPE positions (``get_rope_index`` semantics): text runs advance all three
    components by 1 per token; an image's tokens take (t, h, w) grid coordinates offset by the
    running position, after which the position advances by max(h, w) / merge.
    Returns (pos [3, L] int64, delta = max + 1 - L)."""
    pos = np.zeros((3, L), dtype=np.int64)
    cur, i = 0, 0
    for (s, n), (gt, gh, gw) in zip(spans, grids):
        pos[:, i:s] = np.arange(s - i) + cur
        cur += s - i
        mh, mw = gh // merge, gw // merge
        tt, hh, ww = np.meshgrid(np.arange(gt), np.arange(mh), np.arange(mw), indexing="ij")
        pos[0, s:s + n] = tt.reshape(-1) + cur
        pos[1, s:s + n] = hh.reshape(-1) + cur
        pos[2, s:s + n] = ww.reshape(-1) + cur
        cur += max(mh, mw)
        i = s + n
    pos[:, i:L] = np.arange(L - i) + cur
    return pos, int(pos.max()) + 1 - L if L else 0
