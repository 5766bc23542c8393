"""MiniCPM-V 2.6 (``MiniCPMV``): SigLIP-400M (NaViT variable resolution) + perceiver resampler on a
Qwen2 decoder.

Reference catalog: ``config/runtimes/srt/openbmb/minicpm-v-2-6-rt.yaml`` (``MiniCPMV``, 8B).
Pieces, MI355X-side:

* slicing (``slice_image``): the source image resized to ~``scale_resolution``^2 pixels (sides
  multiples of 14, aspect kept) plus, when the image is larger, a ``cols x rows`` grid of slices
  (1 < cols*rows <= ``max_slice_nums``, the grid whose log aspect is closest to the image's, from
  ceil(area / 448^2) +- 1 slices), each resized the same way; mean / std 0.5;
* vision (:class:`NavitSiglipTower`): every slice keeps its own h x w patch grid; position ids
  are the fractional patch coordinates bucketised into the 70 x 70 table (NaViT), all slices of
  a request packed into one varlen MFMA attention batch (no padding);
* resampler: 64 learned queries (LayerNorm) cross-attend over each slice's kv projection
  (LayerNorm) + a 2-D sin-cos table of that slice's grid (keys only), 128-dim heads;
  LayerNorm, ``@ proj``;
* prompt: each image placeholder becomes ``<image_id>N</image_id><image>`` + 64 feature tokens +
  ``</image>`` and, for sliced images, per grid row ``(<slice>`` + 64 + ``</slice>) x cols`` with
  ``\\n`` between rows -- marker ids read from the checkpoint's ``tokenizer.json``.
The SigLIP layers run through ``gemma3_vision.SiglipVisionTower.encode``; the language model is
the Llama / Qwen2 path of ``llama.py`` (``llm.*`` weights).  transformers ships no MiniCPM-V 2.6
class: ``tests/test_minicpmv_cpu.py`` checks against transformers' SigLIP encoder, torch's
``nn.MultiheadAttention`` and Qwen2 with an independent restatement of the glue (parity of the
image processor itself unpinned).
"""
from __future__ import annotations

import dataclasses
import json
import math
from pathlib import Path

import numpy as np
import torch

from ome_amd import ops
from ome_amd.models.config import ModelConfig
from ome_amd.models.gemma3_vision import SiglipVisionTower
from ome_amd.models.llama import LlamaForCausalLM
from ome_amd.models.quant import linear
from ome_amd.multimodal.inputs import MMInput, load_image, pad_token_id
from ome_amd.parallel import state as pstate

MINICPMV_ARCHS = {"MiniCPMV"}


# ------------------------------------------------------------------ slicing
def _divide(length: float, patch: int) -> int:
    return max(round(length / patch) * patch, patch)


def best_resize(w: float, h: float, scale: int, patch: int, upscale: bool = False) -> tuple[int, int]:
    if w * h > scale * scale or upscale:
        r = w / h
        h = int(scale / math.sqrt(r))
        w = int(h * r)
    return _divide(w, patch), _divide(h, patch)


def sliced_grid(w: int, h: int, max_slices: int, scale: int) -> tuple[int, int] | None:
    """(cols, rows) of the slice grid, or None when the image is not sliced."""
    multiple = min(math.ceil(w * h / (scale * scale)), max_slices)
    if multiple <= 1:
        return None
    log_ratio = math.log(w / h)
    best, err = (1, 1), float("inf")
    for n in (multiple - 1, multiple, multiple + 1):
        if n == 1 or n > max_slices:
            continue
        for m in range(1, n + 1):
            if n % m == 0:
                e = abs(log_ratio - math.log(m / (n // m)))
                if e < err:
                    best, err = (m, n // m), e
    return best


def slice_image(img, max_slices: int = 9, scale: int = 448, patch: int = 14):
    """-> (source image, slices row-major, (cols, rows) or None)."""
    from PIL import Image

    w, h = img.size
    grid = sliced_grid(w, h, max_slices, scale)
    if grid is None:
        return img.resize(best_resize(w, h, scale, patch, True), Image.BICUBIC), [], None
    src = img.resize(best_resize(w, h, scale, patch), Image.BICUBIC)
    cols, rows = grid
    gw, gh = _divide(w, cols) / cols, _divide(h, rows) / rows
    bw, bh = best_resize(gw, gh, scale, patch, True)
    ref = img.resize((bw * cols, bh * rows), Image.BICUBIC)
    slices = [ref.crop((c * bw, r * bh, (c + 1) * bw, (r + 1) * bh)) for r in range(rows) for c in range(cols)]
    return src, slices, grid


def _patches(img, patch: int, mean, std) -> tuple[np.ndarray, tuple[int, int]]:
    a = (np.asarray(img.convert("RGB"), dtype=np.float32) / 255.0 - np.asarray(mean, np.float32)) / \
        np.asarray(std, np.float32)
    H, W = a.shape[0] // patch, a.shape[1] // patch
    a = a[:H * patch, :W * patch].reshape(H, patch, W, patch, 3).transpose(0, 2, 4, 1, 3)   # (h, w, C, ps, ps)
    return np.ascontiguousarray(a.reshape(H * W, 3 * patch * patch)), (H, W)


def preprocess_minicpmv(image, max_slices: int = 9, scale: int = 448, patch: int = 14, mean=(0.5, 0.5, 0.5),
                        std=(0.5, 0.5, 0.5)):
    """-> (patch rows float32 [sum h*w, 3*14*14], per slice (h, w) patch grids (source first),
    (cols, rows) slice layout or None)."""
    src, slices, grid = slice_image(load_image(image), max_slices, scale, patch)
    rows, grids = [], []
    for im in [src] + slices:
        p, g = _patches(im, patch, mean, std)
        rows.append(p)
        grids.append(g)
    return torch.from_numpy(np.concatenate(rows, 0)), grids, grid


def sincos_2d(dim: int, h: int, w: int) -> torch.Tensor:
    """[h, w, dim] table of the MiniCPM-V resampler: the first half encodes grid[0] of
    ``meshgrid(arange(w), arange(h))`` (the column), the second half the row; each half is
    [sin | cos] of pos / 10000^(2i/half)."""
    gw, gh = np.meshgrid(np.arange(w, dtype=np.float32), np.arange(h, dtype=np.float32))

    def one(d, pos):
        om = 1.0 / 10000 ** (np.arange(d // 2, dtype=np.float32) / (d / 2.0))
        out = pos[..., None] * om
        return np.concatenate([np.sin(out), np.cos(out)], -1)

    return torch.from_numpy(np.concatenate([one(dim // 2, gw), one(dim // 2, gh)], -1).astype(np.float32))


# ------------------------------------------------------------------ vision
class NavitSiglipTower(SiglipVisionTower):
    """SigLIP over variable-size patch grids (positions bucketised into the square table)."""

    def pos_ids(self, h: int, w: int) -> torch.Tensor:
        s = self.side
        bounds = torch.arange(1 / s, 1.0, 1 / s)
        fh = torch.clamp(torch.arange(h, dtype=torch.float32) / h, max=1 - 1e-6)
        fw = torch.clamp(torch.arange(w, dtype=torch.float32) / w, max=1 - 1e-6)
        bh = torch.bucketize(fh, bounds, right=True)
        bw = torch.bucketize(fw, bounds, right=True)
        return (bh[:, None] * s + bw[None, :]).reshape(-1)

    def forward_patches(self, rows: torch.Tensor, grids: list[tuple[int, int]], n_layers: int | None = None):
        w = self.w
        x = linear(rows.to(device=self.device, dtype=self.dtype), w["patch.weight"], w["patch.bias"])
        pid = torch.cat([self.pos_ids(h, ww) for h, ww in grids]).to(self.device)
        x = x + w["pos"].index_select(0, pid)
        return self.encode(x, [h * ww for h, ww in grids], n_layers)


class MiniCPMV(LlamaForCausalLM):
    is_multimodal = True

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        ex = cfg.extra or {}
        if str(ex.get("version", "2.6")) not in ("2.5",) and not cfg.attention_bias:
            cfg = dataclasses.replace(cfg, attention_bias=True)   # 2.6: Qwen2 decoder (biased q/k/v)
        super().__init__(cfg, device, dtype, max_positions)
        vc = dict(ex.get("vision_config") or {})
        vc.setdefault("image_size", 980)
        self.visual = NavitSiglipTower(vc, self.device, dtype)
        self.vis_layers = self.visual.depth - (1 if ex.get("drop_vision_last_layer") else 0)
        sc = ex.get("slice_config") or {}
        self.max_slices = int(sc.get("max_slice_nums", ex.get("max_slice_nums", 9)))
        self.slice_scale = int(sc.get("scale_resolution", ex.get("scale_resolution", 448)))
        self.patch = int(sc.get("patch_size", ex.get("patch_size", 14)))
        self.slice_mode = bool(ex.get("slice_mode", True))
        self.use_image_id = bool(ex.get("use_image_id", True))
        self.nq = int(ex.get("query_num", 64))
        self.rheads = max(1, cfg.hidden_size // 128)
        self.rs: dict[str, torch.Tensor] = {}
        self._pos_cache: dict[tuple[int, int], torch.Tensor] = {}
        self._tok = self._token_ids(ex)

    # ------------------------------------------------------------------ token ids
    @staticmethod
    def _token_ids(ex: dict) -> dict[str, int]:
        """Marker / digit / newline ids from tokenizer.json (added tokens + BPE vocab)."""
        got: dict[str, int] = {}
        mp = ex.get("_model_path")
        p = Path(mp) / "tokenizer.json" if mp else None
        if p is not None and p.is_file():
            try:
                tj = json.loads(p.read_text())
            except (OSError, ValueError):
                tj = {}
            for t in tj.get("added_tokens") or []:
                got[t.get("content")] = int(t["id"])
            vocab = (tj.get("model") or {}).get("vocab") or {}
            if isinstance(vocab, dict):
                for k in [str(d) for d in range(10)] + ["Ċ", "\n"]:
                    if k in vocab and k not in got:
                        got[k] = int(vocab[k])
        if "Ċ" in got and "\n" not in got:
            got["\n"] = got["Ċ"]
        for key, name in (("im_start_token_id", "<image>"), ("im_end_token_id", "</image>"),
                          ("slice_start_token_id", "<slice>"), ("slice_end_token_id", "</slice>"),
                          ("im_id_start_token_id", "<image_id>"), ("im_id_end_token_id", "</image_id>")):
            if ex.get(key) is not None:
                got[name] = int(ex[key])
        return got

    # ------------------------------------------------------------------ weights
    def init_random(self, seed: int = 0, std: float = 0.02) -> "MiniCPMV":
        super().init_random(seed, std)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 6007)
        self.visual.init_random(gen, std)
        H, E = self.cfg.hidden_size, self.visual.E
        mk = lambda *s: torch.empty(*s, dtype=self.dtype, device=self.device).normal_(0.0, std, generator=gen)  # noqa
        one = lambda n: torch.ones(n, dtype=self.dtype, device=self.device)  # noqa: E731
        z = lambda n: torch.zeros(n, dtype=self.dtype, device=self.device)  # noqa: E731
        self.rs = {"query": mk(self.nq, H), "kv.weight": mk(H, E), "in.weight": mk(3 * H, H), "in.bias": z(3 * H),
                   "out.weight": mk(H, H), "out.bias": z(H), "ln_q.weight": one(H), "ln_q.bias": z(H),
                   "ln_kv.weight": one(H), "ln_kv.bias": z(H), "ln_post.weight": one(H), "ln_post.bias": z(H),
                   "proj": mk(H, H)}
        return self

    _RS = {"query": "query", "kv_proj.weight": "kv.weight", "attn.in_proj_weight": "in.weight",
           "attn.in_proj_bias": "in.bias", "attn.out_proj.weight": "out.weight", "attn.out_proj.bias": "out.bias",
           "ln_q.weight": "ln_q.weight", "ln_q.bias": "ln_q.bias", "ln_kv.weight": "ln_kv.weight",
           "ln_kv.bias": "ln_kv.bias", "ln_post.weight": "ln_post.weight", "ln_post.bias": "ln_post.bias",
           "proj": "proj"}

    def load_hf_weights(self, weights) -> "MiniCPMV":
        pend: dict = {}

        def lm_only():
            for name, w in weights:
                if name.startswith("llm."):
                    yield name[len("llm."):], w
                elif name.startswith("vpm."):
                    self.visual.load(name[len("vpm."):], w, pend)
                elif name.startswith("resampler."):
                    key = self._RS.get(name[len("resampler."):])
                    if key is not None:
                        self.rs[key] = w.to(device=self.device, dtype=self.dtype).contiguous()
                else:
                    yield name, w

        super().load_hf_weights(lm_only())
        if pend:
            raise ValueError(f"incomplete SigLIP q/k/v projections: {sorted(pend)}")
        return self

    def weight_bytes(self) -> int:
        n = super().weight_bytes() + sum(t.numel() * t.element_size() for t in self.visual.w.values())
        return n + sum(t.numel() * t.element_size() for t in self.rs.values())

    # ------------------------------------------------------------------ multimodal
    @property
    def image_id(self) -> int:
        return self._tok.get("<image>", int((self.cfg.extra or {}).get("image_token_id", 0)))

    def image_prompt_ids(self) -> list[int]:
        return [self.image_id]

    def _markers(self, names) -> list[int]:
        return [self._tok[n] for n in names if n in self._tok]

    def make_mm_input(self, prompt_ids: list[int], images: list):
        where = [i for i, t in enumerate(prompt_ids) if t == self.image_id]
        if len(where) != len(images):
            raise ValueError(f"prompt has {len(where)} image placeholders for {len(images)} images")
        ids, rows, grids, spans, last = [], [], [], [], 0
        for idx, (i, im) in enumerate(zip(where, images)):
            if isinstance(im, tuple):
                px, g, layout = im
            else:
                px, g, layout = preprocess_minicpmv(im, self.max_slices if self.slice_mode else 1, self.slice_scale,
                                                    self.patch)
            ids += prompt_ids[last:i]
            fill = pad_token_id(px, self.cfg.vocab_size)
            if self.use_image_id:
                ids += self._markers(["<image_id>"]) + self._markers(list(str(idx))) + self._markers(["</image_id>"])
            ids += self._markers(["<image>"])
            spans.append((len(ids), self.nq))
            ids += [fill] * self.nq
            ids += self._markers(["</image>"])
            if layout is not None:
                cols, nr = layout
                for r in range(nr):
                    for _ in range(cols):
                        ids += self._markers(["<slice>"])
                        spans.append((len(ids), self.nq))
                        ids += [fill] * self.nq
                        ids += self._markers(["</slice>"])
                    if r < nr - 1:
                        ids += self._markers(["\n"])
            rows.append(px)
            grids += [(1, h, w) for h, w in g]
            last = i + 1
        ids += prompt_ids[last:]
        return ids, MMInput(torch.cat(rows, 0), grids, spans)

    def _pos(self, h: int, w: int) -> torch.Tensor:
        got = self._pos_cache.get((h, w))
        if got is None:
            got = sincos_2d(self.cfg.hidden_size, h, w).reshape(h * w, -1).to(self.device, self.dtype)
            self._pos_cache[(h, w)] = got
        return got

    def resample(self, feats: torch.Tensor, grids: list[tuple[int, int]]) -> torch.Tensor:
        """Per slice: 64 queries cross-attend over that slice's tokens -> [n_slices * 64, H]."""
        r, H, nh = self.rs, self.cfg.hidden_size, self.rheads
        d = H // nh
        kv = ops.layernorm(linear(feats, r["kv.weight"]), r["ln_kv.weight"], r["ln_kv.bias"], 1e-6)
        q = ops.layernorm(r["query"], r["ln_q.weight"], r["ln_q.bias"], 1e-6)
        wq, wk, wv = r["in.weight"].split(H, 0)
        bq, bk, bv = r["in.bias"].split(H, 0)
        qh = linear(q, wq, bq).view(self.nq, nh, d)
        n_kv = [h * w for h, w in grids]
        x = kv[:sum(n_kv)]
        pos = torch.cat([self._pos(h, w) for h, w in grids], 0)
        k = linear((x + pos).contiguous(), wk, bk).view(-1, nh, d)
        v = linear(x.contiguous(), wv, bv).view(-1, nh, d)
        # every slice's 64 queries cross-attend over that slice's tokens: ONE varlen launch
        o = ops.varlen_attention(qh.repeat(len(grids), 1, 1), k, v, [self.nq] * len(grids), d ** -0.5,
                                 k_lengths=n_kv).reshape(len(grids) * self.nq, H)
        o = linear(o, r["out.weight"], r["out.bias"])
        o = ops.layernorm(o, r["ln_post.weight"], r["ln_post.bias"], 1e-6)
        return o @ r["proj"]

    def encode_images(self, pixel_values: torch.Tensor, grids=None) -> torch.Tensor:
        g2 = [(int(h), int(w)) for _, h, w in grids]
        feats = self.visual.forward_patches(pixel_values, g2, self.vis_layers)
        return self.resample(feats, g2)

    def embed_with_images(self, ids: torch.Tensor, rows: torch.Tensor, feats: torch.Tensor) -> torch.Tensor:
        h = pstate.tp_all_reduce(ops.embedding(ids, self.embed, self.tp.vocab_start, self.tp.vocab_end))
        if rows.numel():
            h.index_copy_(0, rows, feats.to(h.dtype))
        return h
