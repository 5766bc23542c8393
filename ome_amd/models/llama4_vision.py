"""Llama 4 multimodal (``Llama4ForConditionalGeneration`` with images: Scout / Maverick, the nine
Llama-4 runtimes of the reference catalog, e.g. ``config/runtimes/srt/meta/llama-4-scout-17b-16e-instruct-rt.yaml``
with ``IMAGE_TEXT_TO_TEXT`` in the base models).

Image path:
* preprocessing (:func:`preprocess_llama4`): best-fit canvas of up to ``max_patches`` 336-px
  tiles (least up-scaling, else least down-scaling, ties -> smallest area, candidate order as
  the reference processor), aspect-preserving bilinear resize capped at one tile of up-scaling,
  zero pad, normalise with mean = std = 0.5, row-major tiles, plus a global 336-px thumbnail when
  there is more than one tile;
* prompt: each ``<|image|>`` of the prompt expands to ``<|image_start|>`` + per tile
  ``<|patch|>`` x tokens-per-tile with ``<|tile_x_separator|>`` / ``<|tile_y_separator|>`` +
  ``<|image|>`` + the thumbnail's patches + ``<|image_end|>``; the ``<|patch|>`` rows of the
  prefill are overwritten with the projected vision features (plain 1D RoPE: no position offsets);
* vision tower (once per request, at the first prefill chunk reaching an image): unfold patch
  GEMM, class token appended last, learned positions, pre-LayerNorm, ``depth`` encoder layers
  (LayerNorm -> fused QKV GEMM -> 2D complex RoPE on (x, y) patch coordinates -> bidirectional
  attention per tile on the varlen MFMA kernel (head dim 88 zero-padded to 96 inside it) ->
  O GEMM; LayerNorm -> GELU MLP), post-LayerNorm, class token dropped, 2x2 pixel shuffle ->
  GELU MLP adapter -> linear projector into the text hidden size.
The language model is :class:`ome_amd.models.llama4.Llama4ForCausalLM` unchanged.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ome_amd import ops
from ome_amd.models.config import ModelConfig
from ome_amd.models.llama4 import Llama4ForCausalLM
from ome_amd.models.quant import linear
from ome_amd.multimodal.inputs import MMInput, load_image
from ome_amd.parallel import state as pstate

# special tokens of the Llama 4 tokenizer (config keys override)
IMAGE_START, IMAGE_END, IMAGE, PATCH, TILE_X, TILE_Y = 200080, 200081, 200090, 200092, 200084, 200085


def supported_canvases(max_chunks: int) -> list[tuple[int, int]]:
    """(tiles_h, tiles_w) candidates in the reference processor's order (by chunk count
    descending, grouped by aspect ratio in first-seen order)."""
    groups: dict[float, list[tuple[int, int]]] = {}
    for n in range(max_chunks, 0, -1):
        for f in sorted({d for d in range(1, n + 1) if n % d == 0}):
            groups.setdefault(f / (n // f), []).append((f, n // f))
    return [hw for v in groups.values() for hw in v]


def best_canvas(h: int, w: int, max_chunks: int, tile: int) -> tuple[int, int]:
    cands = [(a * tile, b * tile) for a, b in supported_canvases(max_chunks)]
    scales = [min(ch / h, cw / w) for ch, cw in cands]
    up = [s for s in scales if s >= 1]
    target = min(up) if up else max(scales)
    best = None
    for (ch, cw), s in zip(cands, scales):
        if s == target and (best is None or ch * cw < best[0] * best[1]):
            best = (ch, cw)
    return best


def preprocess_llama4(image, tile: int = 336, max_patches: int = 16):
    """-> (tiles float32 [n, 3, tile, tile] (row-major tiles, then the thumbnail if n > 1),
    (tiles_h, tiles_w))."""
    from PIL import Image

    img = load_image(image)
    W, H = img.size
    ch, cw = best_canvas(H, W, max_patches, tile)
    th, tw = min(max(H, tile), ch), min(max(W, tile), cw)   # at most one tile of up-scaling
    sw, sh = tw / W, th / H
    if sw < sh:
        nh, nw = min(math.floor(H * sw), th), tw
    else:
        nh, nw = th, min(math.floor(W * sh), tw)
    nh, nw = max(nh, 1), max(nw, 1)

    def norm(a):
        return (np.asarray(a, dtype=np.float32).transpose(2, 0, 1) / 255.0 - 0.5) / 0.5

    canvas = np.zeros((3, ch, cw), dtype=np.float32)
    canvas[:, :nh, :nw] = norm(img.resize((nw, nh), Image.BILINEAR))
    canvas[:, nh:, :] = (0.0 - 0.5) / 0.5   # zero-padded pixels, normalised
    canvas[:, :nh, nw:] = (0.0 - 0.5) / 0.5
    rh, rw = ch // tile, cw // tile
    tiles = canvas.reshape(3, rh, tile, rw, tile).transpose(1, 3, 0, 2, 4).reshape(rh * rw, 3, tile, tile)
    if rh * rw > 1:
        thumb = norm(img.resize((tile, tile), Image.BILINEAR))[None]
        tiles = np.concatenate([tiles, thumb], 0)
    return torch.from_numpy(np.ascontiguousarray(tiles)), (rh, rw)


class Llama4VisionTower:
    def __init__(self, vc: dict, text_hidden: int, device, dtype):
        self.device, self.dtype = device, dtype
        self.E = int(vc.get("hidden_size", 1408))
        self.heads = int(vc.get("num_attention_heads", 16))
        self.D = self.E // self.heads
        self.depth = int(vc.get("num_hidden_layers", 34))
        self.I = int(vc.get("intermediate_size", 5632))
        self.image = int(vc.get("image_size", 336))
        self.patch = int(vc.get("patch_size", 14))
        self.C = int(vc.get("num_channels", 3))
        self.ratio = float(vc.get("pixel_shuffle_ratio", 0.5))
        self.proj_in = int(vc.get("projector_input_dim", 4096))
        self.proj_out = int(vc.get("projector_output_dim", 4096))
        self.out_dim = int(vc.get("vision_output_dim", 4096))
        self.eps = float(vc.get("norm_eps", 1e-5))
        self.text_hidden = text_hidden
        self.side = self.image // self.patch
        self.n_patch = self.side ** 2
        self.tokens_per_tile = int(self.n_patch * self.ratio * self.ratio)
        rp = vc.get("rope_parameters") or {}
        theta = float(rp.get("rope_theta", vc.get("rope_theta", 10000.0)))
        # 2D RoPE on complex pairs: pair j < D/4 rotates by (x + 1) * f_j, pair D/4 + j by (y + 1) * f_j;
        # the class token (last) is not rotated
        fd = self.D // 2
        f = 1.0 / (theta ** (torch.arange(0, fd, 2)[: fd // 2].float() / fd))
        idx = torch.arange(self.n_patch)
        ang = torch.cat([((idx % self.side) + 1)[:, None] * f[None], ((idx // self.side) + 1)[:, None] * f[None]], 1)
        ang = torch.cat([ang, torch.zeros(1, ang.shape[1])])                       # [n_patch + 1, D/2]
        self.cos, self.sin = ang.cos().to(device), ang.sin().to(device)
        self.w: dict[str, torch.Tensor] = {}

    # ------------------------------------------------------------------ weights
    def _shapes(self) -> dict:
        E, I = self.E, self.I
        s = {"patch_embedding.linear.weight": (E, self.C * self.patch ** 2), "class_embedding": (E,),
             "positional_embedding_vlm": (self.n_patch + 1, E), "layernorm_pre.weight": (E,),
             "layernorm_pre.bias": (E,), "layernorm_post.weight": (E,), "layernorm_post.bias": (E,),
             "vision_adapter.mlp.fc1.weight": (self.proj_in, I), "vision_adapter.mlp.fc2.weight": (self.proj_out, self.proj_in),
             "projector.weight": (self.text_hidden, self.out_dim)}
        for b in range(self.depth):
            p = f"layers.{b}."
            s.update({p + "qkv.weight": (3 * E, E), p + "qkv.bias": (3 * E,), p + "o.weight": (E, E),
                      p + "o.bias": (E,), p + "fc1.weight": (I, E), p + "fc1.bias": (I,), p + "fc2.weight": (E, I),
                      p + "fc2.bias": (E,), p + "ln1.weight": (E,), p + "ln1.bias": (E,), p + "ln2.weight": (E,),
                      p + "ln2.bias": (E,)})
        return s

    def init_random(self, gen: torch.Generator, std: float = 0.02) -> None:
        for k, s in self._shapes().items():
            t = torch.empty(*s, dtype=self.dtype, device=self.device)
            if k.endswith(("ln1.weight", "ln2.weight", "layernorm_pre.weight", "layernorm_post.weight")):
                t.fill_(1.0)
            elif len(s) == 1 and k != "class_embedding":
                t.zero_()
            else:
                t.normal_(0.0, std, generator=gen)
            self.w[k] = t

    _REN = {"self_attn.o_proj": "o", "mlp.fc1": "fc1", "mlp.fc2": "fc2", "input_layernorm": "ln1",
            "post_attention_layernorm": "ln2"}

    def load(self, name: str, t: torch.Tensor, pend: dict) -> None:
        """``name`` relative to ``vision_model.`` (or ``multi_modal_projector.linear_1.weight``)."""
        if name.startswith("model.layers."):
            parts = name.split(".")
            b, sub = int(parts[2]), ".".join(parts[3:])
            mod, kind = sub.rsplit(".", 1)
            if mod in ("self_attn.q_proj", "self_attn.k_proj", "self_attn.v_proj"):
                pend.setdefault((b, kind), {})[mod[-6]] = t
                got = pend[(b, kind)]
                if len(got) == 3:
                    self.w[f"layers.{b}.qkv.{kind}"] = self._t(torch.cat([got["q"], got["k"], got["v"]]))
                    del pend[(b, kind)]
                return
            name = f"layers.{b}.{self._REN[mod]}.{kind}"
        self.w[name] = self._t(t)

    def _t(self, t: torch.Tensor) -> torch.Tensor:
        return t.to(device=self.device, dtype=self.dtype).contiguous()

    # ------------------------------------------------------------------ forward
    def _rope(self, x: torch.Tensor, n_tiles: int) -> torch.Tensor:
        """x [T, heads, D] (T = tiles * (n_patch + 1)) -> complex-pair rotation, model dtype."""
        xf = x.float().view(n_tiles, self.n_patch + 1, self.heads, self.D // 2, 2)
        c, s = self.cos[None, :, None, :], self.sin[None, :, None, :]
        re, im = xf[..., 0], xf[..., 1]
        return torch.stack([re * c - im * s, re * s + im * c], -1).reshape(x.shape).to(self.dtype)

    def forward(self, tiles: torch.Tensor) -> torch.Tensor:
        """tiles [n, C, S, S] -> projected features [n * tokens_per_tile, text_hidden]."""
        dev, dt, E, w = self.device, self.dtype, self.E, self.w
        n, P, ps = tiles.shape[0], self.n_patch, self.patch
        x = tiles.to(device=dev, dtype=dt)
        # unfold order: (C, ky, kx) per patch, patches row-major
        x = x.reshape(n, self.C, self.side, ps, self.side, ps).permute(0, 2, 4, 1, 3, 5).reshape(n * P, -1)
        x = linear(x, w["patch_embedding.linear.weight"]).view(n, P, E)
        x = torch.cat([x, w["class_embedding"].view(1, 1, E).expand(n, 1, E)], 1) + w["positional_embedding_vlm"]
        T = n * (P + 1)
        x = ops.layernorm(x.reshape(T, E).contiguous(), w["layernorm_pre.weight"], w["layernorm_pre.bias"], self.eps)
        lens = [P + 1] * n
        for b in range(self.depth):
            p = f"layers.{b}."
            h = ops.layernorm(x, w[p + "ln1.weight"], w[p + "ln1.bias"], self.eps)
            qkv = linear(h, w[p + "qkv.weight"], w[p + "qkv.bias"]).view(T, 3, self.heads, self.D)
            q, k = self._rope(qkv[:, 0], n), self._rope(qkv[:, 1], n)
            a = ops.varlen_attention(q, k, qkv[:, 2], lens, self.D ** -0.5).reshape(T, E)
            x = x + linear(a, w[p + "o.weight"], w[p + "o.bias"])
            h = ops.layernorm(x, w[p + "ln2.weight"], w[p + "ln2.bias"], self.eps)
            x = x + linear(ops.act(linear(h, w[p + "fc1.weight"], w[p + "fc1.bias"]), 3), w[p + "fc2.weight"],
                           w[p + "fc2.bias"])
        x = ops.layernorm(x, w["layernorm_post.weight"], w["layernorm_post.bias"], self.eps)
        x = x.view(n, P + 1, E)[:, :P]
        # 2x2 pixel shuffle (the reference's reshape / permute sequence)
        s, r = self.side, self.ratio
        x = x.reshape(n, s, int(s * r), int(E / r)).permute(0, 2, 1, 3).reshape(n, int(s * r), int(s * r), int(E / r / r))
        x = x.permute(0, 2, 1, 3).reshape(n * self.tokens_per_tile, -1).contiguous()
        x = ops.act(linear(x, w["vision_adapter.mlp.fc1.weight"]), 3)
        x = ops.act(linear(x, w["vision_adapter.mlp.fc2.weight"]), 3)
        return linear(x, w["projector.weight"])


class Llama4ForConditionalGeneration(Llama4ForCausalLM):
    is_multimodal = True

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        ex = cfg.extra or {}
        self.visual = Llama4VisionTower(ex.get("vision_config") or {}, cfg.hidden_size, self.device, dtype)
        self.patch_id = int(ex.get("image_token_index", PATCH))
        self.boi_id = int(ex.get("boi_token_index", IMAGE_START))
        self.eoi_id = int(ex.get("eoi_token_index", IMAGE_END))
        self.image_id = int(ex.get("image_placeholder_token_id", IMAGE))
        self.tile_x = int(ex.get("tile_x_separator_token_id", TILE_X))
        self.tile_y = int(ex.get("tile_y_separator_token_id", TILE_Y))
        self.max_patches = int(ex.get("max_patches", 16))

    def init_random(self, seed: int = 0, std: float = 0.02) -> "Llama4ForConditionalGeneration":
        super().init_random(seed, std)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 4447)
        self.visual.init_random(gen, std)
        return self

    def load_hf_weights(self, weights) -> "Llama4ForConditionalGeneration":
        pend: dict = {}

        def text_only():
            for name, w in weights:
                for pre in ("model.vision_model.", "vision_model."):
                    if name.startswith(pre):
                        self.visual.load(name[len(pre):], w, pend)
                        break
                else:
                    if name.endswith("multi_modal_projector.linear_1.weight"):
                        self.visual.w["projector.weight"] = self.visual._t(w)
                    else:
                        yield name, w

        super().load_hf_weights(text_only())
        if pend:
            raise ValueError(f"incomplete vision q/k/v projections: {sorted(pend)}")
        return self

    def weight_bytes(self) -> int:
        return super().weight_bytes() + sum(t.numel() * t.element_size() for t in self.visual.w.values())

    # ------------------------------------------------------------------ multimodal
    def image_prompt_ids(self) -> list[int]:
        return [self.image_id]

    def _image_tokens(self, ratio: tuple[int, int], patch: int) -> tuple[list[int], list[tuple[int, int]]]:
        """Token layout of one image and its patch runs (offset, length) within it."""
        rh, rw = ratio
        n = self.visual.tokens_per_tile
        ids, runs = [self.boi_id], []

        def patches():
            runs.append((len(ids), n))
            ids.extend([patch] * n)

        if rh * rw > 1:
            for _ in range(rh):
                for x in range(rw):
                    patches()
                    if x < rw - 1:
                        ids.append(self.tile_x)
                ids.append(self.tile_y)
        ids.append(self.image_id)
        patches()
        ids.append(self.eoi_id)
        return ids, runs

    def make_mm_input(self, prompt_ids: list[int], images: list):
        """Expand each ``<|image|>`` of the prompt into the image's tile-token layout.  The patch
        rows carry a content-hash id (:func:`ome_amd.multimodal.inputs.pad_token_id`) so the
        prefix cache only ever matches identical images; the rows are overwritten by the vision
        features, so the id is never embedded."""
        from ome_amd.multimodal.inputs import pad_token_id

        where = [i for i, t in enumerate(prompt_ids) if t == self.image_id]
        if len(where) != len(images):
            raise ValueError(f"prompt has {len(where)} <|image|> tokens for {len(images)} images")
        ids, pvs, grids, spans, last = [], [], [], [], 0
        for i, im in zip(where, images):
            tiles, ratio = im if isinstance(im, tuple) else preprocess_llama4(im, self.visual.image,
                                                                                self.max_patches)
            ids += prompt_ids[last:i]
            toks, runs = self._image_tokens(ratio, pad_token_id(tiles, self.cfg.vocab_size))
            spans += [(len(ids) + o, n) for o, n in runs]
            ids += toks
            pvs.append(tiles)
            grids.append((tiles.shape[0], *ratio))
            last = i + 1
        ids += prompt_ids[last:]
        return ids, MMInput(torch.cat(pvs, 0), grids, spans)

    def encode_images(self, pixel_values: torch.Tensor, grids) -> torch.Tensor:
        return self.visual.forward(pixel_values)

    def embed_with_images(self, ids: torch.Tensor, rows: torch.Tensor, feats: torch.Tensor) -> torch.Tensor:
        h = pstate.tp_all_reduce(ops.embedding(ids, self.embed, self.tp.vocab_start, self.tp.vocab_end))
        if rows.numel():
            h.index_copy_(0, rows, feats.to(h.dtype))
        return h
