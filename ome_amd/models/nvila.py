"""NVILA (``LlavaLlamaModel``, Efficient-Large-Model/NVILA-8B; reference runtime
``config/runtimes/srt/Efficient-Large-Model/nvila-8b-rt.yaml``, model
``config/models/Efficient-Large-Model/NVILA-8B.yaml``).

The VILA code base is remote code that is not importable offline; this follows the published
NVILA design ("scale then compress") and the VILA checkpoint layout; parity is checked against an
fp32 restatement built on transformers' SigLIP and Qwen2 in ``tests/test_nvila_cpu.py`` (parity
with the remote code itself is unpinned):

* checkpoint: one sub-directory per component -- ``llm/`` (Qwen2), ``vision_tower/``
  (SigLIP, 448 px / patch 14) and ``mm_projector/`` -- each with its own config.json
  (``models/loader.py`` reads them with the directory name as a tensor-name prefix);
* Dynamic-S2 multi-scale tiling: every scale but the last is a square resize cut into
  ``(scale / base)^2`` base tiles; the last scale keeps the aspect ratio -- the (cols, rows) grid
  with ``(last / base)^2 <= cols * rows <= max_tiles`` closest to the image's aspect ratio;
* SigLIP tower on all tiles of all scales in ONE varlen batch (``mm_vision_select_layer``: the
  hidden state after that layer, no post-LayerNorm); per scale the tiles are stitched into one
  feature map, every map is area-resized to the last scale's size and the maps are concatenated
  on channels (``mm_hidden_size = E x scales``);
* the merged map is cut back into base-size blocks ("chessboard"), each block goes through the
  projector -- k x k spatial-to-channel folding with zero padding (``mlp_downsample`` k = 2,
  ``mlp_downsample_3x3_fix`` k = 3), then the LayerNorm / Linear / GELU stack as stored -- and the
  blocks are re-assembled: (rows * ceil(side / k)) x (cols * ceil(side / k)) tokens, row-major.
* the language model is ``llama.py`` with the Qwen2 config (``llm_cfg``).
Images only (NVILA's video path samples frames into the same pipeline; not wired here).
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

NVILA_ARCHS = {"LlavaLlamaModel"}
SIGLIP_448 = dict(hidden_size=1152, intermediate_size=4304, num_hidden_layers=27, num_attention_heads=16,
                  image_size=448, patch_size=14, hidden_act="gelu_pytorch_tanh", layer_norm_eps=1e-6)


def closest_grid(w: int, h: int, min_n: int, max_n: int, base: int) -> tuple[int, int]:
    """(cols, rows) with min_n <= cols * rows <= max_n closest to the aspect ratio w / h (ties: the
    larger grid when the image has the pixels for it)."""
    ratios = sorted({(i, j) for n in range(min_n, max_n + 1) for i in range(1, n + 1) for j in range(1, n + 1)
                     if min_n <= i * j <= max_n}, key=lambda r: r[0] * r[1])
    ar, best, best_diff = w / h, (1, 1), float("inf")
    for r in ratios:
        d = abs(ar - r[0] / r[1])
        if d < best_diff:
            best, best_diff = r, d
        elif d == best_diff and w * h > 0.5 * base * base * r[0] * r[1]:
            best = r
    return best


def _norm(a: np.ndarray) -> np.ndarray:
    return ((a / 255.0 - 0.5) / 0.5).transpose(2, 0, 1)


def preprocess_nvila(image, scales: list[int], base: int, max_tiles: int, dynamic: bool = True):
    """-> (float32 [n_tiles, 3, base, base], (rows, cols) of the last scale).  Tile order: scale
    by scale, row-major within a scale."""
    from PIL import Image

    img = load_image(image)
    w, h = img.size
    tiles = []
    last = scales[-1] // base
    for k, s in enumerate(scales):
        if k == len(scales) - 1 and dynamic:
            cols, rows = closest_grid(w, h, last * last, max(max_tiles, last * last), base)
        else:
            cols = rows = s // base
        a = np.asarray(img.resize((cols * base, rows * base), Image.BICUBIC), dtype=np.float32)
        tiles += [a[r * base:(r + 1) * base, c * base:(c + 1) * base] for r in range(rows) for c in range(cols)]
    px = torch.from_numpy(np.ascontiguousarray(np.stack([_norm(t) for t in tiles])))
    return px, (rows, cols)


def fold(x: torch.Tensor, k: int) -> torch.Tensor:
    """[n, H, W, C] -> [n, ceil(H/k), ceil(W/k), k*k*C]: zero-pad bottom / right, fold each k x k
    neighbourhood into channels ordered (row offset, column offset, channel)."""
    n, H, W, C = x.shape
    ph, pw = -H % k, -W % k
    if ph or pw:
        x = F.pad(x, (0, 0, 0, pw, 0, ph))
    H2, W2 = (H + ph) // k, (W + pw) // k
    return x.view(n, H2, k, W2, k, C).permute(0, 1, 3, 2, 4, 5).reshape(n, H2, W2, k * k * C)


class NVILAForCausalLM(LlamaForCausalLM):
    is_multimodal = True

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        ex = cfg.extra or {}
        if pstate.get().tp_size > 1:
            raise NotImplementedError("NVILA: TP > 1 (the reference serves NVILA-8B at TP 1)")
        vc = {**SIGLIP_448, **(ex.get("vision_tower_cfg") or {})}
        vc.pop("architectures", None)
        self.visual = SiglipVisionTower(vc, self.device, dtype)
        self.base = self.visual.image
        self.side = self.visual.side
        sel = int(ex.get("mm_vision_select_layer", -2))
        self.n_layers = sel if sel >= 0 else self.visual.depth + 1 + sel
        aspect = str(ex.get("image_aspect_ratio", "dynamic_s2"))
        s2 = ex.get("s2_scales")
        if "s2" in aspect or s2:
            self.scales = [int(s) for s in str(s2 or "448,896,1344").split(",")]
            self.base = int(ex.get("s2_max_split_size", self.base))
        else:
            self.scales = [self.base]
        if self.base != self.visual.image:
            raise ValueError(f"NVILA: s2_max_split_size {self.base} != tower image size {self.visual.image}")
        self.dynamic = aspect == "dynamic_s2" or bool(ex.get("dynamic_s2", False))
        self.max_tiles = int(ex.get("max_tiles", ex.get("dynamic_max_tiles", 12)))
        pc = ex.get("mm_projector_cfg") or {}
        ptype = str(pc.get("mm_projector_type", ex.get("mm_projector_type", "mlp_downsample_3x3_fix")))
        self.k = {"mlp_downsample": 2, "mlp_downsample_2x2_fix": 2, "mlp_downsample_3x3_fix": 3}.get(ptype)
        if self.k is None:
            raise NotImplementedError(f"NVILA: mm_projector_type {ptype!r}")
        self.image_id = int(ex.get("image_token_id", (ex.get("media_token_ids") or {}).get("image", -200)))
        self.mm_hidden = self.visual.E * len(self.scales)
        self.proj: list[tuple[str, torch.Tensor, torch.Tensor | None]] = []   # ("ln" | "lin", w, b) by index
        self._proj_raw: dict[int, dict[str, torch.Tensor]] = {}

    # ------------------------------------------------------------------ weights
    def _proj_stack(self, raw: dict[int, dict[str, torch.Tensor]]) -> None:
        """Stored Sequential -> ordered (kind, w, b); a missing index after a Linear is its GELU."""
        idx = sorted(raw)
        out = []
        for n, i in enumerate(idx):
            w, b = raw[i]["weight"], raw[i].get("bias")
            t = lambda x: None if x is None else x.to(device=self.device, dtype=self.dtype).contiguous()  # noqa
            if w.dim() == 1:
                out.append(("ln", t(w), t(b)))
            else:
                out.append(("lin", t(w), t(b)))
                if n + 1 < len(idx) and idx[n + 1] != i + 1:
                    out.append(("gelu", None, None))
        self.proj = out

    def init_random(self, seed: int = 0, std: float = 0.02) -> "NVILAForCausalLM":
        super().init_random(seed, std)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 8117)
        self.visual.init_random(gen, std)
        H, C = self.cfg.hidden_size, self.mm_hidden
        kk = self.k * self.k
        mk = lambda *s: torch.empty(*s).normal_(0.0, std)  # noqa: E731
        if self.k == 3:
            raw = {1: {"weight": torch.ones(9 * C), "bias": torch.zeros(9 * C)},
                   2: {"weight": mk(3 * C, 9 * C), "bias": torch.zeros(3 * C)},
                   4: {"weight": torch.ones(3 * C), "bias": torch.zeros(3 * C)},
                   5: {"weight": mk(H, 3 * C), "bias": torch.zeros(H)}, 7: {"weight": mk(H, H), "bias": torch.zeros(H)}}
        else:
            raw = {1: {"weight": torch.ones(kk * C), "bias": torch.zeros(kk * C)},
                   2: {"weight": mk(H, kk * C), "bias": torch.zeros(H)}, 4: {"weight": mk(H, H), "bias": torch.zeros(H)}}
        self._proj_stack(raw)
        return self

    def load_hf_weights(self, weights) -> "NVILAForCausalLM":
        pend: dict = {}
        raw: dict[int, dict[str, torch.Tensor]] = {}

        def lm_only():
            for name, w in weights:
                if name.startswith("vision_tower."):
                    n = name[len("vision_tower."):]
                    for pre in ("vision_tower.vision_model.", "vision_model."):
                        if n.startswith(pre):
                            n = n[len(pre):]
                            break
                    self.visual.load(n, w, pend)
                elif name.startswith("mm_projector."):
                    parts = name.split(".")   # mm_projector.layers.<i>.<weight|bias>
                    raw.setdefault(int(parts[-2]), {})[parts[-1]] = w
                elif name.startswith("llm."):
                    yield name[len("llm."):], w
                else:
                    yield name, w

        super().load_hf_weights(lm_only())
        if pend:
            raise ValueError(f"NVILA: incomplete vision projections: {sorted(pend)}")
        if not raw:
            raise ValueError("NVILA: no mm_projector weights")
        self._proj_stack(raw)
        return self

    def weight_bytes(self) -> int:
        n = super().weight_bytes() + sum(t.numel() * t.element_size() for t in self.visual.w.values())
        return n + sum(t.numel() * t.element_size() for _, w, b in self.proj for t in (w, b) if t is not None)

    # ------------------------------------------------------------------ multimodal
    def image_prompt_ids(self) -> list[int]:
        return [self.image_id]

    def _n_tokens(self, rows: int, cols: int) -> int:
        m = -(-self.side // self.k)
        return rows * m * cols * m

    def make_mm_input(self, prompt_ids: list[int], images: list):
        where = [i for i, t in enumerate(prompt_ids) if t == self.image_id]
        if len(where) != len(images):
            raise ValueError(f"prompt has {len(where)} image tokens for {len(images)} images")
        ids, pvs, grids, spans, last = [], [], [], [], 0
        for i, im in zip(where, images):
            px, (rows, cols) = im if isinstance(im, tuple) else preprocess_nvila(im, self.scales, self.base,
                                                                                 self.max_tiles, self.dynamic)
            n = self._n_tokens(rows, cols)
            ids += prompt_ids[last:i]
            spans.append((len(ids), n))
            ids += [pad_token_id(px, self.cfg.vocab_size)] * n
            pvs.append(px)
            grids.append((rows, cols))
            last = i + 1
        ids += prompt_ids[last:]
        return ids, MMInput(torch.cat(pvs, 0), grids, spans)

    def _project(self, x: torch.Tensor) -> torch.Tensor:
        """[blocks, side, side, C] -> [blocks, m, m, H] (fold + the stored LN / Linear / GELU stack)."""
        f = fold(x, self.k)
        nb, m = f.shape[0], f.shape[1]
        h = f.reshape(nb * m * m, -1).contiguous()
        for kind, w, b in self.proj:
            if kind == "ln":
                h = ops.layernorm(h, w, b, 1e-5)
            elif kind == "lin":
                h = linear(h, w, b)
            else:
                h = ops.act(h, 3)
        return h.view(nb, m, m, -1)

    def encode_images(self, pixel_values: torch.Tensor, grids) -> torch.Tensor:
        s, E, base = self.side, self.visual.E, self.base
        feats = self.visual.forward(pixel_values, self.n_layers, post_norm=False)    # [tiles, s*s, E]
        out, off = [], 0
        for rows, cols in grids:
            maps = []
            for k, sc in enumerate(self.scales):
                r, c = (rows, cols) if k == len(self.scales) - 1 else (sc // base, sc // base)
                t = feats[off:off + r * c].view(r, c, s, s, E)
                off += r * c
                maps.append(t.permute(4, 0, 2, 1, 3).reshape(E, r * s, c * s))   # one stitched map
            size = maps[-1].shape[1:]
            m = torch.cat([mp if mp.shape[1:] == size else
                           F.interpolate(mp[None].float(), size=size, mode="area")[0].to(mp.dtype) for mp in maps], 0)
            # chessboard: base-size blocks of the merged map, projected one by one
            blocks = m.view(-1, rows, s, cols, s).permute(1, 3, 2, 4, 0).reshape(rows * cols, s, s, -1)
            p = self._project(blocks)                                                # [rows*cols, mm, mm, H]
            mm = p.shape[1]
            out.append(p.view(rows, cols, mm, mm, -1).permute(0, 2, 1, 3, 4).reshape(rows * mm * cols * mm, -1))
        return torch.cat(out, 0).contiguous()

    def embed_with_images(self, ids: torch.Tensor, rows: torch.Tensor, feats: torch.Tensor) -> torch.Tensor:
        h = ops.embedding(ids, self.embed, self.tp.vocab_start, self.tp.vocab_end)
        if rows.numel():
            h.index_copy_(0, rows, feats.to(h.dtype))
        return h
