"""DeepSeek-VL2 (``DeepseekVLV2ForCausalLM``): SigLIP-SO400M tiles + 2x2-unfold MLP projector on a
DeepSeekMoE language model with multi-head latent attention.

Reference catalog: ``config/runtimes/srt/deepseek-ai/deepseek-vl2-rt.yaml`` (27B MoE, 4.5B
active).  The language model is ``deepseek.py`` unchanged (absorbed MLA on the latent cache,
grouped MoE routing, shared experts; ``language.*`` weights).  Vision, MI355X-side:

* tiling: the candidate resolution (``candidate_resolutions``) that keeps the most of the image
  at the least padding (LLaVA-NeXT rule) -- one 384-px tile instead when a prompt has more than
  two images -- the image letterboxed (aspect kept, centred, mean-colour fill) into it and cut
  into 384-px tiles, plus a letterboxed 384-px global view first; mean / std 0.5;
* tower (:class:`TimmSiglipTower`): timm's ``vit_so400m_patch14_siglip_384`` body -- 14-px patch
  GEMM (+bias), learned 27x27 positions, 27 pre-norm blocks (fused QKV + bias, bidirectional
  varlen MFMA attention per tile, exact-GELU MLP), final LayerNorm; every tile one varlen sequence;
* projector (``downsample_mlp_gelu``): the 27x27 grid zero-padded to 28x28, 2x2 unfold (channel
  major: c * 4 + 2 * dy + dx) -> GEMM -> GELU -> GEMM;
* layout (``tile_tag: 2D``, ``global_view_pos: head``): the global 14x14 map with a learned
  ``image_newline`` closing each row, the learned ``view_seperator``, then the tiles stitched into
  one (th*14) x (tw*14) map with a newline per row -- all spliced at ``<image>`` token rows.
transformers ships DeepSeek-VL (v1) only: ``tests/test_deepseek_vl2_cpu.py`` checks the vision
path against an independent fp32 restatement and the language model against transformers'
DeepseekV2 (processor pixel parity unpinned).
"""
from __future__ import annotations

import dataclasses

import numpy as np
import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.models.config import ModelConfig
from ome_amd.models.deepseek import DeepseekForCausalLM
from ome_amd.models.nemotron_vl import RadioTower, special_token_ids
from ome_amd.models.quant import linear
from ome_amd.multimodal.inputs import MMInput, load_image, pad_token_id
from ome_amd.parallel import state as pstate

DEEPSEEK_VL2_ARCHS = {"DeepseekVLV2ForCausalLM"}
CANDIDATES = [[384, 384], [384, 768], [768, 384], [384, 1152], [1152, 384], [384, 1536], [1536, 384], [768, 768],
              [384, 1920], [1920, 384], [384, 2304], [2304, 384], [768, 1152], [1152, 768], [384, 2688], [2688, 384],
              [384, 3072], [3072, 384], [768, 1536], [1536, 768], [384, 3456], [3456, 384], [1152, 1152]]


def best_resolution(w: int, h: int, candidates) -> tuple[int, int]:
    """(w, h) of the candidate that keeps the most image pixels, then wastes the fewest."""
    best, fit, waste = None, -1, float("inf")
    for cw, ch in candidates:
        s = min(cw / w, ch / h)
        eff = min(int(w * s) * int(h * s), w * h)
        wst = cw * ch - eff
        if eff > fit or (eff == fit and wst < waste):
            best, fit, waste = (cw, ch), eff, wst
    return best


def letterbox(img, size: tuple[int, int], mean):
    """PIL ``ImageOps.pad``: fit inside ``size`` keeping aspect (bicubic), centred, mean-colour fill."""
    from PIL import Image, ImageOps

    return ImageOps.pad(img, size, method=Image.BICUBIC, color=tuple(int(x * 255) for x in mean))


def preprocess_deepseek_vl2(image, tile: int = 384, crop: bool = True, candidates=CANDIDATES, mean=(0.5, 0.5, 0.5),
                            std=(0.5, 0.5, 0.5)) -> tuple[torch.Tensor, tuple[int, int, int]]:
    """-> (pixels float32 [1 + th*tw, 3, tile, tile] (global view first), (1, th, tw))."""
    img = load_image(image)
    bw, bh = best_resolution(img.width, img.height, candidates) if crop else (tile, tile)
    views = [letterbox(img, (tile, tile), mean)]
    local = letterbox(img, (bw, bh), mean)
    views += [local.crop((x, y, x + tile, y + tile)) for y in range(0, bh, tile) for x in range(0, bw, tile)]
    a = np.stack([np.asarray(v.convert("RGB"), dtype=np.float32) for v in views]) / 255.0
    a = (a - np.asarray(mean, np.float32)) / np.asarray(std, np.float32)
    return torch.from_numpy(np.ascontiguousarray(a.transpose(0, 3, 1, 2))), (1, bh // tile, bw // tile)


def num_image_tokens(th: int, tw: int, s: int = 14) -> int:
    return s * (s + 1) + 1 + (th * s) * (tw * s + 1)


class TimmSiglipTower(RadioTower):
    """timm ViT (no class token, learned positions of the tile grid, final LayerNorm)."""

    def __init__(self, vc: dict, device, dtype):
        vc = dict(vc)
        layers = vc.get("layers") or vc.get("num_hidden_layers") or 27
        sel = int(vc.get("select_layer", -1))
        depth = min(layers, layers + sel + 1) if sel <= 0 else min(layers, sel)
        E = int(vc.get("width") or vc.get("hidden_size") or 1152)
        ratio = float(vc.get("mlp_ratio") or 3.7362)
        super().__init__({"hidden_size": E, "num_attention_heads": vc.get("heads") or vc.get("num_attention_heads") or 16,
                          "num_hidden_layers": depth, "intermediate_size": vc.get("intermediate_size") or int(E * ratio),
                          "patch_size": vc.get("patch_size", 14), "layer_norm_eps": 1e-6, "num_skip": 0},
                         device, dtype, int(vc.get("image_size", 384)), int(vc.get("patch_size", 14)))
        self.n_skip = 0
        self.max_grid = self.side

    def init_random(self, gen: torch.Generator, std: float = 0.02) -> None:
        super().init_random(gen, std)
        self.w["patch.bias"] = torch.zeros(self.E, dtype=self.dtype, device=self.device)
        self.w["cls"] = self.w["cls"][:0]

    def load(self, name: str, t: torch.Tensor) -> None:
        if name.startswith(("attn_pool.", "head.")):
            return
        if name == "patch_embed.proj.weight":
            self.w["patch.weight"] = self._t(t.reshape(t.shape[0], -1))
        elif name == "patch_embed.proj.bias":
            self.w["patch.bias"] = self._t(t)
        elif name == "pos_embed":
            self.w["pos"] = self._t(t.reshape(-1, t.shape[-1]))
            self.max_grid = int(round(self.w["pos"].shape[0] ** 0.5))
        elif name.startswith("blocks."):
            if int(name.split(".")[1]) < self.depth:
                super().load(name, t)
        elif name in ("norm.weight", "norm.bias"):
            super().load(name, t)
        self.w.setdefault("cls", torch.empty(0, self.E, dtype=self.dtype, device=self.device))
        self._pos.clear()


class DeepseekVLV2ForCausalLM(DeepseekForCausalLM):
    is_multimodal = True

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        if not cfg.is_mla:
            raise NotImplementedError("DeepSeek-VL2 without MLA (use_mla: false, the -tiny variant)")
        super().__init__(cfg, device, dtype, max_positions)
        ex = cfg.extra or {}
        self.visual = TimmSiglipTower(ex.get("vision_config") or {}, self.device, dtype)
        pc = ex.get("projector_config") or {}
        if pc.get("projector_type", "downsample_mlp_gelu") != "downsample_mlp_gelu":
            raise NotImplementedError(f"projector {pc.get('projector_type')!r}")
        self.ratio = int(pc.get("downsample_ratio", 2))
        self.depth = int(pc.get("depth", 2))
        self.mlp_ratio = int(pc.get("mlp_ratio", 1))
        if ex.get("tile_tag", "2D") != "2D" or ex.get("global_view_pos", "head") != "head":
            raise NotImplementedError("tile_tag / global_view_pos other than 2D / head")
        self.s = -(-self.visual.side // self.ratio)
        self.candidates = ex.get("candidate_resolutions") or CANDIDATES
        tok = special_token_ids(ex.get("_model_path"), ["<image>"])
        self.image_id = int(ex.get("image_token_id", tok.get("<image>", 128815)))
        self.proj: dict[str, torch.Tensor] = {}

    def init_random(self, seed: int = 0, std: float = 0.02) -> "DeepseekVLV2ForCausalLM":
        super().init_random(seed, std)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 7717)
        self.visual.init_random(gen, std)
        H, C = self.cfg.hidden_size, self.visual.E * self.ratio ** 2
        mk = lambda *s: torch.empty(*s, dtype=self.dtype, device=self.device).normal_(0.0, std, generator=gen)  # noqa
        z = lambda n: torch.zeros(n, dtype=self.dtype, device=self.device)  # noqa: E731
        P = H * self.mlp_ratio
        self.proj = {"layers.0.weight": mk(P, C), "layers.0.bias": z(P), "newline": mk(H), "sep": mk(H)}
        for i in range(1, self.depth):
            self.proj[f"layers.{2 * i}.weight"] = mk(H if i == self.depth - 1 else P, P)
            self.proj[f"layers.{2 * i}.bias"] = z(H if i == self.depth - 1 else P)
        return self

    def load_hf_weights(self, weights) -> "DeepseekVLV2ForCausalLM":
        def lm_only():
            for name, w in weights:
                if name.startswith("language."):
                    yield name[len("language."):], w
                elif name.startswith("vision."):
                    self.visual.load(name[len("vision."):], w)
                elif name.startswith("projector."):
                    self.proj[name[len("projector."):]] = w.to(device=self.device, dtype=self.dtype).contiguous()
                elif name in ("image_newline", "view_seperator"):
                    self.proj["newline" if name == "image_newline" else "sep"] = \
                        w.reshape(-1).to(device=self.device, dtype=self.dtype).contiguous()
                else:
                    yield name, w

        return super().load_hf_weights(lm_only())

    def weight_bytes(self) -> int:
        n = super().weight_bytes() + sum(t.numel() * t.element_size() for t in self.visual.w.values())
        return n + sum(t.numel() * t.element_size() for t in self.proj.values())

    # ------------------------------------------------------------------ multimodal
    def image_prompt_ids(self) -> list[int]:
        return [self.image_id]

    def make_mm_input(self, prompt_ids: list[int], images: list):
        where = [i for i, t in enumerate(prompt_ids) if t == self.image_id]
        if len(where) != len(images):
            raise ValueError(f"prompt has {len(where)} image tokens for {len(images)} images")
        crop = len(images) <= 2
        ids, pvs, grids, spans, last = [], [], [], [], 0
        for i, im in zip(where, images):
            px, g = im if isinstance(im, tuple) else preprocess_deepseek_vl2(im, self.visual.image, crop,
                                                                             self.candidates)
            n = num_image_tokens(g[1], g[2], self.s)
            ids += prompt_ids[last:i]
            spans.append((len(ids), n))
            ids += [pad_token_id(px, self.cfg.vocab_size)] * n
            pvs.append(px)
            grids.append(tuple(int(v) for v in g))
            last = i + 1
        ids += prompt_ids[last:]
        return ids, MMInput(torch.cat(pvs, 0), grids, spans)

    def _project(self, f: torch.Tensor) -> torch.Tensor:
        """[n, side^2, E] tile features -> [n, s*s, H]: zero-pad to even, 2x2 unfold, MLP."""
        n, side, E, r, s = f.shape[0], self.visual.side, self.visual.E, self.ratio, self.s
        x = f.view(n, side, side, E)
        pad = s * r - side
        if pad:
            x = F.pad(x, (0, 0, 0, pad, 0, pad))
        x = x.view(n, s, r, s, r, E).permute(0, 1, 3, 5, 2, 4).reshape(n * s * s, E * r * r).contiguous()
        p = self.proj
        for i in range(self.depth):
            x = linear(x, p[f"layers.{2 * i}.weight"], p[f"layers.{2 * i}.bias"])
            if i < self.depth - 1:
                x = ops.act(x, 3)
        return x.view(n, s * s, -1)

    def encode_images(self, pixel_values: torch.Tensor, grids=None) -> torch.Tensor:
        side, H, s = self.visual.side, self.cfg.hidden_size, self.s
        f = self.visual.forward(pixel_values).view(pixel_values.shape[0], side * side, -1)
        x = self._project(f)
        nl, out, off = self.proj["newline"], [], 0
        for _, th, tw in grids:
            g = x[off].view(s, s, H)
            loc = x[off + 1:off + 1 + th * tw].view(th, tw, s, s, H).permute(0, 2, 1, 3, 4).reshape(th * s, tw * s, H)
            off += 1 + th * tw
            out += [torch.cat([g, nl.view(1, 1, H).expand(s, 1, H)], 1).reshape(-1, H), self.proj["sep"].view(1, H),
                    torch.cat([loc, nl.view(1, 1, H).expand(th * s, 1, H)], 1).reshape(-1, H)]
        return torch.cat(out, 0)

    def embed_with_images(self, ids: torch.Tensor, rows: torch.Tensor, feats: torch.Tensor) -> torch.Tensor:
        h = pstate.tp_all_reduce(ops.embedding(ids, self.embed, self.tp.vocab_start, self.tp.vocab_end))
        if rows.numel():
            h.index_copy_(0, rows, feats.to(h.dtype))
        return h
