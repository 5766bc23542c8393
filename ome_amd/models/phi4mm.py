"""Phi-4-multimodal (``Phi4MMForCausalLM``; reference catalog
``config/runtimes/srt/microsoft/phi-4-multimodal-instruct-rt.yaml``) and the transformers
``Phi4MultimodalForCausalLM`` layout -- text + image serving.

* preprocessing (dynamic HD): the image is fitted into a grid of 448-px crops (up to
  ``dynamic_hd`` = 36; closest aspect ratio when more would be needed), aspect-preserving resize,
  white padding right / bottom, mean / std 0.5; a 448 x 448 global view (bicubic) goes first;
  per crop a 32 x 32 patch mask marks the padding;
* SigLIP tower (the ``gemma3_vision.py`` weights / layers) run to ``feature_layer`` (-2): patch
  GEMM, NaViT bucketed positions over each crop's valid patch rectangle, varlen MFMA attention over
  the valid patches of each crop (queries of padded patches attend to the valid keys -- their
  features reach the 2 x 2 pooling at odd valid extents, exactly as in the reference), 2 x 2
  average pool;
* HD layout per image: sub-image grid cropped to its useful extent, a ``sub_GN`` row separator
  after every row, ``glb_GN``, then the global view's 16 x 16 grid with its separators;
  projector GEMM -> GELU -> GEMM; the image's ``<|endoftext10|>`` placeholder expands to that many
  rows (content-hash ids);
* language model: Phi-4-mini on the Phi-3 path of ``decoder.py`` (fused qkv / gate_up, partial
  rotary, LongRoPE).  Original checkpoints carry the LM as ``base_layer`` weights plus vision /
  speech LoRA adapters: the base weights are served; ``OME_PHI4MM_VISION_LORA=1`` folds the vision
  adapter (``lora_alpha / r`` * B A) into them at load.  The speech encoder is not served
  (the reference runtime's catalog entry serves text + image).
"""
from __future__ import annotations

import dataclasses
import math
import os

import numpy as np
import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.models.config import ModelConfig
from ome_amd.models.decoder import DecoderForCausalLM
from ome_amd.models.gemma3_vision import SiglipVisionTower
from ome_amd.models.quant import linear
from ome_amd.multimodal.inputs import MMInput, load_image, pad_token_id
from ome_amd.parallel import state as pstate

PHI4MM_ARCHS = {"Phi4MMForCausalLM", "Phi4MultimodalForCausalLM"}


def _closest_ratio(aspect: float, ratios, w: int, h: int, size: int):
    best, diff = (1, 1), float("inf")
    for r in ratios:
        d = abs(aspect - r[0] / r[1])
        if d < diff:
            best, diff = r, d
        elif d == diff and w * h > 0.5 * size * size * r[0] * r[1]:
            best = r
    return best


def hd_layout(h: int, w: int, size: int = 448, patch: int = 14, max_num: int = 36):
    """-> (target (cols, rows) crops, resized (w, h), padding (w, h) in px)."""
    wc, hc = math.ceil(w / size), math.ceil(h / size)
    if wc * hc > max_num:
        ratios = sorted({(i, j) for n in range(1, max_num + 1) for i in range(1, n + 1) for j in range(1, n + 1)
                         if i * j <= max_num}, key=lambda r: r[0] * r[1])
        wc, hc = _closest_ratio(w / h, ratios, w, h, size)
    tw, th = size * wc, size * hc
    if tw / w < th / h:
        nw, nh = tw, int(h * tw / w)
    else:
        nw, nh = int(w * th / h), th
    if min(nh, th) < 10 or min(nw, tw) < 10:
        raise ValueError(f"the aspect ratio is very extreme {(nw, nh)}")
    return (wc, hc), (nw, nh), (tw - nw, th - nh)


def preprocess_phi4mm(image, size: int = 448, patch: int = 14, max_num: int = 36):
    """-> (crops float32 [1 + rows * cols, 3, size, size] (global view first), grid
    (rows, cols, padded patch rows, padded patch cols))."""
    from PIL import Image

    img = load_image(image)
    (wc, hc), (nw, nh), (pw, ph) = hd_layout(img.height, img.width, size, patch, max_num)
    a = np.full((nh + ph, nw + pw, 3), 255.0, dtype=np.float32)
    a[:nh, :nw] = np.asarray(img.resize((nw, nh), Image.BILINEAR), dtype=np.float32)
    a = (a / 255.0 - 0.5) / 0.5
    t = torch.from_numpy(np.ascontiguousarray(a.transpose(2, 0, 1)))
    glob = F.interpolate(t[None], size=(size, size), mode="bicubic", align_corners=False)
    crops = t.reshape(3, hc, size, wc, size).permute(1, 3, 0, 2, 4).reshape(-1, 3, size, size)
    pr = ph // patch if ph >= patch else 0
    pc = pw // patch if pw >= patch else 0
    return torch.cat([glob, crops]), (hc, wc, pr, pc)


def crop_masks(grid, side: int) -> torch.Tensor:
    """[1 + rows * cols, side, side] bool valid-patch masks (global view all valid)."""
    hc, wc, pr, pc = grid
    m = torch.ones(hc * side, wc * side, dtype=torch.bool)
    if pc:
        m[:, -pc:] = False
    if pr:
        m[-pr:, :] = False
    m = m.reshape(hc, side, wc, side).transpose(1, 2).reshape(-1, side, side)
    return torch.cat([torch.ones(1, side, side, dtype=torch.bool), m])


def num_image_tokens(grid, side: int = 32) -> int:
    hc, wc, pr, pc = grid
    g = side // 2 + side % 2
    uh = len(range(0, hc * side - pr, 2)) if pr else hc * g
    uw = len(range(0, wc * side - pc, 2)) if pc else wc * g
    return uh * (uw + 1) + 1 + (side // 2) * (side // 2 + 1)


class Phi4MMVisionTower(SiglipVisionTower):
    def _pos_ids(self, mask: torch.Tensor) -> torch.Tensor:
        """NaViT bucketed positions of one crop's patches (0 for padded patches)."""
        s = self.side
        nh, nw = int(mask[:, 0].sum()), int(mask[0, :].sum())
        if nh == 0 or nw == 0:
            return torch.zeros(s * s, dtype=torch.long)
        bounds = torch.arange(1 / s, 1.0, 1 / s)
        fh = torch.clamp(torch.arange(s, dtype=torch.float32) * (1.0 / nh), max=1.0 - 1e-6)
        fw = torch.clamp(torch.arange(s, dtype=torch.float32) * (1.0 / nw), max=1.0 - 1e-6)
        bh, bw = torch.bucketize(fh, bounds, right=True), torch.bucketize(fw, bounds, right=True)
        pos = (bh[:, None] * s + bw[None, :]).reshape(-1)
        return torch.where(mask.reshape(-1), pos, torch.zeros_like(pos))

    def forward_masked(self, pixels: torch.Tensor, masks: torch.Tensor, n_layers: int) -> torch.Tensor:
        """pixels [n, C, S, S], masks [n, s, s] -> hidden state after ``n_layers`` [n, s * s, E];
        keys are restricted to each crop's valid patches."""
        w, E, n, ps, s, dev = self.w, self.E, pixels.shape[0], self.patch, self.side, self.device
        P = s * s
        x = pixels.to(device=dev, dtype=self.dtype)
        x = x.reshape(n, self.C, s, ps, s, ps).permute(0, 2, 4, 1, 3, 5).reshape(n * P, -1)
        pos = torch.cat([self._pos_ids(masks[c]) for c in range(n)]).to(dev)
        x = linear(x, w["patch.weight"], w["patch.bias"]) + w["pos"][pos]
        # valid patches of every crop first (one varlen segment per crop), then the padded ones
        flat = masks.reshape(n, P)
        valid_idx = [torch.nonzero(flat[c]).flatten() + c * P for c in range(n)]
        pad_idx = [torch.nonzero(~flat[c]).flatten() + c * P for c in range(n)]
        nv = [len(v) for v in valid_idx]
        npd = [len(p) for p in pad_idx]
        order = torch.cat(valid_idx + pad_idx).to(dev)
        Nv = sum(nv)
        x = x[order].contiguous()
        T = x.shape[0]
        for b in range(n_layers):
            p = f"layers.{b}."
            h = ops.layernorm(x, w[p + "ln1.weight"], w[p + "ln1.bias"], self.eps)
            qkv = linear(h, w[p + "qkv.weight"], w[p + "qkv.bias"]).view(T, 3, self.heads, self.D)
            a = torch.empty(T, self.heads, self.D, dtype=x.dtype, device=dev)
            ops.varlen_attention(qkv[:Nv, 0], qkv[:Nv, 1], qkv[:Nv, 2], nv, self.D ** -0.5, out=a[:Nv])
            if T > Nv:   # padding queries of each crop attend to that crop's valid tokens (cross lengths)
                ops.varlen_attention(qkv[Nv:, 0], qkv[:Nv, 1], qkv[:Nv, 2], list(npd), self.D ** -0.5,
                                     out=a[Nv:], k_lengths=list(nv))
            x = x + linear(a.reshape(T, E), w[p + "o.weight"], w[p + "o.bias"])
            h = ops.layernorm(x, w[p + "ln2.weight"], w[p + "ln2.bias"], self.eps)
            f = ops.act(linear(h, w[p + "fc1.weight"], w[p + "fc1.bias"]), self.act)
            x = x + linear(f, w[p + "fc2.weight"], w[p + "fc2.bias"])
        out = torch.empty_like(x)
        out[order] = x
        return out.view(n, P, E)


class Phi4MMForCausalLM(DecoderForCausalLM):
    is_multimodal = True

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(dataclasses.replace(cfg, architecture="Phi3ForCausalLM"), device, dtype, max_positions)
        ex = cfg.extra or {}
        vc = dict(ex.get("vision_config") or {})
        if not vc:   # original checkpoints: SigLIP-so400m at 448 px, configured in ``embd_layer``
            vc = dict(hidden_size=1152, intermediate_size=4304, num_hidden_layers=27, num_attention_heads=16,
                      image_size=448, patch_size=14, hidden_act="gelu_pytorch_tanh", layer_norm_eps=1e-6)
        self.visual = Phi4MMVisionTower(vc, self.device, dtype)
        if self.visual.side % 2:
            raise NotImplementedError("odd patch grids (reflection-padded pooling)")
        layer = int(vc.get("feature_layer", -2))
        self.n_layers = self.visual.depth + 1 + layer if layer < 0 else layer
        self.crop = int(vc.get("crop_size", self.visual.image))
        self.max_crops = int(ex.get("dynamic_hd", 36))
        self.image_token_id = int(vc.get("image_token_id", ex.get("image_token_id", 200010)))
        lora = ex.get("vision_lora") or {}
        self.lora_scale = float(lora.get("lora_alpha", 0)) / float(lora.get("r", 1)) if lora else 0.0
        self.merge_lora = os.environ.get("OME_PHI4MM_VISION_LORA", "0") == "1"
        self.proj: dict[str, torch.Tensor] = {}

    def init_random(self, seed: int = 0, std: float = 0.02) -> "Phi4MMForCausalLM":
        super().init_random(seed, std)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 4111)
        self.visual.init_random(gen, std)
        E, H = self.visual.E, self.cfg.hidden_size
        mk = lambda *s: torch.empty(*s, dtype=self.dtype, device=self.device).normal_(0.0, std, generator=gen)  # noqa
        z = lambda k: torch.zeros(k, dtype=self.dtype, device=self.device)  # noqa
        self.proj = {"up.w": mk(H, E), "up.b": z(H), "down.w": mk(H, H), "down.b": z(H), "glb": mk(E), "sub": mk(E)}
        return self

    _PROJ = {"img_projection_up": "up", "img_projection.0": "up", "img_projection_down": "down",
             "img_projection.2": "down"}

    def load_hf_weights(self, weights) -> "Phi4MMForCausalLM":
        pend: dict = {}
        lora: dict[str, dict[str, torch.Tensor]] = {}
        pre = "model.embed_tokens_extend."

        def lm_only():
            for name, w in weights:
                if name.startswith(pre + "image_embed."):
                    n = name[len(pre + "image_embed."):]
                    if n.startswith("img_processor."):
                        self.visual.load(n[len("img_processor."):], w, pend)
                    elif n in ("glb_GN", "global_img_feature_extensor"):
                        self.proj["glb"] = w.reshape(-1).to(device=self.device, dtype=self.dtype)
                    elif n in ("sub_GN", "sub_img_feature_extensor"):
                        self.proj["sub"] = w.reshape(-1).to(device=self.device, dtype=self.dtype)
                    else:
                        mod, kind = n.rsplit(".", 1)
                        self.proj[f"{self._PROJ[mod]}.{'w' if kind == 'weight' else 'b'}"] = \
                            w.to(device=self.device, dtype=self.dtype).contiguous()
                    continue
                if name.startswith(pre) or name.startswith("model.vision_embed_tokens."):
                    continue                                         # speech encoder: not served
                if ".lora_A." in name or ".lora_B." in name:
                    if ".vision." in name:
                        base = name.split(".lora_")[0]
                        lora.setdefault(base, {})["A" if ".lora_A." in name else "B"] = w
                    continue
                yield ("HELD:" if ".base_layer." in name else "") + name.replace(".base_layer.", "."), w

        def merged():
            held = {}   # base_layer weights wait for their LoRA pair (it may come later in the stream)
            for name, w in lm_only():
                if self.merge_lora and name.startswith("HELD:"):
                    held[name[5:]] = w
                    continue
                yield name.removeprefix("HELD:"), w
            for name, w in held.items():
                ab = lora.get(name.rsplit(".", 1)[0])
                if ab is not None:
                    w = (w.float() + self.lora_scale * ab["B"].float() @ ab["A"].float()).to(w.dtype)
                yield name, w

        super().load_hf_weights(merged())
        if pend or len(self.proj) != 6:
            raise ValueError(f"incomplete Phi-4-MM image embedding: {sorted(pend)} {sorted(self.proj)}")
        return self

    def weight_bytes(self) -> int:
        n = super().weight_bytes() + sum(t.numel() * t.element_size() for t in self.visual.w.values())
        return n + sum(t.numel() * t.element_size() for t in self.proj.values())

    # ------------------------------------------------------------------ multimodal
    def image_prompt_ids(self) -> list[int]:
        return [self.image_token_id]

    def make_mm_input(self, prompt_ids: list[int], images: list):
        where = [i for i, t in enumerate(prompt_ids) if t == self.image_token_id]
        if len(where) != len(images):
            raise ValueError(f"prompt has {len(where)} image tokens for {len(images)} images")
        ids, pvs, grids, spans, last = [], [], [], [], 0
        for i, im in zip(where, images):
            px, g = im if isinstance(im, tuple) else preprocess_phi4mm(im, self.crop, self.visual.patch,
                                                                         self.max_crops)
            n = num_image_tokens(g, self.visual.side)
            ids += prompt_ids[last:i]
            spans.append((len(ids), n))
            ids += [pad_token_id(px, self.cfg.vocab_size)] * n
            pvs.append(px)
            grids.append(tuple(int(v) for v in g))
            last = i + 1
        ids += prompt_ids[last:]
        return ids, MMInput(torch.cat(pvs, 0), grids, spans)

    def encode_images(self, pixel_values: torch.Tensor, grids) -> torch.Tensor:
        s, E, g = self.visual.side, self.visual.E, self.visual.side // 2
        masks = torch.cat([crop_masks(gr, s) for gr in grids])
        x = self.visual.forward_masked(pixel_values, masks, self.n_layers)           # [n, s*s, E]
        x = F.avg_pool2d(x.view(-1, s, s, E).permute(0, 3, 1, 2).float(), 2).permute(0, 2, 3, 1).to(x.dtype)
        sub_sep, glb_sep = self.proj["sub"], self.proj["glb"]
        out, c = [], 0
        for gr in grids:
            hc, wc, pr, pc = gr
            glob = torch.cat([x[c], sub_sep.expand(g, 1, E)], 1).reshape(-1, E)
            sub = x[c + 1:c + 1 + hc * wc].view(hc, wc, g, g, E).transpose(1, 2).reshape(hc * g, wc * g, E)
            m = crop_masks(gr, s)[1:].reshape(hc, wc, s, s)[:, :, 0::2, 0::2]
            m = m.transpose(1, 2).reshape(hc * g, wc * g)
            uh, uw = int(m[:, 0].sum()), int(m[0, :].sum())
            sub = torch.cat([sub[:uh, :uw], sub_sep.expand(uh, 1, E)], 1).reshape(-1, E)
            out.append(torch.cat([sub, glb_sep.view(1, E), glob]))
            c += 1 + hc * wc
        feats = torch.cat(out).contiguous()
        h = ops.act(linear(feats, self.proj["up.w"], self.proj["up.b"]).contiguous(), 3)
        return linear(h, self.proj["down.w"], self.proj["down.b"])

    def embed_with_images(self, ids: torch.Tensor, rows: torch.Tensor, feats: torch.Tensor) -> torch.Tensor:
        h = self._embed(ids, None, None)
        if rows.numel():
            h.index_copy_(0, rows, feats.to(h.dtype))
        return h
