"""Phi-3-vision / Phi-3.5-vision (``Phi3VForCausalLM``) on the decoder + CLIP paths.

Reference catalog: ``config/runtimes/srt/microsoft/phi-3-vision-128k-instruct-rt.yaml``.  The
model is a Phi-3 decoder (``decoder.py`` Phi-3 spec: fused ``qkv_proj`` / ``gate_up_proj``,
LongRoPE, head_dim 96 zero-padded to the 128-wide attention tile) fed by the CLIP ViT-L/14-336
tower of ``llava.py`` through Phi-3-V's HD transform:

* preprocessing (``preprocess_phi3v``): transpose portrait images to landscape, scale so the
  width is ``s * 336`` with ``s * ceil(s / ratio) <= num_crops``, pad the height to a multiple of
  336 (centred, white), transpose back; CLIP mean / std; a bicubic 336x336 global view first,
  then the ``h x w`` 336-pixel crops row-major;
* features: hidden states of layer ``layer_idx`` (-2) without the class token, 2x2 patch
  merge (24x24x1024 -> 12x12x4096); the crops are stitched into one ``12h x 12w`` map; a learned
  ``sub_GN`` separator ends every row of both the crop map and the global map, and the learned
  ``glb_GN`` sits between them (``hd_transform_order: sub_glb``); projector
  Linear(4096, H) -> GELU -> Linear(H, H);
* prompt: every ``<|image_N|>`` placeholder (a negative id, as the Phi-3-V processor emits)
  becomes ``(h*w + 1) * 144 + 1 + (h + 1) * 12`` content-hash tokens carrying the features.
The whole vision path runs on the MFMA GEMMs and the varlen attention kernel of the CLIP tower;
only the 2x2 merge and separator splicing are tensor reshapes.  transformers has no Phi-3-V
class, so ``tests/test_phi3v_cpu.py`` checks against HF Phi3 + CLIP modules and an independent
reference of the HD assembly (the processor itself is parity unpinned).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ome_amd import ops
from ome_amd.models.config import ModelConfig
from ome_amd.models.decoder import DecoderForCausalLM
from ome_amd.models.llava import CLIP_L336, CLIPVisionTower
from ome_amd.models.quant import linear
from ome_amd.multimodal.inputs import CLIP_MEAN, CLIP_STD, MMInput, load_image, pad_token_id
from ome_amd.parallel import state as pstate

PHI3V_ARCHS = {"Phi3VForCausalLM"}


def hd_size(w: int, h: int, hd_num: int, crop: int = 336) -> tuple[int, int, int, int]:
    """(resized w, resized h, padded w, padded h) of Phi-3-V's HD transform."""
    trans = w < h
    if trans:
        w, h = h, w
    ratio = w / h
    scale = 1
    while scale * math.ceil(scale / ratio) <= hd_num:
        scale += 1
    scale -= 1
    nw = int(scale * crop)
    nh = int(nw / ratio)
    ph = int(math.ceil(nh / crop) * crop)
    return (nh, nw, ph, nw) if trans else (nw, nh, nw, ph)


def preprocess_phi3v(image, num_crops: int = 16, crop: int = 336) -> tuple[torch.Tensor, tuple[int, int, int]]:
    """-> (pixels float32 [1 + h*w, 3, crop, crop] (global view first), (1, h, w) crops)."""
    from PIL import Image

    img = load_image(image)
    nw, nh, pw, ph = hd_size(img.width, img.height, num_crops, crop)
    img = img.resize((nw, nh), Image.BILINEAR)
    canvas = Image.new("RGB", (pw, ph), (255, 255, 255))
    canvas.paste(img, ((pw - nw) // 2, (ph - nh) // 2))
    a = np.asarray(canvas, dtype=np.float32) / 255.0
    a = (a - np.asarray(CLIP_MEAN, np.float32)) / np.asarray(CLIP_STD, np.float32)
    hd = torch.from_numpy(np.ascontiguousarray(a.transpose(2, 0, 1)))          # [3, ph, pw]
    glob = torch.nn.functional.interpolate(hd[None], size=(crop, crop), mode="bicubic", align_corners=False)
    h, w = ph // crop, pw // crop
    crops = hd.reshape(3, h, crop, w, crop).permute(1, 3, 0, 2, 4).reshape(h * w, 3, crop, crop)
    return torch.cat([glob, crops], 0), (1, h, w)


def num_image_tokens(h: int, w: int, side: int = 12) -> int:
    """Tokens of one image with ``h x w`` crops (``side``: merged patches per crop edge)."""
    return h * side * (w * side + 1) + 1 + side * (side + 1)


class Phi3VForCausalLM(DecoderForCausalLM):
    is_multimodal = True

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        ex = cfg.extra or {}
        ip = ex.get("img_processor") or {}
        vc = {**CLIP_L336, **(ip.get("vision_config") or ex.get("vision_config") or {})}
        self.visual = CLIPVisionTower(vc, self.device, dtype, int(ip.get("layer_idx", -2)), "default")
        if self.visual.side % 2:
            raise NotImplementedError("Phi-3-V 2x2 merge needs an even patch grid")
        self.side = self.visual.side // 2
        self.num_crops = int(ex.get("num_crops", ip.get("num_crops", 16)))
        emb = ex.get("embd_layer") or {}
        if emb.get("hd_transform_order", "sub_glb") != "sub_glb":
            raise NotImplementedError(f"hd_transform_order {emb.get('hd_transform_order')!r}")
        self.proj: dict[str, torch.Tensor] = {}

    def init_random(self, seed: int = 0, std: float = 0.02) -> "Phi3VForCausalLM":
        super().init_random(seed, std)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 3301)
        self.visual.init_random(gen, std)
        H, C = self.cfg.hidden_size, 4 * self.visual.E
        mk = lambda *s: torch.empty(*s, dtype=self.dtype, device=self.device).normal_(0.0, std, generator=gen)  # noqa
        z = lambda n: torch.zeros(n, dtype=self.dtype, device=self.device)  # noqa: E731
        self.proj = {"w0": mk(H, C), "b0": z(H), "w2": mk(H, H), "b2": z(H), "glb": mk(C), "sub": mk(C)}
        return self

    _PROJ = {"img_projection.0.weight": "w0", "img_projection.0.bias": "b0", "img_projection.2.weight": "w2",
             "img_projection.2.bias": "b2", "glb_GN": "glb", "sub_GN": "sub"}

    def load_hf_weights(self, weights) -> "Phi3VForCausalLM":
        pend: dict = {}
        pre = "model.vision_embed_tokens."

        def text_only():
            for name, w in weights:
                if not name.startswith(pre):
                    yield name, w
                    continue
                n = name[len(pre):]
                if n.startswith("img_processor.vision_model."):
                    self.visual.load(n[len("img_processor.vision_model."):], w, pend)
                elif n in self._PROJ:
                    t = w.reshape(-1) if n.endswith("_GN") else w
                    self.proj[self._PROJ[n]] = t.to(device=self.device, dtype=self.dtype).contiguous()
                # wte.weight: a copy of the token embedding

        super().load_hf_weights(text_only())
        if pend:
            raise ValueError(f"incomplete vision q/k/v projections: {sorted(pend)}")
        return self

    def weight_bytes(self) -> int:
        n = super().weight_bytes() + sum(t.numel() * t.element_size() for t in self.visual.w.values())
        return n + sum(t.numel() * t.element_size() for t in self.proj.values())

    # ------------------------------------------------------------------ multimodal
    def image_prompt_ids(self) -> list[int]:
        return [-1]

    def make_mm_input(self, prompt_ids: list[int], images: list):
        where = [i for i, t in enumerate(prompt_ids) if t < 0]
        if len(where) != len(images):
            raise ValueError(f"prompt has {len(where)} image placeholders for {len(images)} images")
        ids, pvs, grids, spans, last = [], [], [], [], 0
        for i, im in zip(where, images):
            if isinstance(im, tuple):
                px, g = im
            else:
                px, g = preprocess_phi3v(im, self.num_crops, self.visual.image)
            n = num_image_tokens(g[1], g[2], self.side)
            ids += prompt_ids[last:i]
            spans.append((len(ids), n))
            ids += [pad_token_id(px, self.cfg.vocab_size)] * n
            pvs.append(px)
            grids.append(tuple(int(v) for v in g))
            last = i + 1
        ids += prompt_ids[last:]
        return ids, MMInput(torch.cat(pvs, 0), grids, spans)

    def _merge(self, f: torch.Tensor) -> torch.Tensor:
        """[N, side^2*4, C] per-crop patch features -> [N, s, s, 4C] (2x2 neighbourhoods concatenated)."""
        N, s, C = f.shape[0], self.side, self.visual.E
        return f.view(N, s, 2, s, 2, C).permute(0, 1, 3, 2, 4, 5).reshape(N, s, s, 4 * C)

    def encode_images(self, pixel_values: torch.Tensor, grids=None) -> torch.Tensor:
        p, s = self.proj, self.side
        C4 = 4 * self.visual.E
        feats = self.visual.forward(pixel_values).view(pixel_values.shape[0], -1, self.visual.E)
        out, off = [], 0
        for _, h, w in grids:
            f = self._merge(feats[off:off + 1 + h * w])
            off += 1 + h * w
            sub = f[1:].view(h, w, s, s, C4).permute(0, 2, 1, 3, 4).reshape(h * s, w * s, C4)
            sub = torch.cat([sub, p["sub"].view(1, 1, C4).expand(h * s, 1, C4)], 1).reshape(-1, C4)
            glb = torch.cat([f[0], p["sub"].view(1, 1, C4).expand(s, 1, C4)], 1).reshape(-1, C4)
            out += [sub, p["glb"].view(1, C4), glb]
        x = linear(torch.cat(out, 0).contiguous(), p["w0"], p["b0"])
        return linear(ops.act(x, 3), p["w2"], p["b2"])

    def embed_with_images(self, ids: torch.Tensor, rows: torch.Tensor, feats: torch.Tensor) -> torch.Tensor:
        h = pstate.tp_all_reduce(ops.embedding(ids, self.embed, self.tp.vocab_start, self.tp.vocab_end))
        if rows.numel():
            h.index_copy_(0, rows, feats.to(h.dtype))
        return h
