"""Janus / Janus-Pro image understanding (reference catalog ``config/runtimes/srt/deepseek-ai/
janus-pro-7b-rt.yaml``: ``JanusMultiModalityCausalLM``; original ``MultiModalityCausalLM``
checkpoints and the transformers ``JanusForConditionalGeneration`` layout).

* preprocessing: longest side -> 384 (bicubic, sides floored at 14 px), pad to a square with the
  mean colour, rescale, mean / std (0.5 for Janus-Pro);
* prompt: each image placeholder becomes ``<begin_of_image>`` + 576 image tokens (content-hash
  ids) + ``<end_of_image>``;
* SigLIP-L/16 tower (the ``gemma3_vision.py`` tower: patch GEMM, learned positions, LayerNorm
  blocks with fused QKV GEMM on the varlen MFMA kernel, exact-GELU MLP, post-LayerNorm), then
  the aligner MLP (GEMM -> GELU -> GEMM) into the Llama language model of ``llama.py``.
The image-GENERATION half of Janus (VQ tokenizer, generation head) is not served -- the
reference runtime serves image understanding (text output) only.
"""
from __future__ import annotations

import torch

from ome_amd import ops
from ome_amd.models.config import ModelConfig
from ome_amd.models.gemma3_vision import SiglipVisionTower
from ome_amd.models.llama import LlamaForCausalLM
from ome_amd.models.quant import linear
from ome_amd.multimodal.inputs import MMInput, load_image, pad_token_id
from ome_amd.parallel import state as pstate

JANUS_ARCHS = {"JanusForConditionalGeneration", "MultiModalityCausalLM", "JanusMultiModalityCausalLM"}
# SigLIP-L/16-384 of the original checkpoints (their vision config only names the timm model)
SIGLIP_L16_384 = dict(hidden_size=1024, intermediate_size=4096, num_hidden_layers=24, num_attention_heads=16,
                      image_size=384, patch_size=16, hidden_act="gelu", layer_norm_eps=1e-6)


def preprocess_janus(image, size: int = 384, mean=(0.5, 0.5, 0.5), std=(0.5, 0.5, 0.5), min_size: int = 14):
    """-> float32 [1, 3, size, size]."""
    import numpy as np
    from PIL import Image

    img = load_image(image)
    w, h = img.size
    d = size / max(w, h)
    nw, nh = max(round(w * d), min_size), max(round(h * d), min_size)
    img = img.resize((nw, nh), Image.BICUBIC)
    a = np.asarray(img, dtype=np.float32)
    side = max(nw, nh)
    bg = np.empty((side, side, 3), dtype=np.float32)
    bg[:] = np.asarray([int(x * 255) for x in mean], np.float32)
    if nw > nh:
        top = (side - nh) // 2
        bg[top:top + nh, :] = a
    else:
        left = (side - nw) // 2
        bg[:, left:left + nw] = a
    bg = (bg / 255.0 - np.asarray(mean, np.float32)) / np.asarray(std, np.float32)
    return torch.from_numpy(np.ascontiguousarray(bg.transpose(2, 0, 1)))[None]


class JanusVisionTower(SiglipVisionTower):
    _REN = {**SiglipVisionTower._REN, "self_attn.projection_layer": "o"}

    def load(self, name: str, t: torch.Tensor, pend: dict) -> None:
        """transformers names (``embeddings.*``, ``encoder.layers.*``, ``post_layernorm.*``) or the
        timm names of the original checkpoints (``patch_embed.*``, ``pos_embed``, ``blocks.*``, ``norm.*``)."""
        if name.startswith(("attn_pool.", "head.")):
            return
        if name.startswith("patch_embed.proj."):
            name = "embeddings.patch_embedding." + name.split(".")[-1]
        elif name == "pos_embed":
            self.w["pos"] = self._t(t.reshape(-1, t.shape[-1]))
            return
        elif name.startswith("norm."):
            name = "post_layernorm." + name.split(".")[-1]
        elif name.startswith("blocks."):
            p = name.split(".")
            b, mod, kind = p[1], ".".join(p[2:-1]), p[-1]
            if mod == "attn.qkv":
                self.w[f"layers.{b}.qkv.{kind}"] = self._t(t)
                return
            mod = {"attn.proj": "self_attn.out_proj", "norm1": "layer_norm1", "norm2": "layer_norm2"}.get(mod, mod)
            name = f"encoder.layers.{b}.{mod}.{kind}"
        super().load(name, t, pend)


class JanusForConditionalGeneration(LlamaForCausalLM):
    is_multimodal = True

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        ex = cfg.extra or {}
        self.orig = cfg.architecture != "JanusForConditionalGeneration"
        vc = dict(ex.get("vision_config") or {})
        if self.orig:
            params = vc.get("params") or {}
            vc = {**SIGLIP_L16_384, "image_size": int(params.get("image_size", 384))}
            ap = (ex.get("aligner_config") or {}).get("params") or {}
            self.aligner_depth = int(ap.get("depth", 2))
        else:
            vc.setdefault("intermediate_size", int(vc.get("hidden_size", 1024) * float(vc.get("mlp_ratio", 4.0))))
            self.aligner_depth = int(vc.get("depth", 2))
        self.visual = JanusVisionTower(vc, self.device, dtype)
        self.n_tokens = self.visual.n_patch
        self.image_id = int(ex.get("image_token_id", ex.get("image_token_index", 100581)))
        self.boi = int(ex.get("boi_token_id", 100016))
        self.eoi = int(ex.get("eoi_token_id", 100593))
        self.mean = tuple(ex.get("image_mean") or (0.5, 0.5, 0.5))
        self.std = tuple(ex.get("image_std") or (0.5, 0.5, 0.5))
        self.align: list[tuple[torch.Tensor, torch.Tensor | None]] = []

    def init_random(self, seed: int = 0, std: float = 0.02) -> "JanusForConditionalGeneration":
        super().init_random(seed, std)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 4493)
        self.visual.init_random(gen, std)
        H, E = self.cfg.hidden_size, self.visual.E
        mk = lambda *s: torch.empty(*s, dtype=self.dtype, device=self.device).normal_(0.0, std, generator=gen)  # noqa
        z = torch.zeros(H, dtype=self.dtype, device=self.device)
        self.align = [(mk(H, E), z)] + [(mk(H, H), z) for _ in range(1, self.aligner_depth)]
        return self

    def load_hf_weights(self, weights) -> "JanusForConditionalGeneration":
        pend: dict = {}
        al: dict[int, dict[str, torch.Tensor]] = {}

        def lm_only():
            for name, w in weights:
                n = name[len("model."):] if name.startswith("model.") and not self.orig else name
                if n.startswith("vision_model.vision_tower."):          # original
                    self.visual.load(n[len("vision_model.vision_tower."):], w, pend)
                elif n.startswith("vision_model."):                      # transformers
                    self.visual.load(n[len("vision_model."):], w, pend)
                elif n.startswith("aligner."):
                    p = n.split(".")
                    if p[1] == "fc1":                                    # transformers: fc1, hidden_layers.k
                        idx = 0
                    elif p[1] == "hidden_layers":
                        idx = int(p[2]) + 1
                    else:                                                # original: layers.0, layers.2, ...
                        idx = int(p[2]) // 2
                    al.setdefault(idx, {})[p[-1]] = w.to(device=self.device, dtype=self.dtype).contiguous()
                elif n.startswith("language_model."):
                    rest = n[len("language_model."):]
                    yield (rest if rest.startswith(("model.", "lm_head.")) else "model." + rest), w
                elif n.startswith(("gen_", "generation_", "vqmodel.")) or ".gen_" in n:
                    continue                                             # image-generation half: not served
                else:
                    yield name, w

        super().load_hf_weights(lm_only())
        if pend:
            raise ValueError(f"incomplete vision projections: {sorted(pend)}")
        self.align = [(al[i]["weight"], al[i].get("bias")) for i in sorted(al)]
        return self

    def weight_bytes(self) -> int:
        n = super().weight_bytes() + sum(t.numel() * t.element_size() for t in self.visual.w.values())
        return n + sum(w.numel() * w.element_size() for w, _ in self.align)

    # ------------------------------------------------------------------ multimodal
    def image_prompt_ids(self) -> list[int]:
        return [self.boi, self.image_id, self.eoi]

    def make_mm_input(self, prompt_ids: list[int], images: list):
        where = [i for i, t in enumerate(prompt_ids) if t == self.image_id]
        if len(where) != len(images):
            raise ValueError(f"prompt has {len(where)} image tokens for {len(images)} images")
        ids, pvs, spans, last = [], [], [], 0
        for i, im in zip(where, images):
            px = im if isinstance(im, torch.Tensor) else preprocess_janus(im, self.visual.image, self.mean, self.std)
            ids += prompt_ids[last:i]
            spans.append((len(ids), self.n_tokens))
            ids += [pad_token_id(px, self.cfg.vocab_size)] * self.n_tokens
            pvs.append(px)
            last = i + 1
        ids += prompt_ids[last:]
        return ids, MMInput(torch.cat(pvs, 0), [(1, self.visual.side, self.visual.side)] * len(pvs), spans)

    def encode_images(self, pixel_values: torch.Tensor, grids=None) -> torch.Tensor:
        x = self.visual.forward(pixel_values).reshape(-1, self.visual.E)
        for k, (w, b) in enumerate(self.align):
            if k:
                x = ops.act(x, 3)
            x = linear(x, w, b)
        return x

    def embed_with_images(self, ids: torch.Tensor, rows: torch.Tensor, feats: torch.Tensor) -> torch.Tensor:
        h = pstate.tp_all_reduce(ops.embedding(ids, self.embed, self.tp.vocab_start, self.tp.vocab_end))
        if rows.numel():
            h.index_copy_(0, rows, feats.to(h.dtype))
        return h
