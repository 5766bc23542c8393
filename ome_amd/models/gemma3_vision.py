"""Gemma 3 with images (``Gemma3ForConditionalGeneration``: gemma-3-4b/12b/27b-it; reference
catalog ``config/runtimes/srt/google/gemma-3-27b-it-rt.yaml`` and its base model with
``IMAGE_TEXT_TO_TEXT``).

* preprocessing: resize to the tower's square input (896 px, bilinear), rescale, normalise with
  mean = std = 0.5 (SigLIP);
* prompt: each ``<start_of_image>`` of the prompt becomes ``\\n\\n <start_of_image>``
  + ``mm_tokens_per_image`` soft tokens + ``<end_of_image> \\n\\n`` (the reference processor's
  ``full_image_sequence``); the soft-token rows carry a content-hash id (prefix cache safety) and
  are overwritten with the projected features, which are NOT multiplied by the embedding
  normaliser (only token embeddings are);
* attention: the soft tokens of one image attend to each other bidirectionally
  (OR(causal, same image block), AND the sliding window on local layers) -- a per-row last
  visible key (``row_hi``) in the MFMA prefill kernels; the scheduler never splits an image block
  across prefill chunks (``MMInput.atomic``);
* vision tower: SigLIP -- patch conv as one GEMM (+bias), learned positions, ``depth`` pre-LN
  layers (LayerNorm -> fused QKV GEMM -> bidirectional varlen MFMA attention per image, head dim
  72 -> O GEMM; LayerNorm -> GELU-tanh MLP), post-LayerNorm; projector: 4 x 4 average pool to
  ``mm_tokens_per_image`` tokens, Gemma RMSNorm (1 + w), GEMM into the text hidden size.
The language model is :class:`ome_amd.models.gemma.GemmaForCausalLM` (Gemma 3 text) unchanged.
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.models.config import ModelConfig
from ome_amd.models.gemma import GemmaForCausalLM
from ome_amd.models.quant import linear
from ome_amd.multimodal.inputs import MMInput, load_image, pad_token_id
from ome_amd.parallel import state as pstate

NEWLINE2 = 108   # "\n\n" in the Gemma 3 tokenizer


def preprocess_gemma3(image, size: int = 896) -> torch.Tensor:
    """-> float32 [1, 3, size, size]."""
    from PIL import Image

    img = load_image(image).resize((size, size), Image.BILINEAR)
    a = (np.asarray(img, dtype=np.float32).transpose(2, 0, 1) / 255.0 - 0.5) / 0.5
    return torch.from_numpy(np.ascontiguousarray(a))[None]


class SiglipVisionTower:
    def __init__(self, vc: dict, device, dtype):
        self.device, self.dtype = device, dtype
        self.E = int(vc.get("hidden_size", 1152))
        self.heads = int(vc.get("num_attention_heads", 16))
        self.D = self.E // self.heads
        self.depth = int(vc.get("num_hidden_layers", 27))
        self.I = int(vc.get("intermediate_size", 4304))
        self.image = int(vc.get("image_size", 896))
        self.patch = int(vc.get("patch_size", 14))
        self.C = int(vc.get("num_channels", 3))
        self.eps = float(vc.get("layer_norm_eps", 1e-6))
        act = vc.get("hidden_act", "gelu_pytorch_tanh")
        self.act = {"gelu_pytorch_tanh": 1, "gelu": 3, "quick_gelu": None}.get(act, 1)
        self.side = self.image // self.patch
        self.n_patch = self.side ** 2
        self.w: dict[str, torch.Tensor] = {}

    def _t(self, t):
        return t.to(device=self.device, dtype=self.dtype).contiguous()

    def init_random(self, gen: torch.Generator, std: float = 0.02) -> None:
        E, I = self.E, self.I
        shapes = {"patch.weight": (E, self.C * self.patch ** 2), "patch.bias": (E,), "pos": (self.n_patch, E),
                  "post_ln.weight": (E,), "post_ln.bias": (E,)}
        for b in range(self.depth):
            p = f"layers.{b}."
            shapes.update({p + "qkv.weight": (3 * E, E), p + "qkv.bias": (3 * E,), p + "o.weight": (E, E),
                           p + "o.bias": (E,), p + "fc1.weight": (I, E), p + "fc1.bias": (I,), p + "fc2.weight": (E, I),
                           p + "fc2.bias": (E,), p + "ln1.weight": (E,), p + "ln1.bias": (E,), p + "ln2.weight": (E,),
                           p + "ln2.bias": (E,)})
        for k, s in shapes.items():
            t = torch.empty(*s, dtype=self.dtype, device=self.device)
            if k.endswith(("ln1.weight", "ln2.weight", "post_ln.weight")):
                t.fill_(1.0)
            elif len(s) == 1:
                t.zero_()
            else:
                t.normal_(0.0, std, generator=gen)
            self.w[k] = t

    _REN = {"self_attn.out_proj": "o", "mlp.fc1": "fc1", "mlp.fc2": "fc2", "layer_norm1": "ln1", "layer_norm2": "ln2"}

    def load(self, name: str, t: torch.Tensor, pend: dict) -> None:
        """``name`` relative to the tower (``embeddings.*``, ``encoder.layers.*``, ``post_layernorm.*``)."""
        if name.startswith("head."):
            return  # attention-pooling head: unused (the LM takes every patch)
        if name == "embeddings.patch_embedding.weight":
            self.w["patch.weight"] = self._t(t.reshape(t.shape[0], -1))
        elif name == "embeddings.patch_embedding.bias":
            self.w["patch.bias"] = self._t(t)
        elif name == "embeddings.position_embedding.weight":
            self.w["pos"] = self._t(t)
        elif name.startswith("post_layernorm."):
            self.w["post_ln." + name.split(".")[-1]] = self._t(t)
        elif name.startswith("encoder.layers."):
            parts = name.split(".")
            b, mod, kind = int(parts[2]), ".".join(parts[3:-1]), parts[-1]
            if mod in ("self_attn.q_proj", "self_attn.k_proj", "self_attn.v_proj"):
                got = pend.setdefault((b, kind), {})
                got[mod[-6]] = t
                if len(got) == 3:
                    self.w[f"layers.{b}.qkv.{kind}"] = self._t(torch.cat([got["q"], got["k"], got["v"]]))
                    del pend[(b, kind)]
                return
            self.w[f"layers.{b}.{self._REN[mod]}.{kind}"] = self._t(t)

    def forward(self, pixels: torch.Tensor, n_layers: int | None = None, post_norm: bool = True) -> torch.Tensor:
        """pixels [n, C, S, S] -> last hidden state [n, n_patch, E] (post-LayerNorm); ``n_layers`` /
        ``post_norm=False``: the hidden state after that many layers (LLaVA-OneVision features)."""
        w, E, n, ps, s = self.w, self.E, pixels.shape[0], self.patch, self.side
        x = pixels.to(device=self.device, dtype=self.dtype)
        x = x.reshape(n, self.C, s, ps, s, ps).permute(0, 2, 4, 1, 3, 5).reshape(n * self.n_patch, -1)
        x = (linear(x, w["patch.weight"], w["patch.bias"]).view(n, self.n_patch, E) + w["pos"]).reshape(-1, E)
        return self.encode(x, [self.n_patch] * n, n_layers, post_norm).view(n, self.n_patch, E)

    def encode(self, x: torch.Tensor, lens: list[int], n_layers: int | None = None,
               post_norm: bool = True) -> torch.Tensor:
        """Encoder layers over packed embeddings x [T, E] of sequences of lengths ``lens``
        (bidirectional varlen MFMA attention per sequence) -> [T, E]."""
        w, E, T = self.w, self.E, x.shape[0]
        for b in range(self.depth if n_layers is None else n_layers):
            p = f"layers.{b}."
            h = ops.layernorm(x.contiguous(), w[p + "ln1.weight"], w[p + "ln1.bias"], self.eps)
            qkv = linear(h, w[p + "qkv.weight"], w[p + "qkv.bias"]).view(T, 3, self.heads, self.D)
            a = ops.varlen_attention(qkv[:, 0], qkv[:, 1], qkv[:, 2], lens, self.D ** -0.5).reshape(T, E)
            x = x + linear(a, w[p + "o.weight"], w[p + "o.bias"])
            h = ops.layernorm(x, w[p + "ln2.weight"], w[p + "ln2.bias"], self.eps)
            f = linear(h, w[p + "fc1.weight"], w[p + "fc1.bias"])
            f = ops.act(f, self.act) if self.act is not None else f * torch.sigmoid(1.702 * f)
            x = x + linear(f, w[p + "fc2.weight"], w[p + "fc2.bias"])
        if not post_norm:
            return x
        return ops.layernorm(x, w["post_ln.weight"], w["post_ln.bias"], self.eps)


class Gemma3ForConditionalGeneration(GemmaForCausalLM):
    is_multimodal = True
    bidirectional_images = True

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        ex = cfg.extra or {}
        self.visual = SiglipVisionTower(ex.get("vision_config") or {}, self.device, dtype)
        self.mm_tokens = int(ex.get("mm_tokens_per_image", 256))
        self.tok_side = int(round(math.sqrt(self.mm_tokens)))
        self.pool = self.visual.side // self.tok_side
        self.image_id = int(ex.get("image_token_index", ex.get("image_token_id", 262144)))
        self.boi_id = int(ex.get("boi_token_index", 255999))
        self.eoi_id = int(ex.get("eoi_token_index", 256000))
        self.nl2 = int(ex.get("image_newline_token_id", NEWLINE2))
        self.proj_w = self.proj_norm = None   # [H_text, E_vision] (GEMM layout), Gemma RMSNorm (1 + w folded)

    def init_random(self, seed: int = 0, std: float = 0.02) -> "Gemma3ForConditionalGeneration":
        super().init_random(seed, std)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 4451)
        self.visual.init_random(gen, std)
        E = self.visual.E
        self.proj_w = torch.empty(self.cfg.hidden_size, E, dtype=self.dtype, device=self.device).normal_(
            0.0, std, generator=gen)
        self.proj_norm = torch.ones(E, dtype=self.dtype, device=self.device)
        return self

    def load_hf_weights(self, weights) -> "Gemma3ForConditionalGeneration":
        pend: dict = {}

        def text_only():
            for name, w in weights:
                for pre in ("model.vision_tower.vision_model.", "vision_tower.vision_model.", "model.vision_tower.",
                            "vision_tower."):
                    if name.startswith(pre):
                        self.visual.load(name[len(pre):], w, pend)
                        break
                else:
                    if name.endswith("multi_modal_projector.mm_input_projection_weight"):
                        self.proj_w = w.t().to(device=self.device, dtype=self.dtype).contiguous()
                    elif name.endswith("multi_modal_projector.mm_soft_emb_norm.weight"):
                        self.proj_norm = (w.float() + 1.0).to(device=self.device, dtype=self.dtype)
                    else:
                        yield name, w

        super().load_hf_weights(text_only())
        if pend:
            raise ValueError(f"incomplete vision q/k/v projections: {sorted(pend)}")
        return self

    def weight_bytes(self) -> int:
        n = super().weight_bytes() + sum(t.numel() * t.element_size() for t in self.visual.w.values())
        return n + sum(t.numel() * t.element_size() for t in (self.proj_w, self.proj_norm) if t is not None)

    # ------------------------------------------------------------------ multimodal
    def image_prompt_ids(self) -> list[int]:
        return [self.boi_id]

    def make_mm_input(self, prompt_ids: list[int], images: list):
        where = [i for i, t in enumerate(prompt_ids) if t == self.boi_id]
        if len(where) != len(images):
            raise ValueError(f"prompt has {len(where)} <start_of_image> tokens for {len(images)} images")
        ids, pvs, spans, last = [], [], [], 0
        for i, im in zip(where, images):
            px = im if isinstance(im, torch.Tensor) else preprocess_gemma3(im, self.visual.image)
            tok = pad_token_id(px, self.cfg.vocab_size)
            ids += prompt_ids[last:i] + [self.nl2, self.boi_id]
            spans.append((len(ids), self.mm_tokens))
            ids += [tok] * self.mm_tokens + [self.eoi_id, self.nl2]
            pvs.append(px)
            last = i + 1
        ids += prompt_ids[last:]
        # atomic: bidirectional image blocks are never split across prefill chunks
        return ids, MMInput(torch.cat(pvs, 0), [(1, self.visual.side, self.visual.side)] * len(pvs), spans,
                            atomic=True)

    def encode_images(self, pixel_values: torch.Tensor, grids=None) -> torch.Tensor:
        h = self.visual.forward(pixel_values)                                   # [n, P, E]
        n, E, s, k = h.shape[0], self.visual.E, self.visual.side, self.pool
        h = h.transpose(1, 2).reshape(n, E, s, s).float()
        h = F.avg_pool2d(h, k, k).flatten(2).transpose(1, 2).reshape(-1, E).to(self.dtype).contiguous()
        h = ops.rmsnorm(h, self.proj_norm, self.visual.eps)
        return linear(h, self.proj_w)

    def embed_with_images(self, ids: torch.Tensor, rows: torch.Tensor, feats: torch.Tensor) -> torch.Tensor:
        h = pstate.tp_all_reduce(ops.embedding(ids, self.embed, self.tp.vocab_start, self.tp.vocab_end))
        h = h * self.normalizer
        if rows.numel():
            h.index_copy_(0, rows, feats.to(h.dtype))
        return h
