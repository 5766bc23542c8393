"""CLIP as an embedding model (``CLIPModel``: reference catalog
``config/runtimes/srt/openai/clip-vit-large-patch14-336-rt.yaml``): text and image embeddings in
one joint space, served through ``/v1/embeddings`` (text inputs, and ``{"image": <data URL>}``
items).

* text: token + absolute position embeddings, encoder layers with CAUSAL attention (the varlen
  MFMA kernel's causal mode over the packed prompts), final LayerNorm, the row of the first EOS
  token (the highest id for legacy configs with ``eos_token_id == 2``), ``text_projection``;
* image: the CLIP tower of ``llava.py`` run to the last layer, class token -> post-LayerNorm ->
  ``visual_projection``;
* embeddings are L2-normalised (cosine-ready, like the other embedders here).
Encoder-only: no KV cache, no decode graphs.
"""
from __future__ import annotations

import math

import torch

from ome_amd import ops
from ome_amd.models.common import AttnMeta, PagedKVCache
from ome_amd.models.config import ModelConfig
from ome_amd.models.llava import CLIPVisionTower, preprocess_clip
from ome_amd.models.quant import linear
from ome_amd.multimodal.inputs import MMInput


class _TP:
    def __init__(self, heads: int, vocab: int):
        self.tp, self.rank, self.hq, self.hkv = 1, 0, heads, heads
        self.vocab, self.vocab_start, self.vocab_end = vocab, 0, vocab


class CLIPModel:
    encoder_only = True
    tune_gemms = False
    is_multimodal = True
    mm_cross = True   # images are consumed whole by the embed path (no placeholder rows to splice)

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        ex = cfg.extra or {}
        self.cfg, self.device, self.dtype = cfg, torch.device(device), dtype
        # the text config's keys are merged into ``extra`` (ModelConfig.from_hf); vision stays nested
        tc, vc = ex.get("text_config") or ex, ex.get("vision_config") or {}
        self.E = int(tc.get("hidden_size", 768))
        self.heads = int(tc.get("num_attention_heads", 12))
        self.D = self.E // self.heads
        self.depth = int(tc.get("num_hidden_layers", 12))
        self.I = int(tc.get("intermediate_size", 3072))
        self.V = int(tc.get("vocab_size", 49408))
        self.max_pos = int(tc.get("max_position_embeddings", 77))
        self.eps = float(tc.get("layer_norm_eps", 1e-5))
        self.quick = tc.get("hidden_act", "quick_gelu") == "quick_gelu"
        self.eos = int(tc.get("eos_token_id", 2))
        self.proj_dim = int(vc.get("projection_dim") or ex.get("projection_dim") or 512)
        self.tp = _TP(self.heads, self.V)
        self.layers = list(range(self.depth))
        self.kv_layers: list[int] = []
        vdepth = int(vc.get("num_hidden_layers", 24))
        self.visual = CLIPVisionTower(vc, self.device, dtype, feature_layer=vdepth, strategy="full")
        self.w: dict[str, torch.Tensor] = {}

    def _t(self, t):
        return t.to(device=self.device, dtype=self.dtype).contiguous()

    # ------------------------------------------------------------------ weights
    def init_random(self, seed: int = 0, std: float = 0.02) -> "CLIPModel":
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed)
        E, I, P = self.E, self.I, self.proj_dim
        shapes = {"tok": (self.V, E), "pos": (self.max_pos, E), "final_ln.weight": (E,), "final_ln.bias": (E,),
                  "text_proj": (P, E), "visual_proj": (P, self.visual.E), "post_ln.weight": (self.visual.E,),
                  "post_ln.bias": (self.visual.E,)}
        for b in self.layers:
            p = f"layers.{b}."
            shapes.update({p + "qkv.weight": (3 * E, E), p + "qkv.bias": (3 * E,), p + "o.weight": (E, E),
                           p + "o.bias": (E,), p + "fc1.weight": (I, E), p + "fc1.bias": (I,), p + "fc2.weight": (E, I),
                           p + "fc2.bias": (E,), p + "ln1.weight": (E,), p + "ln1.bias": (E,), p + "ln2.weight": (E,),
                           p + "ln2.bias": (E,)})
        for k, s in shapes.items():
            t = torch.empty(*s, dtype=self.dtype, device=self.device)
            if k.endswith(("ln1.weight", "ln2.weight", "final_ln.weight", "post_ln.weight")):
                t.fill_(1.0)
            elif len(s) == 1:
                t.zero_()
            else:
                t.normal_(0.0, std, generator=gen)
            self.w[k] = t
        self.visual.init_random(gen, std)
        return self

    _REN = {"self_attn.out_proj": "o", "mlp.fc1": "fc1", "mlp.fc2": "fc2", "layer_norm1": "ln1", "layer_norm2": "ln2"}

    def load_hf_weights(self, weights) -> "CLIPModel":
        tpend, vpend = {}, {}
        for name, t in weights:
            n = name[len("model."):] if name.startswith("model.") else name
            if n.startswith("vision_model."):
                r = n[len("vision_model."):]
                if r.startswith("post_layernorm."):
                    self.w["post_ln." + r.split(".")[-1]] = self._t(t)
                else:
                    self.visual.load(r, t, vpend)
            elif n == "visual_projection.weight":
                self.w["visual_proj"] = self._t(t)
            elif n == "text_projection.weight":
                self.w["text_proj"] = self._t(t)
            elif n.startswith("text_model."):
                r = n[len("text_model."):]
                if r == "embeddings.token_embedding.weight":
                    self.w["tok"] = self._t(t)
                elif r == "embeddings.position_embedding.weight":
                    self.w["pos"] = self._t(t)
                elif r.startswith("final_layer_norm."):
                    self.w["final_ln." + r.split(".")[-1]] = self._t(t)
                elif r.startswith("encoder.layers."):
                    parts = r.split(".")
                    b, mod, kind = int(parts[2]), ".".join(parts[3:-1]), parts[-1]
                    if mod in ("self_attn.q_proj", "self_attn.k_proj", "self_attn.v_proj"):
                        got = tpend.setdefault((b, kind), {})
                        got[mod[-6]] = t
                        if len(got) == 3:
                            self.w[f"layers.{b}.qkv.{kind}"] = self._t(torch.cat([got["q"], got["k"], got["v"]]))
                            del tpend[(b, kind)]
                    else:
                        self.w[f"layers.{b}.{self._REN[mod]}.{kind}"] = self._t(t)
        if tpend or vpend:
            raise ValueError("incomplete CLIP q/k/v projections")
        return self

    def weight_bytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in list(self.w.values()) + list(self.visual.w.values()))

    # ------------------------------------------------------------------ text
    def forward(self, ids: torch.Tensor, meta: AttnMeta, kv: PagedKVCache | None = None) -> torch.Tensor:
        lengths = meta.extra.get("lengths")
        if lengths is None:
            cu = meta.cu_q.tolist()
            lengths = [b - a for a, b in zip(cu[:-1], cu[1:])]
        w, E = self.w, self.E
        self._ids = ids
        x = (w["tok"][ids.long()] + w["pos"][meta.positions.long()]).contiguous()
        T = x.shape[0]
        for b in self.layers:
            p = f"layers.{b}."
            h = ops.layernorm(x, w[p + "ln1.weight"], w[p + "ln1.bias"], self.eps)
            qkv = linear(h, w[p + "qkv.weight"], w[p + "qkv.bias"]).view(T, 3, self.heads, self.D)
            a = ops.varlen_attention(qkv[:, 0], qkv[:, 1], qkv[:, 2], lengths, self.D ** -0.5, causal=True)
            x = x + linear(a.reshape(T, E), w[p + "o.weight"], w[p + "o.bias"])
            h = ops.layernorm(x, w[p + "ln2.weight"], w[p + "ln2.bias"], self.eps)
            f = linear(h, w[p + "fc1.weight"], w[p + "fc1.bias"])
            f = f * torch.sigmoid(1.702 * f) if self.quick else ops.act(f, 3)
            x = x + linear(f, w[p + "fc2.weight"], w[p + "fc2.bias"])
        return ops.layernorm(x, w["final_ln.weight"], w["final_ln.bias"], self.eps)

    def pool(self, hidden: torch.Tensor, cu: torch.Tensor) -> torch.Tensor:
        ids, rows = self._ids, []
        for s, (a, b) in enumerate(zip(cu[:-1].tolist(), cu[1:].tolist())):
            seq = ids[a:b]
            if self.eos == 2:   # legacy configs: the EOT token is the highest id
                rows.append(a + int(seq.argmax()))
            else:
                hit = (seq == self.eos).nonzero()
                rows.append(a + (int(hit[0]) if hit.numel() else b - a - 1))
        pooled = hidden.index_select(0, torch.tensor(rows, device=hidden.device))
        e = linear(pooled, self.w["text_proj"]).float()
        return torch.nn.functional.normalize(e, dim=-1)

    # ------------------------------------------------------------------ images
    def make_mm_input(self, prompt_ids: list[int], images: list):
        if len(images) != 1:
            raise ValueError("one image per CLIP embedding request")
        im = images[0]
        px = im if isinstance(im, torch.Tensor) else preprocess_clip(im, self.visual.image)
        return [self.eos], MMInput(px, [(1, self.visual.side, self.visual.side)], [])

    def embed_images(self, pixel_values: torch.Tensor) -> torch.Tensor:
        n, L = pixel_values.shape[0], self.visual.tokens
        h = self.visual.forward(pixel_values).view(n, L, -1)[:, 0].contiguous()   # class token
        h = ops.layernorm(h, self.w["post_ln.weight"], self.w["post_ln.bias"], self.visual.eps)
        return torch.nn.functional.normalize(linear(h, self.w["visual_proj"]).float(), dim=-1)
