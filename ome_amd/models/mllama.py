"""Llama 3.2 Vision (``MllamaForConditionalGeneration``) on the ome_amd kernels.

Reference catalog: ten ClusterServingRuntimes serve this architecture through SGLang
(``config/runtimes/srt/meta/llama-3-2-11b-vision-instruct-rt.yaml``, the 90B variants, ...).

Language model: a Llama decoder whose ``cross_attention_layers`` are tanh-gated cross-attention
blocks over the request's vision tokens.  Self-attention layers run the Llama path unchanged
(fused RoPE + paged KV, MFMA paged attention); only they own paged KV pages (``kv_layers``).
A cross layer: ``h += tanh(g_attn) * O(attn(q_norm(Q(norm1 h)), vision K/V))`` then
``h += tanh(g_mlp) * mask_row * MLP(norm2 h)``.

Vision tokens live in a model-owned paged cache (one K/V page pool per cross layer, the same
[pages, Hkv, 16, D] / [pages, Hkv, D, 16] layouts as the self-attention cache) filled once per
request, at its first prefill chunk: vision tower -> projector -> per cross layer K (with
k_norm) / V -> ``ome_kv_cache_write``.  Real tiles of all images are stored first, padding tiles
after, so every text row's visible set (``multimodal/mllama.py``: its image group, or for rows
before the first image *all* vision tokens) is one key range [lo, hi); cross attention is then
the GQA paged *decode* kernel with one query row per text token and a per-row first key
(``row_lo``) -- the same kernel for prefill rows, decode rows and HIP-graph decode.  Per-slot
range tables on the device map (request slot, position) -> (lo, hi, gates), so decode graphs
need no host input beyond the request slots they already carry.  Text-only requests get a zero
range and zero gates (the cross layer is an identity for them, as in HF where it is skipped).

Vision tower (run once per image): Conv2d patch embedding as a GEMM over unfolded patches,
gated pre / post tile-aspect embeddings, gated position + tile-position embeddings, a local
encoder (its intermediate layers concatenated to the output) and a tanh-gated global encoder;
LayerNorms on ``ome_layernorm``, GEMMs on hipBLASLt, bidirectional attention on PyTorch SDPA
with the Mllama padding mask (a query/key pair is masked only when both are padding).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.models.common import AttnMeta, PagedKVCache
from ome_amd.models.config import ModelConfig
from ome_amd.models.llama import LlamaForCausalLM
from ome_amd.models.quant import dequant_fp8_stream, linear
from ome_amd.parallel import state as pstate

MLLAMA_ARCHS = {"MllamaForConditionalGeneration"}
P_CACHE = 16


def _vcfg(cfg: ModelConfig) -> dict:
    return (cfg.extra or {}).get("vision_config") or {}


class MllamaVision:
    """Vision tower + multi-modal projector (weights as a flat dict of tensors)."""

    def __init__(self, vc: dict, out_dim: int, device, dtype):
        self.C = int(vc.get("hidden_size", 1280))
        self.heads = int(vc.get("attention_heads", 16))
        self.tile = int(vc.get("image_size", 560))
        self.patch = int(vc.get("patch_size", 14))
        self.max_tiles = int(vc.get("max_num_tiles", 4))
        self.L = int(vc.get("num_hidden_layers", 32))
        self.Lg = int(vc.get("num_global_layers", 8))
        self.inter_idx = list(vc.get("intermediate_layers_indices", [3, 7, 15, 23, 30]))
        self.I = int(vc.get("intermediate_size", 5120))
        self.eps = float(vc.get("norm_eps", 1e-5))
        self.act = {"gelu": 3, "gelu_pytorch_tanh": 1, "gelu_new": 1, "quick_gelu": 6}.get(vc.get("hidden_act", "gelu"), 3)
        self.P = (self.tile // self.patch) ** 2 + 1       # patches + class token per tile
        self.Pp = self.P + (8 - self.P % 8) % 8           # padded to a multiple of 8
        self.out_dim = out_dim
        self.device, self.dtype = device, dtype
        self.w: dict[str, torch.Tensor] = {}

    def init_random(self, gen, std: float = 0.02) -> None:
        C, I, mt = self.C, self.I, self.max_tiles
        r = lambda *s, sd=std: (torch.randn(*s, generator=gen, device=self.device) * sd).to(self.dtype)  # noqa: E731
        one = lambda n: torch.ones(n, dtype=self.dtype, device=self.device)  # noqa: E731
        zero = lambda n: torch.zeros(n, dtype=self.dtype, device=self.device)  # noqa: E731
        w = self.w
        w["patch"] = r(C, 3 * self.patch * self.patch)
        w["cls"] = r(C)
        w["pos"], w["pos_gate"], w["tile_pos"] = r(self.P, C), torch.zeros(1, device=self.device), r(9, mt * self.P * C)
        for k in ("pre", "post"):
            w[f"{k}_tile"], w[f"{k}_gate"] = r(9, mt * C), torch.zeros(1, device=self.device)
        for k in ("ln_pre", "ln_post"):
            w[f"{k}.w"], w[f"{k}.b"] = one(C), zero(C)
        for enc, n in (("t", self.L), ("g", self.Lg)):
            for i in range(n):
                p = f"{enc}{i}."
                w[p + "qkv"] = r(3 * C, C)
                w[p + "o"] = r(C, C)
                w[p + "ln1.w"], w[p + "ln1.b"], w[p + "ln2.w"], w[p + "ln2.b"] = one(C), zero(C), one(C), zero(C)
                w[p + "fc1.w"], w[p + "fc1.b"], w[p + "fc2.w"], w[p + "fc2.b"] = r(I, C), zero(I), r(C, I), zero(C)
                if enc == "g":
                    w[p + "gate_attn"] = torch.full((1,), math.pi / 4, device=self.device)
                    w[p + "gate_ffn"] = torch.full((1,), math.pi / 4, device=self.device)
        k_in = C * (len(self.inter_idx) + 1)
        w["proj.w"], w["proj.b"] = r(self.out_dim, k_in), zero(self.out_dim)

    def load(self, name: str, t: torch.Tensor) -> bool:
        """Checkpoint name (``vision_model.*`` / ``multi_modal_projector.*``) -> internal key."""
        put = lambda x: x.to(device=self.device, dtype=self.dtype).contiguous()  # noqa: E731
        w = self.w
        if name.startswith("multi_modal_projector."):
            w["proj.w" if name.endswith("weight") else "proj.b"] = put(t)
            return True
        if not name.startswith("vision_model."):
            return False
        n = name[len("vision_model."):]
        simple = {"class_embedding": "cls", "gated_positional_embedding.embedding": "pos",
                  "gated_positional_embedding.tile_embedding.weight": "tile_pos",
                  "pre_tile_positional_embedding.embedding.weight": "pre_tile",
                  "post_tile_positional_embedding.embedding.weight": "post_tile",
                  "layernorm_pre.weight": "ln_pre.w", "layernorm_pre.bias": "ln_pre.b",
                  "layernorm_post.weight": "ln_post.w", "layernorm_post.bias": "ln_post.b"}
        gates = {"gated_positional_embedding.gate": "pos_gate", "pre_tile_positional_embedding.gate": "pre_gate",
                 "post_tile_positional_embedding.gate": "post_gate"}
        if n in simple:
            w[simple[n]] = put(t)
        elif n in gates:
            w[gates[n]] = t.float().to(self.device)
        elif n == "patch_embedding.weight":
            w["patch"] = put(t.reshape(t.shape[0], -1))
        elif n.startswith(("transformer.layers.", "global_transformer.layers.")):
            enc = "t" if n.startswith("transformer.") else "g"
            rest = n.split("layers.", 1)[1]
            i, sub = rest.split(".", 1)
            p = f"{enc}{i}."
            m = {"input_layernorm.weight": "ln1.w", "input_layernorm.bias": "ln1.b",
                 "post_attention_layernorm.weight": "ln2.w", "post_attention_layernorm.bias": "ln2.b",
                 "mlp.fc1.weight": "fc1.w", "mlp.fc1.bias": "fc1.b", "mlp.fc2.weight": "fc2.w", "mlp.fc2.bias": "fc2.b",
                 "self_attn.o_proj.weight": "o"}
            if sub in m:
                w[p + m[sub]] = put(t)
            elif sub in ("gate_attn", "gate_ffn"):
                w[p + sub] = t.float().to(self.device)
            elif sub.startswith("self_attn.") and sub.endswith("_proj.weight"):
                w.setdefault(p + "_qkv", {})[sub[10]] = t
                parts = w[p + "_qkv"]
                if len(parts) == 3:
                    w[p + "qkv"] = put(torch.cat([parts["q"], parts["k"], parts["v"]], 0))
                    del w[p + "_qkv"]
        else:
            return False
        return True

    # ------------------------------------------------------------------ forward
    def _ln(self, x, k):
        return ops.layernorm(x.contiguous(), self.w[k + ".w"], self.w[k + ".b"], self.eps)

    def _layer(self, p: str, x: torch.Tensor, mask, gated: bool) -> torch.Tensor:
        """``mask`` = (pad_rows, real_rows, pad counts, real counts): a (query, key) pair is masked
        only when both are padding, i.e. real queries see every key of their image and padding
        queries see the image's real keys -- two varlen launches (self, then cross lengths for
        the padding rows) instead of a dense [S, S] bias."""
        n, S, C = x.shape
        w, h = self.w, self.heads
        D = C // h
        qkv = linear(self._ln(x, p + "ln1").view(n * S, C), w[p + "qkv"]).view(n * S, 3, h, D)
        a = ops.varlen_attention(qkv[:, 0], qkv[:, 1], qkv[:, 2], [S] * n, D ** -0.5)
        pad_rows, real_rows, n_pad, n_real = mask
        if pad_rows.numel():
            q = qkv[:, 0].index_select(0, pad_rows)
            kv = qkv[:, 1:].index_select(0, real_rows)
            a.index_copy_(0, pad_rows, ops.varlen_attention(q, kv[:, 0], kv[:, 1], n_pad, D ** -0.5,
                                                            k_lengths=n_real))
        a = linear(a.reshape(n * S, C), w[p + "o"]).view(n, S, C)
        x = x + (torch.tanh(w[p + "gate_attn"]).to(x.dtype) * a if gated else a)
        m = linear(self._ln(x, p + "ln2").view(n * S, C), w[p + "fc1.w"], w[p + "fc1.b"])
        m = ops.act(m.contiguous(), self.act) if self.act != 6 else m * torch.sigmoid(1.702 * m)
        m = linear(m, w[p + "fc2.w"], w[p + "fc2.b"]).view(n, S, C)
        return x + (torch.tanh(w[p + "gate_ffn"]).to(x.dtype) * m if gated else m)

    def forward(self, pixels: torch.Tensor, ar_ids: torch.Tensor, ar_mask: torch.Tensor) -> torch.Tensor:
        """pixels [n, T, 3, s, s] (T = max tiles), ar_ids [n], ar_mask [n, T] -> projected vision
        tokens [n, T, P, out_dim] (padding patches removed)."""
        w, C, P, Pp, ps = self.w, self.C, self.P, self.Pp, self.patch
        n, T = pixels.shape[:2]
        px = pixels.reshape(n * T, 3, self.tile, self.tile).to(self.dtype)
        cols = F.unfold(px, kernel_size=ps, stride=ps).transpose(1, 2)        # [nT, patches, 3*ps*ps]
        x = linear(cols.reshape(-1, cols.shape[-1]).contiguous(), w["patch"]).view(n, T, P - 1, C)
        x = x + (torch.tanh(w["pre_gate"]).to(x.dtype) * w["pre_tile"][ar_ids].view(n, T, 1, C))
        x = torch.cat([w["cls"].view(1, 1, 1, C).expand(n, T, 1, C), x], 2)
        g = torch.tanh(w["pos_gate"]).to(x.dtype)
        x = x + (1 - g) * w["pos"].view(1, 1, P, C) + g * w["tile_pos"][ar_ids].view(n, T, P, C)
        x = self._ln(x, "ln_pre")
        x = F.pad(x, (0, 0, 0, Pp - P))
        # a (query, key) pair is masked only when both are padding (padded patch or padded tile)
        pad = torch.ones(n, T, Pp, dtype=torch.bool, device=x.device)
        pad[:, :, :P] = ~ar_mask.bool()[:, :, None]
        pad = pad.view(n * T * Pp)
        rows = torch.arange(n * T * Pp, device=x.device)
        n_pad = pad.view(n, T * Pp).sum(1).tolist()
        bias = (rows[pad], rows[~pad], n_pad, [T * Pp - c for c in n_pad])   # see _layer
        x = x.view(n, T * Pp, C)
        inter = []
        for i in range(self.L):
            x = self._layer(f"t{i}.", x, bias, False)
            if i in self.inter_idx:
                inter.append(x)
        x = self._ln(x, "ln_post").view(n, T, Pp, C)
        x = x + torch.tanh(w["post_gate"]).to(x.dtype) * w["post_tile"][ar_ids].view(n, T, 1, C)
        x = x.view(n, T * Pp, C)
        for i in range(self.Lg):
            x = self._layer(f"g{i}.", x, bias, True)
        x = x.view(n, T, Pp, C)[:, :, :P]
        inter_t = torch.stack([inter[self.inter_idx.index(i)] for i in self.inter_idx], -1)  # [n, T*Pp, C, k]
        inter_t = inter_t.reshape(n, T, Pp, -1)[:, :, :P]
        feats = torch.cat([x, inter_t], -1)
        return linear(feats.reshape(n * T * P, -1).contiguous(), w["proj.w"], w["proj.b"]).view(n, T, P, -1)


class MllamaForConditionalGeneration(LlamaForCausalLM):
    is_multimodal = True
    mm_cross = True
    stateful = True   # per request slot: vision-token ranges (``alloc_state``), per-row slots in meta

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        hf = cfg.extra or {}
        tc = hf.get("text_config") or hf
        self.cross = sorted(int(i) for i in tc.get("cross_attention_layers", []))
        self.cross_set = set(self.cross)
        self.kv_layers = [i for i in self.layers if i not in self.cross_set]
        self.image_token_id = int(hf.get("image_token_index", hf.get("image_token_id", 128256)))
        self.vision = MllamaVision(_vcfg(cfg), cfg.hidden_size, self.device, dtype)
        self.tokens_per_tile = self.vision.P
        self.max_tiles = self.vision.max_tiles
        L = cfg.num_layers
        self.w_xq: list[torch.Tensor | None] = [None] * L
        self.w_xkv: list[torch.Tensor | None] = [None] * L   # [2 * hkv * D, H]: this rank's k rows then v rows
        self.gates: dict[int, tuple[float, float]] = {}
        self.max_images = int(hf.get("max_images_per_request", 4))
        self.pool_images = int(hf.get("vision_cache_images", 0))  # 0: sized in alloc_state
        self.image_mean = tuple(hf.get("image_mean") or (0.48145466, 0.4578275, 0.40821073))
        self.image_std = tuple(hf.get("image_std") or (0.26862954, 0.26130258, 0.27577711))

    # ------------------------------------------------------------------ weights
    def init_random(self, seed: int = 0, std: float = 0.02) -> "MllamaForConditionalGeneration":
        super().init_random(seed, std)
        cfg, tp, D = self.cfg, self.tp, self.D
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 31337)
        H = cfg.hidden_size
        for i in self.cross:
            if i not in self._layer_set:
                continue
            self.w_qkv[i] = None
            self.w_xq[i] = self._alloc(tp.hq * D, H, std=std, gen=gen)
            self.w_xkv[i] = self._alloc(2 * tp.hkv * D, H, std=std, gen=gen)
            self.qn[i], self.kn[i] = self._alloc(D, std=None, gen=gen), self._alloc(D, std=None, gen=gen)
            self.gates[i] = (math.tanh(0.5), math.tanh(0.5))
        self.embed = torch.cat([self.embed, self._alloc(8, H, std=1.0, gen=gen)], 0) if self.tp.tp == 1 else \
            self._full_embed_random(gen)
        self.vision.init_random(gen, std)
        return self

    def _full_embed_random(self, gen):
        V = self.cfg.vocab_size + 8
        return self._alloc(V, self.cfg.hidden_size, std=1.0, gen=gen)

    def load_hf_weights(self, weights) -> "MllamaForConditionalGeneration":
        tp, D = self.tp, self.D
        if self.fp8:   # e.g. RedHatAI Llama-3.2-90B-Vision-Instruct-FP8-dynamic: per-channel weight_scale
            weights = dequant_fp8_stream(weights, self.fp8_block, self.dtype)
        xparts: dict[int, dict[str, torch.Tensor]] = {}
        rest = []
        embed_full = None

        def put(t):
            return t.to(device=self.device, dtype=self.dtype).contiguous()

        for name, w in weights:
            if self.vision.load(name, w):
                continue
            n = name
            for pre in ("language_model.model.", "model.language_model.", "language_model."):
                if n.startswith(pre):
                    n = n[len(pre):]
                    break
            if n == "embed_tokens.weight":  # vocab + 8 special rows, kept whole on every rank
                embed_full = w
            parts = n.split(".")
            if parts[0] == "layers" and int(parts[1]) in self.cross_set:
                i, sub = int(parts[1]), ".".join(parts[2:])
                if sub in ("cross_attn_attn_gate", "cross_attn_mlp_gate"):
                    xparts.setdefault(i, {})[sub] = w
                    continue
                if sub.startswith("cross_attn."):
                    xparts.setdefault(i, {})[sub[len("cross_attn."):]] = w
                    continue
            rest.append(("model." + n if not n.startswith("lm_head") else n, w))
        # the Llama loader requires self-attention weights for every layer: cross layers have none
        for i in self.cross:
            if i in self._layer_set:
                rest += [(f"model.layers.{i}.self_attn.{c}_proj.weight",
                          torch.zeros((self.cfg.num_heads if c == "q" else self.cfg.num_kv_heads) * D, 1))
                         for c in "qkv"]
        super().load_hf_weights(iter(rest))
        if embed_full is None:
            raise ValueError("checkpoint has no embed_tokens")
        self.embed = put(embed_full)
        for i, p in xparts.items():
            if i not in self._layer_set:
                continue
            self.w_qkv[i] = None
            self.w_xq[i] = put(p["q_proj.weight"].narrow(0, tp.rank * tp.hq * D, tp.hq * D))
            k = p["k_proj.weight"].narrow(0, tp.kv_start * D, tp.hkv * D)
            v = p["v_proj.weight"].narrow(0, tp.kv_start * D, tp.hkv * D)
            self.w_xkv[i] = put(torch.cat([k, v], 0))
            self.w_o[i] = put(p["o_proj.weight"].narrow(1, tp.rank * tp.hq * D, tp.hq * D))
            self.qn[i], self.kn[i] = put(p["q_norm.weight"]), put(p["k_norm.weight"])
            self.gates[i] = (math.tanh(float(p["cross_attn_attn_gate"].float().reshape(-1)[0])),
                             math.tanh(float(p["cross_attn_mlp_gate"].float().reshape(-1)[0])))
        return self

    def weight_bytes(self) -> int:
        n = super().weight_bytes()
        n += sum(t.numel() * t.element_size() for t in self.w_xq + self.w_xkv if t is not None)
        return n + sum(t.numel() * t.element_size() for t in self.vision.w.values() if isinstance(t, torch.Tensor))

    # ------------------------------------------------------------------ per-slot vision-token state
    def alloc_state(self, slots: int) -> None:
        """Per request slot: visibility segments (text start, lo, hi, mlp gate) on the device, and a
        page pool for the vision-token K/V of ``pool_images`` images per cross layer."""
        tp, D = self.tp, self.D
        NS = self.max_images + 1
        dv = self.device
        self.seg_start = torch.full((slots, NS), 1 << 30, dtype=torch.int32, device=dv)
        self.seg_lo = torch.zeros(slots, NS, dtype=torch.int32, device=dv)
        self.seg_hi = torch.zeros(slots, NS, dtype=torch.int32, device=dv)
        self.seg_mlp = torch.zeros(slots, NS, dtype=torch.float32, device=dv)
        self.has_img = torch.zeros(slots, dtype=torch.float32, device=dv)
        per_img = -(-self.max_tiles * self.tokens_per_tile // P_CACHE)
        self.max_xpages = per_img * self.max_images
        self.xtable = torch.zeros(slots, self.max_xpages, dtype=torch.int32, device=dv)
        n_img = self.pool_images or max(4, min(slots, 32 if dv.type == "cuda" else 4))
        self.n_xpages = per_img * n_img + 1
        self.xk = {i: torch.zeros(self.n_xpages, tp.hkv, P_CACHE, D, dtype=self.dtype, device=dv) for i in self.cross
                   if i in self._layer_set}
        self.xv = {i: torch.zeros(self.n_xpages, tp.hkv, D, P_CACHE, dtype=self.dtype, device=dv) for i in self.cross
                   if i in self._layer_set}
        self._xfree = list(range(self.n_xpages - 1, 0, -1))  # page 0: scratch target of text-only rows
        self._slot_pages: dict[int, list[int]] = {}

    def _free_slot(self, slot: int) -> None:
        pages = self._slot_pages.pop(slot, None)
        if pages:
            self._xfree.extend(pages)
        self.has_img[slot] = 0.0
        self.seg_start[slot] = 1 << 30

    def prepare_chunks(self, chunks) -> None:
        """Host hook before an eager step: a request's first chunk (re)initialises its slot; one
        with images runs the vision tower and fills its vision-token cache and segments."""
        for c in chunks:
            r = c.req
            if c.start != 0:
                continue
            slot = r.req_slot
            self._free_slot(slot)
            mm = getattr(r, "mm", None)
            if mm is None or not getattr(mm, "cross_only", False):
                continue
            self._encode_request(slot, mm)
            mm.release = (lambda s=slot: self._free_slot(s))

    @torch.no_grad()
    def _encode_request(self, slot: int, mm) -> None:
        n = len(mm.image_pos)
        if n > self.max_images:
            raise ValueError(f"at most {self.max_images} images per request")
        Tm, Pt, D = self.max_tiles, self.tokens_per_tile, self.D
        total = n * Tm * Pt
        need = -(-total // P_CACHE)
        if need > len(self._xfree):
            raise RuntimeError("vision-token cache exhausted (raise vision_cache_images)")
        pages = [self._xfree.pop() for _ in range(need)]
        self._slot_pages[slot] = pages
        dv = self.device
        pix = mm.pixel_values.to(dv)
        ar_ids = torch.tensor(mm.ar_ids, dtype=torch.long, device=dv)
        ar_mask = torch.zeros(n, Tm, dtype=torch.bool, device=dv)
        for k, t in enumerate(mm.num_tiles):
            ar_mask[k, :t] = True
        feats = self.vision.forward(pix, ar_ids, ar_mask)           # [n, Tm, Pt, H]
        real = torch.cat([feats[k, :t].reshape(-1, feats.shape[-1]) for k, t in enumerate(mm.num_tiles)], 0)
        pad = [feats[k, t:].reshape(-1, feats.shape[-1]) for k, t in enumerate(mm.num_tiles) if t < Tm]
        states = torch.cat([real] + pad, 0) if pad else real                     # [total, H]
        pg = torch.tensor(pages, dtype=torch.int64, device=dv)
        tok = torch.arange(total, device=dv)
        cache_slots = (pg[tok // P_CACHE] * P_CACHE + tok % P_CACHE).to(torch.int32)
        hkv = self.tp.hkv
        for i in self.xk:
            kv = linear(states, self.w_xkv[i]).view(total, 2, hkv, D)
            k = ops.rmsnorm(kv[:, 0].contiguous(), self.kn[i], self.eps)
            ops.kv_cache_write(k, kv[:, 1].contiguous(), self.xk[i], self.xv[i], cache_slots)
        self.xtable[slot, :need] = pg.to(torch.int32)
        segs = mm.segments(Pt, Tm)
        NS = self.seg_start.shape[1]
        st = [s[0] for s in segs] + [1 << 30] * (NS - len(segs))
        lo = [s[1] for s in segs] + [0] * (NS - len(segs))
        hi = [s[2] for s in segs] + [0] * (NS - len(segs))
        ml = [float(s[3]) for s in segs] + [0.0] * (NS - len(segs))
        self.seg_start[slot] = torch.tensor(st, dtype=torch.int32, device=dv)
        self.seg_lo[slot] = torch.tensor(lo, dtype=torch.int32, device=dv)
        self.seg_hi[slot] = torch.tensor(hi, dtype=torch.int32, device=dv)
        self.seg_mlp[slot] = torch.tensor(ml, dtype=torch.float32, device=dv)
        self.has_img[slot] = 1.0

    # ------------------------------------------------------------------ forward
    def _row_slots(self, meta: AttnMeta, T: int) -> torch.Tensor:
        cu, slot, _ = meta.extra["ssm"]
        if cu.shape[0] - 1 == T:  # one row per sequence (decode graphs)
            return slot
        return torch.repeat_interleave(slot, (cu[1:] - cu[:-1]).long(), output_size=T)

    def _cross_rows(self, meta: AttnMeta, T: int):
        rs = self._row_slots(meta, T).long()
        pos = meta.positions
        seg = (self.seg_start.index_select(0, rs) <= pos[:, None]).sum(-1, keepdim=True) - 1  # [T, 1]
        seg = seg.clamp(min=0)
        lo = self.seg_lo.index_select(0, rs).gather(1, seg)[:, 0]
        hi = self.seg_hi.index_select(0, rs).gather(1, seg)[:, 0]
        mlp = self.seg_mlp.index_select(0, rs).gather(1, seg)[:, 0]
        has = self.has_img.index_select(0, rs)
        hi = torch.where(has > 0, hi, torch.ones_like(hi))  # text-only rows: one scratch key, zero gate
        bt = self.xtable.index_select(0, rs)
        return bt, lo.contiguous(), hi.to(torch.int32).contiguous(), has, mlp

    def _cross_block(self, i: int, x: torch.Tensor, rows) -> torch.Tensor:
        tp, D = self.tp, self.D
        T = x.shape[0]
        bt, lo, hi, has, _ = rows
        q = ops.rmsnorm(linear(x, self.w_xq[i]).view(T * tp.hq, D), self.qn[i], self.eps).view(T, tp.hq, D)
        a = ops.paged_decode(q, self.xk[i], self.xv[i], bt, hi, self.scale, self._xws(T), row_lo=lo)
        return linear(a.view(T, tp.hq * D), self.w_o[i])

    def _xws(self, T: int):
        """One split-free workspace for every row count: a text row's key range fits one decode
        partition (<= images x tiles x tokens), so the split-K buffers are never touched."""
        if self.device.type != "cuda":
            return None
        ws = getattr(self, "_xws1", None)
        if ws is None:
            span = self.max_images * self.max_tiles * self.tokens_per_tile + P_CACHE
            ws = ops.DecodeWorkspace(1, self.tp.hq, self.D, span, -(-span // 128) * 128, self.device)
            self._xws1 = ws
        return ws

    def forward(self, ids: torch.Tensor, meta: AttnMeta, kv: PagedKVCache,
                input_embeds: torch.Tensor | None = None) -> torch.Tensor:
        cfg, tp, D = self.cfg, self.tp, self.D
        T = ids.shape[0]
        x, residual = self._stage_input(ids, input_embeds)
        rows = self._cross_rows(meta, T) if "ssm" in meta.extra else None
        for i in self.layers:
            if i > 0:
                ops.fused_add_rmsnorm(x, residual, self.ln1[i], self.eps)
            if i in self.cross_set:
                if rows is None:  # no per-row slots (single-sequence tools): text only, identity
                    x = torch.zeros_like(x)
                    continue
                ga, gm = self.gates[i]
                a = pstate.tp_all_reduce(self._cross_block(i, x, rows))
                a = a * (ga * rows[3]).to(a.dtype)[:, None]
                ops.fused_add_rmsnorm(a, residual, self.ln2[i], self.eps)
                m = self.mlp(i, a)
                x = m * (gm * rows[3] * rows[4]).to(m.dtype)[:, None]
                continue
            qkv = linear(x, self.w_qkv[i], self.b_qkv[i])
            q = torch.empty(T, tp.hq, D, dtype=self.dtype, device=x.device)
            k_cache, v_cache = kv.layer(i)
            ks, vs = kv.scales(i)
            ops.rope_qkv_cache(qkv, meta.positions, self.cos_sin, cfg.rot_dim, q, k_cache, v_cache, meta.slots,
                               tp.hq, tp.hkv, D, True, None, None, self.eps, ks, vs)
            attn = self.attention(q, k_cache, v_cache, meta, ks, vs)
            o = pstate.tp_all_reduce(linear(attn.view(T, tp.hq * D), self.w_o[i]))
            ops.fused_add_rmsnorm(o, residual, self.ln2[i], self.eps)
            x = self.mlp(i, o)
        return self._stage_output(x, residual)

    def _stage_input(self, ids: torch.Tensor, input_embeds: torch.Tensor | None):
        if input_embeds is None:
            h = ops.embedding(ids, self.embed)  # whole table (vocab + 8 specials) on every rank
        else:
            h = input_embeds
        return ops.rmsnorm(h, self.ln1[0], self.eps), h

    # ------------------------------------------------------------------ requests
    def make_mm_input(self, prompt_ids: list[int], images: list):
        from ome_amd.multimodal.mllama import CrossMMInput, preprocess_image

        pos = [k for k, t in enumerate(prompt_ids) if t == self.image_token_id]
        if len(pos) != len(images):
            raise ValueError(f"{len(images)} images but {len(pos)} <|image|> tokens in the prompt")
        pvs, ars, nts = [], [], []
        for im in images:
            if isinstance(im, tuple):  # preprocessed (pixel_values, aspect_ratio_id, num_tiles)
                pv, ar, nt = im
            else:
                pv, ar, nt = preprocess_image(im, tile=self.vision.tile, max_tiles=self.max_tiles,
                                              mean=self.image_mean, std=self.image_std)
            pvs.append(torch.as_tensor(pv, dtype=torch.float32))
            ars.append(int(ar))
            nts.append(int(nt))
        return list(prompt_ids), CrossMMInput(torch.stack(pvs), ars, nts, pos)

    def image_prompt_ids(self) -> list[int]:
        return [self.image_token_id]
