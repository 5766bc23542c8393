"""Qwen2-VL (``Qwen2VLForConditionalGeneration``; reference catalog
``config/runtimes/srt/qwen/qwen2-vl-*``) on the ome_amd kernels.

* Language model: the Qwen2 dense decoder of ``llama.py`` (q/k/v biases), unchanged on the hot
  path.  M-RoPE (``mrope_section`` [t, h, w] split of the rotary frequencies) only differs from
  1D RoPE for image tokens: text tokens carry three equal components, which IS 1D RoPE at that
  position.  So decode rows (HIP-graph path) just use ``position + rope_delta``; prefill chunks
  that contain image tokens get a per-token cos/sin table built from their 3D positions
  (:meth:`mrope_table`) and run through the same fused RoPE / KV-cache kernel with row-indexed
  positions (``meta.extra['rope']``).
* Vision tower (runs once per image, at the first prefill chunk that reaches it): Conv3d patch
  embedding as one GEMM over (C, T, ps, ps) patches, ``depth`` pre-LN ViT blocks with 2D
  (h, w) rotary embeddings, bidirectional attention within each image, quick-GELU MLPs, and the
  2x2 patch merger (LN -> GEMM -> GELU -> GEMM) into the LM hidden size.  LayerNorms run on the
  ``ome_layernorm`` HIP kernel, GEMMs on hipBLASLt, attention per image on PyTorch SDPA (not a
  serving hot path: one pass per image).
* Image placeholder rows of the prompt are overwritten with the merged vision features
  (``Request.mm.spans``) before the first decoder layer.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.models.common import AttnMeta, PagedKVCache
from ome_amd.models.config import ModelConfig
from ome_amd.models.llama import LlamaForCausalLM
from ome_amd.models.quant import linear
from ome_amd.parallel import state as pstate

QWEN2_VL_ARCHS = {"Qwen2VLForConditionalGeneration", "Qwen2_5_VLForConditionalGeneration"}


class Qwen2VisionTower:
    def __init__(self, vc: dict, out_hidden: int, device, dtype):
        self.device, self.dtype = device, dtype
        self.E = int(vc.get("embed_dim", 1280))
        self.depth = int(vc.get("depth", 32))
        self.heads = int(vc.get("num_heads", 16))
        self.hd = self.E // self.heads
        self.mlp = int(self.E * float(vc.get("mlp_ratio", 4)))
        self.patch = int(vc.get("patch_size", 14))
        self.merge = int(vc.get("spatial_merge_size", 2))
        self.temporal = int(vc.get("temporal_patch_size", 2))
        self.cin = int(vc.get("in_channels", 3))
        self.out_hidden = out_hidden
        if vc.get("hidden_act", "quick_gelu") != "quick_gelu":
            raise NotImplementedError(f"vision hidden_act {vc.get('hidden_act')!r}")
        self.w: dict[str, torch.Tensor] = {}
        rd = self.hd // 2
        self.inv = 1.0 / (10000.0 ** (torch.arange(0, rd, 2, dtype=torch.float32) / rd))

    def init_random(self, gen: torch.Generator, std: float = 0.02) -> None:
        E, M, mh = self.E, self.mlp, self.E * self.merge ** 2
        shapes = {"patch_embed.proj.weight": (E, self.cin * self.temporal * self.patch ** 2),
                  "merger.ln_q.weight": (E,), "merger.ln_q.bias": (E,), "merger.mlp.0.weight": (mh, mh),
                  "merger.mlp.0.bias": (mh,), "merger.mlp.2.weight": (self.out_hidden, mh),
                  "merger.mlp.2.bias": (self.out_hidden,)}
        for b in range(self.depth):
            p = f"blocks.{b}."
            shapes.update({p + "norm1.weight": (E,), p + "norm1.bias": (E,), p + "norm2.weight": (E,),
                           p + "norm2.bias": (E,), p + "attn.qkv.weight": (3 * E, E), p + "attn.qkv.bias": (3 * E,),
                           p + "attn.proj.weight": (E, E), p + "attn.proj.bias": (E,), p + "mlp.fc1.weight": (M, E),
                           p + "mlp.fc1.bias": (M,), p + "mlp.fc2.weight": (E, M), p + "mlp.fc2.bias": (E,)})
        for k, s in shapes.items():
            t = torch.empty(*s, dtype=self.dtype, device=self.device)
            if k.endswith("norm1.weight") or k.endswith("norm2.weight") or k.endswith("ln_q.weight"):
                t.fill_(1.0)
            elif len(s) == 1:
                t.zero_()
            else:
                t.normal_(0.0, std, generator=gen)
            self.w[k] = t

    def load(self, name: str, t: torch.Tensor) -> None:
        if name == "patch_embed.proj.weight":
            t = t.reshape(t.shape[0], -1)
        self.w[name] = t.to(device=self.device, dtype=self.dtype).contiguous()

    def _ln(self, x, p):
        return ops.layernorm(x, self.w[p + ".weight"], self.w[p + ".bias"], 1e-6)

    def rot_pos(self, grids) -> torch.Tensor:
        """[N, hd/2] rotary angles of each patch (h then w frequencies), merge-block-major order."""
        m, out = self.merge, []
        for t, h, w in grids:
            hp = torch.arange(h).view(h, 1).expand(h, w)
            wp = torch.arange(w).view(1, w).expand(h, w)
            blk = (h // m, m, w // m, m)
            hp = hp.reshape(blk).transpose(1, 2).reshape(-1)
            wp = wp.reshape(blk).transpose(1, 2).reshape(-1)
            out.append(torch.stack([hp, wp], -1).repeat(t, 1))
        pos = torch.cat(out).float()
        return (pos[:, :, None] * self.inv[None, None, :]).reshape(pos.shape[0], -1)

    def forward(self, pixel_values: torch.Tensor, grids: list[tuple[int, int, int]]) -> torch.Tensor:
        dev, dt, E, Hh, D = self.device, self.dtype, self.E, self.heads, self.hd
        x = linear(pixel_values.to(device=dev, dtype=dt), self.w["patch_embed.proj.weight"])
        ang = self.rot_pos(grids).to(dev)
        emb = torch.cat([ang, ang], -1)
        cos, sin = emb.cos()[:, None, :], emb.sin()[:, None, :]
        lens = [h * w for t, h, w in grids for _ in range(t)]
        N = x.shape[0]

        def rope(t):
            tf = t.float()
            half = D // 2
            rot = torch.cat([-tf[..., half:], tf[..., :half]], -1)
            return (tf * cos + rot * sin).to(dt)

        for b in range(self.depth):
            p = f"blocks.{b}."
            h = self._ln(x, p + "norm1")
            qkv = linear(h, self.w[p + "attn.qkv.weight"], self.w[p + "attn.qkv.bias"]).view(N, 3, Hh, D)
            q, k, v = rope(qkv[:, 0]), rope(qkv[:, 1]), qkv[:, 2]
            # bidirectional attention within each image / frame: one varlen MFMA launch
            a = ops.varlen_attention(q, k, v, lens, D ** -0.5).reshape(N, E)
            x = x + linear(a, self.w[p + "attn.proj.weight"], self.w[p + "attn.proj.bias"])
            h = self._ln(x, p + "norm2")
            f = linear(h, self.w[p + "mlp.fc1.weight"], self.w[p + "mlp.fc1.bias"])
            f = f * torch.sigmoid(1.702 * f)
            x = x + linear(f, self.w[p + "mlp.fc2.weight"], self.w[p + "mlp.fc2.bias"])
        h = self._ln(x, "merger.ln_q").reshape(-1, E * self.merge ** 2)
        h = F.gelu(linear(h, self.w["merger.mlp.0.weight"], self.w["merger.mlp.0.bias"]))
        return linear(h, self.w["merger.mlp.2.weight"], self.w["merger.mlp.2.bias"])


class Qwen2VLForConditionalGeneration(LlamaForCausalLM):
    is_multimodal = True
    tower_cls = Qwen2VisionTower

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        ex = cfg.extra or {}
        rp = ex.get("rope_parameters") or ex.get("rope_scaling") or {}
        sec = list(rp.get("mrope_section") or [16, 24, 24])
        half = cfg.rot_dim // 2
        if sum(sec) != half:
            raise ValueError(f"mrope_section {sec} does not cover {half} rotary frequencies")
        self.mrope_sec = torch.tensor(np.repeat(np.arange(3), sec), dtype=torch.long)
        self.inv = 1.0 / (cfg.rope_theta ** (torch.arange(0, cfg.rot_dim, 2, dtype=torch.float64) / cfg.rot_dim))
        self.image_token_id = int(ex.get("image_token_id", 151655))
        self.vision_start_id = int(ex.get("vision_start_token_id", 151652))
        self.vision_end_id = int(ex.get("vision_end_token_id", 151653))
        self.visual = self.tower_cls(ex.get("vision_config") or {}, cfg.hidden_size, self.device, dtype)
        self.merge = self.visual.merge

    # ------------------------------------------------------------------ weights
    def init_random(self, seed: int = 0, std: float = 0.02) -> "Qwen2VLForConditionalGeneration":
        super().init_random(seed, std)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 4243)
        self.visual.init_random(gen, std)
        return self

    def load_hf_weights(self, weights) -> "Qwen2VLForConditionalGeneration":
        lm = []
        for name, w in weights:
            for pre in ("model.visual.", "visual."):
                if name.startswith(pre):
                    self.visual.load(name[len(pre):], w)
                    break
            else:
                if name.startswith("model.language_model."):
                    name = "model." + name[len("model.language_model."):]
                lm.append((name, w))
        return super().load_hf_weights(iter(lm))

    def weight_bytes(self) -> int:
        return super().weight_bytes() + sum(t.numel() * t.element_size() for t in self.visual.w.values())

    # ------------------------------------------------------------------ multimodal
    def encode_images(self, pixel_values: torch.Tensor, grids) -> torch.Tensor:
        return self.visual.forward(pixel_values, grids)

    def mrope_table(self, pos3: torch.Tensor) -> torch.Tensor:
        """pos3 [3, T] -> per-row cos|sin table [T, rot_dim] (float32, model device)."""
        p = pos3.to(torch.float64).t()[:, self.mrope_sec]          # [T, rot/2]
        ang = p * self.inv[None, :]
        return torch.cat([ang.cos(), ang.sin()], -1).float().to(self.device)

    def embed_with_images(self, ids: torch.Tensor, rows: torch.Tensor, feats: torch.Tensor) -> torch.Tensor:
        h = pstate.tp_all_reduce(ops.embedding(ids, self.embed, self.tp.vocab_start, self.tp.vocab_end))
        if rows.numel():
            h.index_copy_(0, rows, feats.to(h.dtype))
        return h

    # ------------------------------------------------------------------ forward
    def forward(self, ids: torch.Tensor, meta: AttnMeta, kv: PagedKVCache,
                input_embeds: torch.Tensor | None = None) -> torch.Tensor:
        rope = meta.extra.get("rope") if meta.extra else None
        if rope is None:
            return super().forward(ids, meta, kv, input_embeds)
        cfg, tp, D = self.cfg, self.tp, self.D
        rpos, table = rope
        ds = meta.extra.get("deepstack")
        T = ids.shape[0]
        x, residual = self._stage_input(ids, input_embeds)
        for i in self.layers:
            if i > 0:
                ops.fused_add_rmsnorm(x, residual, self.ln1[i], self.eps)
            qkv = linear(x, self.w_qkv[i], self.b_qkv[i])
            q = torch.empty(T, tp.hq, D, dtype=self.dtype, device=x.device)
            k_cache, v_cache = kv.layer(i)
            ks, vs = kv.scales(i)
            ops.rope_qkv_cache(qkv, rpos, table, cfg.rot_dim, q, k_cache, v_cache, meta.slots,
                               tp.hq, tp.hkv, D, True, self.qn[i], self.kn[i], self.eps, ks, vs)
            attn = self.attention(q, k_cache, v_cache, meta, ks, vs)
            o = pstate.tp_all_reduce(linear(attn.view(T, tp.hq * D), self.w_o[i]))
            ops.fused_add_rmsnorm(o, residual, self.ln2[i], self.eps)
            x = self.mlp(i, o)
            if ds is not None and i < len(ds[1]):   # Qwen3-VL deepstack: layer i output += level-i features
                x.index_add_(0, ds[0], ds[1][i].to(x.dtype))
        return self._stage_output(x, residual)


def num_image_tokens(grid: tuple[int, int, int], merge: int) -> int:
    t, h, w = grid
    return t * h * w // (merge * merge)



# ---------------------------------------------------------------------------------------------
# Qwen2.5-VL (reference catalog ``config/runtimes/srt/Qwen/Qwen2.5-VL-7B-Instruct-rt.yaml``,
# ``.../XiaomiMiMo/mimo-vl-7b-rl-rt.yaml``): same language model, processor and M-RoPE as
# Qwen2-VL; the vision tower adds windowed attention (windows of ``window_size`` px, i.e. 4 x 4
# merge blocks at 112 / 14 / 2), full attention only in ``fullatt_block_indexes``, RMSNorm and a
# biased SwiGLU MLP.  Patches are permuted window-major once at the start (each window is then a
# contiguous varlen segment of the ``ome_varlen_attention`` launch, the full-attention layers use
# the per-image segments, which the permutation keeps contiguous) and the merged features are
# permuted back at the end.
# ---------------------------------------------------------------------------------------------
class Qwen25VisionTower(Qwen2VisionTower):
    def __init__(self, vc: dict, out_hidden: int, device, dtype):
        self.device, self.dtype = device, dtype
        self.E = int(vc.get("hidden_size", 1280))
        self.depth = int(vc.get("depth", 32))
        self.heads = int(vc.get("num_heads", 16))
        self.hd = self.E // self.heads
        self.inter = int(vc.get("intermediate_size", 3420))
        self.inter_pad = -(-self.inter // 8) * 8   # act_and_mul tiles 8 columns: zero-padded lanes
        self.patch = int(vc.get("patch_size", 14))
        self.merge = int(vc.get("spatial_merge_size", 2))
        self.temporal = int(vc.get("temporal_patch_size", 2))
        self.cin = int(vc.get("in_channels", vc.get("in_chans", 3)))
        self.window = int(vc.get("window_size", 112))
        self.full = set(int(i) for i in (vc.get("fullatt_block_indexes") or []))
        self.out_hidden = int(vc.get("out_hidden_size") or out_hidden)
        act = vc.get("hidden_act", "silu")
        self.act = {"silu": 0, "swish": 0, "gelu_pytorch_tanh": 1}.get(act)
        if self.act is None:
            raise NotImplementedError(f"vision hidden_act {act!r}")
        self.w: dict[str, torch.Tensor] = {}
        rd = self.hd // 2
        self.inv = 1.0 / (10000.0 ** (torch.arange(0, rd, 2, dtype=torch.float32) / rd))

    def init_random(self, gen: torch.Generator, std: float = 0.02) -> None:
        E, I, mh = self.E, self.inter, self.E * self.merge ** 2
        shapes = {"patch_embed.proj.weight": (E, self.cin * self.temporal * self.patch ** 2),
                  "merger.ln_q.weight": (E,), "merger.mlp.0.weight": (mh, mh), "merger.mlp.0.bias": (mh,),
                  "merger.mlp.2.weight": (self.out_hidden, mh), "merger.mlp.2.bias": (self.out_hidden,)}
        for b in range(self.depth):
            p = f"blocks.{b}."
            shapes.update({p + "norm1.weight": (E,), p + "norm2.weight": (E,), p + "attn.qkv.weight": (3 * E, E),
                           p + "attn.qkv.bias": (3 * E,), p + "attn.proj.weight": (E, E), p + "attn.proj.bias": (E,),
                           p + "mlp.gate_proj.weight": (I, E), p + "mlp.gate_proj.bias": (I,),
                           p + "mlp.up_proj.weight": (I, E), p + "mlp.up_proj.bias": (I,),
                           p + "mlp.down_proj.weight": (E, I), p + "mlp.down_proj.bias": (E,)})
        for k, s in shapes.items():
            t = torch.empty(*s, dtype=self.dtype, device=self.device)
            if k.endswith(("norm1.weight", "norm2.weight", "ln_q.weight")):
                t.fill_(1.0)
            elif len(s) == 1:
                t.zero_()
            else:
                t.normal_(0.0, std, generator=gen)
            self.w[k] = t

    def _fused_mlp(self, b: int):
        """(gate|up [2*I_pad, E], bias, down [E, I_pad]) of block ``b``, built once from the
        checkpoint's gate / up / down projections with zero padding to ``inter_pad``."""
        key = f"blocks.{b}.mlp._fused"
        f = self.w.get(key)
        if f is None:
            p, I, Ip = f"blocks.{b}.mlp.", self.inter, self.inter_pad

            def pad_rows(t):
                return F.pad(t, (0, 0, 0, Ip - I)) if t.dim() == 2 else F.pad(t, (0, Ip - I))

            gu = torch.cat([pad_rows(self.w[p + "gate_proj.weight"]), pad_rows(self.w[p + "up_proj.weight"])])
            gub = torch.cat([pad_rows(self.w[p + "gate_proj.bias"]), pad_rows(self.w[p + "up_proj.bias"])])
            dn = F.pad(self.w[p + "down_proj.weight"], (0, Ip - I))
            f = (gu.contiguous(), gub.contiguous(), dn.contiguous())
            self.w[key] = f
            for n in ("gate_proj.weight", "gate_proj.bias", "up_proj.weight", "up_proj.bias", "down_proj.weight"):
                del self.w[p + n]
        return f

    def window_index(self, grids) -> tuple[torch.Tensor, list[int]]:
        """Merge-block permutation to window-major order + the window lengths (in patches)."""
        vws = self.window // self.merge // self.patch
        U = self.merge ** 2
        idx, lens, base = [], [], 0
        for t, h, w in grids:
            gh, gw = h // self.merge, w // self.merge
            index = torch.arange(t * gh * gw).reshape(t, gh, gw)
            ph, pw = vws - gh % vws, vws - gw % vws
            nh, nw = (gh + ph) // vws, (gw + pw) // vws
            padded = F.pad(index, (0, pw, 0, ph), "constant", -100)
            padded = padded.reshape(t, nh, vws, nw, vws).permute(0, 1, 3, 2, 4).reshape(t, nh * nw, vws * vws)
            counts = (padded != -100).sum(-1).reshape(-1)
            flat = padded.reshape(-1)
            idx.append(flat[flat != -100] + base)
            lens.extend(int(c) * U for c in counts if int(c) > 0)
            base += t * gh * gw
        return torch.cat(idx), lens

    def forward(self, pixel_values: torch.Tensor, grids: list[tuple[int, int, int]]) -> torch.Tensor:
        dev, dt, E, Hh, D = self.device, self.dtype, self.E, self.heads, self.hd
        U = self.merge ** 2
        x = linear(pixel_values.to(device=dev, dtype=dt), self.w["patch_embed.proj.weight"])
        N = x.shape[0]
        widx, win_lens = self.window_index(grids)
        widx_d = widx.to(dev)
        x = x.view(N // U, U, E).index_select(0, widx_d).reshape(N, E)
        ang = self.rot_pos(grids).to(dev)
        ang = ang.view(N // U, U, -1).index_select(0, widx_d).reshape(N, -1)
        emb = torch.cat([ang, ang], -1)
        cos, sin = emb.cos()[:, None, :], emb.sin()[:, None, :]
        full_lens = [h * w for t, h, w in grids for _ in range(t)]

        def rope(t):
            tf = t.float()
            half = D // 2
            rot = torch.cat([-tf[..., half:], tf[..., :half]], -1)
            return (tf * cos + rot * sin).to(dt)

        for b in range(self.depth):
            p = f"blocks.{b}."
            h = ops.rmsnorm(x, self.w[p + "norm1.weight"], 1e-6)
            qkv = linear(h, self.w[p + "attn.qkv.weight"], self.w[p + "attn.qkv.bias"]).view(N, 3, Hh, D)
            q, k, v = rope(qkv[:, 0]), rope(qkv[:, 1]), qkv[:, 2]
            a = ops.varlen_attention(q, k, v, full_lens if b in self.full else win_lens, D ** -0.5).reshape(N, E)
            x = x + linear(a, self.w[p + "attn.proj.weight"], self.w[p + "attn.proj.bias"])
            h = ops.rmsnorm(x, self.w[p + "norm2.weight"], 1e-6)
            gu, gub, dn = self._fused_mlp(b)
            f = ops.act_and_mul(linear(h, gu, gub), self.act)
            x = x + linear(f, dn, self.w[p + "mlp.down_proj.bias"])
        h = ops.rmsnorm(x, self.w["merger.ln_q.weight"], 1e-6).reshape(-1, E * U)
        h = F.gelu(linear(h, self.w["merger.mlp.0.weight"], self.w["merger.mlp.0.bias"]))
        out = linear(h, self.w["merger.mlp.2.weight"], self.w["merger.mlp.2.bias"])
        return out.index_select(0, torch.argsort(widx).to(dev))


class Qwen2_5_VLForConditionalGeneration(Qwen2VLForConditionalGeneration):
    tower_cls = Qwen25VisionTower

    def weight_bytes(self) -> int:
        n = LlamaForCausalLM.weight_bytes(self)
        for v in self.visual.w.values():
            n += sum(t.numel() * t.element_size() for t in (v if isinstance(v, tuple) else (v,)))
        return n
