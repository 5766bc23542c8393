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

QWEN2_VL_ARCHS = {"Qwen2VLForConditionalGeneration"}


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
        self.visual = Qwen2VisionTower(ex.get("vision_config") or {}, cfg.hidden_size, self.device, dtype)
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
        return self._stage_output(x, residual)


def num_image_tokens(grid: tuple[int, int, int], merge: int) -> int:
    t, h, w = grid
    return t * h * w // (merge * merge)

