"""Phi-3-small (``Phi3SmallForCausalLM``, microsoft/Phi-3-small-8k-instruct / -128k-instruct).

Reference catalog entry: ``config/models/microsoft/Phi-3-small-8k-instruct.yaml``.  The modelling
code is remote code (``modeling_phi3_small.py``) that is not importable offline, so this follows the
published architecture; parity is checked against an fp32 restatement of it in
``tests/test_phi3small_cpu.py`` (parity with the remote code itself is unpinned):

* LayerNorm (weight + bias) before attention and MLP, final LayerNorm;
* fused, biased ``query_key_value`` in kv-group order ``[kv_heads][q_per_kv + 2][head_dim]``
  (the decoder's ``groups`` layout), biased ``dense`` output projection, NeoX RoPE with base
  ``rope_embedding_base``;
* muP scalings: embeddings x ``mup_embedding_multiplier``, softmax scale
  ``mup_attn_multiplier / head_dim`` (not 1/sqrt), logits / ``mup_width_multiplier``;
* GeGELU MLP: ``up_proj`` (biased, [2 * ff, H]) holds the gate and linear halves interleaved row
  by row (``::2`` / ``1::2``); they are de-interleaved at load into the [gate; up] layout so the
  fused ``act_and_mul`` kernel (act 3: quick-GELU(min(g, 20)) * (clamp(u, -20, 20) + 1)) applies;
* block-sparse attention on every layer except each ``dense_attention_every_n_layers``-th: blocks
  of ``blocksparse_block_size`` tokens, a band of ``blocksparse_num_local_blocks`` local blocks plus
  every ``blocksparse_vert_stride``-th block, the stripe offset rotating with the head
  (``blocksparse_homo_head_pattern`` false).  The paged attention kernels apply it as a score mask
  (``ops.paged_decode`` / ``ops.paged_prefill`` ``blocksparse=``; attention.hip ``bs_visible``).
"""
from __future__ import annotations

import torch

from ome_amd import ops
from ome_amd.models.common import AttnMeta, PagedKVCache
from ome_amd.models.config import ModelConfig
from ome_amd.models.decoder import DecoderForCausalLM
from ome_amd.models.quant import linear


class Phi3SmallForCausalLM(DecoderForCausalLM):
    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        hf = cfg.extra or {}
        if float(hf.get("gegelu_limit", 20.0)) != 20.0:
            raise NotImplementedError("Phi-3-small GeGELU limit other than 20")
        self.act = 3
        L = cfg.num_layers
        self.b_gu: list[torch.Tensor | None] = [None] * L
        every = int(hf.get("dense_attention_every_n_layers") or 0)
        self.sparse_layer = [bool(every) and (i + 1) % every != 0 for i in range(L)]
        vert = int(hf.get("blocksparse_vert_stride", 8))
        step = 0 if hf.get("blocksparse_homo_head_pattern", False) else max(1, vert // cfg.num_heads)
        # the kernels see this rank's heads 0 .. hq-1: the global offset of the stripe pattern
        self.bs = (int(hf.get("blocksparse_block_size", 64)), int(hf.get("blocksparse_num_local_blocks", 16)), vert,
                   step, self.tp.rank * self.tp.hq * step)
        self._layer_bs = None

    # ------------------------------------------------------------------ weights
    def init_random(self, seed: int = 0, std: float = 0.02) -> "Phi3SmallForCausalLM":
        super().init_random(seed, std)
        g = torch.Generator(device="cpu").manual_seed(seed + 11)
        for i in self.layers:
            self.b_gu[i] = (torch.randn(self.w_gu[i].shape[0], generator=g) * std).to(self.device, self.dtype)
        return self

    def load_hf_weights(self, weights) -> "Phi3SmallForCausalLM":
        def deinterleave():
            for name, w in weights:
                if ".mlp.up_proj." in name:   # rows g0, u0, g1, u1, ... -> [g; u]
                    w = torch.cat([w[0::2], w[1::2]], 0)
                    name = name.replace(".mlp.up_proj.", ".mlp.gate_up_il.")
                yield name, w

        return super().load_hf_weights(deinterleave())

    def _load_mlp(self, i: int, p: dict, put) -> None:
        super()._load_mlp(i, p, put)
        if "gate_up.bias" in p:
            tp = self.tp
            g, u = p["gate_up.bias"].chunk(2, 0)
            self.b_gu[i] = put(torch.cat([g.narrow(0, tp.rank * tp.inter, tp.inter),
                                          u.narrow(0, tp.rank * tp.inter, tp.inter)], 0))

    def weight_bytes(self) -> int:
        return super().weight_bytes() + sum(b.numel() * b.element_size() for b in self.b_gu if b is not None)

    # ------------------------------------------------------------------ forward
    def _mlp(self, i: int, x: torch.Tensor) -> torch.Tensor:
        return linear(ops.act_and_mul(linear(x, self.w_gu[i], self.b_gu[i]), self.act), self.w_d[i], self.b_d[i])

    def _attn_block(self, i: int, x: torch.Tensor, meta: AttnMeta, kv: PagedKVCache) -> torch.Tensor:
        self._layer_bs = self.bs if self.sparse_layer[i] else None
        return super()._attn_block(i, x, meta, kv)

    def attention(self, q, k_cache, v_cache, meta: AttnMeta, ks: float = 1.0, vs: float = 1.0) -> torch.Tensor:
        bs = self._layer_bs
        if bs is None:
            return super().attention(q, k_cache, v_cache, meta, ks, vs)
        if meta.is_decode:
            return ops.paged_decode(q, k_cache, v_cache, meta.block_tables, meta.seq_lens, self.scale,
                                    meta.decode_ws, self.window, order=meta.order, k_scale=ks, v_scale=vs,
                                    blocksparse=bs)
        if meta.mode == "mixed":
            n = meta.num_prefill
            out = torch.empty_like(q)
            ops.paged_prefill(q[:n], k_cache, v_cache, meta.block_tables, meta.cu_q, meta.kv_lens, meta.items,
                              self.scale, self.window, out=out[:n], k_scale=ks, v_scale=vs, blocksparse=bs)
            ops.paged_decode(q[n:], k_cache, v_cache, meta.dec_block_tables, meta.seq_lens, self.scale,
                             meta.decode_ws, self.window, out=out[n:], order=meta.order, k_scale=ks, v_scale=vs,
                             blocksparse=bs)
            return out
        return ops.paged_prefill(q, k_cache, v_cache, meta.block_tables, meta.cu_q, meta.kv_lens, meta.items,
                                 self.scale, self.window, k_scale=ks, v_scale=vs, blocksparse=bs)
