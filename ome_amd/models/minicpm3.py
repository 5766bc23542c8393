"""MiniCPM3 (``MiniCPM3ForCausalLM``; reference catalog ``config/runtimes/srt/openbmb/minicpm3-4b-rt.yaml``).

MiniCPM3 is multi-head latent attention with a narrower latent than DeepSeek: kv_lora_rank 256 +
qk_rope_head_dim 32, so every layer caches ONE 288-wide latent row per token (the (288, 256)
instance of ``csrc/kernels/mla.hip``; 40 heads run as head groups of 16 with a partial last
group), non-interleaved (NeoX) RoPE with LongRoPE factors, and a dense SwiGLU MLP.  The
muP-style scalings of the family are folded into weights once, so the forward is the
DeepSeek MLA path of ``deepseek.py`` unchanged:
* ``scale_emb`` into the embedding table (the LM head keeps its own unscaled copy when tied);
* the residual-branch factor ``scale_depth / sqrt(num_layers)`` into ``o_proj`` and ``down_proj``;
* the logit divisor ``hidden_size / dim_model_base`` into the final RMSNorm weight.
"""
from __future__ import annotations

import math

import torch

from ome_amd.models.config import ModelConfig
from ome_amd.models.deepseek import DeepseekForCausalLM


class MiniCPM3ForCausalLM(DeepseekForCausalLM):
    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        ex = cfg.extra or {}
        self.interleaved_rope = False   # MiniCPM3 rotates halves (rotate_half), not DeepSeek's pairs
        self.scale_emb = float(ex.get("scale_emb", 1.0))
        depth = ex.get("scale_depth")
        self.res_scale = (float(depth) / math.sqrt(cfg.num_layers)) if depth is not None else 1.0
        base = ex.get("dim_model_base")
        self.logit_div = cfg.hidden_size / float(base) if base else 1.0

    def _post_load(self) -> None:
        for lst in (self.w_o, self.w_d):
            for i in self.layers:
                if lst[i] is not None:
                    lst[i] = (lst[i].float() * self.res_scale).to(self.dtype)
        if self.norm is not None:
            self.norm = (self.norm.float() / self.logit_div).to(self.dtype)
        if self.embed is not None:
            if self.lm_head is self.embed:
                self.lm_head = self.embed.clone()
            self.embed = (self.embed.float() * self.scale_emb).to(self.dtype)
        super()._post_load()
