"""XVERSE MoE (``XverseMoeForCausalLM``, XVERSE-MoE-A36B; reference catalog
``config/runtimes/srt/xverse/xverse-moe-a36b-rt.yaml``).

Llama attention (separate q / k / v / o, no biases) and a sparse MoE MLP: softmax top-``moe_top_k``
router (``mlp.router``; renormalised only with ``norm_topk_prob``), SwiGLU experts of width
``intermediate_size``, and ``num_shared_experts`` always-on experts fused into one SwiGLU of width
``num_shared_experts * intermediate_size`` (no gate) -- the ``moe.py`` path with the config keys
and checkpoint names mapped.  Parity: no transformers implementation exists; the test pins the
mapping against an equivalent re-laid transformers Qwen2-MoE (XVERSE semantics parity-unpinned).
"""
from __future__ import annotations

import dataclasses

import torch

from ome_amd.models.config import ModelConfig
from ome_amd.models.moe import MoEForCausalLM


def _xverse_cfg(cfg: ModelConfig) -> ModelConfig:
    ex = cfg.extra or {}
    I = int(ex.get("intermediate_size") or cfg.intermediate_size)
    ns = int(ex.get("num_shared_experts") or 0)
    return dataclasses.replace(cfg, num_experts=int(ex.get("num_experts") or cfg.num_experts),
                               num_experts_per_tok=int(ex.get("moe_top_k") or cfg.num_experts_per_tok or 2),
                               moe_intermediate_size=I, shared_expert_intermediate_size=ns * I, num_shared_experts=ns,
                               norm_topk_prob=bool(ex.get("norm_topk_prob", False)), attention_bias=False)


class XverseMoeForCausalLM(MoEForCausalLM):
    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(_xverse_cfg(cfg), device, dtype, max_positions)

    def load_hf_weights(self, weights) -> "XverseMoeForCausalLM":
        def renamed():
            for name, w in weights:
                if ".mlp.router." in name:
                    yield name.replace(".mlp.router.", ".mlp.gate."), w
                elif ".mlp.shared_experts." in name:
                    yield name.replace(".mlp.shared_experts.", ".mlp.shared_expert."), w
                else:
                    yield name, w

        return super().load_hf_weights(renamed())
