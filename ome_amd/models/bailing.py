"""Bailing MoE (Ling-lite / Ling-plus, ``BailingMoeForCausalLM``; reference catalog
``config/runtimes/srt/inclusionAI/ling-lite-rt.yaml``, ``ling-plus-rt.yaml``).

A Llama-style decoder whose MLPs are sparse MoE: softmax top-k router (``norm_topk_prob``
renormalisation), SwiGLU experts, ``num_shared_experts`` always-on experts fused into one
SwiGLU of width ``num_shared_experts * moe_intermediate_size`` (no gate), optional dense first
layers (``first_k_dense_replace``) -- i.e. the ``moe.py`` path, with the checkpoint's names
mapped at load:
* ``word_embeddings`` -> embeddings; fused ``attention.query_key_value`` ([q | k | v] rows,
  bias with ``use_qkv_bias``) -> the fused QKV projection; ``attention.dense`` -> o_proj;
  ``mlp.shared_experts.*`` -> the shared expert;
* ``norm_head``: the LM head is L2-normalised over the vocabulary dimension (each hidden
  column, eps 1e-7) once at load.
Parity: there is no transformers implementation of this family; the test checks the mapping
against an equivalent transformers Qwen2-MoE (the shared-expert gate held at sigmoid(0) and
compensated in the shared down projection) -- the Bailing semantics themselves are parity-unpinned.
"""
from __future__ import annotations

import dataclasses

import torch

from ome_amd.models.config import ModelConfig
from ome_amd.models.moe import MoEForCausalLM


def _bailing_cfg(cfg: ModelConfig) -> ModelConfig:
    ex = cfg.extra or {}
    ns = int(ex.get("num_shared_experts") or 0)
    return dataclasses.replace(cfg, shared_expert_intermediate_size=ns * int(cfg.moe_intermediate_size or 0),
                               num_shared_experts=ns,
                               attention_bias=bool(ex.get("use_qkv_bias", False) or ex.get("use_bias", False)))


class BailingMoeForCausalLM(MoEForCausalLM):
    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(_bailing_cfg(cfg), device, dtype, max_positions)
        ex = cfg.extra or {}
        if ex.get("use_bias", False):
            raise NotImplementedError("Bailing use_bias (biased dense / MLP projections)")
        self.norm_head = bool(ex.get("norm_head", False))

    def load_hf_weights(self, weights) -> "BailingMoeForCausalLM":
        cfg, D = self.cfg, self.D
        q_rows, kv_rows = cfg.num_heads * D, cfg.num_kv_heads * D

        def renamed():
            for name, w in weights:
                n = name[len("model."):] if name.startswith("model.") else name
                if n == "word_embeddings.weight":
                    yield "model.embed_tokens.weight", w
                elif n == "lm_head.weight" or name == "lm_head.weight":
                    if self.norm_head:
                        w = torch.nn.functional.normalize(w.float(), dim=0, eps=1e-7)
                    yield "lm_head.weight", w
                elif ".attention.query_key_value." in n:
                    pre, kind = n.split(".attention.query_key_value.")
                    q, k, v = w.split([q_rows, kv_rows, kv_rows], 0)
                    for nm, t in (("q_proj", q), ("k_proj", k), ("v_proj", v)):
                        yield f"model.{pre}.self_attn.{nm}.{kind}", t
                elif ".attention.dense." in n:
                    pre, kind = n.split(".attention.dense.")
                    yield f"model.{pre}.self_attn.o_proj.{kind}", w
                elif ".mlp.shared_experts." in n:
                    yield "model." + n.replace(".mlp.shared_experts.", ".mlp.shared_expert."), w
                else:
                    yield name, w

        return super().load_hf_weights(renamed())
