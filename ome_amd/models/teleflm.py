"""Tele-FLM (CofeAI, ``TeleFLMModel``) on the dense Llama path.

Reference catalog: ``config/runtimes/srt/CofeAI/tele-flm-rt.yaml:14`` (52B, served with
``--trust-remote-code``).  Tele-FLM is a Llama-layout decoder (RMSNorm, RoPE, SwiGLU, GQA) trained
with muP width scaling; serving it needs only the two muP multipliers of its remote code:

* token embeddings are scaled by ``input_mult`` (when ``use_mup``);
* LM-head logits are scaled by ``output_mult / mup_scale_factor`` (when ``use_mup``).

Everything else -- fused QKV / gate_up GEMMs, the stream-K GEMM routing, rank-sliced TP loading,
HIP graphs -- is the Llama path unchanged (``plain_layout``).  At bf16 the 52B checkpoint
(~104 GB) fits one MI355X (288 GB HBM3E) at TP=1.  transformers has no Tele-FLM class, so parity
with the remote code is unpinned beyond ``tests/test_teleflm_cpu.py``'s fp32 reference.
"""
from __future__ import annotations

import torch

from ome_amd import ops
from ome_amd.models.config import ModelConfig
from ome_amd.models.llama import LlamaForCausalLM
from ome_amd.parallel import state as pstate

TELEFLM_ARCHS = {"TeleFLMModel", "TeleFLMForCausalLM"}


class TeleFLMForCausalLM(LlamaForCausalLM):
    plain_layout = True

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        ex = cfg.extra or {}
        mup = bool(ex.get("use_mup", False))
        self.input_mult = float(ex.get("input_mult", 1.0)) if mup else 1.0
        self.logit_mult = float(ex.get("output_mult", 1.0)) / float(ex.get("mup_scale_factor", 1.0)) if mup else 1.0

    def _stage_input(self, ids: torch.Tensor, input_embeds: torch.Tensor | None):
        st = pstate.get()
        if (st.pp_size > 1 and not st.is_first_pp) or input_embeds is not None or self.input_mult == 1.0:
            return super()._stage_input(ids, input_embeds)
        h = pstate.tp_all_reduce(ops.embedding(ids, self.embed, self.tp.vocab_start, self.tp.vocab_end))
        h = h * self.input_mult
        return ops.rmsnorm(h, self.ln1[0], self.eps), h

    def compute_logits(self, hidden: torch.Tensor) -> torch.Tensor:
        logits = super().compute_logits(hidden)
        if self.logit_mult != 1.0:
            logits = (logits.float() * self.logit_mult).to(logits.dtype)
        return logits
