"""Grok-1 / Grok-2 (xAI) sparse MoE decoders on the ome_amd kernels.

Reference catalog: ``config/runtimes/srt/xai-org/grok-1-rt.yaml:14`` (``Grok1ModelForCausalLM``,
314B, 8 experts top-2) and ``grok-2-rt.yaml:14`` (``Grok1ForCausalLM``, the xai-org/grok-2
checkpoint).  On MI355X the bf16 weights (~630 GB) fit one 8-GPU xGMI node at TP=8 with ~210 GB
of HBM3E left per GPU for KV; experts are tensor-parallel over their intermediate dimension so
every MoE layer costs exactly one all-reduce, like the dense family.

Differences from the Mixtral path (``moe.py``), all inside the same kernels:

* sandwich RMSNorms: ``pre_attn_norm`` -> attention -> ``post_attn_norm`` -> residual add,
  ``pre_moe_norm`` -> MoE -> ``post_moe_norm`` -> residual add (plain ``w * x`` norms);
* embeddings scaled by ``embedding_multiplier_scale``, logits by ``output_multiplier_scale``;
* attention logits scaled by ``attn_output_multiplier`` and soft-capped
  (``max_attn_value`` / ``attn_logit_softcapping``: ``cap * tanh(s / cap)`` inside the MFMA
  attention kernels);
* GELU (tanh) gated experts; softmax top-2 routing *without* renormalisation;
* Grok-2 only: router-logit soft-capping, final-logit soft-capping, and ``residual_moe`` -- a
  dense GeGLU MLP beside the experts, ``(mlp(x) + moe(x)) / sqrt(2)``, both partial sums sharing
  one TP all-reduce.

Weight names: the hpcai-tech Grok-1 layout (``attn.*``, ``moe_block.experts.N.linear /
linear_v / linear_1``) and the xai-org/SGLang layout (``self_attn.*``, ``block_sparse_moe.experts.N.
w1 / w3 / w2``, residual ``mlp.*``) both load.  Grok-2's ``attn_temperature_len`` (a
length-dependent query temperature) is not modelled -- parity unpinned, no reference
implementation is importable here.
"""
from __future__ import annotations

import logging
import math

import torch

from ome_amd import ops
from ome_amd.models.common import AttnMeta, PagedKVCache
from ome_amd.models.config import ModelConfig
from ome_amd.models.moe import MoEForCausalLM
from ome_amd.models.quant import linear
from ome_amd.parallel import state as pstate

GROK_ARCHS = {"Grok1ModelForCausalLM", "Grok1ForCausalLM"}
log = logging.getLogger("ome_amd.models.grok")

_EXPERT_NAMES = {"linear": "w1", "linear_v": "w3", "linear_1": "w2"}


class GrokForCausalLM(MoEForCausalLM):
    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        ex = cfg.extra or {}
        self.act = 1                 # GELU (tanh approximation, as jax.nn.gelu) gated experts
        self.renorm = False          # softmax top-k weights are used as they are
        self.scale = float(ex.get("attn_output_multiplier") or cfg.head_dim ** -0.5)
        self.softcap = float(ex.get("attn_logit_softcapping") or ex.get("max_attn_value") or 0.0)
        self.router_cap = float(ex.get("router_logit_softcapping") or 0.0)
        self.final_cap = float(ex.get("final_logit_softcapping") or 0.0)
        self.emb_mult = float(ex.get("embedding_multiplier_scale") or 1.0)
        self.out_mult = float(ex.get("output_multiplier_scale") or 1.0)
        self.residual_moe = bool(ex.get("residual_moe", False))
        if ex.get("attn_temperature_len", -1) and ex.get("attn_temperature_len", -1) > 0:
            log.warning("grok: attn_temperature_len=%s is not modelled", ex["attn_temperature_len"])
        L = cfg.num_layers
        self.post_attn: list[torch.Tensor | None] = [None] * L
        self.post_moe: list[torch.Tensor | None] = [None] * L
        self.w_rgu: list[torch.Tensor | None] = [None] * L    # residual dense MLP (Grok-2)
        self.w_rd: list[torch.Tensor | None] = [None] * L

    # ------------------------------------------------------------------ weights
    def init_random(self, seed: int = 0, std: float = 0.02) -> "GrokForCausalLM":
        super().init_random(seed, std)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 65537 + 7919 * pstate.get().tp_rank)
        H, I = self.cfg.hidden_size, self.tp.inter
        for i in self.layers:
            self.post_attn[i] = self._alloc(H, std=None, gen=None)
            self.post_moe[i] = self._alloc(H, std=None, gen=None)
            if self.residual_moe:
                self.w_rgu[i] = self._alloc(2 * I, H, std=std, gen=gen)
                self.w_rd[i] = self._alloc(H, I, std=std / math.sqrt(2 * self.cfg.num_layers), gen=gen)
        return self

    @staticmethod
    def _rename(name: str) -> str | None:
        """Checkpoint name -> the Mixtral-style names the MoE loader reads (None: captured here)."""
        parts = name.split(".")
        if "layers" not in parts:
            return name
        j = parts.index("layers") + 2
        if j >= len(parts):
            return name
        head, mod, rest = parts[:j], parts[j], parts[j + 1:]
        if mod == "attn":
            mod = "self_attn"
        elif mod == "moe_block":
            mod = "block_sparse_moe"
            if len(rest) >= 3 and rest[0] == "experts" and rest[2] in _EXPERT_NAMES:
                rest = rest[:2] + [_EXPERT_NAMES[rest[2]]] + rest[3:]
        elif mod == "pre_attn_norm":
            mod = "input_layernorm"
        elif mod == "pre_moe_norm":
            mod = "post_attention_layernorm"
        elif mod in ("post_attn_norm", "post_moe_norm", "mlp"):
            return None
        return ".".join(head + [mod] + rest)

    def load_hf_weights(self, weights) -> "GrokForCausalLM":
        tp = self.tp
        caught: dict[tuple[int, str], torch.Tensor] = {}

        def stream():
            for name, w in weights:
                new = self._rename(name)
                if new is not None:
                    yield new, w
                    continue
                parts = name.split(".")
                j = parts.index("layers")
                i = int(parts[j + 1])
                if i in self._layer_set:
                    caught[(i, ".".join(parts[j + 2:]))] = w

        super().load_hf_weights(stream())
        put = lambda t: t.to(device=self.device, dtype=self.dtype).contiguous()  # noqa: E731
        I = tp.inter
        for i in self.layers:
            self.post_attn[i] = put(caught.pop((i, "post_attn_norm.weight")))
            self.post_moe[i] = put(caught.pop((i, "post_moe_norm.weight")))
            if self.residual_moe:
                g, u = caught.pop((i, "mlp.gate_proj.weight")), caught.pop((i, "mlp.up_proj.weight"))
                d = caught.pop((i, "mlp.down_proj.weight"))
                s = tp.rank * I
                self.w_rgu[i] = put(torch.cat([g.narrow(0, s, min(I, g.shape[0] - s)),
                                               u.narrow(0, s, min(I, u.shape[0] - s))], 0))
                self.w_rd[i] = put(d.narrow(1, s, min(I, d.shape[1] - s)))
        return self

    def weight_bytes(self) -> int:
        n = super().weight_bytes()
        for lst in (self.post_attn, self.post_moe, self.w_rgu, self.w_rd):
            n += sum(t.numel() * t.element_size() for t in lst if t is not None)
        return n

    # ------------------------------------------------------------------ forward
    def router_logits(self, i: int, x: torch.Tensor) -> torch.Tensor:
        logits = super().router_logits(i, x)
        if self.router_cap > 0:
            c = self.router_cap
            logits = torch.tanh(logits.float() / c) * c
        return logits

    def mlp(self, i: int, x: torch.Tensor) -> torch.Tensor:
        out = self._moe_partial(i, x)
        if self.residual_moe:
            dense = linear(ops.act_and_mul(linear(x, self.w_rgu[i]), self.act), self.w_rd[i])
            out = (out + dense) * (1.0 / math.sqrt(2.0))
        return pstate.tp_all_reduce(out)

    def _stage_input(self, ids: torch.Tensor, input_embeds: torch.Tensor | None):
        st = pstate.get()
        T, H = ids.shape[0], self.cfg.hidden_size
        if st.pp_size > 1 and not st.is_first_pp:
            return pstate.pp_recv(((T, H), self.dtype, ids.device), ((T, H), self.dtype, ids.device))
        if input_embeds is None:
            h = pstate.tp_all_reduce(ops.embedding(ids, self.embed, self.tp.vocab_start, self.tp.vocab_end))
            h = h * self.emb_mult
        else:
            h = input_embeds
        return ops.rmsnorm(h, self.ln1[self.layers[0]], self.eps), h

    def forward(self, ids: torch.Tensor, meta: AttnMeta, kv: PagedKVCache,
                input_embeds: torch.Tensor | None = None) -> torch.Tensor:
        cfg, tp, D = self.cfg, self.tp, self.D
        T = ids.shape[0]
        x, residual = self._stage_input(ids, input_embeds)
        for i in self.layers:
            if i > 0:   # previous layer's (post-normed) MoE output joins the residual stream
                ops.fused_add_rmsnorm(x, residual, self.ln1[i], self.eps)
            qkv = linear(x, self.w_qkv[i], self.b_qkv[i])
            q = torch.empty(T, tp.hq, D, dtype=self.dtype, device=x.device)
            k_cache, v_cache = kv.layer(i)
            ks, vs = kv.scales(i)
            ops.rope_qkv_cache(qkv, meta.positions, self.cos_sin, cfg.rot_dim, q, k_cache, v_cache, meta.slots,
                               tp.hq, tp.hkv, D, True, self.qn[i], self.kn[i], self.eps, ks, vs)
            attn = self.attention(q, k_cache, v_cache, meta, ks, vs)
            o = pstate.tp_all_reduce(linear(attn.view(T, tp.hq * D), self.w_o[i]))
            o = ops.rmsnorm(o, self.post_attn[i], self.eps)
            ops.fused_add_rmsnorm(o, residual, self.ln2[i], self.eps)
            x = ops.rmsnorm(self.mlp(i, o), self.post_moe[i], self.eps)
        return self._stage_output(x, residual)

    def compute_logits(self, hidden: torch.Tensor) -> torch.Tensor:
        logits = super().compute_logits(hidden)
        if self.out_mult != 1.0 or self.final_cap > 0:
            lf = logits.float() * self.out_mult
            if self.final_cap > 0:
                lf = torch.tanh(lf / self.final_cap) * self.final_cap
            logits = lf.to(logits.dtype)
        return logits
