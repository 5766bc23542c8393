"""LayerNorm decoder families: Starcoder2 (``Starcoder2ForCausalLM``), GPT-NeoX / Pythia
(``GPTNeoXForCausalLM``) and Phi-1/1.5/2 (``PhiForCausalLM``) on the ome_amd kernels.

Reference catalog entries: ``config/runtimes/srt/bigcode/starcoder2-*`` style runtimes and the
generic HF-architecture runtime match (``pkg/runtimeselector`` picks a runtime by
``modelArchitecture``); the reference serves these through its SGLang/vLLM images.  What differs
from the Llama path (``llama.py``):

* LayerNorm with bias (mean/variance) instead of RMSNorm: ``ops.layernorm`` /
  ``ops.fused_add_layernorm`` (HIP ``ome_layernorm``; the residual add is fused the same way the
  RMSNorm kernel fuses it);
* biases on every projection; the row-parallel biases (attention output, MLP down) are loaded on
  TP rank 0 only so the all-reduce adds them once;
* non-gated MLP ``proj(act(fc(x)))`` with GELU-tanh (Starcoder2) or exact GELU (GPT-NeoX),
  run in place by ``ops.act`` (HIP ``ome_act``) between two hipBLASLt GEMMs;
* GPT-NeoX: fused per-head ``query_key_value`` [heads, 3, D] re-ordered at load time into the
  [Q; K; V] layout of the fused RoPE/KV-cache kernel, partial rotary (``rotary_pct``; the kernel
  rotates the first ``rot_dim`` dims, NeoX ``rotate_half`` form) and the *parallel residual*
  ``h + attn(ln1(h)) + mlp(ln2(h))`` -- the two row-parallel partial sums are added before ONE
  TP all-reduce per layer (half the collectives of the sequential form);
* Starcoder2: GQA, sliding window (``sliding_window``), tied embeddings.
* Phi-2: parallel residual with ONE shared LayerNorm per layer (``h + attn(ln(h)) + mlp(ln(h))``:
  the norm output feeds both branches, no second norm launch), partial rotary
  (``partial_rotary_factor`` 0.4), GELU-tanh MLP ``fc1``/``fc2`` and a biased ``lm_head`` (the bias is
  vocab-sharded with the head so each TP rank adds its slice before the all-gather).  Phi-2's
  head_dim 80 is zero-padded per head to the 128 kernel tile at load time (``cfg.attn_head_dim``
  keeps 80 for the softmax scale); the pad costs 1.6x KV bytes but keeps the MFMA tiles.
"""
from __future__ import annotations

import math

import torch

from ome_amd import ops
from ome_amd.models.common import AttnMeta, PagedKVCache
from ome_amd.models.config import ModelConfig
from ome_amd.models.llama import LlamaForCausalLM
from ome_amd.models.quant import linear
from ome_amd.parallel import state as pstate

LAYERNORM_ARCHS = {"Starcoder2ForCausalLM", "GPTNeoXForCausalLM", "PhiForCausalLM"}

_ACTS = {"gelu_pytorch_tanh": 1, "gelu_new": 1, "gelu_fast": 1, "gelu": 3, "silu": 0, "swish": 0}


class LayerNormForCausalLM(LlamaForCausalLM):
    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        hf = cfg.extra or {}
        self.neox = cfg.model_type == "gpt_neox" or cfg.architecture == "GPTNeoXForCausalLM"
        self.phi = cfg.model_type == "phi" or cfg.architecture == "PhiForCausalLM"
        if self.phi and hf.get("qk_layernorm"):
            raise NotImplementedError("Phi qk_layernorm")
        self.Dt = cfg.attn_head_dim or self.D  # checkpoint head dim (< D when zero-padded, Phi-2)
        if self.Dt != self.D:
            self.scale = 1.0 / math.sqrt(self.Dt)
        self.parallel_residual = self.phi or (self.neox and bool(hf.get("use_parallel_residual", True)))
        act = cfg.hidden_act
        if act not in _ACTS:
            raise NotImplementedError(f"hidden_act {act!r}")
        self.act = _ACTS[act]
        L = cfg.num_layers
        self.ln1b: list[torch.Tensor | None] = [None] * L
        self.ln2b: list[torch.Tensor | None] = [None] * L
        self.b_o: list[torch.Tensor | None] = [None] * L
        self.b_fc: list[torch.Tensor | None] = [None] * L
        self.b_d: list[torch.Tensor | None] = [None] * L
        self.norm_b: torch.Tensor | None = None
        self.lm_head_b: torch.Tensor | None = None

    # ------------------------------------------------------------------ weights
    def init_random(self, seed: int = 0, std: float = 0.02) -> "LayerNormForCausalLM":
        cfg, tp, D = self.cfg, self.tp, self.D
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 7919 * pstate.get().tp_rank)
        H, r0 = cfg.hidden_size, tp.rank == 0
        rows = (tp.hq + 2 * tp.hkv) * D
        zeros = lambda *s: torch.zeros(*s, dtype=self.dtype, device=self.device)  # noqa: E731
        for i in self.layers:
            self.w_qkv[i] = self._alloc(rows, H, std=std, gen=gen)
            self.b_qkv[i] = self._alloc(rows, std=std, gen=gen)
            self.w_o[i] = self._alloc(H, tp.hq * D, std=std / math.sqrt(2 * cfg.num_layers), gen=gen)
            self.b_o[i] = self._alloc(H, std=std, gen=gen) if r0 else zeros(H)
            self.ln1[i], self.ln2[i] = self._alloc(H, std=None, gen=gen), self._alloc(H, std=None, gen=gen)
            self.ln1b[i], self.ln2b[i] = zeros(H), zeros(H)
            self.w_gu[i] = self._alloc(tp.inter, H, std=std, gen=gen)
            self.b_fc[i] = self._alloc(tp.inter, std=std, gen=gen)
            self.w_d[i] = self._alloc(H, tp.inter, std=std / math.sqrt(2 * cfg.num_layers), gen=gen)
            self.b_d[i] = self._alloc(H, std=std, gen=gen) if r0 else zeros(H)
            if self.Dt != D:  # zero the per-head pad dims, as a padded checkpoint has them
                self.w_qkv[i].view(-1, D, H)[:, self.Dt:].zero_()
                self.b_qkv[i].view(-1, D)[:, self.Dt:].zero_()
                self.w_o[i].view(H, -1, D)[:, :, self.Dt:].zero_()
        self.embed = self._alloc(tp.vocab, H, std=1.0, gen=gen)
        self.norm, self.norm_b = self._alloc(H, std=None, gen=gen), zeros(H)
        self.lm_head = self.embed if cfg.tie_word_embeddings else self._alloc(tp.vocab, H, std=std, gen=gen)
        if self.phi:
            self.lm_head_b = self._alloc(tp.vocab, std=std, gen=gen)
        self._post_load()
        return self

    def load_hf_weights(self, weights) -> "LayerNormForCausalLM":
        cfg, tp, D = self.cfg, self.tp, self.D
        H, nh = cfg.hidden_size, cfg.num_heads
        qkv: dict[int, dict[str, torch.Tensor]] = {}
        r0 = tp.rank == 0

        def put(t):
            return t.to(device=self.device, dtype=self.dtype).contiguous()

        def inter_rows(t):  # column-parallel fc: rows of this rank
            n = min(tp.inter, t.shape[0] - tp.rank * tp.inter)
            return t.narrow(0, tp.rank * tp.inter, n)

        Dt = self.Dt

        def pad_rows(t):  # [heads * Dt, ...] -> [heads * D, ...], zero-padding every head
            if Dt == D:
                return t
            t = t.reshape(-1, Dt, *t.shape[1:])
            z = t.new_zeros(t.shape[0], D - Dt, *t.shape[2:])
            return torch.cat([t, z], 1).reshape(-1, *t.shape[2:])

        def row_bias(t):  # row-parallel bias: rank 0 only
            return put(t) if r0 else torch.zeros(t.shape, dtype=self.dtype, device=self.device)

        for name, w in weights:
            for pre in ("gpt_neox.", "model."):
                if name.startswith(pre):
                    name = name[len(pre):]
                    break
            if name in ("embed_in.weight", "embed_tokens.weight"):
                self.embed = put(self._vocab_shard(w))
                continue
            if name in ("embed_out.weight", "lm_head.weight"):
                self.lm_head = put(self._vocab_shard(w))
                continue
            if name == "lm_head.bias":
                self.lm_head_b = put(self._vocab_shard(w[:, None])[:, 0])
                continue
            if name in ("final_layer_norm.weight", "norm.weight", "final_layernorm.weight"):
                self.norm = put(w)
                continue
            if name in ("final_layer_norm.bias", "norm.bias", "final_layernorm.bias"):
                self.norm_b = put(w)
                continue
            parts = name.split(".")
            if parts[0] != "layers":
                continue
            i, rest = int(parts[1]), ".".join(parts[2:])
            if i not in self._layer_set:
                continue
            kind = rest.rsplit(".", 1)[-1]  # weight / bias
            if rest.startswith("attention.query_key_value."):
                # [heads, 3, D, (H)] -> this rank's heads, split into q / k / v
                t = w.reshape(nh, 3, D, *w.shape[1:]).narrow(0, tp.rank * tp.hq, tp.hq)
                d = qkv.setdefault(i, {})
                for j, c in enumerate("qkv"):
                    d[c + kind] = t[:, j].reshape(tp.hq * D, *w.shape[1:])
            elif rest.startswith("self_attn.q_proj."):
                qkv.setdefault(i, {})["q" + kind] = pad_rows(w.narrow(0, tp.rank * tp.hq * Dt, tp.hq * Dt))
            elif rest.startswith(("self_attn.k_proj.", "self_attn.v_proj.")):
                qkv.setdefault(i, {})[rest[10] + kind] = pad_rows(w.narrow(0, tp.kv_start * Dt, tp.hkv * Dt))
            elif rest in ("attention.dense.weight", "self_attn.o_proj.weight", "self_attn.dense.weight"):
                self.w_o[i] = put(pad_rows(w.narrow(1, tp.rank * tp.hq * Dt, tp.hq * Dt).t()).t())
            elif rest in ("attention.dense.bias", "self_attn.o_proj.bias", "self_attn.dense.bias"):
                self.b_o[i] = row_bias(w)
            elif rest in ("mlp.dense_h_to_4h.weight", "mlp.c_fc.weight", "mlp.fc1.weight"):
                self.w_gu[i] = put(inter_rows(w))
            elif rest in ("mlp.dense_h_to_4h.bias", "mlp.c_fc.bias", "mlp.fc1.bias"):
                self.b_fc[i] = put(inter_rows(w))
            elif rest in ("mlp.dense_4h_to_h.weight", "mlp.c_proj.weight", "mlp.fc2.weight"):
                self.w_d[i] = put(w.narrow(1, tp.rank * tp.inter, min(tp.inter, w.shape[1] - tp.rank * tp.inter)))
            elif rest in ("mlp.dense_4h_to_h.bias", "mlp.c_proj.bias", "mlp.fc2.bias"):
                self.b_d[i] = row_bias(w)
            elif rest.startswith("input_layernorm."):
                (self.ln1 if kind == "weight" else self.ln1b)[i] = put(w)
            elif rest.startswith("post_attention_layernorm."):
                (self.ln2 if kind == "weight" else self.ln2b)[i] = put(w)
        for i, p in qkv.items():
            self.w_qkv[i] = put(torch.cat([p["qweight"], p["kweight"], p["vweight"]], 0))
            if "qbias" in p:
                self.b_qkv[i] = put(torch.cat([p["qbias"], p["kbias"], p["vbias"]], 0))
        if self.lm_head is None:
            self.lm_head = self.embed
        missing = [i for i in self.layers if self.w_qkv[i] is None or self.w_gu[i] is None or self.w_d[i] is None]
        if missing or self.embed is None:
            raise ValueError(f"checkpoint incomplete: layers missing {missing[:4]}...")
        self._post_load()
        return self

    def weight_bytes(self) -> int:
        n = super().weight_bytes()
        for lst in (self.ln1b, self.ln2b, self.b_o, self.b_fc, self.b_d, [self.norm_b, self.lm_head_b]):
            n += sum(t.numel() * t.element_size() for t in lst if t is not None)
        return n

    # ------------------------------------------------------------------ forward
    def mlp(self, i: int, x: torch.Tensor, reduce: bool = True) -> torch.Tensor:
        h = linear(x, self.w_gu[i], self.b_fc[i])
        ops.act(h, self.act)
        y = linear(h, self.w_d[i], self.b_d[i])
        return pstate.tp_all_reduce(y) if reduce else y

    def _stage_input(self, ids: torch.Tensor, input_embeds: torch.Tensor | None):
        st = pstate.get()
        T, H = ids.shape[0], self.cfg.hidden_size
        if st.pp_size > 1 and not st.is_first_pp:
            return pstate.pp_recv(((T, H), self.dtype, ids.device), ((T, H), self.dtype, ids.device))
        if input_embeds is None:
            h = pstate.tp_all_reduce(ops.embedding(ids, self.embed, self.tp.vocab_start, self.tp.vocab_end))
        else:
            h = input_embeds
        return ops.layernorm(h, self.ln1[0], self.ln1b[0], self.eps), h

    def _attn_block(self, i: int, x: torch.Tensor, meta: AttnMeta, kv: PagedKVCache) -> torch.Tensor:
        """Attention sub-block up to the row-parallel output projection (not yet reduced)."""
        cfg, tp, D = self.cfg, self.tp, self.D
        T = x.shape[0]
        qkv = linear(x, self.w_qkv[i], self.b_qkv[i])
        q = torch.empty(T, tp.hq, D, dtype=self.dtype, device=x.device)
        k_cache, v_cache = kv.layer(i)
        ks, vs = kv.scales(i)
        ops.rope_qkv_cache(qkv, meta.positions, self.cos_sin, cfg.rot_dim, q, k_cache, v_cache, meta.slots,
                           tp.hq, tp.hkv, D, True, None, None, self.eps, ks, vs)
        attn = self.attention(q, k_cache, v_cache, meta, ks, vs)
        return linear(attn.view(T, tp.hq * D), self.w_o[i], self.b_o[i])

    def forward(self, ids: torch.Tensor, meta: AttnMeta, kv: PagedKVCache,
                input_embeds: torch.Tensor | None = None) -> torch.Tensor:
        x, residual = self._stage_input(ids, input_embeds)
        for i in self.layers:
            if i > 0:  # x holds the previous layer's block output: add it, normalise for this layer
                ops.fused_add_layernorm(x, residual, self.ln1[i], self.ln1b[i], self.eps)
            if self.parallel_residual:
                x2 = x if self.phi else ops.layernorm(residual, self.ln2[i], self.ln2b[i], self.eps)
                o = self._attn_block(i, x, meta, kv)
                x = pstate.tp_all_reduce(o + self.mlp(i, x2, reduce=False))
            else:
                o = pstate.tp_all_reduce(self._attn_block(i, x, meta, kv))
                ops.fused_add_layernorm(o, residual, self.ln2[i], self.ln2b[i], self.eps)
                x = self.mlp(i, o)
        return self._stage_output(x, residual)

    def _stage_output(self, x: torch.Tensor, residual: torch.Tensor) -> torch.Tensor | None:
        st = pstate.get()
        if st.pp_size > 1 and not st.is_last_pp:
            pstate.pp_send(x, residual)
            return None
        ops.fused_add_layernorm(x, residual, self.norm, self.norm_b, self.eps)
        return x

    def compute_logits(self, hidden: torch.Tensor) -> torch.Tensor:
        if self.lm_head_b is None:
            return super().compute_logits(hidden)
        logits = linear(hidden, self.lm_head, self.lm_head_b)
        if self.tp.tp > 1:
            logits = pstate.tp_all_gather(logits, dim=-1)
        return logits[:, : self.cfg.vocab_size]
