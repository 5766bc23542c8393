"""DeciLM / Llama-Nemotron NAS decoders (``DeciLMForCausalLM``: Llama-3.3-Nemotron-Super-49B,
Llama-3.1-Nemotron-Ultra-253B; reference catalog ``config/runtimes/srt/nvidia/llama-3-3-nemotron-super-49b-v1-rt.yaml``,
``config/runtimes/vllm/llama-3-1-nemotron-ultra-253b-v1-rt.yaml``).

A Llama decoder whose blocks were searched per layer (``block_configs``):
* attention: GQA with a per-layer group size ``n_heads_in_group`` (so a per-layer KV-head count:
  the paged KV cache holds per-layer [pages, Hkv_i, P, D] tensors), ``no_op`` (the block has no
  attention and no input norm) or ``replace_with_linear`` (norm -> one H x H GEMM);
* FFN: SwiGLU with a per-layer width ``find_multiple(int(2 * ffn_mult * H / 3), 256)``, ``no_op``,
  or ``replace_with_linear``.
Residual adds are chained through the fused add + RMSNorm kernel (the pending block output is
added when the next norm runs).  Tensor parallelism splits heads / FFN width per layer; linear
replacements are replicated (no collective).  Only real attention layers own KV pages.  Pipeline
stages hand over (pending block output, residual stream) -- a zero block output when the
boundary layer ended on a no-op.
The remote-code model is not importable here: tests compose transformers' Llama modules per the
block config (parity with the remote code itself unpinned).
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


def ffn_mult_to_intermediate(mult: float, hidden: int) -> int:
    n = int(2 * mult * hidden / 3)
    return n if n % 256 == 0 else n + 256 - n % 256


def block_kinds(cfg: ModelConfig) -> list[dict]:
    """Per layer: {attn: 'attn'|'linear'|'none', group: int, ffn: 'mlp'|'linear'|'none', inter: int}."""
    out = []
    for b in (cfg.extra or {}).get("block_configs") or []:
        a, f = b.get("attention") or {}, b.get("ffn") or {}
        ak = "none" if a.get("no_op") else "linear" if a.get("replace_with_linear") else "attn"
        fk = "none" if f.get("no_op") else "linear" if f.get("replace_with_linear") else "mlp"
        out.append({"attn": ak, "group": int(a.get("n_heads_in_group") or 1), "ffn": fk,
                    "inter": ffn_mult_to_intermediate(float(f.get("ffn_mult") or 0.0), cfg.hidden_size) if fk == "mlp"
                    else 0})
    if len(out) != cfg.num_layers:
        raise ValueError(f"block_configs has {len(out)} entries for {cfg.num_layers} layers")
    return out


class DeciLMForCausalLM(LlamaForCausalLM):
    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        st = pstate.get()
        self.blocks = block_kinds(cfg)
        tp, nh = st.tp_size, cfg.num_heads
        self.hkv: dict[int, int] = {}
        self.kv_start: dict[int, int] = {}
        self.inter: dict[int, int] = {}
        for i, b in enumerate(self.blocks):
            if b["attn"] == "attn":
                kvh = nh // b["group"]
                self.hkv[i] = kvh // tp if kvh >= tp else 1
                self.kv_start[i] = st.tp_rank * self.hkv[i] if kvh >= tp else st.tp_rank * kvh // tp
            if b["ffn"] == "mlp":
                self.inter[i] = -(-b["inter"] // tp)
        self.kv_layers = [i for i in self.layers if self.blocks[i]["attn"] == "attn"]
        self.kv_heads_per_layer = {i: self.hkv[i] for i in self.kv_layers}
        self.w_lin_attn: list[torch.Tensor | None] = [None] * cfg.num_layers
        self.w_lin_mlp: list[torch.Tensor | None] = [None] * cfg.num_layers

    # ------------------------------------------------------------------ weights
    def init_random(self, seed: int = 0, std: float = 0.02) -> "DeciLMForCausalLM":
        cfg, tp, D, H = self.cfg, self.tp, self.D, self.cfg.hidden_size
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 7919 * pstate.get().tp_rank)
        so = std / math.sqrt(2 * cfg.num_layers)
        for i in self.layers:
            b = self.blocks[i]
            if b["attn"] != "none":
                self.ln1[i] = self._alloc(H, std=None, gen=gen)
            if b["attn"] == "attn":
                self.w_qkv[i] = self._alloc((tp.hq + 2 * self.hkv[i]) * D, H, std=std, gen=gen)
                self.w_o[i] = self._alloc(H, tp.hq * D, std=so, gen=gen)
            elif b["attn"] == "linear":
                self.w_lin_attn[i] = self._alloc(H, H, std=so, gen=gen)
            if b["ffn"] != "none":
                self.ln2[i] = self._alloc(H, std=None, gen=gen)
            if b["ffn"] == "mlp":
                self.w_gu[i] = self._alloc(2 * self.inter[i], H, std=std, gen=gen)
                self.w_d[i] = self._alloc(H, self.inter[i], std=so, gen=gen)
            elif b["ffn"] == "linear":
                self.w_lin_mlp[i] = self._alloc(H, H, std=so, gen=gen)
        self.embed = self._alloc(tp.vocab, H, std=1.0, gen=gen)
        self.norm = self._alloc(H, std=None, gen=gen)
        self.lm_head = self.embed if cfg.tie_word_embeddings else self._alloc(tp.vocab, H, std=std, gen=gen)
        return self

    def load_hf_weights(self, weights) -> "DeciLMForCausalLM":
        tp, D = self.tp, self.D
        parts: dict[int, dict[str, torch.Tensor]] = {}

        def put(t):
            return t.to(device=self.device, dtype=self.dtype).contiguous()

        for name, w in weights:
            n = name[len("model."):] if name.startswith("model.") else name
            if n == "embed_tokens.weight":
                self.embed = put(self._vocab_shard(w))
            elif n == "norm.weight":
                self.norm = put(w)
            elif n == "lm_head.weight":
                self.lm_head = put(self._vocab_shard(w))
            elif n.startswith("layers."):
                p = n.split(".")
                i, rest = int(p[1]), ".".join(p[2:])
                if i in self._layer_set:
                    parts.setdefault(i, {})[rest] = w
        for i in self.layers:
            p, b = parts.get(i, {}), self.blocks[i]
            if b["attn"] != "none":
                self.ln1[i] = put(p["input_layernorm.weight"])
            if b["attn"] == "attn":
                hk, ks = self.hkv[i], self.kv_start[i]
                q = p["self_attn.q_proj.weight"].narrow(0, tp.rank * tp.hq * D, tp.hq * D)
                k = p["self_attn.k_proj.weight"].narrow(0, ks * D, hk * D)
                v = p["self_attn.v_proj.weight"].narrow(0, ks * D, hk * D)
                self.w_qkv[i] = put(torch.cat([q, k, v]))
                self.w_o[i] = put(p["self_attn.o_proj.weight"].narrow(1, tp.rank * tp.hq * D, tp.hq * D))
            elif b["attn"] == "linear":
                self.w_lin_attn[i] = put(p["self_attn.linear_attn.weight"])
            if b["ffn"] != "none":
                self.ln2[i] = put(p["post_attention_layernorm.weight"])
            if b["ffn"] == "mlp":
                I = self.inter[i]
                g, u, dn = p["mlp.gate_proj.weight"], p["mlp.up_proj.weight"], p["mlp.down_proj.weight"]
                n_ = min(I, g.shape[0] - tp.rank * I)
                self.w_gu[i] = put(torch.cat([g.narrow(0, tp.rank * I, n_), u.narrow(0, tp.rank * I, n_)]))
                self.w_d[i] = put(dn.narrow(1, tp.rank * I, n_))
            elif b["ffn"] == "linear":
                self.w_lin_mlp[i] = put(p["mlp.linear_mlp.weight"])
        if self.lm_head is None:
            self.lm_head = self.embed
        if self.embed is None:
            raise ValueError("checkpoint incomplete: no embed_tokens")
        return self

    def weight_bytes(self) -> int:
        n = super().weight_bytes()
        for lst in (self.w_lin_attn, self.w_lin_mlp):
            n += sum(t.numel() * t.element_size() for t in lst if t is not None)
        return n

    # ------------------------------------------------------------------ forward
    def forward(self, ids: torch.Tensor, meta: AttnMeta, kv: PagedKVCache,
                input_embeds: torch.Tensor | None = None) -> torch.Tensor:
        cfg, tp, D = self.cfg, self.tp, self.D
        T = ids.shape[0]
        st = pstate.get()
        pend = None   # block output still to be added to the residual stream h
        if st.pp_size > 1 and not st.is_first_pp:
            spec = ((T, cfg.hidden_size), self.dtype, ids.device)
            pend, h = pstate.pp_recv(spec, spec)
        else:
            h = input_embeds if input_embeds is not None else \
                pstate.tp_all_reduce(ops.embedding(ids, self.embed, tp.vocab_start, tp.vocab_end))

        def norm(w):
            nonlocal pend
            if pend is None:
                return ops.rmsnorm(h, w, self.eps)
            x, pend = pend, None
            ops.fused_add_rmsnorm(x, h, w, self.eps)   # h += x; x <- rmsnorm(h) * w
            return x

        for i in self.layers:
            b = self.blocks[i]
            if b["attn"] == "attn":
                x = norm(self.ln1[i])
                hk = self.hkv[i]
                qkv = linear(x, self.w_qkv[i])
                q = torch.empty(T, tp.hq, D, dtype=self.dtype, device=x.device)
                k_cache, v_cache = kv.layer(i)
                ks, vs = kv.scales(i)
                ops.rope_qkv_cache(qkv, meta.positions, self.cos_sin, cfg.rot_dim, q, k_cache, v_cache, meta.slots,
                                   tp.hq, hk, D, True, None, None, self.eps, ks, vs)
                attn = self.attention(q, k_cache, v_cache, meta, ks, vs)
                pend = pstate.tp_all_reduce(linear(attn.view(T, tp.hq * D), self.w_o[i]))
            elif b["attn"] == "linear":
                pend = linear(norm(self.ln1[i]), self.w_lin_attn[i])
            if b["ffn"] == "mlp":
                pend = self.mlp(i, norm(self.ln2[i]))
            elif b["ffn"] == "linear":
                pend = linear(norm(self.ln2[i]), self.w_lin_mlp[i])
        if st.pp_size > 1 and not st.is_last_pp:
            pstate.pp_send(pend if pend is not None else torch.zeros_like(h), h)
            return None
        return norm(self.norm)
