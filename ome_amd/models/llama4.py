"""Llama 4 text decoders (``Llama4ForCausalLM`` / the language model of
``Llama4ForConditionalGeneration``: Scout 17B-16E, Maverick 17B-128E) on the ome_amd kernels.

Reference: the Llama-4 runtimes of the catalog (``config/runtimes/srt/meta/llama-4-*``) and the
weekly benchmark model ``llama-4-scout-17b-16e-instruct`` (``.github/workflows/benchmark.yaml``).
What differs from the Llama / MoE paths, and where it runs:

* interleaved (complex-pair) RoPE: the q/k projection rows of every head are permuted at load time
  from the pair layout ``(2i, 2i+1)`` to the NeoX halves ``(i, i + D/2)`` the fused RoPE/KV-cache
  kernel rotates (q.k is invariant under the common permutation; V / O are untouched);
* NoPE layers (every ``no_rope_layer_interval``-th layer): no rotation (``apply_rope=False`` in the
  same kernel) and full causal attention with the attention-temperature tuning
  ``q *= 1 + attn_scale * log1p(floor((pos + 1) / floor_scale))``;
* RoPE layers: chunked attention (``attention_chunk_size``: a query sees only keys of its own chunk)
  -- a ``window < -1`` mode of the decode / prefill attention kernels (``attn_lo`` in
  ``attention.hip``) -- and the weightless L2 q/k norm, which commutes with the rotation, so it
  runs as the kernel's RMS q/k-norm with unit weights;
* MoE: sigmoid of the top-k router logits scales the expert INPUT (``routed_in = x * s``) before
  the grouped MFMA GEMMs (combine weight 1), plus an always-on shared expert; HF stores the experts
  as ``gate_up_proj`` [E, H, 2I] / ``down_proj`` [E, I, H] and they are transposed into the
  kernels' [E, 2I, H] / [E, H, I] at load time;
* dense layers between MoE layers (Maverick, ``interleave_moe_layer_step``) use
  ``intermediate_size_mlp``.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.models.common import AttnMeta, PagedKVCache
from ome_amd.models.config import ModelConfig
from ome_amd.models.moe import MoEForCausalLM
from ome_amd.models.quant import linear
from ome_amd.parallel import state as pstate

LLAMA4_ARCHS = {"Llama4ForCausalLM", "Llama4ForConditionalGeneration"}


def _hf(cfg: ModelConfig) -> dict:
    ex = cfg.extra or {}
    return {**ex, **(ex.get("text_config") or {})}


def pair_to_halves(w: torch.Tensor, heads: int, D: int) -> torch.Tensor:
    """Rows of a per-head projection [heads*D, ...]: interleaved pairs -> NeoX halves."""
    perm = torch.cat([torch.arange(0, D, 2), torch.arange(1, D, 2)]).to(w.device)
    return w.reshape(heads, D, *w.shape[1:]).index_select(1, perm).reshape(w.shape)


class Llama4ForCausalLM(MoEForCausalLM):
    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        hf = _hf(cfg)
        L, tp = cfg.num_layers, self.tp
        self.tp.inter = -(-int(hf.get("intermediate_size_mlp") or cfg.intermediate_size) // tp.tp)
        self.shared_inter = -(-int(hf.get("intermediate_size") or cfg.moe_intermediate_size) // tp.tp)
        step = int(hf.get("interleave_moe_layer_step") or 1)
        moe = hf.get("moe_layers")
        if moe is None:
            moe = list(range(step - 1, L, step))
        self.moe_layers = {i for i in moe if i in self._layer_set}
        from ome_amd.parallel import eplb

        eplb.attach(self)  # again: the EPLB slots follow this family's MoE layer set
        interval = int(hf.get("no_rope_layer_interval") or 4)
        nrl = hf.get("no_rope_layers") or [int((i + 1) % interval != 0) for i in range(L)]
        self.use_rope = [bool(nrl[i]) for i in range(L)]
        chunk = hf.get("attention_chunk_size")
        self.windows = [-int(chunk) if (chunk and self.use_rope[i]) else -1 for i in range(L)]
        self.qk_l2 = bool(hf.get("use_qk_norm", True))
        self.temp_tuning = bool(hf.get("attn_temperature_tuning", True))
        fs, asc = float(hf.get("floor_scale") or 8192), float(hf.get("attn_scale") or 0.1)
        mp = self.cos_sin.shape[0]
        pos = torch.arange(mp, dtype=torch.float64)
        self.temp = (torch.log1p(torch.floor((pos + 1.0) / fs)) * asc + 1.0).float().to(self.device)
        self.unit = torch.ones(self.D, dtype=dtype, device=self.device)

    # ------------------------------------------------------------------ weights
    def init_random(self, seed: int = 0, std: float = 0.02) -> "Llama4ForCausalLM":
        super().init_random(seed, std)
        for i in self.moe_layers:
            self.w_sgate[i] = None  # Llama 4's shared expert has no sigmoid gate
        return self

    def load_hf_weights(self, weights) -> "Llama4ForCausalLM":
        cfg, tp = self.cfg, self.tp
        D, I, SI = self.D, self.moe_inter, self.shared_inter
        experts: dict[int, dict[str, torch.Tensor]] = {}
        shared: dict[int, dict[str, torch.Tensor]] = {}
        base = []

        def put(t):
            return t.to(device=self.device, dtype=self.dtype).contiguous()

        for name, w in weights:
            if name.startswith(("vision_model.", "multi_modal_projector.")):
                continue
            if name.startswith("language_model."):
                name = name[len("language_model."):]
            n = name[len("model."):] if name.startswith("model.") else name
            parts = n.split(".")
            if parts[0] == "layers" and len(parts) > 3:
                i, sub = int(parts[1]), ".".join(parts[2:])
                if i not in self._layer_set:
                    continue
                if sub == "self_attn.q_proj.weight":
                    w = pair_to_halves(w, cfg.num_heads, D)
                elif sub == "self_attn.k_proj.weight":
                    w = pair_to_halves(w, cfg.num_kv_heads, D)
                if sub.startswith("feed_forward.") and i in self.moe_layers:
                    rest = sub[len("feed_forward."):]
                    if rest == "router.weight":
                        self.w_router[i] = put(w)
                    elif rest.startswith("experts."):
                        experts.setdefault(i, {})[rest.split(".")[1]] = w
                    elif rest.startswith("shared_expert."):
                        shared.setdefault(i, {})[rest.split(".")[1]] = w
                    continue
                if sub.startswith("feed_forward."):
                    sub = "mlp." + sub[len("feed_forward."):]
                base.append(("model.layers.%d.%s" % (i, sub), w))
                continue
            base.append((name, w))
        self._load_base(base)
        idx = self.local_experts
        for i, d in experts.items():
            gu, dn = d["gate_up_proj"], d["down_proj"]  # [E, H, 2I], [E, I, H]
            Ifull = gu.shape[-1] // 2
            sel = torch.tensor(idx(i), dtype=torch.long, device=gu.device)
            gu, dn = gu.index_select(0, sel), dn.index_select(0, sel)
            n = min(I, Ifull - tp.rank * I)
            g = gu[..., tp.rank * I: tp.rank * I + n]
            u = gu[..., Ifull + tp.rank * I: Ifull + tp.rank * I + n]
            self.w13[i] = put(torch.cat([g, u], -1).transpose(1, 2))
            self.w2[i] = put(dn[:, tp.rank * I: tp.rank * I + n, :].transpose(1, 2))
            self.w_gu[i] = self.w_d[i] = None
        for i, d in shared.items():
            g, u, dn = d["gate_proj"], d["up_proj"], d["down_proj"]
            n = min(SI, g.shape[0] - tp.rank * SI)
            self.w_sgu[i] = put(torch.cat([g.narrow(0, tp.rank * SI, n), u.narrow(0, tp.rank * SI, n)], 0))
            self.w_sd[i] = put(dn.narrow(1, tp.rank * SI, n))
        return self

    # ------------------------------------------------------------------ forward
    def mlp(self, i: int, x: torch.Tensor) -> torch.Tensor:
        if i not in self.moe_layers:
            return super().mlp(i, x)
        T, H = x.shape
        logits = F.linear(x, self.w_router[i])
        tw, tid = ops.moe_route(logits, self.k, False, "sigmoid")
        s = tw.to(x.dtype)
        if self.k == 1:
            xr = x * s
        else:  # one routed copy of the row per selected expert, each top-1
            xr = (x[:, None, :] * s[..., None]).reshape(T * self.k, H)
            tid = tid.reshape(T * self.k, 1)
        ones = torch.ones(tid.shape, dtype=torch.float32, device=x.device)
        if self.ep > 1:
            from ome_amd.parallel.ep import moe_ep

            tables = None
            if self.eplb is not None:
                self.eplb.record(i, tid)
                tables = self.eplb.tables[i]
            out = moe_ep(xr, ones, tid, self.w13[i], self.w2[i], self.act, 1.0, self.E, tables)
        else:
            out = ops.fused_moe(xr, ones, tid, self.w13[i], self.w2[i], self.act)
        if self.k > 1:
            out = out.view(T, self.k, H).sum(1)
        sh = linear(ops.act_and_mul(linear(x, self.w_sgu[i]), self.act), self.w_sd[i])
        return pstate.tp_all_reduce(out + sh)

    def forward(self, ids: torch.Tensor, meta: AttnMeta, kv: PagedKVCache,
                input_embeds: torch.Tensor | None = None) -> torch.Tensor:
        cfg, tp, D = self.cfg, self.tp, self.D
        T = ids.shape[0]
        x, residual = self._stage_input(ids, input_embeds)
        for i in self.layers:
            if i > 0:
                ops.fused_add_rmsnorm(x, residual, self.ln1[i], self.eps)
            qkv = linear(x, self.w_qkv[i], self.b_qkv[i])
            q = torch.empty(T, tp.hq, D, dtype=self.dtype, device=x.device)
            k_cache, v_cache = kv.layer(i)
            ks, vs = kv.scales(i)
            rope = self.use_rope[i]
            nw = self.unit if (rope and self.qk_l2) else None
            ops.rope_qkv_cache(qkv, meta.positions, self.cos_sin, cfg.rot_dim, q, k_cache, v_cache, meta.slots,
                               tp.hq, tp.hkv, D, rope, nw, nw, self.eps, ks, vs)
            if not rope and self.temp_tuning:
                q.mul_(self.temp.index_select(0, meta.positions.long()).view(T, 1, 1))
            self.window = self.windows[i]
            attn = self.attention(q, k_cache, v_cache, meta, ks, vs)
            o = pstate.tp_all_reduce(linear(attn.view(T, tp.hq * D), self.w_o[i]))
            ops.fused_add_rmsnorm(o, residual, self.ln2[i], self.eps)
            x = self.mlp(i, o)
        return self._stage_output(x, residual)
