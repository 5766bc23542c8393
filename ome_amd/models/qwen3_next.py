"""Qwen3-Next hybrid decoder (``Qwen3NextForCausalLM``; reference catalog
``config/runtimes/srt/Qwen/qwen3-next-80b-a3b-*-rt.yaml``) on the ome_amd kernels.

Layers follow ``layer_types`` (by default three Gated-DeltaNet layers, then one full-attention
layer); every layer's MLP is the sparse MoE of ``moe.py`` (softmax top-k with renorm, fused
grouped-GEMM experts, a shared expert scaled by ``sigmoid(shared_expert_gate(x))``).

* Gated DeltaNet (linear attention): ONE GEMM for [q | k | v | z | b | a] (``in_proj_qkvz`` /
  ``in_proj_ba`` rows are permuted at load from HF's per-k-head-group interleaving into
  per-tensor blocks, so the conv input and the recurrence read plain row-strided views) ->
  causal depthwise conv1d + SiLU over q|k|v (``ome_ssm_conv1d``, per-slot conv state) ->
  ``ome_gdn_scan`` (L2-norm of q / k, ``g`` / ``beta`` from a / b, the delta-rule recurrence with
  each v-head's fp32 state spread over DPP rows of lanes in VGPRs, per request slot) -> norm-then-gate
  RMSNorm ``w * norm(o) * silu(z)`` (``ome_gated_rmsnorm`` norm_first) -> out_proj GEMM.
* Gated attention: q_proj's per-head [query | gate] halves are split at load into one fused
  [q | k | v | gate] projection; per-head q / k RMSNorm + partial NeoX RoPE (rot_dim = D / 4)
  + paged KV write in ``ome_rope_qkv_cache``; paged MFMA attention; ``o * sigmoid(gate)``.
* every RMSNorm of this family scales by ``1 + w``: folded into the stored weights at load
  (in fp32, before the cast), so the standard norm kernels apply.

Only the attention layers own KV pages (``kv_layers``); recurrent state lives per request slot
(``alloc_state``: conv [n_lin, slots, conv_dim, K-1] in the model dtype, delta-rule state
[n_lin, slots, Hv, dv, dk] fp32, transposed -- ~2 MiB per layer-slot at the 80B shape, sized
before the KV pool).  The prefix cache is off for stateful models.

Tensor parallelism: the Gated-DeltaNet layers split by key-head groups (rank r owns k-heads
[r*Hk/tp, (r+1)*Hk/tp) and the v-heads of those groups -- the q / k / v / z / b / a rows, the
conv channels, A_log / dt_bias and out_proj's columns), so the recurrence needs no exchange; the
gated attention splits by query heads as the Llama base does, the MoE by experts' intermediate
dim (``moe.py``); each mixer's out projection is row-parallel and all-reduced with the residual
add + RMSNorm.  80B bf16 (~160 GB) also fits one MI355X, where TP=1 is the default.
"""
from __future__ import annotations

import math

import torch

from ome_amd import ops
from ome_amd.models.common import AttnMeta, PagedKVCache
from ome_amd.models.config import ModelConfig
from ome_amd.models.moe import MoEForCausalLM
from ome_amd.models.quant import linear
from ome_amd.parallel import state as pstate

QWEN3_NEXT_ARCHS = {"Qwen3NextForCausalLM"}


def layer_types(hf: dict, n: int) -> list[str]:
    t = hf.get("layer_types")
    if t:
        return list(t)
    k = int(hf.get("full_attention_interval", 4))
    return ["full_attention" if (i + 1) % k == 0 else "linear_attention" for i in range(n)]


class Qwen3NextForCausalLM(MoEForCausalLM):
    stateful = True

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        if pstate.get().pp_size > 1:
            raise NotImplementedError("Qwen3-Next: pipeline parallelism (TP is supported)")
        hf = cfg.extra or {}
        self.types = layer_types(hf, cfg.num_layers)
        self.kv_layers = [i for i in self.layers if self.types[i] == "full_attention"]
        self.lin_layers = [i for i in self.layers if self.types[i] == "linear_attention"]
        self.li = {i: k for k, i in enumerate(self.lin_layers)}
        self.Hk_full = int(hf.get("linear_num_key_heads", 16))
        self.Hv_full = int(hf.get("linear_num_value_heads", 32))
        self.dk = int(hf.get("linear_key_head_dim", 128))
        self.dv = int(hf.get("linear_value_head_dim", 128))
        self.K = int(hf.get("linear_conv_kernel_dim", 4))
        ntp, r = self.tp.tp, self.tp.rank
        if self.Hk_full % ntp:
            raise ValueError(f"Qwen3-Next: {self.Hk_full} linear-attention key heads do not split over TP={ntp}")
        self.Hk, self.Hv = self.Hk_full // ntp, self.Hv_full // ntp   # this rank's heads
        self.hk0 = r * self.Hk
        self.kd, self.vd = self.Hk * self.dk, self.Hv * self.dv
        self.conv_dim = 2 * self.kd + self.vd
        step = int(hf.get("decoder_sparse_step", 1) or 1)
        dense = set(hf.get("mlp_only_layers") or [])
        self.moe_layers = {i for i in self.layers if i not in dense and (i + 1) % step == 0}
        from ome_amd.parallel import eplb

        eplb.attach(self)   # again: the MoE layer set changed
        L = cfg.num_layers
        self.w_lin: list[torch.Tensor | None] = [None] * L     # [q | k | v | z | b | a] rows
        self.conv_w: list[torch.Tensor | None] = [None] * L
        self.A_log: list[torch.Tensor | None] = [None] * L
        self.dt_bias: list[torch.Tensor | None] = [None] * L
        self.gnorm: list[torch.Tensor | None] = [None] * L
        self.w_out: list[torch.Tensor | None] = [None] * L
        self.conv_state: torch.Tensor | None = None
        self.rec_state: torch.Tensor | None = None

    def alloc_state(self, slots: int) -> None:
        n = len(self.lin_layers)
        self.conv_state = torch.zeros(n, slots, self.conv_dim, self.K - 1, dtype=self.dtype, device=self.device)
        self.rec_state = torch.zeros(n, slots, self.Hv, self.dv, self.dk, dtype=torch.float32, device=self.device)

    # ------------------------------------------------------------------ weights
    def init_random(self, seed: int = 0, std: float = 0.02) -> "Qwen3NextForCausalLM":
        super().init_random(seed, std)   # embeddings, norms, MoE / dense MLPs, (placeholder) attention
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 31337)
        H, D, tp = self.cfg.hidden_size, self.D, self.tp
        f32 = dict(dtype=torch.float32, device=self.device)
        for i in self.layers:
            if self.types[i] == "linear_attention":
                self.w_qkv[i] = self.b_qkv[i] = self.w_o[i] = self.qn[i] = self.kn[i] = None
                self.w_lin[i] = self._alloc(self.conv_dim + self.vd + 2 * self.Hv, H, std=std, gen=gen)
                self.conv_w[i] = self._alloc(self.conv_dim, self.K, std=0.2, gen=gen)
                self.A_log[i] = torch.log(torch.linspace(1.0, 16.0, self.Hv, **f32))
                self.dt_bias[i] = torch.ones(self.Hv, **f32)
                self.gnorm[i] = self._alloc(self.dv, std=None, gen=gen)
                self.w_out[i] = self._alloc(H, self.vd, std=std / math.sqrt(2 * self.cfg.num_layers), gen=gen)
            else:
                self.w_qkv[i] = self._alloc((2 * tp.hq + 2 * tp.hkv) * D, H, std=std, gen=gen)
                self.qn[i] = self._alloc(D, std=None, gen=gen)
                self.kn[i] = self._alloc(D, std=None, gen=gen)
        return self

    def _qkvz_order(self) -> tuple[torch.Tensor, torch.Tensor]:
        """Row gathers: HF's per-k-head groups [q k v z] / [b a] -> [all q | all k | all v | all z]
        and [all b | all a], over this rank's k-head groups only."""
        Hk, dk, dv, r = self.Hk, self.dk, self.dv, self.Hv // self.Hk
        g = 2 * dk + 2 * r * dv
        heads = self.hk0 + torch.arange(Hk)
        base = heads[:, None] * g
        q = (base + torch.arange(dk)).reshape(-1)
        k = (base + dk + torch.arange(dk)).reshape(-1)
        v = (base + 2 * dk + torch.arange(r * dv)).reshape(-1)
        z = (base + 2 * dk + r * dv + torch.arange(r * dv)).reshape(-1)
        gb = heads[:, None] * (2 * r)
        b = (gb + torch.arange(r)).reshape(-1)
        a = (gb + r + torch.arange(r)).reshape(-1)
        return torch.cat([q, k, v, z]), torch.cat([b, a])

    def load_hf_weights(self, weights) -> "Qwen3NextForCausalLM":
        lin: dict[int, dict[str, torch.Tensor]] = {}
        attn: dict[int, dict[str, torch.Tensor]] = {}

        def one_plus(t):   # Qwen3NextRMSNorm: x * (1 + w)
            return (1.0 + t.float()).to(device=self.device, dtype=self.dtype).contiguous()

        def ours(weights):
            for name, w in weights:
                n = name[len("model."):] if name.startswith("model.") else name
                if n == "norm.weight":
                    self.norm = one_plus(w)
                    continue
                parts = n.split(".")
                if parts[0] == "layers" and len(parts) > 3:
                    i, sub = int(parts[1]), ".".join(parts[2:])
                    if i not in self._layer_set:
                        continue
                    if sub.startswith("linear_attn."):
                        lin.setdefault(i, {})[sub[len("linear_attn."):]] = w
                        continue
                    if sub in ("self_attn.q_proj.weight", "self_attn.k_proj.weight", "self_attn.v_proj.weight"):
                        attn.setdefault(i, {})[sub[10]] = w
                        continue
                    norm = {"self_attn.q_norm.weight": self.qn, "self_attn.k_norm.weight": self.kn,
                            "input_layernorm.weight": self.ln1, "post_attention_layernorm.weight": self.ln2}.get(sub)
                    if norm is not None:
                        norm[i] = one_plus(w)
                        continue
                yield name, w

        placeholder = torch.empty(0, device=self.device)
        for i in self.layers:
            self.w_qkv[i] = placeholder   # assembled below (the base loader checks presence)
        super().load_hf_weights(ours(weights))

        def put(t, dtype=None):
            return t.to(device=self.device, dtype=dtype or self.dtype).contiguous()

        pq, pb = self._qkvz_order()
        D, hq = self.D, self.tp.hq
        for i in self.layers:
            self.w_qkv[i] = None
            if self.types[i] == "linear_attention":
                d = lin.get(i, {})
                need = ("in_proj_qkvz.weight", "in_proj_ba.weight", "conv1d.weight", "A_log", "dt_bias",
                        "norm.weight", "out_proj.weight")
                miss = [k for k in need if k not in d]
                if miss:
                    raise ValueError(f"layer {i}: missing linear_attn weights {miss}")
                qkvz, ba = d["in_proj_qkvz.weight"], d["in_proj_ba.weight"]
                self.w_lin[i] = put(torch.cat([qkvz[pq.to(qkvz.device)], ba[pb.to(ba.device)]], 0))
                kdf = self.Hk_full * self.dk
                cw = d["conv1d.weight"].reshape(2 * kdf + self.Hv_full * self.dv, -1)   # [q | k | v] channels
                k0, v0 = self.hk0 * self.dk, self.hk0 * (self.Hv // self.Hk) * self.dv
                self.conv_w[i] = put(torch.cat([cw[k0:k0 + self.kd], cw[kdf + k0:kdf + k0 + self.kd],
                                                cw[2 * kdf + v0:2 * kdf + v0 + self.vd]], 0))
                h0 = v0 // self.dv
                self.A_log[i] = put(d["A_log"][h0:h0 + self.Hv], torch.float32)
                self.dt_bias[i] = put(d["dt_bias"][h0:h0 + self.Hv], torch.float32)
                self.gnorm[i] = put(d["norm.weight"])
                self.w_out[i] = put(d["out_proj.weight"][:, v0:v0 + self.vd])
            else:
                d = attn.get(i, {})
                if len(d) != 3:
                    raise ValueError(f"layer {i}: missing attention projections")
                tp = self.tp
                qg = d["q"].reshape(-1, 2, D, d["q"].shape[-1])[tp.rank * hq:(tp.rank + 1) * hq]
                kv = slice(tp.kv_start * D, (tp.kv_start + tp.hkv) * D)
                self.w_qkv[i] = put(torch.cat([qg[:, 0].reshape(hq * D, -1), d["k"][kv], d["v"][kv],
                                               qg[:, 1].reshape(hq * D, -1)], 0))
        return self

    def weight_bytes(self) -> int:
        n = super().weight_bytes()
        for lst in (self.w_lin, self.conv_w, self.gnorm, self.w_out):
            n += sum(t.numel() * t.element_size() for t in lst if t is not None)
        return n

    # ------------------------------------------------------------------ forward
    def gated_delta(self, i: int, x: torch.Tensor, seqs) -> torch.Tensor:
        cu, slot, reset = seqs
        kd, vd, cd, Hv = self.kd, self.vd, self.conv_dim, self.Hv
        j = self.li[i]
        p = linear(x, self.w_lin[i])                                    # [T, q | k | v | z | b | a]
        conv = ops.ssm_conv1d(p[:, :cd], self.conv_w[i], None, self.conv_state[j], cu, slot, reset)
        o = ops.gdn_scan(conv[:, :kd], conv[:, kd:2 * kd], conv[:, 2 * kd:], p[:, cd + vd + Hv:],
                         p[:, cd + vd:cd + vd + Hv], self.A_log[i], self.dt_bias[i], self.rec_state[j], cu, slot,
                         reset, Hv, self.Hk)
        o = ops.gated_rmsnorm(o, p[:, cd:cd + vd], self.gnorm[i], self.dv, self.eps, norm_first=True)
        return self._row_parallel(o, self.w_out[i])   # partial sums under TP

    def gated_attention(self, i: int, x: torch.Tensor, meta: AttnMeta, kv: PagedKVCache) -> torch.Tensor:
        tp, D, T = self.tp, self.D, x.shape[0]
        p = linear(x, self.w_qkv[i])                                    # [T, q | k | v | gate]
        q = torch.empty(T, tp.hq, D, dtype=self.dtype, device=x.device)
        k_cache, v_cache = kv.layer(i)
        ks, vs = kv.scales(i)
        ops.rope_qkv_cache(p, meta.positions, self.cos_sin, self.cfg.rot_dim, q, k_cache, v_cache, meta.slots,
                           tp.hq, tp.hkv, D, True, self.qn[i], self.kn[i], self.eps, ks, vs)
        a = self.attention(q, k_cache, v_cache, meta, ks, vs).view(T, tp.hq * D)
        a = a * torch.sigmoid(p[:, (tp.hq + 2 * tp.hkv) * D:])
        return self._row_parallel(a, self.w_o[i])

    def forward(self, ids: torch.Tensor, meta: AttnMeta, kv: PagedKVCache,
                input_embeds: torch.Tensor | None = None) -> torch.Tensor:
        seqs = meta.extra["ssm"]
        x, residual = self._stage_input(ids, input_embeds)
        for i in self.layers:
            if i > 0:
                ops.fused_add_rmsnorm(x, residual, self.ln1[i], self.eps)
            if self.types[i] == "linear_attention":
                o = self.gated_delta(i, x, seqs)
            else:
                o = self.gated_attention(i, x, meta, kv)
            o = self._reduce_add_norm(o, residual, self.ln2[i])   # TP all-reduce + add + norm
            x = self.mlp(i, o)
        return self._stage_output(x, residual)
