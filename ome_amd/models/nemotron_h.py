"""NemotronH hybrid Mamba-2 / attention / MLP decoders (``NemotronHForCausalLM``; reference catalog
``config/runtimes/srt/nvidia/nemotron-h-*`` runtimes) on the ome_amd kernels.

Layer types (``layers_block_type`` / the legacy ``hybrid_override_pattern`` M * - E): every block
is ``h + mixer(RMSNorm(h))`` with

* ``M`` Mamba-2 mixer: in_proj GEMM -> [z | xBC | dt] -> causal depthwise conv1d + SiLU
  (``ome_ssm_conv1d``) -> selective scan with per-head A, D, dt_bias and n_groups shared B/C
  (``ome_ssm_scan``: recurrent, fp32 state held in VGPRs across a sequence's rows) -> gated
  group RMSNorm ``w * norm(y * silu(z))`` (``ome_gated_rmsnorm``) -> out_proj GEMM;
* ``*`` attention without positional encoding (GQA, the fused QKV / paged-KV kernel with
  ``apply_rope=False``, paged decode / prefill attention) -- only these layers own KV pages;
* ``-`` MLP ``down(relu(up(x))^2)`` (``ome_act`` ReLU^2 in place between two GEMMs);
* ``E`` sparse MoE (Nemotron-3 Nano / Super): fp32 router logits -> sigmoid scores with the
  ``e_score_correction_bias`` used for selection only, grouped top-k (``ome_moe_route`` noaux_tc
  mode), renormalised and scaled by ``routed_scaling_factor``; NON-gated ReLU^2 experts on the
  grouped MFMA GEMMs (``fused_moe(gated=False)``), optionally inside a latent projection
  (``moe_latent_size``), plus an always-on ReLU^2 shared expert.

Recurrent state lives per request slot (the row of the page-table pool, ``Request.req_slot``):
conv state [slots, conv_dim, K-1] (model dtype) and SSM state [slots, H, P, N] (fp32) per Mamba
layer; a sequence's first prefill chunk starts from zeros (``reset``), later chunks and decode
rows continue.  The prefix cache is disabled for this family (a prefix's SSM state is not paged).
HIP-graph decode captures the same kernels with one-row sequences.  The dt clamp
``time_step_min`` is applied on every row (HF clamps in its chunked prefill path only).

Tensor parallelism: a Mamba-2 mixer splits by SSM heads in whole B/C groups (rank r owns heads
[r*H/tp, (r+1)*H/tp) and groups [r*G/tp, ...): its z / x / B / C / dt rows of in_proj, those conv
channels, A / D / dt_bias, the gated-norm weight slice and out_proj's columns), so the scan needs
no exchange; attention splits by heads, the ReLU^2 MLP / experts / shared expert by intermediate
dim (router and latent projections replicated).  Every mixer's output is a row-parallel partial
sum, all-reduced with the next residual add + RMSNorm.
"""
from __future__ import annotations

import math

import torch

from ome_amd import ops
from ome_amd.models.common import AttnMeta, PagedKVCache
from ome_amd.models.config import ModelConfig
from ome_amd.models.llama import LlamaForCausalLM
from ome_amd.models.quant import dequant_fp8_stream, linear
from ome_amd.parallel import state as pstate

NEMOTRON_H_ARCHS = {"NemotronHForCausalLM"}
_CODES = {"M": "linear_attention", "*": "full_attention", "-": "mlp", "E": "moe"}
_LEGACY = {"mamba": "linear_attention", "attention": "full_attention", "mlp": "mlp", "moe": "moe"}


def layer_types(hf: dict) -> list[str]:
    t = hf.get("layers_block_type") or hf.get("layer_types")
    if t:
        return [_LEGACY.get(x, x) for x in t]
    pat = hf.get("hybrid_override_pattern")
    if pat:
        return [_CODES[c] for c in pat]
    return ["linear_attention", "moe", "full_attention", "mlp"]


class NemotronHForCausalLM(LlamaForCausalLM):
    stateful = True

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        if pstate.get().pp_size > 1:
            raise NotImplementedError("NemotronH: pipeline parallelism (TP is supported)")
        hf = cfg.extra or {}
        self.types = layer_types(hf)
        self.kv_layers = [i for i in self.layers if self.types[i] == "full_attention"]
        self.mamba_layers = [i for i in self.layers if self.types[i] == "linear_attention"]
        self.mi = {i: k for k, i in enumerate(self.mamba_layers)}
        ntp = self.tp.tp
        self.H_full = int(hf.get("mamba_num_heads", 128))
        self.P = int(hf.get("mamba_head_dim", 64))
        self.N = int(hf.get("ssm_state_size", 128))
        self.G_full = int(hf.get("n_groups", 8))
        self.K = int(hf.get("conv_kernel", 4))
        if self.H_full % ntp or self.G_full % ntp:
            raise ValueError(f"NemotronH: {self.H_full} SSM heads / {self.G_full} groups do not split over TP={ntp}")
        self.H, self.G = self.H_full // ntp, self.G_full // ntp   # this rank's heads / groups
        self.I = self.H * self.P
        self.conv_dim = self.I + 2 * self.G * self.N
        self.dt_min = float(hf.get("time_step_min", 0.001) or 0.0)
        self.inter_full = int(hf.get("intermediate_size", cfg.intermediate_size))
        self.inter = self._split(self.inter_full, "intermediate_size")
        self.mlp_act = {"relu2": 4, "silu": 0, "gelu": 3}[hf.get("mlp_hidden_act", "relu2")]
        L = cfg.num_layers
        self.w_in: list[torch.Tensor | None] = [None] * L
        self.conv_w: list[torch.Tensor | None] = [None] * L
        self.conv_b: list[torch.Tensor | None] = [None] * L
        self.A: list[torch.Tensor | None] = [None] * L
        self.Dp: list[torch.Tensor | None] = [None] * L
        self.dt_bias: list[torch.Tensor | None] = [None] * L
        self.gnorm: list[torch.Tensor | None] = [None] * L
        self.w_out: list[torch.Tensor | None] = [None] * L
        self.conv_state: torch.Tensor | None = None
        self.ssm_state: torch.Tensor | None = None
        # MoE blocks
        self.E = int(hf.get("n_routed_experts") or hf.get("num_local_experts") or 0)
        self.topk = int(hf.get("num_experts_per_tok", 2))
        self.moe_I = self._split(int(hf.get("moe_intermediate_size", 0) or 0), "moe_intermediate_size")
        self.shared_I = self._split(int(hf.get("moe_shared_expert_intermediate_size", 0) or 0),
                                    "moe_shared_expert_intermediate_size")
        self.latent = int(hf.get("moe_latent_size") or 0)
        self.n_group = int(hf.get("n_group", 1) or 1)
        self.topk_group = int(hf.get("topk_group", 1) or 1)
        self.routed_scale = float(hf.get("routed_scaling_factor", 1.0) or 1.0)
        self.renorm = bool(hf.get("norm_topk_prob", True))
        self.w_router: list[torch.Tensor | None] = [None] * L      # fp32 [E, H]
        self.e_bias: list[torch.Tensor | None] = [None] * L        # fp32 [E]
        self.w_eu: list[torch.Tensor | None] = [None] * L          # [E, I, H'] (H' = latent or hidden)
        self.w_ed: list[torch.Tensor | None] = [None] * L          # [E, H', I]
        self.w_su: list[torch.Tensor | None] = [None] * L
        self.w_sd: list[torch.Tensor | None] = [None] * L
        self.w_l1: list[torch.Tensor | None] = [None] * L          # latent in / out projections
        self.w_l2: list[torch.Tensor | None] = [None] * L

    def _split(self, n: int, what: str) -> int:
        if n % self.tp.tp:
            raise ValueError(f"NemotronH: {what}={n} does not split over TP={self.tp.tp}")
        return n // self.tp.tp

    def _mamba_slices(self):
        """(in_proj row index, conv channel index, head slice, inner slice) of this rank."""
        r, I, H, G, N = self.tp.rank, self.I, self.H, self.G, self.N
        If, GNf = self.H_full * self.P, self.G_full * self.N
        ar = torch.arange
        xs = ar(r * I, (r + 1) * I)
        bs, cs = ar(r * G * N, (r + 1) * G * N), ar(r * G * N, (r + 1) * G * N)
        conv = torch.cat([xs, If + bs, If + GNf + cs])
        rows = torch.cat([xs, If + conv, 2 * If + 2 * GNf + ar(r * H, (r + 1) * H)])
        return rows, conv, slice(r * H, (r + 1) * H), slice(r * I, (r + 1) * I)

    def alloc_state(self, slots: int) -> None:
        nm = len(self.mamba_layers)
        self.conv_state = torch.zeros(nm, slots, self.conv_dim, self.K - 1, dtype=self.dtype, device=self.device)
        self.ssm_state = torch.zeros(nm, slots, self.H, self.P, self.N, dtype=torch.float32, device=self.device)

    # ------------------------------------------------------------------ weights
    def init_random(self, seed: int = 0, std: float = 0.02) -> "NemotronHForCausalLM":
        cfg, tp, D = self.cfg, self.tp, self.D
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed)
        Hd = cfg.hidden_size
        f32 = dict(dtype=torch.float32, device=self.device)
        for i in self.layers:
            self.ln1[i] = self._alloc(Hd, std=None, gen=gen)
            t = self.types[i]
            if t == "linear_attention":
                self.w_in[i] = self._alloc(self.I + self.conv_dim + self.H, Hd, std=std, gen=gen)
                self.conv_w[i] = self._alloc(self.conv_dim, self.K, std=0.2, gen=gen)
                self.conv_b[i] = self._alloc(self.conv_dim, std=std, gen=gen)
                self.A[i] = -torch.arange(1, self.H + 1, **f32)
                self.Dp[i] = torch.ones(self.H, **f32)
                self.dt_bias[i] = torch.full((self.H,), math.log(math.expm1(0.01)), **f32)
                self.gnorm[i] = self._alloc(self.I, std=None, gen=gen)
                self.w_out[i] = self._alloc(Hd, self.I, std=std / math.sqrt(2 * cfg.num_layers), gen=gen)
            elif t == "full_attention":
                self.w_qkv[i] = self._alloc((tp.hq + 2 * tp.hkv) * D, Hd, std=std, gen=gen)
                self.w_o[i] = self._alloc(Hd, tp.hq * D, std=std / math.sqrt(2 * cfg.num_layers), gen=gen)
            elif t == "moe":
                Hl, dstd = self.latent or Hd, std / math.sqrt(2 * cfg.num_layers)
                self.w_router[i] = torch.randn(self.E, Hd, generator=gen, **f32) * std
                self.e_bias[i] = torch.zeros(self.E, **f32)
                self.w_eu[i] = self._alloc(self.E, self.moe_I, Hl, std=std, gen=gen)
                self.w_ed[i] = self._alloc(self.E, Hl, self.moe_I, std=dstd, gen=gen)
                self.w_su[i] = self._alloc(self.shared_I, Hd, std=std, gen=gen)
                self.w_sd[i] = self._alloc(Hd, self.shared_I, std=dstd, gen=gen)
                if self.latent:
                    self.w_l1[i] = self._alloc(Hl, Hd, std=std, gen=gen)
                    self.w_l2[i] = self._alloc(Hd, Hl, std=std, gen=gen)
            else:
                self.w_gu[i] = self._alloc(self.inter, Hd, std=std, gen=gen)
                self.w_d[i] = self._alloc(Hd, self.inter, std=std / math.sqrt(2 * cfg.num_layers), gen=gen)
        self.embed = self._alloc(tp.vocab, Hd, std=1.0, gen=gen)
        self.norm = self._alloc(Hd, std=None, gen=gen)
        self.lm_head = self.embed if cfg.tie_word_embeddings else self._alloc(tp.vocab, Hd, std=std, gen=gen)
        return self

    def load_hf_weights(self, weights) -> "NemotronHForCausalLM":
        if self.fp8:   # FP8 checkpoints (ModelOpt / compressed-tensors / block-scaled): dequantised to bf16
            weights = dequant_fp8_stream(weights, self.fp8_block, self.dtype)

        def put(t, dtype=None):
            return t.to(device=self.device, dtype=dtype or self.dtype).contiguous()

        tp, D = self.tp, self.D
        rows_in, conv_ch, hs, isl = self._mamba_slices()
        r = tp.rank

        def part(t, n, dim):   # this rank's n-wide block of dim
            return t.narrow(dim, r * n, n) if tp.tp > 1 else t

        qkv: dict[int, dict[str, torch.Tensor]] = {}
        experts: dict[int, dict[tuple[int, str], torch.Tensor]] = {}
        for name, w in weights:
            for pre in ("backbone.", "model."):
                if name.startswith(pre):
                    name = name[len(pre):]
                    break
            if name in ("embedding.weight", "embeddings.weight", "embed_tokens.weight"):
                self.embed = put(self._vocab_shard(w))
                continue
            if name in ("norm_f.weight", "norm.weight"):
                self.norm = put(w)
                continue
            if name == "lm_head.weight":
                self.lm_head = put(self._vocab_shard(w))
                continue
            parts = name.split(".")
            if parts[0] != "layers":
                continue
            i, sub = int(parts[1]), ".".join(parts[2:])
            if i not in self._layer_set:
                continue
            if sub == "norm.weight":
                self.ln1[i] = put(w)
            elif sub == "mixer.in_proj.weight":
                self.w_in[i] = put(w[rows_in.to(w.device)])
            elif sub == "mixer.conv1d.weight":
                self.conv_w[i] = put(w.reshape(w.shape[0], -1)[conv_ch.to(w.device)])
            elif sub == "mixer.conv1d.bias":
                self.conv_b[i] = put(w[conv_ch.to(w.device)])
            elif sub == "mixer.A_log":
                self.A[i] = -torch.exp(w[hs].float()).to(self.device)
            elif sub == "mixer.D":
                self.Dp[i] = put(w[hs], torch.float32)
            elif sub == "mixer.dt_bias":
                self.dt_bias[i] = put(w[hs], torch.float32)
            elif sub == "mixer.norm.weight":
                self.gnorm[i] = put(w[isl])
            elif sub == "mixer.out_proj.weight":
                self.w_out[i] = put(w[:, isl])
            elif sub in ("mixer.q_proj.weight", "mixer.k_proj.weight", "mixer.v_proj.weight"):
                qkv.setdefault(i, {})[sub[6]] = w
            elif sub == "mixer.o_proj.weight":
                self.w_o[i] = put(part(w, tp.hq * D, 1))
            elif sub == "mixer.up_proj.weight":
                self.w_gu[i] = put(part(w, self.inter, 0))
            elif sub == "mixer.down_proj.weight":
                self.w_d[i] = put(part(w, self.inter, 1))
            elif sub == "mixer.gate.weight":
                self.w_router[i] = put(w, torch.float32)
            elif sub == "mixer.gate.e_score_correction_bias":
                self.e_bias[i] = put(w, torch.float32)
            elif sub == "mixer.experts.up_proj":             # fused [E, I, H']
                self.w_eu[i] = put(part(w, self.moe_I, 1))
            elif sub == "mixer.experts.down_proj":
                self.w_ed[i] = put(part(w, self.moe_I, 2))
            elif sub.startswith("mixer.experts.") and sub.endswith(".weight"):   # per expert
                e, kind = int(sub.split(".")[2]), sub.split(".")[3]
                experts.setdefault(i, {})[(e, kind)] = w
            elif sub == "mixer.shared_experts.up_proj.weight":
                self.w_su[i] = put(part(w, self.shared_I, 0))
            elif sub == "mixer.shared_experts.down_proj.weight":
                self.w_sd[i] = put(part(w, self.shared_I, 1))
            elif sub == "mixer.fc1_latent_proj.weight":
                self.w_l1[i] = put(w)
            elif sub == "mixer.fc2_latent_proj.weight":
                self.w_l2[i] = put(w)
        for i, d in experts.items():
            self.w_eu[i] = put(torch.stack([part(d[(e, "up_proj")], self.moe_I, 0) for e in range(self.E)]))
            self.w_ed[i] = put(torch.stack([part(d[(e, "down_proj")], self.moe_I, 1) for e in range(self.E)]))
        for i in self.layers:
            if self.types[i] == "moe":
                if self.e_bias[i] is None:
                    self.e_bias[i] = torch.zeros(self.E, dtype=torch.float32, device=self.device)
                if self.w_router[i] is None or self.w_eu[i] is None or self.w_ed[i] is None:
                    raise ValueError(f"layer {i}: incomplete MoE weights")
        for i, d in qkv.items():
            kv = slice(tp.kv_start * D, (tp.kv_start + tp.hkv) * D)
            self.w_qkv[i] = put(torch.cat([d["q"][r * tp.hq * D:(r + 1) * tp.hq * D], d["k"][kv], d["v"][kv]], 0))
        if self.lm_head is None:
            self.lm_head = self.embed
        return self

    def weight_bytes(self) -> int:
        n = super().weight_bytes()
        for lst in (self.w_in, self.conv_w, self.conv_b, self.gnorm, self.w_out, self.w_router, self.w_eu, self.w_ed,
                    self.w_su, self.w_sd, self.w_l1, self.w_l2):
            n += sum(t.numel() * t.element_size() for t in lst if t is not None)
        return n

    # ------------------------------------------------------------------ forward
    def mamba(self, i: int, x: torch.Tensor, seqs) -> torch.Tensor:
        cu, slot, reset = seqs
        I, cd, H, G, N = self.I, self.conv_dim, self.H, self.G, self.N
        k = self.mi[i]
        zxd = linear(x, self.w_in[i])
        z, xbc, dt = zxd[:, :I], zxd[:, I:I + cd], zxd[:, I + cd:]
        conv = ops.ssm_conv1d(xbc, self.conv_w[i], self.conv_b[i], self.conv_state[k], cu, slot, reset)
        xs, B, C = conv[:, :I], conv[:, I:I + G * N], conv[:, I + G * N:]
        y = ops.ssm_scan(xs, dt, B, C, self.A[i], self.Dp[i], self.dt_bias[i], self.dt_min, self.ssm_state[k], cu,
                         slot, reset, H, self.P, N, G)
        y = ops.gated_rmsnorm(y, z, self.gnorm[i], I // G, self.eps)
        return linear(y, self.w_out[i])

    def moe(self, i: int, x: torch.Tensor) -> torch.Tensor:
        logits = torch.nn.functional.linear(x.float(), self.w_router[i])      # HF routes in fp32
        tw, tid = ops.moe_route(logits, self.topk, self.renorm, "sigmoid", bias=self.e_bias[i],
                                n_group=self.n_group, topk_group=self.topk_group, group_mode=2)
        h = linear(x, self.w_l1[i]) if self.latent else x
        out = ops.fused_moe(h, tw, tid, self.w_eu[i], self.w_ed[i], self.mlp_act, self.routed_scale, gated=False)
        if self.latent:
            out = linear(out, self.w_l2[i])
        if self.w_su[i] is not None:
            out = out + linear(ops.act(linear(x, self.w_su[i]), self.mlp_act), self.w_sd[i])
        return out

    def forward(self, ids: torch.Tensor, meta: AttnMeta, kv: PagedKVCache,
                input_embeds: torch.Tensor | None = None) -> torch.Tensor:
        tp, D = self.tp, self.D
        T = ids.shape[0]
        seqs = meta.extra["ssm"]
        x, residual = self._stage_input(ids, input_embeds)
        for i in self.layers:
            if i > 0:   # the previous mixer's partial sums: TP all-reduce + residual add + norm
                x = self._reduce_add_norm(x, residual, self.ln1[i])
            t = self.types[i]
            if t == "linear_attention":
                x = self.mamba(i, x, seqs)
            elif t == "full_attention":
                qkv = linear(x, self.w_qkv[i])
                q = torch.empty(T, tp.hq, D, dtype=self.dtype, device=x.device)
                k_cache, v_cache = kv.layer(i)
                ks, vs = kv.scales(i)
                ops.rope_qkv_cache(qkv, meta.positions, self.cos_sin, self.cfg.rot_dim, q, k_cache, v_cache,
                                   meta.slots, tp.hq, tp.hkv, D, False, None, None, self.eps, ks, vs)
                attn = self.attention(q, k_cache, v_cache, meta, ks, vs)
                x = linear(attn.view(T, tp.hq * D), self.w_o[i])
            elif t == "moe":
                x = self.moe(i, x)
            else:
                x = linear(ops.act(linear(x, self.w_gu[i]), self.mlp_act), self.w_d[i])
        if self.layers and tp.tp > 1:
            x = pstate.tp_all_reduce(x)
        return self._stage_output(x, residual)
