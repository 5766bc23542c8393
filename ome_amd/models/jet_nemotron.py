"""Jet-Nemotron (``JetNemotronForCausalLM``, jet-ai/Jet-Nemotron-2B; reference runtime
``config/runtimes/srt/jet-ai/jet-nemotron-2b-rt.yaml``, model ``config/models/jet-ai/Jet-Nemotron-2B.yaml``).

A Qwen2.5 decoder (biased QKV, RMSNorm, SwiGLU) in which most attention layers are replaced by
JetBlocks (linear attention found by PostNAS); a few full-attention and sliding-window layers are
kept.  The modelling code is remote code that is not importable offline, so this follows the
published architecture; ``tests/test_jet_nemotron_cpu.py`` checks it against an independent fp32
restatement (parity with the remote code itself is unpinned).

JetBlock, per token x (after the input RMSNorm):
  q = silu(W_q x), k = silu(W_k x)                     (no static conv on q / k)
  v = silu(dynconv(W_v x))  with causal taps generated per token:
      taps = W_2 silu(W_1 x) + b_2   -> [value_dim / cpk, K]  (cpk = 1 per channel, head_v_dim per head)
  g = -exp(A_log) softplus(W_a x + dt_bias), beta = sigmoid(W_b x)
  o = gated delta rule over (l2norm(q) / sqrt(dk), l2norm(k), v, g, beta)      (ome_gdn_scan)
  out = W_o (RMSNorm(o) * w * silu(W_g x))                                         (ome_gated_rmsnorm)

Kernels: ONE GEMM for [q | k | v | g | a | b], the generator's two GEMMs, ``ome_dyn_conv1d``
(the per-token-tap conv with per-slot state), ``ome_gdn_scan`` (dk 64 / 128 / 256, any dv), the
gated RMSNorm and the out GEMM.  Attention layers are the Llama path (RoPE + paged KV write,
paged MFMA attention; ``swa`` layers with their window).  Only attention layers own KV pages;
JetBlock state (conv window + fp32 delta-rule state) lives per request slot like Qwen3-Next's.

Config: ``layer_types`` entries ``jet`` / ``attn`` / ``swa`` (aliases ``linear_attention``,
``full_attention``, ``sliding_attention``), else ``efficient_attention_config`` /
top-level ``full_attention_layers`` + ``swa_layers`` index lists, else the published 2B layout
(full attention at layers 15 and 20, sliding window at 21 and 22).  JetBlock shape from
``efficient_attention_config["jet"]``: ``num_heads``, ``head_dim``, ``expand_v``, ``conv_size``,
``dconv_generator_reduction``, ``norm_eps``.  TP = 1 (the reference runs --tp-size 1).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.models.common import AttnMeta, PagedKVCache
from ome_amd.models.config import ModelConfig
from ome_amd.models.llama import LlamaForCausalLM
from ome_amd.models.quant import linear
from ome_amd.parallel import state as pstate

JET_ARCHS = {"JetNemotronForCausalLM"}
_ALIAS = {"jet": "jet", "linear": "jet", "linear_attention": "jet", "jet_block": "jet",
          "attn": "attn", "full": "attn", "full_attention": "attn", "attention": "attn",
          "swa": "swa", "sliding_attention": "swa", "sliding_window": "swa"}


def jet_layer_types(hf: dict, n: int) -> list[str]:
    t = hf.get("layer_types")
    if t:
        out = [_ALIAS.get(str(x).lower()) for x in t]
        if None in out or len(out) != n:
            raise ValueError(f"Jet-Nemotron: unsupported layer_types {t}")
        return out
    eac = hf.get("efficient_attention_config") or {}
    full = eac.get("full_attention_layers", hf.get("full_attention_layers"))
    swa = eac.get("swa_layers", hf.get("swa_layers"))
    if full is None and swa is None:
        full, swa = ([15, 20], [21, 22]) if n == 28 else ([], [])
    full, swa = set(full or []), set(swa or [])
    return ["attn" if i in full else "swa" if i in swa else "jet" for i in range(n)]


class JetNemotronForCausalLM(LlamaForCausalLM):
    stateful = True

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        hf = cfg.extra or {}
        if "attention_bias" not in hf:
            cfg.attention_bias = True   # Qwen2.5 backbone: biased q / k / v
        super().__init__(cfg, device, dtype, max_positions)
        st = pstate.get()
        if st.tp_size > 1 or st.pp_size > 1:
            raise NotImplementedError("Jet-Nemotron: TP / PP > 1 (the reference serves the 2B model at TP 1)")
        L = cfg.num_layers
        self.types = jet_layer_types(hf, L)
        self.kv_layers = [i for i in self.layers if self.types[i] != "jet"]
        self.jet_layers = [i for i in self.layers if self.types[i] == "jet"]
        self.ji = {i: k for k, i in enumerate(self.jet_layers)}
        eac = hf.get("efficient_attention_config") or {}
        jc = eac.get("jet") or {}
        swa_cfg = eac.get("swa") or {}
        self.swa_window = int(swa_cfg.get("window_size") or hf.get("swa_window_size") or hf.get("sliding_window")
                              or 4096)
        self.Hn = int(jc.get("num_heads", max(1, cfg.num_heads // 2)))
        self.dk = int(jc.get("head_dim", 256))
        self.dv = int(self.dk * float(jc.get("expand_v", 2.0)))
        self.K = int(jc.get("conv_size", 4))
        self.red = int(jc.get("dconv_generator_reduction", 8))
        self.jeps = float(jc.get("norm_eps", cfg.rms_norm_eps))
        self.kd, self.vd = self.Hn * self.dk, self.Hn * self.dv
        self.cpk = 1   # channels per generated kernel (set from the checkpoint's generator shape)
        self.w_jet: list[torch.Tensor | None] = [None] * L   # [q | k | v | g | a | b] rows
        self.gen1: list[torch.Tensor | None] = [None] * L
        self.gen2: list[torch.Tensor | None] = [None] * L
        self.gen2_b: list[torch.Tensor | None] = [None] * L
        self.A_log: list[torch.Tensor | None] = [None] * L
        self.dt_bias: list[torch.Tensor | None] = [None] * L
        self.onorm: list[torch.Tensor | None] = [None] * L
        self.w_out: list[torch.Tensor | None] = [None] * L
        self.conv_state: torch.Tensor | None = None
        self.rec_state: torch.Tensor | None = None

    def alloc_state(self, slots: int) -> None:
        n = len(self.jet_layers)
        self.conv_state = torch.zeros(n, slots, self.vd, self.K - 1, dtype=self.dtype, device=self.device)
        self.rec_state = torch.zeros(n, slots, self.Hn, self.dv, self.dk, dtype=torch.float32, device=self.device)

    @property
    def jet_rows(self) -> int:
        return 2 * self.kd + 2 * self.vd + 2 * self.Hn

    # ------------------------------------------------------------------ weights
    def init_random(self, seed: int = 0, std: float = 0.02) -> "JetNemotronForCausalLM":
        super().init_random(seed, std)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 4242)
        H = self.cfg.hidden_size
        R = max(1, H // self.red)
        f32 = dict(dtype=torch.float32, device=self.device)
        for i in self.jet_layers:
            self.w_qkv[i] = self.b_qkv[i] = self.w_o[i] = None
            self.w_jet[i] = self._alloc(self.jet_rows, H, std=std, gen=gen)
            self.gen1[i] = self._alloc(R, H, std=std, gen=gen)
            self.gen2[i] = self._alloc(self.vd * self.K, R, std=std, gen=gen)
            self.gen2_b[i] = self._alloc(self.vd * self.K, std=0.2, gen=gen)
            self.A_log[i] = torch.log(torch.linspace(1.0, 16.0, self.Hn, **f32))
            self.dt_bias[i] = torch.ones(self.Hn, **f32)
            self.onorm[i] = self._alloc(self.dv, std=None, gen=gen)
            self.w_out[i] = self._alloc(H, self.vd, std=std / math.sqrt(2 * self.cfg.num_layers), gen=gen)
        return self

    _JET = {"q_proj.weight": "q", "k_proj.weight": "k", "v_proj.weight": "v", "g_proj.weight": "g",
            "a_proj.weight": "a", "b_proj.weight": "b", "o_proj.weight": "o", "A_log": "A_log",
            "dt_bias": "dt_bias", "o_norm.weight": "norm", "norm.weight": "norm",
            "dynamic_conv1d.kernel_generator.0.weight": "gen1", "dynamic_conv1d.kernel_generator.2.weight": "gen2",
            "dynamic_conv1d.kernel_generator.2.bias": "gen2_b"}

    def load_hf_weights(self, weights) -> "JetNemotronForCausalLM":
        jet: dict[int, dict[str, torch.Tensor]] = {}

        def ours(weights):
            for name, w in weights:
                n = name[len("model."):] if name.startswith("model.") else name
                parts = n.split(".")
                if parts[0] == "layers" and len(parts) > 3 and int(parts[1]) in self.ji:
                    sub = ".".join(parts[3:]) if parts[2] in ("self_attn", "attn", "mixer", "jet") else None
                    key = self._JET.get(sub) if sub is not None else None
                    if key is not None:
                        jet.setdefault(int(parts[1]), {})[key] = w
                        continue
                yield name, w

        placeholder = torch.empty(0, device=self.device)
        for i in self.jet_layers:
            self.w_qkv[i] = placeholder   # the base loader checks every layer's presence
        super().load_hf_weights(ours(weights))

        def put(t, dtype=None):
            return t.to(device=self.device, dtype=dtype or self.dtype).contiguous()

        for i in self.jet_layers:
            self.w_qkv[i] = self.b_qkv[i] = None
            d = jet.get(i, {})
            miss = [k for k in ("q", "k", "v", "g", "a", "b", "o", "A_log", "dt_bias", "norm", "gen1", "gen2")
                    if k not in d]
            if miss:
                raise ValueError(f"Jet-Nemotron layer {i}: missing JetBlock weights {miss}")
            self.w_jet[i] = put(torch.cat([d["q"], d["k"], d["v"], d["g"], d["a"], d["b"]], 0))
            if self.w_jet[i].shape[0] != self.jet_rows:
                raise ValueError(f"Jet-Nemotron layer {i}: projection rows {self.w_jet[i].shape[0]} != "
                                 f"{self.jet_rows} (num_heads {self.Hn}, head_dim {self.dk}, dv {self.dv})")
            g2 = d["gen2"]
            if g2.shape[0] == self.vd * self.K:
                self.cpk = 1
            elif g2.shape[0] == self.Hn * self.K:
                self.cpk = self.dv
            else:
                raise ValueError(f"Jet-Nemotron layer {i}: kernel generator rows {g2.shape[0]}")
            self.gen1[i], self.gen2[i] = put(d["gen1"]), put(g2)
            self.gen2_b[i] = put(d["gen2_b"]) if "gen2_b" in d else None
            self.A_log[i] = put(d["A_log"], torch.float32)
            self.dt_bias[i] = put(d["dt_bias"], torch.float32)
            self.onorm[i] = put(d["norm"])
            self.w_out[i] = put(d["o"])
        return self

    def weight_bytes(self) -> int:
        n = super().weight_bytes()
        for lst in (self.w_jet, self.gen1, self.gen2, self.gen2_b, self.onorm, self.w_out):
            n += sum(t.numel() * t.element_size() for t in lst if t is not None)
        return n

    # ------------------------------------------------------------------ forward
    def jet_block(self, i: int, x: torch.Tensor, seqs) -> torch.Tensor:
        cu, slot, reset = seqs
        kd, vd, Hn = self.kd, self.vd, self.Hn
        j = self.ji[i]
        T = x.shape[0]
        p = linear(x, self.w_jet[i])                      # [T, q | k | v | g | a | b]
        qkv = torch.empty(T, 2 * kd + vd, dtype=x.dtype, device=x.device)
        qkv[:, :2 * kd] = F.silu(p[:, :2 * kd])
        taps = linear(F.silu(linear(x, self.gen1[i])), self.gen2[i], self.gen2_b[i])
        ops.dyn_conv1d(p[:, 2 * kd:2 * kd + vd], taps, self.conv_state[j], cu, slot, reset, self.cpk,
                       out=qkv[:, 2 * kd:])
        oa = 2 * kd + 2 * vd
        o = ops.gdn_scan(qkv[:, :kd], qkv[:, kd:2 * kd], qkv[:, 2 * kd:], p[:, oa:oa + Hn], p[:, oa + Hn:],
                         self.A_log[i], self.dt_bias[i], self.rec_state[j], cu, slot, reset, Hn, Hn)
        o = ops.gated_rmsnorm(o, p[:, 2 * kd + vd:oa], self.onorm[i], self.dv, self.jeps, norm_first=True)
        return linear(o, self.w_out[i])

    def attn_block(self, i: int, x: torch.Tensor, meta: AttnMeta, kv: PagedKVCache) -> torch.Tensor:
        cfg, tp, D, T = self.cfg, self.tp, self.D, x.shape[0]
        qkv = linear(x, self.w_qkv[i], self.b_qkv[i])
        q = torch.empty(T, tp.hq, D, dtype=self.dtype, device=x.device)
        k_cache, v_cache = kv.layer(i)
        ks, vs = kv.scales(i)
        ops.rope_qkv_cache(qkv, meta.positions, self.cos_sin, cfg.rot_dim, q, k_cache, v_cache, meta.slots,
                           tp.hq, tp.hkv, D, True, None, None, self.eps, ks, vs)
        self.window = self.swa_window if self.types[i] == "swa" else -1
        a = self.attention(q, k_cache, v_cache, meta, ks, vs)
        return linear(a.view(T, tp.hq * D), self.w_o[i])

    def forward(self, ids: torch.Tensor, meta: AttnMeta, kv: PagedKVCache,
                input_embeds: torch.Tensor | None = None) -> torch.Tensor:
        seqs = meta.extra["ssm"]
        x, residual = self._stage_input(ids, input_embeds)
        for i in self.layers:
            if i > 0:
                ops.fused_add_rmsnorm(x, residual, self.ln1[i], self.eps)
            o = self.jet_block(i, x, seqs) if self.types[i] == "jet" else self.attn_block(i, x, meta, kv)
            ops.fused_add_rmsnorm(o, residual, self.ln2[i], self.eps)
            x = self._mlp_partial(i, o)
        return self._stage_output(x, residual)
