"""DeepSeek-V2 / V2-Lite / V3 / R1 and Kimi-K2 (``DeepseekV2ForCausalLM``, ``DeepseekV3ForCausalLM``)
on the ome_amd kernels.  The reference serves these through SGLang runtimes
(``config/runtimes/srt/deepseek-rdma-pd-rt.yaml:20`` and the Kimi-K2 PD runtime); SURVEY.md §2.9
K6 (MLA), K10 (grouped top-k routing), K11 (grouped GEMM), K8 (block-FP8).

Attention is multi-head latent attention run in the *absorbed* form for every step kind:

  x --[q_a | kv_a] fused GEMM--> q_a -> RMSNorm -> q_b GEMM -> q [T, H, nope + rope]
                            \\-> c_kv (512) -> RMSNorm ; k_pe (64)
  RoPE(q_pe, k_pe) -> latent cache row [c_kv | k_pe] (576 wide, ONE per token for all heads)
  q_lat = [q_nope . W_UK | q_pe]  (batched GEMM over heads)
  o_lat = ome_mla_attn(q_lat, latent cache)           [T, H, 512]   (csrc/kernels/mla.hip)
  o     = o_lat . W_UV^T -> o_proj -> TP all-reduce
So the KV cache is 576 x 2 B per token per layer (70 KB/token for V3's 61 layers) regardless of
the head count, and decode is MQA-shaped: all heads of a token share every latent byte read.

The MLP is dense for the first ``first_k_dense_replace`` layers and routed MoE afterwards:
sigmoid (V3) / softmax (V2) scores, group-limited top-k (``noaux_tc`` with
``e_score_correction_bias`` for V3, ``group_limited_greedy`` for V2) in ``ome_moe_route``,
grouped MFMA GEMMs, ``routed_scaling_factor``, plus the always-on shared experts.
Heads, expert intermediates and the dense MLP are tensor-parallel; the latent cache is
replicated per rank.
"""
from __future__ import annotations

import math

import torch

from ome_amd import ops
from ome_amd.models.common import AttnMeta, PagedKVCache
from ome_amd.models.config import ModelConfig, rope_cos_sin
from ome_amd.models.llama import LlamaForCausalLM
from ome_amd.models.quant import dequant_fp8_stream, linear
from ome_amd.parallel import state as pstate

KV_LATENT = 512
ROPE_DIM = 64
#: (kv_lora_rank, qk_rope_head_dim) pairs with a compiled MLA kernel (csrc/kernels/mla.hip)
MLA_SHAPES = {(512, 64), (256, 32)}


def _yarn_mscale(scale: float, m: float) -> float:
    return 1.0 if scale <= 1 else 0.1 * m * math.log(scale) + 1.0


class DeepseekForCausalLM(LlamaForCausalLM):
    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        if (cfg.kv_lora_rank, cfg.qk_rope_head_dim) not in MLA_SHAPES:
            raise ValueError(f"MLA kernel is built for (kv_lora_rank, qk_rope_head_dim) in {sorted(MLA_SHAPES)} "
                             f"(got {cfg.kv_lora_rank}, {cfg.qk_rope_head_dim})")
        # the dense base sets up TP shapes from num_heads; MLA has no kv heads of its own
        super().__init__(cfg, device, dtype, max_positions)
        st = pstate.get()
        if cfg.num_heads % st.tp_size:
            raise ValueError("num_heads must divide by tp")
        self.Hl = cfg.num_heads // st.tp_size
        self.nope, self.rope, self.vd = cfg.qk_nope_head_dim, cfg.qk_rope_head_dim, cfg.v_head_dim
        self.lat = cfg.kv_lora_rank      # latent width; cache rows are [lat | rope]
        self.qk_dim = self.nope + self.rope
        self.qlr = cfg.q_lora_rank
        scale = self.qk_dim ** -0.5
        sc = cfg.rope_scaling or {}
        if sc.get("mscale_all_dim"):
            scale *= _yarn_mscale(sc.get("factor", 1.0), sc["mscale_all_dim"]) ** 2
        self.scale = scale
        rc = ModelConfig(**{**cfg.__dict__, "head_dim": self.rope, "partial_rotary_factor": 1.0})
        mp = max_positions or cfg.max_position_embeddings
        self.cos_sin = rope_cos_sin(rc, mp, device=self.device)
        self.interleaved_rope = bool((cfg.extra or {}).get("rope_interleave", True))
        # MoE (expert parallelism under DP attention: this rank owns experts [e0, e0 + E_local))
        self.E, self.k = cfg.num_experts, cfg.num_experts_per_tok
        self.ep = st.ep_size
        if self.E and self.E % self.ep:
            raise ValueError(f"{self.E} experts do not split over ep={self.ep}")
        self.E_local = self.E // self.ep if self.E else 0
        self.e0 = st.ep_rank * self.E_local
        self.moe_inter = -(-cfg.moe_intermediate_size // st.tp_size) if cfg.num_experts else 0
        self.shared_inter = -(-(cfg.num_shared_experts * cfg.moe_intermediate_size) // st.tp_size) \
            if cfg.num_shared_experts else 0
        topk_method = (cfg.extra or {}).get("topk_method", "noaux_tc" if cfg.model_type == "deepseek_v3" else
                                            "greedy")
        self.group_mode = {"greedy": 0, "group_limited_greedy": 1, "noaux_tc": 2}.get(topk_method, 0)
        self.routed_scale = cfg.routed_scaling_factor
        if cfg.model_type == "deepseek_v2" and cfg.norm_topk_prob:
            self.routed_scale = 1.0  # V2 applies the factor only to unnormalised weights
        L = cfg.num_layers
        step = max(1, cfg.moe_layer_freq)
        self.moe_layers = {i for i in self.layers if cfg.num_experts and i >= cfg.first_k_dense_replace and
                           i % step == 0}
        from ome_amd.parallel import eplb

        eplb.attach(self)  # expert slots per rank (+ redundant replicas) under expert parallelism
        self.w_qa: list = [None] * L      # [q_lora + 576, H] fused q_a / kv_a (or [576, H] if no q_lora)
        self.qa_ln: list = [None] * L
        self.w_qb: list = [None] * L      # [Hl * qk_dim, q_lora] (or [Hl * qk_dim, H] = q_proj)
        self.kva_ln: list = [None] * L
        self.w_uk: list = [None] * L      # [Hl, nope, 512]
        self.w_uv: list = [None] * L      # [Hl, 512, vd]
        self.w_router: list = [None] * L
        self.b_router: list = [None] * L  # e_score_correction_bias (f32)
        self.w13: list = [None] * L
        self.w2: list = [None] * L
        self.w_sgu: list = [None] * L
        self.w_sd: list = [None] * L
        self.kv_layout = (1, self.lat + self.rope, 0)
        self.tune_gemms = False  # TunableOp pre-capture tuning is validated on the dense family only
        self._ws = None
        self._arange = None

    # ------------------------------------------------------------------ weights
    def init_random(self, seed: int = 0, std: float = 0.02) -> "DeepseekForCausalLM":
        cfg = self.cfg
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 7919 * pstate.get().tp_rank)
        H, Hl = cfg.hidden_size, self.Hl
        out_std = std / math.sqrt(2 * cfg.num_layers)
        st = pstate.get()
        inter = -(-cfg.intermediate_size // st.tp_size)
        for i in self.layers:
            self.w_qa[i] = self._alloc(self.qlr + self.lat + self.rope, H, std=std, gen=gen)
            if self.qlr:
                self.qa_ln[i] = self._alloc(self.qlr, std=None, gen=gen)
            self.w_qb[i] = self._alloc(Hl * self.qk_dim, self.qlr or H, std=std, gen=gen)
            self.kva_ln[i] = self._alloc(self.lat, std=None, gen=gen)
            self.w_uk[i] = self._alloc(Hl, self.nope, self.lat, std=std, gen=gen)
            self.w_uv[i] = self._alloc(Hl, self.lat, self.vd, std=std, gen=gen)
            self.w_o[i] = self._alloc(H, Hl * self.vd, std=out_std, gen=gen)
            self.ln1[i] = self._alloc(H, std=None, gen=gen)
            self.ln2[i] = self._alloc(H, std=None, gen=gen)
            if i in self.moe_layers:
                I = self.moe_inter
                self.w_router[i] = self._alloc(self.E, H, std=std, gen=gen)
                if self.group_mode == 2:
                    self.b_router[i] = torch.zeros(self.E, dtype=torch.float32, device=self.device)
                idx = torch.tensor(self.local_experts(i), dtype=torch.long, device=self.device)
                self.w13[i] = self._alloc(self.E, 2 * I, H, std=std, gen=gen).index_select(0, idx).contiguous()
                self.w2[i] = self._alloc(self.E, H, I, std=out_std, gen=gen).index_select(0, idx).contiguous()
                if self.shared_inter:
                    self.w_sgu[i] = self._alloc(2 * self.shared_inter, H, std=std, gen=gen)
                    self.w_sd[i] = self._alloc(H, self.shared_inter, std=out_std, gen=gen)
            else:
                self.w_gu[i] = self._alloc(2 * inter, H, std=std, gen=gen)
                self.w_d[i] = self._alloc(H, inter, std=out_std, gen=gen)
        tp = self.tp
        self.embed = self._alloc(tp.vocab, H, std=1.0, gen=gen)
        self.norm = self._alloc(H, std=None, gen=gen)
        self.lm_head = self.embed if cfg.tie_word_embeddings else self._alloc(tp.vocab, H, std=std, gen=gen)
        self._post_load()
        return self

    def _post_load(self) -> None:
        if not self.fp8:
            return
        from ome_amd.models.quant import quantize_moe_experts, quantize_weight

        for lst in (self.w_qa, self.w_qb, self.w_o, self.w_gu, self.w_d, self.w_sgu, self.w_sd):
            for i in self.layers:
                if self._quantizable(lst[i]):
                    lst[i] = quantize_weight(lst[i], self.fp8_block, tp=self.tp.tp)
        quantize_moe_experts(self)   # routed experts stay fp8 (block-scaled grouped GEMM)

    def _deinterleave_rows(self, w: torch.Tensor, head_dim: int, n_heads: int) -> torch.Tensor:
        """HF DeepSeek rotates interleaved (x0,x1),(x2,x3)... pairs of the rope dims; permute the
        projection rows once so the rope dims come out as [evens | odds] (NeoX layout)."""
        if not self.interleaved_rope:
            return w
        R = self.rope
        perm = torch.cat([torch.arange(0, R, 2), torch.arange(1, R, 2)])
        idx = []
        for h in range(n_heads):
            base = h * head_dim + head_dim - R
            idx.append(torch.arange(h * head_dim, base))
            idx.append(base + perm)
        return w[torch.cat(idx).to(w.device)]

    def load_hf_weights(self, weights) -> "DeepseekForCausalLM":
        cfg = self.cfg
        st = pstate.get()
        r, Hl = st.tp_rank, self.Hl
        inter = -(-cfg.intermediate_size // st.tp_size)
        I, SI = self.moe_inter, self.shared_inter
        if self.fp8:
            weights = dequant_fp8_stream(weights, self.fp8_block, self.dtype)
        parts: dict[int, dict[str, torch.Tensor]] = {}
        experts: dict[int, dict[int, dict[str, torch.Tensor]]] = {}

        def put(t, dtype=None):
            return t.to(device=self.device, dtype=dtype or self.dtype).contiguous()

        def rows(t, n):
            return t.narrow(0, r * n, min(n, t.shape[0] - r * n))

        def cols(t, n):
            return t.narrow(1, r * n, min(n, t.shape[1] - r * n))

        for name, w in weights:
            n = name[len("model."):] if name.startswith("model.") else name
            if n == "embed_tokens.weight":
                self.embed = put(self._vocab_shard(w))
                continue
            if n == "norm.weight":
                self.norm = put(w)
                continue
            if n == "lm_head.weight":
                self.lm_head = put(self._vocab_shard(w))
                continue
            p = n.split(".")
            if p[0] != "layers" or int(p[1]) not in self._layer_set:
                continue
            i, rest = int(p[1]), ".".join(p[2:])
            d = parts.setdefault(i, {})
            if rest in ("mlp.experts.gate_up_proj", "mlp.experts.down_proj"):
                # transformers >= 5 fused expert tensors: [E, 2I, H] (gate | up) / [E, H, I]
                for e in range(w.shape[0]):
                    de = experts.setdefault(i, {}).setdefault(e, {})
                    if p[4] == "down_proj":
                        de["down_proj"] = w[e]
                    else:
                        de["gate_proj"], de["up_proj"] = w[e].chunk(2, 0)
            elif rest.startswith("mlp.experts."):
                e = int(p[4])
                experts.setdefault(i, {}).setdefault(e, {})[p[5]] = w
            elif rest in ("self_attn.q_proj.weight", "self_attn.q_b_proj.weight"):
                full = self._deinterleave_rows(w, self.qk_dim, cfg.num_heads)
                self.w_qb[i] = put(rows(full, Hl * self.qk_dim))
            elif rest == "self_attn.kv_b_proj.weight":
                kvb = rows(w, Hl * (self.nope + self.vd)).reshape(Hl, self.nope + self.vd, self.lat)
                self.w_uk[i] = put(kvb[:, : self.nope, :])
                self.w_uv[i] = put(kvb[:, self.nope:, :].transpose(1, 2))
            elif rest == "self_attn.o_proj.weight":
                self.w_o[i] = put(cols(w, Hl * self.vd))
            elif rest == "self_attn.q_a_layernorm.weight":
                self.qa_ln[i] = put(w)
            elif rest == "self_attn.kv_a_layernorm.weight":
                self.kva_ln[i] = put(w)
            elif rest == "input_layernorm.weight":
                self.ln1[i] = put(w)
            elif rest == "post_attention_layernorm.weight":
                self.ln2[i] = put(w)
            elif rest == "mlp.gate.weight":
                self.w_router[i] = put(w)
            elif rest == "mlp.gate.e_score_correction_bias":
                self.b_router[i] = put(w, torch.float32)
            else:
                d[rest] = w
        for i, d in parts.items():
            if "self_attn.kv_a_proj_with_mqa.weight" in d:
                kva = self._deinterleave_rows(d["self_attn.kv_a_proj_with_mqa.weight"], self.lat + self.rope, 1)
                qa = d.get("self_attn.q_a_proj.weight")
                self.w_qa[i] = put(torch.cat([qa, kva], 0) if qa is not None else kva)
            if "mlp.gate_proj.weight" in d:
                self.w_gu[i] = put(torch.cat([rows(d["mlp.gate_proj.weight"], inter),
                                              rows(d["mlp.up_proj.weight"], inter)], 0))
                self.w_d[i] = put(cols(d["mlp.down_proj.weight"], inter))
            if "mlp.shared_experts.gate_proj.weight" in d:
                self.w_sgu[i] = put(torch.cat([rows(d["mlp.shared_experts.gate_proj.weight"], SI),
                                               rows(d["mlp.shared_experts.up_proj.weight"], SI)], 0))
                self.w_sd[i] = put(cols(d["mlp.shared_experts.down_proj.weight"], SI))
        for i, ex in experts.items():
            gs, ds = [], []
            for e in self.local_experts(i):
                de = ex[e]
                gs.append(torch.cat([rows(de["gate_proj"], I), rows(de["up_proj"], I)], 0))
                ds.append(cols(de["down_proj"], I))
            self.w13[i] = put(torch.stack(gs))
            self.w2[i] = put(torch.stack(ds))
        if self.lm_head is None:
            self.lm_head = self.embed
        missing = [i for i in self.layers if self.w_qa[i] is None or self.w_uk[i] is None or
                   (i in self.moe_layers and self.w13[i] is None) or (i not in self.moe_layers and self.w_gu[i] is None)]
        if missing or self.embed is None:
            raise ValueError(f"checkpoint incomplete: layers missing {missing[:4]}")
        self._post_load()
        return self

    def local_experts(self, i: int) -> list[int]:
        from ome_amd.parallel import eplb

        return eplb.local_experts(self, i)

    def weight_bytes(self) -> int:
        from ome_amd.models.quant import Fp8Weight

        n = 0
        seen = set()
        for lst in (self.w_qa, self.qa_ln, self.w_qb, self.kva_ln, self.w_uk, self.w_uv, self.w_o, self.ln1, self.ln2,
                    self.w_gu, self.w_d, self.w_router, self.w13, self.w2, self.w_sgu, self.w_sd,
                    [self.embed, self.norm, self.lm_head]):
            for t in lst:
                if isinstance(t, Fp8Weight) or hasattr(t, "nbytes") and callable(getattr(t, "nbytes", None)):
                    n += t.nbytes()
                elif t is not None and t.data_ptr() not in seen:
                    seen.add(t.data_ptr())
                    n += t.numel() * t.element_size()
        return n

    # ------------------------------------------------------------------ forward
    def _token_rows(self, meta: AttnMeta, T: int):
        """(tok_row, kv_lens) per query token, plus the block table they index."""
        if self._arange is None or self._arange.numel() < T:
            self._arange = torch.arange(max(T, 4096), dtype=torch.int32, device=self.device)
        kv_lens = (meta.positions + 1).to(torch.int32)
        if meta.is_decode:
            return [(0, T, meta.block_tables, self._arange[:T], meta.seq_lens)]
        n = meta.num_prefill if meta.mode == "mixed" else T
        seg = []
        if n:
            cu = meta.cu_q
            rows = torch.searchsorted(cu[1:].contiguous(), self._arange[:n].to(cu.dtype), right=True).to(torch.int32)
            seg.append((0, n, meta.block_tables, rows, kv_lens[:n]))
        if n < T:
            seg.append((n, T, meta.dec_block_tables, self._arange[: T - n], meta.seq_lens))
        return seg

    def attention_block(self, i: int, x: torch.Tensor, meta: AttnMeta, kv: PagedKVCache) -> torch.Tensor:
        T = x.shape[0]
        Hl = self.Hl
        a = linear(x, self.w_qa[i])
        if self.qlr:
            qa = ops.rmsnorm(a[:, : self.qlr], self.qa_ln[i], self.eps)   # row-strided view, no copy
            q = linear(qa, self.w_qb[i])
        else:
            q = linear(x, self.w_qb[i])
        lat = self.lat
        q = q.view(T, Hl, self.qk_dim)
        cache = kv.k[i]
        flat = cache.view(-1, lat + self.rope)
        q_full = torch.empty(T, Hl, lat + self.rope, dtype=x.dtype, device=x.device)   # [q_nope . W_UK | q_pe]
        # kv_a_layernorm + RoPE(k_pe) -> latent cache row, RoPE(q_pe) -> q_full: one kernel
        # (padding rows carry slot -1: parked in the scratch page 0)
        ops.mla_prep(a, self.qlr, lat, self.rope, self.kva_ln[i], self.eps, meta.positions, self.cos_sin, meta.slots,
                     flat, q, self.nope, q_full)
        # strided batched GEMMs read the head-major views in place (no transpose copies)
        q_nope = q[..., : self.nope].transpose(0, 1)                       # [Hl, T, nope] view
        # written straight into q_full's latent columns (a [Hl, T, lat] view with unit inner
        # stride: the batched GEMM takes it as its output layout, no copy pass)
        torch.bmm(q_nope, self.w_uk[i], out=q_full[:, :, :lat].transpose(0, 1))
        o_lat = torch.empty(T, Hl, lat, dtype=x.dtype, device=x.device)
        ws = None
        if x.is_cuda:   # one split-K workspace per stream (two-batch overlap runs two at once)
            if self._ws is None:
                self._ws = {}
            sid = torch.cuda.current_stream(x.device).cuda_stream
            ws = self._ws.get(sid)
            if ws is None:
                ws = self._ws[sid] = ops.MLAWorkspace(x.device)
        cache3 = cache.view(cache.shape[0], -1, lat + self.rope)
        for s, e, bt, rows, lens in self._token_rows(meta, T):
            ops.mla_attn(q_full[s:e], cache3, bt, rows, lens, self.scale, ws, out=o_lat[s:e], dv=lat)
        o = torch.empty(T, Hl * self.vd, dtype=x.dtype, device=x.device)
        torch.bmm(o_lat.transpose(0, 1), self.w_uv[i], out=o.view(T, Hl, self.vd).transpose(0, 1))   # token-major
        return pstate.tp_all_reduce(linear(o, self.w_o[i]))

    def mlp(self, i: int, x: torch.Tensor) -> torch.Tensor:
        if i not in self.moe_layers:
            return super().mlp(i, x)
        cfg = self.cfg
        logits = torch.nn.functional.linear(x, self.w_router[i])
        tw, tid = ops.moe_route(logits, self.k, cfg.norm_topk_prob and self.k > 1, cfg.scoring_func,
                                bias=self.b_router[i], n_group=cfg.n_group, topk_group=cfg.topk_group,
                                group_mode=self.group_mode)
        if self.ep > 1:
            from ome_amd.parallel.ep import moe_ep

            tables = None
            if self.eplb is not None:
                self.eplb.record(i, tid)
                tables = self.eplb.tables[i]
            out = moe_ep(x, tw, tid, self.w13[i], self.w2[i], self.act, self.routed_scale, self.E, tables)
            if self.w_sgu[i] is not None:
                out = out + linear(ops.act_and_mul(linear(x, self.w_sgu[i]), self.act), self.w_sd[i])
        elif self.w_sgu[i] is not None:   # shared experts first; the routed sum lands on them in the combine
            sh = linear(ops.act_and_mul(linear(x, self.w_sgu[i]), self.act), self.w_sd[i])
            out = ops.fused_moe(x, tw, tid, self.w13[i], self.w2[i], self.act, self.routed_scale, add=sh.contiguous())
        else:
            out = ops.fused_moe(x, tw, tid, self.w13[i], self.w2[i], self.act, self.routed_scale)
        return pstate.tp_all_reduce(out)

    def forward(self, ids: torch.Tensor, meta: AttnMeta, kv: PagedKVCache,
                input_embeds: torch.Tensor | None = None) -> torch.Tensor:
        x, residual = self._stage_input(ids, input_embeds)
        for i in self.layers:
            if i > 0:
                ops.fused_add_rmsnorm(x, residual, self.ln1[i], self.eps)
            o = self.attention_block(i, x, meta, kv)
            ops.fused_add_rmsnorm(o, residual, self.ln2[i], self.eps)
            x = self.mlp(i, o)
        return self._stage_output(x, residual)
