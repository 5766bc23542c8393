"""Dense decoder family (Llama 2/3/3.1/3.2, Mistral, Qwen2/2.5, Qwen3) on the ome_amd kernels.

Per layer (SURVEY.md §3.6 hot loop):
  fused_add_rmsnorm -> QKV GEMM (hipBLASLt) -> fused RoPE + paged KV write (HIP) ->
  paged attention (HIP, MFMA) -> O GEMM -> TP all-reduce -> fused_add_rmsnorm ->
  gate_up GEMM -> SiLU*mul (HIP) -> down GEMM -> TP all-reduce.
Tensor parallelism is Megatron-style: QKV / gate_up column-parallel, O / down row-parallel,
vocab-parallel embedding and LM head.  KV heads are replicated when tp > num_kv_heads.
"""
from __future__ import annotations

import math
import os

import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.models.common import AttnMeta, PagedKVCache, mixed_attention
from ome_amd.models.config import ModelConfig, rope_cos_sin
from ome_amd.models.quant import _GEMV_ROWS, Fp8Weight, dequant_fp8_stream, fp8_block_size, linear, quantize_weight
from ome_amd.parallel import state as pstate

# fused SwiGLU + down GEMV at batch <= 4: opt-in.  Measured slower at c=1 (256.9 vs 279.0 tok/s):
# every wave of the GEMV recomputes SiLU over the whole K (N/R waves x K exps), which costs more
# VALU time than the act_and_mul launch it removes.
_GEMV_ACT = os.environ.get("OME_GEMV_ACT", "0") == "1"


def _dtype(name: str) -> torch.dtype:
    return {"bfloat16": torch.bfloat16, "float16": torch.float16, "float32": torch.float32}.get(
        str(name).replace("torch.", ""), torch.bfloat16)


class TPShape:
    """Local (per-rank) shapes of a dense decoder under tensor parallelism."""

    def __init__(self, cfg: ModelConfig, tp: int, rank: int):
        if cfg.num_heads % tp:
            raise ValueError(f"num_heads {cfg.num_heads} not divisible by tp {tp}")
        self.tp, self.rank = tp, rank
        self.hq = cfg.num_heads // tp
        if cfg.num_kv_heads >= tp:
            if cfg.num_kv_heads % tp:
                raise ValueError(f"num_kv_heads {cfg.num_kv_heads} not divisible by tp {tp}")
            self.hkv = cfg.num_kv_heads // tp
            self.kv_start = rank * self.hkv
        else:  # replicate kv heads
            self.hkv = 1
            self.kv_start = rank * cfg.num_kv_heads // tp
        inter = cfg.intermediate_size
        self.inter = -(-inter // tp)
        self.vocab = -(-cfg.vocab_size // tp)
        self.vocab_start = rank * self.vocab
        self.vocab_end = min(cfg.vocab_size, self.vocab_start + self.vocab)


class LlamaForCausalLM:
    """Weights live as plain tensors in per-layer lists (no nn.Module dispatch on the hot path)."""

    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        self.cfg, self.device, self.dtype = cfg, torch.device(device), dtype
        st = pstate.get()
        self.tp = TPShape(cfg, st.tp_size, st.tp_rank)
        self.D = cfg.head_dim
        self.eps = cfg.rms_norm_eps
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        self.window = cfg.sliding_window or -1
        self.act = 0 if cfg.hidden_act in ("silu", "swish") else 1
        L = cfg.num_layers
        # pipeline parallelism: this stage owns a contiguous slice of the decoder layers; the
        # per-layer lists stay indexed by the global layer id (other stages' entries are None)
        self.layers = pstate.stage_layers(L, st.pp_size, st.pp_rank)
        self._layer_set = set(self.layers)
        self.kv_scales: dict[int, tuple[float, float]] = {}  # checkpoint fp8 KV scales per layer
        self.w_qkv: list[torch.Tensor] = [None] * L
        self.b_qkv: list[torch.Tensor | None] = [None] * L
        self.w_o: list[torch.Tensor] = [None] * L
        self.ln1: list[torch.Tensor] = [None] * L
        self.ln2: list[torch.Tensor] = [None] * L
        self.w_gu: list[torch.Tensor] = [None] * L
        self.w_d: list[torch.Tensor] = [None] * L
        self.qn: list[torch.Tensor | None] = [None] * L
        self.kn: list[torch.Tensor | None] = [None] * L
        self.embed: torch.Tensor | None = None
        self.norm: torch.Tensor | None = None
        self.lm_head: torch.Tensor | None = None
        mp = max_positions or cfg.max_position_embeddings
        self.cos_sin = rope_cos_sin(cfg, mp, device=self.device)
        self.fp8 = (cfg.quantization or "").lower() in ("fp8", "fbgemm_fp8")
        self.fp8_block = fp8_block_size(cfg) if self.fp8 else 0

    # ------------------------------------------------------------------ weights
    def _alloc(self, *shape, std: float | None, gen: torch.Generator | None) -> torch.Tensor:
        t = torch.empty(*shape, dtype=self.dtype, device=self.device)
        if std is None:
            t.fill_(1.0)
        else:
            t.normal_(0.0, std, generator=gen)
        return t

    def init_random(self, seed: int = 0, std: float = 0.02) -> "LlamaForCausalLM":
        """Random-init weights of this architecture (BASELINE rule: synthetic weights)."""
        cfg, tp, D = self.cfg, self.tp, self.D
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 7919 * pstate.get().tp_rank)
        H = cfg.hidden_size
        qkv_rows = (tp.hq + 2 * tp.hkv) * D
        for i in self.layers:
            self.w_qkv[i] = self._alloc(qkv_rows, H, std=std, gen=gen)
            if cfg.attention_bias:
                self.b_qkv[i] = self._alloc(qkv_rows, std=std, gen=gen)
            self.w_o[i] = self._alloc(H, tp.hq * D, std=std / math.sqrt(2 * cfg.num_layers), gen=gen)
            self.ln1[i] = self._alloc(H, std=None, gen=gen)
            self.ln2[i] = self._alloc(H, std=None, gen=gen)
            self.w_gu[i] = self._alloc(2 * tp.inter, H, std=std, gen=gen)
            self.w_d[i] = self._alloc(H, tp.inter, std=std / math.sqrt(2 * cfg.num_layers), gen=gen)
            if cfg.qk_norm:
                self.qn[i] = self._alloc(D, std=None, gen=gen)
                self.kn[i] = self._alloc(D, std=None, gen=gen)
        self.embed = self._alloc(tp.vocab, H, std=1.0, gen=gen)
        self.norm = self._alloc(H, std=None, gen=gen)
        self.lm_head = self.embed if cfg.tie_word_embeddings else self._alloc(tp.vocab, H, std=std, gen=gen)
        self._post_load()
        return self

    def _quantizable(self, w) -> bool:
        return isinstance(w, torch.Tensor) and w.dim() == 2 and w.numel() > 0 and w.shape[0] % 64 == 0 and \
            w.shape[1] % 128 == 0

    plain_layout = False   # subclass keeps the Llama weight layout, loader and MLP (e.g. TeleFLM)

    def _plain(self) -> bool:
        return type(self) is LlamaForCausalLM or type(self).__dict__.get("plain_layout", False)

    softcap = 0.0   # attention-logit soft-capping cap * tanh(s / cap) (0: off)
    gu_il = False   # gate_up rows interleaved in 16-row blocks (fused SiLU*mul GEMM epilogue)

    def _post_load(self) -> None:
        """``quantization: fp8``: the QKV / O / gate-up / down projections become W8A8 (the
        embedding, LM head and norms stay bf16, as in the reference runtimes).  bf16 SwiGLU on a
        GPU: gate_up weights are interleaved in 16-row blocks so the stream-K GEMM can apply
        SiLU(gate) * up in its epilogue (no act_and_mul pass, no [T, 2I] intermediate)."""
        if not self.fp8 and self._plain() and self.act == 0 and self.device.type == "cuda" and \
                self.dtype == torch.bfloat16 and os.environ.get("OME_GATE_UP_INTERLEAVE", "1") == "1" and \
                all(isinstance(self.w_gu[i], torch.Tensor) and self.w_gu[i].shape[0] % 32 == 0 for i in self.layers):
            for i in self.layers:
                self.w_gu[i] = ops.interleave_gate_up(self.w_gu[i])
            self.gu_il = True
        if not self.fp8:
            return
        kept = 0
        for lst in (self.w_qkv, self.w_o, self.w_gu, self.w_d):
            for i in self.layers:
                if self._quantizable(lst[i]):
                    lst[i] = quantize_weight(lst[i], self.fp8_block, tp=self.tp.tp)
                elif isinstance(lst[i], torch.Tensor) and lst[i].numel():
                    kept += 1
        import logging

        from ome_amd.models.quant import fp8_bf16_copy_bytes

        log = logging.getLogger("ome_amd.models")
        if kept:
            log.warning("fp8: %d projections keep bf16 (shape not 64x128-tileable)", kept)
        if fp8_bf16_copy_bytes():
            log.info("fp8: bf16 copies of the small projections: %.1f MiB in this process",
                     fp8_bf16_copy_bytes() / 2 ** 20)

    # ------------------------------------------------------------------ rank-aware loading
    _presliced = False   # set by build_model when the loader already applied shard_plan

    def sharded(self) -> bool:
        """Whether this rank reads only its shard of the checkpoint (dense Llama family under
        TP / PP; fp8 checkpoints keep whole-tensor reads: their scales follow the block grid)."""
        st = pstate.get()
        return self._plain() and not self.fp8 and (self.tp.tp > 1 or st.pp_size > 1)

    def shard_plan(self, name: str, shape) -> tuple[str, int, int] | None:
        """This rank's slice of checkpoint tensor ``name`` (full ``shape``), mirroring
        :meth:`load_hf_weights`: column-parallel q/k/v/gate/up and the vocab-parallel embedding
        / LM head by rows, row-parallel o/down by columns; other pipeline stages' layers are not
        read at all (("rows", 0, 0))."""
        tp, D = self.tp, self.D
        n = name[len("model."):] if name.startswith("model.") else name
        if n in ("embed_tokens.weight", "lm_head.weight"):
            return "rows", tp.vocab_start, max(0, min(tp.vocab, shape[0] - tp.vocab_start))
        parts = n.split(".")
        if parts[0] != "layers" or len(parts) < 3:
            return None
        if int(parts[1]) not in self._layer_set:
            return "rows", 0, 0
        rest = ".".join(parts[2:])
        if rest in ("self_attn.q_proj.weight", "self_attn.q_proj.bias"):
            return "rows", tp.rank * tp.hq * D, tp.hq * D
        if rest in ("self_attn.k_proj.weight", "self_attn.k_proj.bias", "self_attn.v_proj.weight",
                    "self_attn.v_proj.bias"):
            return "rows", tp.kv_start * D, tp.hkv * D
        if rest == "self_attn.o_proj.weight":
            return "cols", tp.rank * tp.hq * D, tp.hq * D
        if rest in ("mlp.gate_proj.weight", "mlp.up_proj.weight"):
            return "rows", tp.rank * tp.inter, max(0, min(tp.inter, shape[0] - tp.rank * tp.inter))
        if rest == "mlp.down_proj.weight":
            return "cols", tp.rank * tp.inter, max(0, min(tp.inter, shape[1] - tp.rank * tp.inter))
        return None

    def load_hf_weights(self, weights) -> "LlamaForCausalLM":
        """Load from an iterator of (hf_name, tensor) — shards / fuses for this TP rank (tensors
        arrive already sliced when the loader applied :meth:`shard_plan`)."""
        cfg, tp, D = self.cfg, self.tp, self.D
        qkv_parts: dict[int, dict[str, torch.Tensor]] = {}
        gu_parts: dict[int, dict[str, torch.Tensor]] = {}
        pre = self._presliced

        def rows(t, start, n):
            return t if pre else t.narrow(0, start, n)

        def cols(t, start, n):
            return t if pre else t.narrow(1, start, n)

        def put(t):
            return t.to(device=self.device, dtype=self.dtype).contiguous()

        if self.fp8:
            weights = dequant_fp8_stream(weights, self.fp8_block, self.dtype)
        for name, w in weights:
            if name.startswith("model."):
                name = name[len("model."):]
            if name == "embed_tokens.weight":
                self.embed = put(self._vocab_shard(w))
                continue
            if name == "norm.weight":
                self.norm = put(w)
                continue
            if name == "lm_head.weight":
                self.lm_head = put(self._vocab_shard(w))
                continue
            parts = name.split(".")
            if parts[0] != "layers":
                continue
            i, rest = int(parts[1]), ".".join(parts[2:])
            if i not in self._layer_set:
                continue
            if rest in ("self_attn.q_proj.weight", "self_attn.q_proj.bias"):
                qkv_parts.setdefault(i, {})["q" + rest[-1]] = rows(w, tp.rank * tp.hq * D, tp.hq * D)
            elif rest in ("self_attn.k_proj.weight", "self_attn.k_proj.bias"):
                qkv_parts.setdefault(i, {})["k" + rest[-1]] = rows(w, tp.kv_start * D, tp.hkv * D)
            elif rest in ("self_attn.v_proj.weight", "self_attn.v_proj.bias"):
                qkv_parts.setdefault(i, {})["v" + rest[-1]] = rows(w, tp.kv_start * D, tp.hkv * D)
            elif rest == "self_attn.o_proj.weight":
                self.w_o[i] = put(cols(w, tp.rank * tp.hq * D, tp.hq * D))
            elif rest == "mlp.gate_proj.weight":
                gu_parts.setdefault(i, {})["g"] = rows(w, tp.rank * tp.inter, min(tp.inter, w.shape[0] - tp.rank * tp.inter))
            elif rest == "mlp.up_proj.weight":
                gu_parts.setdefault(i, {})["u"] = rows(w, tp.rank * tp.inter, min(tp.inter, w.shape[0] - tp.rank * tp.inter))
            elif rest == "mlp.down_proj.weight":
                self.w_d[i] = put(cols(w, tp.rank * tp.inter, min(tp.inter, w.shape[1] - tp.rank * tp.inter)))
            elif rest == "input_layernorm.weight":
                self.ln1[i] = put(w)
            elif rest == "post_attention_layernorm.weight":
                self.ln2[i] = put(w)
            elif rest == "self_attn.q_norm.weight":
                self.qn[i] = put(w)
            elif rest == "self_attn.k_norm.weight":
                self.kn[i] = put(w)
            elif rest.endswith((".k_scale", ".v_scale")) and rest.startswith("self_attn."):
                # fp8 KV-cache scales (``self_attn.k_scale`` / ``self_attn.attn.k_scale`` /
                # ``self_attn.k_proj.k_scale`` spellings), consumed by --kv-cache-dtype fp8
                ks, vs = self.kv_scales.get(i, (1.0, 1.0))
                val = float(w.float().max())
                self.kv_scales[i] = (val, vs) if rest.endswith(".k_scale") else (ks, val)
        for i, p in qkv_parts.items():
            self.w_qkv[i] = put(torch.cat([p["qt"], p["kt"], p["vt"]], 0))
            if "qs" in p:
                self.b_qkv[i] = put(torch.cat([p["qs"], p["ks"], p["vs"]], 0))
        for i, p in gu_parts.items():
            self.w_gu[i] = put(torch.cat([p["g"], p["u"]], 0))
        if self.lm_head is None:
            self.lm_head = self.embed
        missing = [i for i in self.layers if self.w_qkv[i] is None or self.w_gu[i] is None]
        if missing or self.embed is None:
            raise ValueError(f"checkpoint incomplete: layers missing {missing[:4]}...")
        self._post_load()
        return self

    def gate_up_weight(self, i: int) -> torch.Tensor:
        """Layer i's gate_up weight in checkpoint order ([gate; up] rows), whatever the layout
        the kernels use."""
        w = self.w_gu[i]
        if not self.gu_il:
            return w
        g, u = ops.deinterleave_gate_up(w.t())
        return torch.cat([g.t(), u.t()], 0)

    def _vocab_shard(self, w: torch.Tensor) -> torch.Tensor:
        tp = self.tp
        sh = w if self._presliced else w[tp.vocab_start:tp.vocab_end]
        if sh.shape[0] < tp.vocab:
            sh = torch.cat([sh, sh.new_zeros(tp.vocab - sh.shape[0], sh.shape[1])], 0)
        return sh

    def weight_bytes(self) -> int:
        seen, n = set(), 0
        for lst in (self.w_qkv, self.b_qkv, self.w_o, self.ln1, self.ln2, self.w_gu, self.w_d, self.qn, self.kn,
                    [self.embed, self.norm, self.lm_head]):
            for t in lst:
                if isinstance(t, Fp8Weight):
                    n += t.nbytes()
                elif t is not None and t.data_ptr() not in seen:
                    seen.add(t.data_ptr())
                    n += t.numel() * t.element_size()
        return n

    # ------------------------------------------------------------------ forward
    def attention(self, q: torch.Tensor, k_cache, v_cache, meta: AttnMeta, ks: float = 1.0,
                  vs: float = 1.0) -> torch.Tensor:
        """``ks`` / ``vs``: the layer's fp8 KV dequantisation scales (1 for a bf16 cache)."""
        cap = self.softcap
        if meta.is_decode:
            return ops.paged_decode(q, k_cache, v_cache, meta.block_tables, meta.seq_lens, self.scale,
                                    meta.decode_ws, self.window, order=meta.order, k_scale=ks, v_scale=vs, softcap=cap)
        if meta.mode == "mixed":
            return mixed_attention(
                q, meta.num_prefill,
                lambda qp, op: ops.paged_prefill(qp, k_cache, v_cache, meta.block_tables, meta.cu_q, meta.kv_lens,
                                                 meta.items, self.scale, self.window, out=op, k_scale=ks, v_scale=vs,
                                                 softcap=cap),
                lambda qd, od: ops.paged_decode(qd, k_cache, v_cache, meta.dec_block_tables, meta.seq_lens,
                                                self.scale, meta.decode_ws, self.window, out=od, order=meta.order,
                                                k_scale=ks, v_scale=vs, softcap=cap))
        return ops.paged_prefill(q, k_cache, v_cache, meta.block_tables, meta.cu_q, meta.kv_lens, meta.items,
                                 self.scale, self.window, k_scale=ks, v_scale=vs, softcap=cap)

    def gemm_probe(self, i: int, x: torch.Tensor, a: torch.Tensor) -> None:
        """Layer i's projection GEMMs exactly as the forward routes them (QKV, O, gate_up with its
        SiLU epilogue, down), without the TP all-reduce: the row-count cost probe of
        ``runtime/step_cost.py``.  ``x`` [M, hidden], ``a`` [M, O-projection input width]."""
        linear(x, self.w_qkv[i], self.b_qkv[i])
        self._row_parallel(a, self.w_o[i])
        self._mlp_partial(i, x)

    def gemm_probe_widths(self) -> tuple[int, int] | None:
        """(hidden, O-projection input width) when this model's layers run exactly the dense
        QKV / O / gate_up / down projections :meth:`gemm_probe` times, else None (MoE, MLA and
        other subclasses that reuse the class with a different layer)."""
        i = self.layers[0] if self.layers else None
        if i is None or not self._plain() or any(lst[i] is None for lst in (self.w_qkv, self.w_o, self.w_gu, self.w_d)):
            return None
        return self.cfg.hidden_size, self.tp.hq * self.D

    def mlp(self, i: int, x: torch.Tensor) -> torch.Tensor:
        return pstate.tp_all_reduce(self._mlp_partial(i, x))

    def _mlp_partial(self, i: int, x: torch.Tensor) -> torch.Tensor:
        """gate_up -> SiLU*mul -> down: this rank's partial sums (before the TP all-reduce),
        written straight into the all-reduce's staging buffer when there is one."""
        wd = self.w_d[i]
        if self.gu_il:
            w = self.w_gu[i]
            plan = ops.gemm_sk_plan(x.shape[0], w.shape[0], w.shape[1], 2) if x.shape[0] > _GEMV_ROWS else None
            if plan is not None and x.stride(1) == 1 and x.stride(0) % 8 == 0:
                a = ops.gemm_sk(x, w, epi=2, bn=plan[0], nwg=plan[1], bm=plan[2])
            else:
                a = ops.act_and_mul(linear(x, w), self.act, interleaved=True)
            return self._row_parallel(a, wd)
        gu = linear(x, self.w_gu[i])
        if _GEMV_ACT and self.act == 0 and gu.is_cuda and type(wd) is torch.Tensor and gu.dim() == 2 and \
                gu.shape[0] <= _GEMV_ROWS and gu.dtype == wd.dtype == torch.bfloat16 and gu.stride(1) == 1 and \
                gu.stride(0) % 8 == 0 and gu.data_ptr() % 16 == 0 and wd.data_ptr() % 16 == 0:
            # decode at batch <= 4: SwiGLU folded into the down-projection GEMV's operand load
            st = pstate.tp_ar_staging((gu.shape[0], self.cfg.hidden_size), self.dtype, gu.device) \
                if self.tp.tp > 1 else None
            return ops.gemv_act(gu, wd, out=st)
        a = ops.act_and_mul(gu, self.act)
        return self._row_parallel(a, wd)

    def _row_parallel(self, a: torch.Tensor, w, bias=None) -> torch.Tensor:
        if self.tp.tp > 1:
            st = pstate.tp_ar_staging((a.shape[0], self.cfg.hidden_size), self.dtype, a.device)
            if st is not None:
                return linear(a, w, bias, out=st)
        return linear(a, w, bias)

    def _reduce_add_norm(self, part: torch.Tensor, residual: torch.Tensor, w: torch.Tensor,
                         reduce: bool = True) -> torch.Tensor:
        """residual += allreduce(part); return rmsnorm(residual) * w -- one fused xGMI kernel at
        decode sizes under TP, all-reduce + fused_add_rmsnorm otherwise (``reduce=False``: the
        input is already reduced)."""
        if self.tp.tp > 1 and reduce:
            y = pstate.tp_all_reduce_add_rmsnorm(part, residual, w, self.eps)
            if y is not None:
                return y
            part = pstate.tp_all_reduce(part)
        ops.fused_add_rmsnorm(part, residual, w, self.eps)
        return part

    def forward(self, ids: torch.Tensor, meta: AttnMeta, kv: PagedKVCache,
                input_embeds: torch.Tensor | None = None) -> torch.Tensor:
        """ids [T] int32 -> final normed hidden [T, H]."""
        cfg, tp, D = self.cfg, self.tp, self.D
        T = ids.shape[0]
        x, residual = self._stage_input(ids, input_embeds)
        st = pstate.get()
        first = self.layers[0] if self.layers else 0
        # subclasses that override mlp() (MoE) return already-reduced outputs
        partial = type(self).mlp is LlamaForCausalLM.mlp
        for i in self.layers:
            if i > 0:  # the previous layer's MLP partial sums -> all-reduce + add + norm (a pipeline
                # stage's first layer receives the previous stage's already-reduced output)
                x = self._reduce_add_norm(x, residual, self.ln1[i], reduce=partial and i > first)
            qkv = linear(x, self.w_qkv[i], self.b_qkv[i])
            q = torch.empty(T, tp.hq, D, dtype=self.dtype, device=x.device)
            k_cache, v_cache = kv.layer(i)
            ks, vs = kv.scales(i)
            ops.rope_qkv_cache(qkv, meta.positions, self.cos_sin, cfg.rot_dim, q, k_cache, v_cache, meta.slots,
                               tp.hq, tp.hkv, D, True, self.qn[i], self.kn[i], self.eps, ks, vs)
            attn = self.attention(q, k_cache, v_cache, meta, ks, vs)
            o = self._reduce_add_norm(self._row_parallel(attn.view(T, tp.hq * D), self.w_o[i]), residual,
                                      self.ln2[i])
            x = self._mlp_partial(i, o) if partial else self.mlp(i, o)
        if self.layers and (st.pp_size == 1 or st.is_last_pp):
            return self._reduce_add_norm(x, residual, self.norm, reduce=partial)   # final norm
        if self.layers and partial:
            x = pstate.tp_all_reduce(x)
        return self._stage_output(x, residual)

    def _stage_input(self, ids: torch.Tensor, input_embeds: torch.Tensor | None):
        """(x, residual) entering this stage's first layer: embedding + first RMSNorm on the
        first pipeline stage, received from the previous stage otherwise."""
        st = pstate.get()
        T, H = ids.shape[0], self.cfg.hidden_size
        if st.pp_size > 1 and not st.is_first_pp:
            x, residual = pstate.pp_recv(((T, H), self.dtype, ids.device), ((T, H), self.dtype, ids.device))
            return x, residual
        if input_embeds is None:
            h = pstate.tp_all_reduce(ops.embedding(ids, self.embed, self.tp.vocab_start, self.tp.vocab_end))
        else:
            h = input_embeds
        return ops.rmsnorm(h, self.ln1[0], self.eps), h

    def _stage_output(self, x: torch.Tensor, residual: torch.Tensor) -> torch.Tensor | None:
        """Last stage: final norm -> hidden states.  Earlier stages: ship (x, residual) on and
        return None (the sampled tokens come back via :func:`pstate.pp_broadcast_from_last`)."""
        st = pstate.get()
        if st.pp_size > 1 and not st.is_last_pp:
            pstate.pp_send(x, residual)
            return None
        ops.fused_add_rmsnorm(x, residual, self.norm, self.eps)
        return x

    def compute_logits(self, hidden: torch.Tensor) -> torch.Tensor:
        logits = linear(hidden, self.lm_head)
        if self.tp.tp > 1:
            logits = pstate.tp_all_gather(logits, dim=-1)
        return logits[:, : self.cfg.vocab_size]
