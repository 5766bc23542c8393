"""Gemma family (Gemma 1, Gemma 2, Gemma 3 text) on the ome_amd kernels.

Reference catalog entries: ``config/runtimes/srt/google/gemma-2-*-rt.yaml`` (Gemma2ForCausalLM) and
``gemma-3-*-rt.yaml`` (Gemma3ForConditionalGeneration; the language model is served here, image
inputs are not).  Differences from the Llama path (``llama.py``), all kept inside the same
kernels:

* RMSNorm scales by ``(1 + w)``: the ``1`` is folded into the weights at load time, so the
  standard ``rmsnorm`` / ``fused_add_rmsnorm`` kernels apply unchanged (also for Gemma-3 q/k-norm
  inside the fused RoPE kernel);
* embeddings are scaled by ``sqrt(hidden)`` (rounded to the model dtype, as HF does);
* Gemma 2/3 "sandwich" norms: the attention and MLP outputs are RMS-normalised again before the
  residual add (``post_attention_layernorm`` / ``post_feedforward_layernorm``); the pre-MLP norm
  is ``pre_feedforward_layernorm``;
* GeGLU MLP (``gelu_pytorch_tanh``), head_dim 256, attention scale ``query_pre_attn_scalar^-1/2``;
* Gemma 2 attention-logit soft-capping (``cap * tanh(s / cap)``, done inside the MFMA attention
  kernels) and final-logit soft-capping;
* per-layer sliding windows (``layer_types``; Gemma 2 alternates local/global, Gemma 3 has one
  global layer in six) and, for Gemma 3, a separate RoPE table for the local layers
  (``rope_local_base_freq``).

``Gemma2ForSequenceClassification`` (reward models such as Skywork-Reward-Gemma-2-27B-v0.2,
reference ``config/models/Skywork/Skywork-Reward-Gemma-2-27B-v0.2.yaml``): the same decoder, the
final norm's last-token row through the ``score`` Linear (no bias, no logit soft-capping), served as
an embedding-style model (``pool``).
"""
from __future__ import annotations

import torch

from ome_amd import ops
from ome_amd.models.common import AttnMeta, PagedKVCache
from ome_amd.models.config import ModelConfig, rope_cos_sin
from ome_amd.models.llama import LlamaForCausalLM
from ome_amd.models.quant import linear
from ome_amd.parallel import state as pstate

GEMMA_ARCHS = {"GemmaForCausalLM", "Gemma2ForCausalLM", "Gemma3ForCausalLM", "Gemma3ForConditionalGeneration",
               "Gemma2ForSequenceClassification"}


def _hf(cfg: ModelConfig) -> dict:
    ex = cfg.extra or {}
    return ex.get("text_config") or ex


class GemmaForCausalLM(LlamaForCausalLM):
    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        hf = {**(cfg.extra or {}), **_hf(cfg)}
        mt = cfg.model_type
        self.gen = 1 if mt == "gemma" else (2 if mt == "gemma2" else 3)
        self.sandwich = self.gen >= 2
        qpas = hf.get("query_pre_attn_scalar") or cfg.head_dim
        self.scale = float(qpas) ** -0.5
        self.attn_softcap = float(hf.get("attn_logit_softcapping") or 0.0)
        self.final_softcap = float(hf.get("final_logit_softcapping") or 0.0)
        self.act = 1  # gelu_pytorch_tanh (GeGLU)
        L = cfg.num_layers
        sw = hf.get("sliding_window") or cfg.sliding_window
        types = hf.get("layer_types")
        if not types:
            if self.gen == 2:
                types = ["sliding_attention" if i % 2 == 0 else "full_attention" for i in range(L)]
            elif self.gen == 3:
                pat = hf.get("sliding_window_pattern", 6)
                types = ["full_attention" if (i + 1) % pat == 0 else "sliding_attention" for i in range(L)]
            else:
                types = ["full_attention"] * L
        self.windows = [int(sw) if (sw and types[i] == "sliding_attention") else -1 for i in range(L)]
        self.post_attn: list[torch.Tensor | None] = [None] * L
        self.post_ff: list[torch.Tensor | None] = [None] * L
        mp = max_positions or cfg.max_position_embeddings
        self.cos_sin_local = self.cos_sin
        rp = hf.get("rope_parameters") or {}
        local_theta = (rp.get("sliding_attention") or {}).get("rope_theta") or hf.get("rope_local_base_freq")
        if self.gen == 3 and local_theta:
            lc = ModelConfig(**{**cfg.__dict__, "rope_theta": float(local_theta), "rope_scaling": None})
            self.cos_sin_local = rope_cos_sin(lc, mp, device=self.device)
        self.normalizer = torch.tensor(cfg.hidden_size ** 0.5, dtype=dtype).item()
        self.is_cls = cfg.architecture.endswith("ForSequenceClassification")
        self.num_labels = int(hf.get("num_labels") or len(hf.get("id2label") or {}) or 1)
        self.score: torch.Tensor | None = None   # [num_labels, H] sequence-classification head

    # ------------------------------------------------------------------ weights
    def init_random(self, seed: int = 0, std: float = 0.02) -> "GemmaForCausalLM":
        super().init_random(seed, std)
        H = self.cfg.hidden_size
        for i in self.layers:
            if self.sandwich:
                self.post_attn[i] = self._alloc(H, std=None, gen=None)
                self.post_ff[i] = self._alloc(H, std=None, gen=None)
            if self.gen == 3 and self.qn[i] is None:
                self.qn[i] = self._alloc(self.D, std=None, gen=None)
                self.kn[i] = self._alloc(self.D, std=None, gen=None)
        if self.is_cls:
            g = torch.Generator(device="cpu").manual_seed(seed + 7)
            self.score = (torch.randn(self.num_labels, self.cfg.hidden_size, generator=g) * std).to(
                device=self.device, dtype=self.dtype)
        return self

    def load_hf_weights(self, weights) -> "GemmaForCausalLM":
        def renamed():
            for name, w in weights:
                for pre in ("model.language_model.", "language_model.model.", "language_model."):
                    if name.startswith(pre):
                        name = "model." + name[len(pre):]
                        break
                if name.startswith(("vision_tower.", "multi_modal_projector.", "model.vision_tower.",
                                    "model.multi_modal_projector.")):
                    continue  # image encoder: not served (text-only Gemma 3)
                if self.sandwich:
                    if name.endswith(".post_attention_layernorm.weight"):
                        name = name.replace(".post_attention_layernorm.", ".gemma_post_attn.")
                    elif name.endswith(".pre_feedforward_layernorm.weight"):
                        name = name.replace(".pre_feedforward_layernorm.", ".post_attention_layernorm.")
                    elif name.endswith(".post_feedforward_layernorm.weight"):
                        name = name.replace(".post_feedforward_layernorm.", ".gemma_post_ff.")
                yield name, w

        extra: dict[tuple[int, str], torch.Tensor] = {}

        def capture():
            for name, w in renamed():
                n = name[len("model."):] if name.startswith("model.") else name
                parts = n.split(".")
                if parts[0] == "layers" and len(parts) >= 4 and parts[2] in ("gemma_post_attn", "gemma_post_ff"):
                    extra[(int(parts[1]), parts[2])] = w
                    continue
                if name == "score.weight":
                    self.score = w.to(device=self.device, dtype=self.dtype).contiguous()
                    continue
                yield name, w

        super().load_hf_weights(capture())
        for (i, kind), w in extra.items():
            if i not in self._layer_set:
                continue
            t = w.to(device=self.device, dtype=self.dtype).contiguous()
            (self.post_attn if kind == "gemma_post_attn" else self.post_ff)[i] = t
        # RMSNorm (1 + w): fold the 1 into every norm weight (in fp32, then the model dtype)
        one = lambda t: None if t is None else (t.float() + 1.0).to(self.dtype)  # noqa: E731
        for lst in (self.ln1, self.ln2, self.post_attn, self.post_ff, self.qn, self.kn):
            for i in self.layers:
                lst[i] = one(lst[i])
        self.norm = one(self.norm)
        return self

    # ------------------------------------------------------------------ forward
    def _stage_input(self, ids: torch.Tensor, input_embeds: torch.Tensor | None):
        st = pstate.get()
        T, H = ids.shape[0], self.cfg.hidden_size
        if st.pp_size > 1 and not st.is_first_pp:
            return pstate.pp_recv(((T, H), self.dtype, ids.device), ((T, H), self.dtype, ids.device))
        if input_embeds is None:
            h = pstate.tp_all_reduce(ops.embedding(ids, self.embed, self.tp.vocab_start, self.tp.vocab_end))
            h = h * self.normalizer
        else:
            h = input_embeds
        return ops.rmsnorm(h, self.ln1[self.layers[0]], self.eps), h

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
            cs = self.cos_sin_local if self.windows[i] > 0 else self.cos_sin
            ops.rope_qkv_cache(qkv, meta.positions, cs, cfg.rot_dim, q, k_cache, v_cache, meta.slots,
                               tp.hq, tp.hkv, D, True, self.qn[i], self.kn[i], self.eps, ks, vs)
            attn = self._attention(i, q, k_cache, v_cache, meta, ks, vs)
            o = pstate.tp_all_reduce(linear(attn.view(T, tp.hq * D), self.w_o[i]))
            if self.sandwich:
                o = ops.rmsnorm(o, self.post_attn[i], self.eps)
            ops.fused_add_rmsnorm(o, residual, self.ln2[i], self.eps)
            x = self.mlp(i, o)
            if self.sandwich:
                x = ops.rmsnorm(x, self.post_ff[i], self.eps)
        return self._stage_output(x, residual)

    def _attention(self, i: int, q, k_cache, v_cache, meta: AttnMeta, ks: float, vs: float) -> torch.Tensor:
        w, cap = self.windows[i], self.attn_softcap
        if meta.is_decode:
            return ops.paged_decode(q, k_cache, v_cache, meta.block_tables, meta.seq_lens, self.scale, meta.decode_ws,
                                    w, order=meta.order, k_scale=ks, v_scale=vs, softcap=cap)
        hi = meta.extra.get("row_hi") if meta.extra else None  # Gemma 3 bidirectional image blocks
        if meta.mode == "mixed":
            n = meta.num_prefill
            out = torch.empty_like(q)
            ops.paged_prefill(q[:n], k_cache, v_cache, meta.block_tables, meta.cu_q, meta.kv_lens, meta.items,
                              self.scale, w, out=out[:n], k_scale=ks, v_scale=vs, softcap=cap,
                              row_hi=None if hi is None else hi[:n])
            ops.paged_decode(q[n:], k_cache, v_cache, meta.dec_block_tables, meta.seq_lens, self.scale,
                             meta.decode_ws, w, out=out[n:], order=meta.order, k_scale=ks, v_scale=vs, softcap=cap)
            return out
        return ops.paged_prefill(q, k_cache, v_cache, meta.block_tables, meta.cu_q, meta.kv_lens, meta.items,
                                 self.scale, w, k_scale=ks, v_scale=vs, softcap=cap, row_hi=hi)

    def pool(self, hidden: torch.Tensor, cu: torch.Tensor) -> torch.Tensor:
        """Per sequence (rows ``cu[s]:cu[s+1]``): the classification head's raw scores of the last
        token (``Gemma2ForSequenceClassification``), else last-token pooling + L2 norm."""
        if self.score is None:
            return ops.pool(hidden, cu, 0, True)
        last = hidden.index_select(0, (cu[1:] - 1).long())
        return linear(last, self.score).float()

    def compute_logits(self, hidden: torch.Tensor) -> torch.Tensor:
        logits = super().compute_logits(hidden)
        if self.final_softcap > 0:
            c = self.final_softcap
            logits = (torch.tanh(logits.float() / c) * c).to(logits.dtype)
        return logits

    def weight_bytes(self) -> int:
        n = super().weight_bytes()
        if self.score is not None:
            n += self.score.numel() * self.score.element_size()
        for lst in (self.post_attn, self.post_ff):
            n += sum(t.numel() * t.element_size() for t in lst if t is not None)
        return n
