"""GPT-OSS (``GptOssForCausalLM``; reference catalog ``config/runtimes/srt/openai/gpt-oss-*-rt.yaml``)
on the ome_amd kernels.

What differs from the Llama / MoE paths, and where it runs:

* attention sinks: a learned per-head logit that joins every softmax as an extra column with no
  value -- added to the softmax denominator inside the MFMA decode / prefill attention kernels
  (``sinks`` argument; also in the split-K reduce);
* alternating sliding-window (128) / full layers (``layer_types``), head_dim 64, q/k/v/o biases
  (the o bias lives on TP rank 0 only, so the all-reduce adds it once);
* YaRN RoPE (factor 32, ``truncate: false``) in the NeoX layout the fused RoPE kernel uses;
* MoE: router with bias, top-k then softmax over the selected logits (identical to softmax +
  renormalise, i.e. ``ome_moe_route``), experts with per-expert biases in both grouped MFMA
  GEMMs and the clamped SwiGLU ``(clamp(u, +-7) + 1) * g * sigmoid(1.702 g)``, g = min(g, 7)
  (``act_and_mul`` ACT 2).  HF stores gate/up interleaved in the last dim of ``gate_up_proj``
  [E, H, 2I]; they are de-interleaved into the kernels' [E, 2I, H] (gate rows, then up rows)
  at load time;
* MXFP4 expert checkpoints (``*_blocks`` / ``*_scales``, e2m1 pairs + e8m0 exponents) are
  dequantised to bf16 while streaming (``dequant_mxfp4``, checked against transformers'
  ``convert_moe_packed_tensors``).
Experts are tensor-parallel over the intermediate dimension (like ``moe.py`` TP mode), or, under
DP attention, expert-parallel: rank r owns experts [r*E/ep, (r+1)*E/ep) with their biases and the
tokens travel by all-to-all (``parallel/ep.py``, RCCL path: the expert biases keep the
low-latency exchange off).
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

FP4_VALUES = (0.0, 0.5, 1.0, 1.5, 2.0, 3.0, 4.0, 6.0, -0.0, -0.5, -1.0, -1.5, -2.0, -3.0, -4.0, -6.0)


def dequant_mxfp4(blocks: torch.Tensor, scales: torch.Tensor, dtype=torch.float32) -> torch.Tensor:
    """MXFP4 -> dense, in the checkpoint's [E, out, in] order: ``blocks`` [E, out, in/32, 16] uint8
    (two e2m1 codes per byte, low nibble first), ``scales`` [E, out, in/32] uint8 (e8m0, bias 127)."""
    lut = torch.tensor(FP4_VALUES, dtype=torch.float32, device=blocks.device)
    b = blocks.to(torch.uint8)
    lo, hi = lut[(b & 0x0F).long()], lut[(b >> 4).long()]
    vals = torch.stack([lo, hi], -1).reshape(*b.shape[:-1], b.shape[-1] * 2)  # [..., G, 32]
    vals = torch.ldexp(vals, (scales.to(torch.int32) - 127)[..., None].to(torch.float32))
    return vals.reshape(*b.shape[:-2], -1).to(dtype)


class GptOssForCausalLM(LlamaForCausalLM):
    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        hf = cfg.extra or {}
        st = pstate.get()
        self.E, self.k = cfg.num_experts, cfg.num_experts_per_tok
        self.ep = st.ep_size
        if self.E % self.ep:
            raise ValueError(f"{self.E} experts do not split over ep={self.ep}")
        self.E_local = self.E // self.ep            # expert slots on this rank (all of them without EP)
        self.e0 = st.ep_rank * self.E_local if self.ep > 1 else 0
        self.expert_biases = True
        self.I = -(-cfg.moe_intermediate_size // self.tp.tp)
        self.act = 2
        L = cfg.num_layers
        sw = hf.get("sliding_window") or 128
        types = hf.get("layer_types") or ["sliding_attention" if i % 2 == 0 else "full_attention" for i in range(L)]
        self.windows = [int(sw) if types[i] == "sliding_attention" else -1 for i in range(L)]
        self.sinks: list[torch.Tensor | None] = [None] * L
        self.b_o: list[torch.Tensor | None] = [None] * L
        self.w_router: list[torch.Tensor | None] = [None] * L
        self.b_router: list[torch.Tensor | None] = [None] * L
        self.w13: list[torch.Tensor | None] = [None] * L
        self.b13: list[torch.Tensor | None] = [None] * L
        self.w2: list[torch.Tensor | None] = [None] * L
        self.b2: list[torch.Tensor | None] = [None] * L
        self.tune_gemms = False

    # ------------------------------------------------------------------ weights
    def init_random(self, seed: int = 0, std: float = 0.02) -> "GptOssForCausalLM":
        super().init_random(seed, std)
        cfg, tp = self.cfg, self.tp
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 31337 + 7919 * tp.rank)
        H, I, E = cfg.hidden_size, self.I, self.E_local
        bias_here = tp.rank == 0 or self.ep > 1     # TP: added once by rank 0; EP: by each owner
        for i in self.layers:
            self.w_gu[i] = self.w_d[i] = None
            self.sinks[i] = torch.randn(tp.hq, generator=gen, device=self.device, dtype=torch.float32)
            self.b_o[i] = self._alloc(H, std=std, gen=gen) if tp.rank == 0 else None
            self.w_router[i] = self._alloc(self.E, H, std=std, gen=gen)
            self.b_router[i] = self._alloc(self.E, std=std, gen=gen)
            self.w13[i] = self._alloc(E, 2 * I, H, std=std, gen=gen)
            self.b13[i] = self._alloc(E, 2 * I, std=std, gen=gen)
            self.w2[i] = self._alloc(E, H, I, std=std / math.sqrt(2 * cfg.num_layers), gen=gen)
            self.b2[i] = self._alloc(E, H, std=std, gen=gen) if bias_here else torch.zeros(
                E, H, dtype=self.dtype, device=self.device)
            if self.b_qkv[i] is None:
                self.b_qkv[i] = self._alloc((tp.hq + 2 * tp.hkv) * self.D, std=std, gen=gen)
        return self

    def load_hf_weights(self, weights) -> "GptOssForCausalLM":
        tp, I, D = self.tp, self.I, self.D
        pending: dict[tuple[int, str], dict[str, torch.Tensor]] = {}
        mlp: dict[int, dict[str, torch.Tensor]] = {}

        def put(t, dtype=None):
            return t.to(device=self.device, dtype=dtype or self.dtype).contiguous()

        def rest():
            for name, w in weights:
                n = name[len("model."):] if name.startswith("model.") else name
                parts = n.split(".")
                if parts[0] == "layers" and len(parts) >= 4:
                    i = int(parts[1])
                    sub = ".".join(parts[2:])
                    if i not in self._layer_set:
                        continue
                    if sub == "self_attn.sinks":
                        self.sinks[i] = put(w.narrow(0, tp.rank * tp.hq, tp.hq), torch.float32)
                        continue
                    if sub == "self_attn.o_proj.bias":
                        self.b_o[i] = put(w) if tp.rank == 0 else None
                        continue
                    if sub.startswith("mlp."):
                        key = sub[len("mlp."):]
                        for suf in ("_blocks", "_scales"):
                            if key.endswith(suf):
                                pending.setdefault((i, key[: -len(suf)]), {})[suf] = w
                                break
                        else:
                            mlp.setdefault(i, {})[key] = w
                        continue
                yield name, w

        # the base loader handles embeddings, norms and q/k/v(+bias)/o; MLP weights are ours
        placeholder = torch.empty(0, device=self.device)
        for i in self.layers:
            self.w_gu[i] = placeholder
        super().load_hf_weights(rest())
        for (i, key), d in pending.items():  # MXFP4 experts -> dense [E, in, out] (the bf16 param layout)
            mlp.setdefault(i, {})[key] = dequant_mxfp4(d["_blocks"], d["_scales"]).transpose(1, 2)
        ex = slice(self.e0, self.e0 + self.E_local)         # this rank's experts (EP), all otherwise
        for i, d in mlp.items():
            gu = d["experts.gate_up_proj"][ex].float()        # [E, H, 2I] gate/up interleaved
            gb = d["experts.gate_up_proj_bias"][ex].float()   # [E, 2I]
            g, u = gu[..., 0::2], gu[..., 1::2]               # [E, H, I_full]
            sl = slice(tp.rank * I, tp.rank * I + I)
            self.w13[i] = put(torch.cat([g[..., sl], u[..., sl]], -1).transpose(1, 2))    # [E, 2I, H]
            self.b13[i] = put(torch.cat([gb[:, 0::2][:, sl], gb[:, 1::2][:, sl]], -1))
            dn = d["experts.down_proj"][ex].float()           # [E, I_full, H]
            self.w2[i] = put(dn[:, sl, :].transpose(1, 2))    # [E, H, I]
            b2 = d["experts.down_proj_bias"][ex]
            self.b2[i] = put(b2) if tp.rank == 0 or self.ep > 1 else torch.zeros_like(put(b2))
            self.w_router[i] = put(d["router.weight"])
            self.b_router[i] = put(d["router.bias"])
            self.w_gu[i] = self.w_d[i] = None
        missing = [i for i in self.layers if self.w13[i] is None or self.sinks[i] is None]
        if missing:
            raise ValueError(f"GPT-OSS checkpoint incomplete: layers {missing[:4]}")
        return self

    def weight_bytes(self) -> int:
        n = super().weight_bytes()
        for lst in (self.w13, self.b13, self.w2, self.b2, self.w_router, self.b_router, self.b_o, self.sinks):
            n += sum(t.numel() * t.element_size() for t in lst if t is not None)
        return n

    # ------------------------------------------------------------------ forward
    def forward(self, ids: torch.Tensor, meta: AttnMeta, kv: PagedKVCache,
                input_embeds: torch.Tensor | None = None) -> torch.Tensor:
        cfg, tp, D = self.cfg, self.tp, self.D
        T = ids.shape[0]
        x, residual = self._stage_input(ids, input_embeds)
        first = self.layers[0]
        for i in self.layers:
            if i > first:
                ops.fused_add_rmsnorm(x, residual, self.ln1[i], self.eps)
            qkv = linear(x, self.w_qkv[i], self.b_qkv[i])
            q = torch.empty(T, tp.hq, D, dtype=self.dtype, device=x.device)
            k_cache, v_cache = kv.layer(i)
            ks, vs = kv.scales(i)
            ops.rope_qkv_cache(qkv, meta.positions, self.cos_sin, cfg.rot_dim, q, k_cache, v_cache, meta.slots,
                               tp.hq, tp.hkv, D, True, None, None, self.eps, ks, vs)
            attn = self._attention(i, q, k_cache, v_cache, meta, ks, vs)
            o = pstate.tp_all_reduce(linear(attn.view(T, tp.hq * D), self.w_o[i], self.b_o[i]))
            ops.fused_add_rmsnorm(o, residual, self.ln2[i], self.eps)
            x = self.mlp(i, o)
        return self._stage_output(x, residual)

    def _attention(self, i: int, q, k_cache, v_cache, meta: AttnMeta, ks: float, vs: float) -> torch.Tensor:
        w, sk = self.windows[i], self.sinks[i]
        if meta.is_decode:
            return ops.paged_decode(q, k_cache, v_cache, meta.block_tables, meta.seq_lens, self.scale, meta.decode_ws,
                                    w, order=meta.order, k_scale=ks, v_scale=vs, sinks=sk)
        if meta.mode == "mixed":
            n = meta.num_prefill
            out = torch.empty_like(q)
            ops.paged_prefill(q[:n], k_cache, v_cache, meta.block_tables, meta.cu_q, meta.kv_lens, meta.items,
                              self.scale, w, out=out[:n], k_scale=ks, v_scale=vs, sinks=sk)
            ops.paged_decode(q[n:], k_cache, v_cache, meta.dec_block_tables, meta.seq_lens, self.scale,
                             meta.decode_ws, w, out=out[n:], order=meta.order, k_scale=ks, v_scale=vs, sinks=sk)
            return out
        return ops.paged_prefill(q, k_cache, v_cache, meta.block_tables, meta.cu_q, meta.kv_lens, meta.items,
                                 self.scale, w, k_scale=ks, v_scale=vs, sinks=sk)

    def mlp(self, i: int, x: torch.Tensor) -> torch.Tensor:
        logits = F.linear(x, self.w_router[i], self.b_router[i])
        tw, tid = ops.moe_route(logits, self.k, True)
        if self.ep > 1:
            from ome_amd.parallel.ep import moe_ep

            out = moe_ep(x, tw, tid, self.w13[i], self.w2[i], self.act, 1.0, self.E, None, self.b13[i], self.b2[i])
        else:
            out = ops.fused_moe(x, tw, tid, self.w13[i], self.w2[i], self.act, 1.0, self.b13[i], self.b2[i])
        return pstate.tp_all_reduce(out)
