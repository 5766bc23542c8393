"""Sparse MoE decoders (Mixtral, Qwen2-MoE, Qwen3-MoE, PhiMoE) on the ome_amd kernels.

Attention is the dense-family path (``llama.py``); the MLP becomes:
  router GEMM (hipBLASLt) -> ``ome_moe_route`` (softmax top-k, renorm) ->
  ``ome_moe_align`` (device counting sort) -> grouped MFMA GEMM gate_up (A rows gathered) ->
  SiLU*mul -> grouped MFMA GEMM down -> ``ome_moe_combine`` (+ shared expert, Qwen2-MoE) ->
  TP all-reduce.
Experts are tensor-parallel over the intermediate dimension (every rank holds a 1/tp slice of
every expert), so the collective pattern matches the dense family; expert parallelism with
all-to-all dispatch is the alternative for very large expert counts.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from ome_amd import ops
from ome_amd.models.llama import LlamaForCausalLM
from ome_amd.parallel import state as pstate


class MoEForCausalLM(LlamaForCausalLM):
    def __init__(self, cfg, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        tp = self.tp
        st = pstate.get()
        self.E = cfg.num_experts
        # expert parallelism (DP attention): this rank owns experts [e0, e0 + E_local)
        self.ep = st.ep_size
        if self.E % self.ep:
            raise ValueError(f"{self.E} experts do not split over ep={self.ep}")
        self.E_local = self.E // self.ep
        self.e0 = st.ep_rank * self.E_local
        self.tune_gemms = False  # TunableOp pre-capture tuning is validated on the dense family only
        self.k = cfg.num_experts_per_tok
        self.renorm = cfg.norm_topk_prob
        self.moe_inter = -(-cfg.moe_intermediate_size // tp.tp)
        self.shared_inter = -(-(cfg.shared_expert_intermediate_size or 0) // tp.tp)
        L = cfg.num_layers
        self.w_router: list[torch.Tensor] = [None] * L
        self.w13: list[torch.Tensor] = [None] * L     # [E, 2*I_local, H]
        self.w2: list[torch.Tensor] = [None] * L      # [E, H, I_local]
        self.w_sgu: list[torch.Tensor | None] = [None] * L   # shared expert gate_up
        self.w_sd: list[torch.Tensor | None] = [None] * L    # shared expert down
        self.w_sgate: list[torch.Tensor | None] = [None] * L  # shared expert sigmoid gate [1, H]
        step = max(1, cfg.moe_layer_freq)
        self.moe_layers = {i for i in self.layers if i >= cfg.first_k_dense_replace and (i + 1) % step == 0} \
            if step > 1 else {i for i in self.layers if i >= cfg.first_k_dense_replace}
        from ome_amd.parallel import eplb

        eplb.attach(self)  # expert slots per rank (+ redundant replicas) under expert parallelism

    def init_random(self, seed: int = 0, std: float = 0.02) -> "MoEForCausalLM":
        super().init_random(seed, std)
        cfg = self.cfg
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 104729 + 7919 * pstate.get().tp_rank)
        H, I = cfg.hidden_size, self.moe_inter
        for i in self.layers:
            if i not in self.moe_layers:
                continue
            self.w_gu[i] = self.w_d[i] = None  # dense MLP replaced by experts
            self.w_router[i] = self._alloc(self.E, H, std=std, gen=gen)
            idx = torch.tensor(self.local_experts(i), dtype=torch.long, device=self.device)
            self.w13[i] = self._alloc(self.E, 2 * I, H, std=std, gen=gen).index_select(0, idx).contiguous()
            self.w2[i] = self._alloc(self.E, H, I, std=std / math.sqrt(2 * cfg.num_layers),
                                     gen=gen).index_select(0, idx).contiguous()
            if self.shared_inter:
                self.w_sgu[i] = self._alloc(2 * self.shared_inter, H, std=std, gen=gen)
                self.w_sd[i] = self._alloc(H, self.shared_inter, std=std / math.sqrt(2 * cfg.num_layers), gen=gen)
                self.w_sgate[i] = self._alloc(1, H, std=std, gen=gen)
        self._quantize_experts()
        return self

    def load_hf_weights(self, weights) -> "MoEForCausalLM":
        tp = self.tp
        I, SI = self.moe_inter, self.shared_inter
        experts: dict[int, dict[int, dict[str, torch.Tensor]]] = {}
        fused: dict[int, dict[str, torch.Tensor]] = {}
        shared: dict[int, dict[str, torch.Tensor]] = {}
        rest_iter = []
        if self.fp8:
            from ome_amd.models.quant import dequant_fp8_stream

            weights = dequant_fp8_stream(weights, self.fp8_block, self.dtype)

        def put(t):
            return t.to(device=self.device, dtype=self.dtype).contiguous()

        def rows(t, n):
            return t.narrow(0, tp.rank * n, min(n, t.shape[0] - tp.rank * n))

        def cols(t, n):
            return t.narrow(1, tp.rank * n, min(n, t.shape[1] - tp.rank * n))

        for name, w in weights:
            n = name[len("model."):] if name.startswith("model.") else name
            parts = n.split(".")
            if parts[0] == "layers" and len(parts) > 3 and parts[2] in ("block_sparse_moe", "mlp") and \
                    int(parts[1]) in self.moe_layers:
                i = int(parts[1])
                sub = ".".join(parts[3:])
                if sub == "gate.weight":
                    self.w_router[i] = put(w)
                elif sub in ("experts.gate_up_proj", "experts.down_proj"):   # fused per layer (Qwen3-VL-MoE)
                    fused.setdefault(i, {})[parts[4]] = w
                elif sub.startswith("experts."):
                    e = int(parts[4])
                    kind = parts[5]  # w1/w2/w3 (Mixtral) or gate_proj/up_proj/down_proj
                    experts.setdefault(i, {}).setdefault(e, {})[kind] = w
                elif sub.startswith("shared_expert."):
                    shared.setdefault(i, {})[parts[4]] = w
                elif sub == "shared_expert_gate.weight":
                    self.w_sgate[i] = put(w)
                continue
            rest_iter.append((name, w))
        # dense / attention / embeddings through the base loader (it tolerates missing MLPs below)
        self._load_base(rest_iter)
        for i, ex in experts.items():
            gs, ds = [], []
            for e in self.local_experts(i):
                d = ex[e]
                g = d.get("w1", d.get("gate_proj"))
                u = d.get("w3", d.get("up_proj"))
                dn = d.get("w2", d.get("down_proj"))
                if g is None or u is None or dn is None:
                    raise ValueError(f"layer {i} expert {e}: missing weights")
                gs.append(torch.cat([rows(g, I), rows(u, I)], 0))
                ds.append(cols(dn, I))
            self.w13[i] = put(torch.stack(gs))
            self.w2[i] = put(torch.stack(ds))
            self.w_gu[i] = self.w_d[i] = None
        H = self.cfg.hidden_size
        for i, d in fused.items():   # gate_up [E, H, 2I] (or [E, 2I, H]), down [E, I, H] (or [E, H, I])
            gu, dn = d["gate_up_proj"], d["down_proj"]
            if gu.shape[1] == H and gu.shape[2] != H:
                gu = gu.transpose(1, 2)
            if dn.shape[2] == H and dn.shape[1] != H:
                dn = dn.transpose(1, 2)
            sel = torch.tensor(self.local_experts(i), dtype=torch.long, device=gu.device)
            gu, dn = gu.index_select(0, sel), dn.index_select(0, sel)
            g, u = gu.chunk(2, 1)
            self.w13[i] = put(torch.cat([g.narrow(1, tp.rank * I, min(I, g.shape[1] - tp.rank * I)),
                                         u.narrow(1, tp.rank * I, min(I, u.shape[1] - tp.rank * I))], 1))
            self.w2[i] = put(dn.narrow(2, tp.rank * I, min(I, dn.shape[2] - tp.rank * I)))
            self.w_gu[i] = self.w_d[i] = None
        for i, d in shared.items():
            self.w_sgu[i] = put(torch.cat([rows(d["gate_proj"], SI), rows(d["up_proj"], SI)], 0))
            self.w_sd[i] = put(cols(d["down_proj"], SI))
        self._quantize_experts()
        return self

    def _load_base(self, weights) -> None:
        # the base loader validates dense MLP weights; present them as satisfied for MoE layers
        saved = [self.w_gu[i] for i in self.layers]
        placeholder = torch.empty(0, device=self.device)
        for i in self.moe_layers:
            self.w_gu[i] = placeholder
        super().load_hf_weights(iter(weights))
        for i in self.moe_layers:
            if self.w_gu[i] is placeholder:
                self.w_gu[i] = saved[i]

    def _quantize_experts(self) -> None:
        """``quantization: fp8``: routed experts are stored as fp8 with 128x128 block scales and
        run on the block-scaled grouped GEMM (no dequantisation to bf16 at load)."""
        if self.fp8:
            from ome_amd.models.quant import quantize_moe_experts

            quantize_moe_experts(self)

    def local_experts(self, i: int) -> list[int]:
        from ome_amd.parallel import eplb

        return eplb.local_experts(self, i)

    def weight_bytes(self) -> int:
        n = super().weight_bytes()
        for lst in (self.w_router, self.w13, self.w2, self.w_sgu, self.w_sd, self.w_sgate):
            n += sum(t.nbytes() if hasattr(t, "scale") else t.numel() * t.element_size() for t in lst if t is not None)
        return n

    def router_logits(self, i: int, x: torch.Tensor) -> torch.Tensor:
        return F.linear(x, self.w_router[i])

    def mlp(self, i: int, x: torch.Tensor) -> torch.Tensor:
        if i not in self.moe_layers:
            return super().mlp(i, x)
        return pstate.tp_all_reduce(self._moe_partial(i, x))

    def _moe_partial(self, i: int, x: torch.Tensor) -> torch.Tensor:
        """Routed experts (+ shared expert): this rank's partial sums, before the TP all-reduce."""
        tw, tid = ops.moe_route(self.router_logits(i, x), self.k, self.renorm)
        if self.ep > 1:
            from ome_amd.parallel.ep import moe_ep

            tables = None
            if self.eplb is not None:
                self.eplb.record(i, tid)
                tables = self.eplb.tables[i]
            out = moe_ep(x, tw, tid, self.w13[i], self.w2[i], self.act, 1.0, self.E, tables)
        else:
            out = ops.fused_moe(x, tw, tid, self.w13[i], self.w2[i], self.act)
        if self.w_sgu[i] is not None:
            sh = F.linear(ops.act_and_mul(F.linear(x, self.w_sgu[i]), self.act), self.w_sd[i])
            if self.w_sgate[i] is not None:
                sh = sh * torch.sigmoid(F.linear(x, self.w_sgate[i]))
            out = out + sh
        return out
