"""Sparse-MoE variants of the spec-driven decoder (``models/decoder.py``): OLMoE, Granite-MoE,
DBRX, ERNIE-4.5-MoE and MiniMax-M2 from the reference runtime catalog
(``config/runtimes/srt/allenai/olmoe-1b-7b-0924-rt.yaml``, ``ibm-granite/granite-3-0-3b-a800m-instruct-rt.yaml``,
``databricks/dbrx-instruct-rt.yaml``, ``baidu/ernie-4-5-21b-a3b-pt-rt.yaml``, ``minimax/minimax-m2-rt.yaml``).

Attention, norms and residual forms come from the family's :class:`DecoderSpec`; the MLP of the
MoE layers runs on the same kernels as the Mixtral / Qwen-MoE path (``models/moe.py``):
``ome_moe_route`` (softmax or sigmoid scores, optional e_score_correction_bias used for the
selection only, optional renormalisation -- this one kernel covers all five routers) ->
``ome_moe_align`` -> grouped MFMA GEMM gate_up -> SiLU*mul -> grouped MFMA GEMM down ->
``ome_moe_combine``, plus an optional always-on shared expert (ERNIE).  Experts are tensor-parallel
over the intermediate dimension, so the block output is one partial sum and the decoder's
single TP all-reduce per block still applies; under DP attention they are expert-parallel
instead (rank r owns experts [r*E/ep, (r+1)*E/ep), tokens by all-to-all, ``parallel/ep.py``).

Checkpoint expert layouts accepted: per expert (``experts.<e>.{gate,up,down}_proj`` / ``w1,w3,w2``),
fused per layer (``experts.gate_up_proj`` [E, 2I, H] + ``experts.down_proj`` [E, H, I]),
Granite-MoE ``input_linear`` / ``output_linear`` and DBRX ``w1`` / ``v1`` / ``w2`` ([E*I, H]).
"""
from __future__ import annotations

import math

import torch

from ome_amd import ops
from ome_amd.models.config import ModelConfig
from ome_amd.models.decoder import DecoderForCausalLM
from ome_amd.models.quant import linear
from ome_amd.parallel import state as pstate

_L = r"(?:model\.)?layers\.(\d+)\."


def _moe_names(arch: str) -> list:
    if arch == "OlmoeForCausalLM":
        return [(_L + r"mlp\.gate\.weight", r"L.\1.router.weight"),
                (_L + r"mlp\.experts\.(\d+)\.(gate|up|down)_proj\.weight", r"L.\1.experts.\2.\3"),
                (_L + r"mlp\.experts\.(gate_up|down)_proj", r"L.\1.experts.\2")]
    if arch == "GraniteMoeForCausalLM":
        return [(_L + r"block_sparse_moe\.router\.layer\.weight", r"L.\1.router.weight"),
                (_L + r"block_sparse_moe\.input_linear\.weight", r"L.\1.experts.gate_up"),
                (_L + r"block_sparse_moe\.output_linear\.weight", r"L.\1.experts.down")]
    if arch == "DbrxForCausalLM":
        return [(r"blocks\.(\d+)\.ffn\.router\.layer\.weight", r"L.\1.router.weight"),
                (r"blocks\.(\d+)\.ffn\.experts\.mlp\.(w1|v1|w2)", r"L.\1.experts.dbrx_\2")]
    if arch == "Ernie4_5_MoeForCausalLM":
        return [(_L + r"mlp\.gate\.weight", r"L.\1.router.weight"),
                (_L + r"mlp\.moe_statics\.e_score_correction_bias", r"L.\1.router.bias"),
                (_L + r"mlp\.experts\.(\d+)\.(gate|up|down)_proj\.weight", r"L.\1.experts.\2.\3"),
                (_L + r"mlp\.experts\.(gate_up|down)_proj", r"L.\1.experts.\2"),
                (_L + r"mlp\.shared_experts\.(gate|up|down)_proj\.weight", r"L.\1.shared.\2")]
    if arch == "MiniMaxM2ForCausalLM":
        return [(_L + r"block_sparse_moe\.gate\.weight", r"L.\1.router.weight"),
                (_L + r"block_sparse_moe\.e_score_correction_bias", r"L.\1.router.bias"),
                (_L + r"block_sparse_moe\.experts\.(\d+)\.w(1|2|3)\.weight", r"L.\1.experts.\2.w\3"),
                (_L + r"block_sparse_moe\.experts\.(gate_up|down)_proj", r"L.\1.experts.\2")]
    raise NotImplementedError(arch)


DECODER_MOE_ARCHS = {"OlmoeForCausalLM", "GraniteMoeForCausalLM", "DbrxForCausalLM", "Ernie4_5_MoeForCausalLM",
                     "MiniMaxM2ForCausalLM"}


class DecoderMoEForCausalLM(DecoderForCausalLM):
    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16, max_positions: int | None = None):
        super().__init__(cfg, device, dtype, max_positions)
        st, tp, hf, arch = pstate.get(), self.tp, cfg.extra or {}, cfg.architecture
        self.ep = st.ep_size
        if cfg.num_experts % self.ep:
            raise ValueError(f"{cfg.num_experts} experts do not split over ep={self.ep}")
        self.E_local = cfg.num_experts // self.ep
        self.e0 = st.ep_rank * self.E_local if self.ep > 1 else 0
        self.spec.names = list(self.spec.names) + _moe_names(arch)
        self.E, self.k = cfg.num_experts, cfg.num_experts_per_tok
        self.scoring = "sigmoid" if arch == "MiniMaxM2ForCausalLM" else "softmax"
        self.renorm = True if arch in ("GraniteMoeForCausalLM", "Ernie4_5_MoeForCausalLM", "MiniMaxM2ForCausalLM") \
            else cfg.norm_topk_prob
        self.moe_inter = -(-cfg.moe_intermediate_size // tp.tp)
        n_sh = int(hf.get("moe_num_shared_experts") or 0)
        self.shared_inter = -(-(n_sh * cfg.moe_intermediate_size) // tp.tp) if n_sh else 0
        L = cfg.num_layers
        if arch == "Ernie4_5_MoeForCausalLM":
            lo, hi, step = hf.get("moe_layer_start_index", 1), hf.get("moe_layer_end_index", L - 1), \
                hf.get("moe_layer_interval", 1)
            hi = L - 1 if hi in (None, -1) else hi
            self.moe_layers = {i for i in self.layers if (i + 1) % step == 0 and lo <= i <= hi}
        else:
            self.moe_layers = set(self.layers)
        self.w_router: list[torch.Tensor | None] = [None] * L
        self.b_router: list[torch.Tensor | None] = [None] * L   # e_score_correction_bias (selection only)
        self.w13: list[torch.Tensor | None] = [None] * L        # [E, 2*I_local, H]
        self.w2: list[torch.Tensor | None] = [None] * L         # [E, H, I_local]
        self.w_sgu: list[torch.Tensor | None] = [None] * L
        self.w_sd: list[torch.Tensor | None] = [None] * L

    # ------------------------------------------------------------------ weights
    def init_random(self, seed: int = 0, std: float = 0.02) -> "DecoderMoEForCausalLM":
        super().init_random(seed, std)
        gen = torch.Generator(device=self.device)
        gen.manual_seed(seed + 104729 + 7919 * pstate.get().tp_rank)
        H, I, E = self.cfg.hidden_size, self.moe_inter, self.E_local
        for i in self.moe_layers:
            self.w_router[i] = self._alloc(self.E, H, std=std, gen=gen)
            self.w13[i] = self._alloc(E, 2 * I, H, std=std, gen=gen)
            self.w2[i] = self._alloc(E, H, I, std=std / math.sqrt(2 * self.cfg.num_layers), gen=gen)
            if self.scoring == "sigmoid" or self.cfg.architecture == "Ernie4_5_MoeForCausalLM":
                self.b_router[i] = torch.zeros(self.E, dtype=torch.float32, device=self.device)
            if self.shared_inter:
                self.w_sgu[i] = self._alloc(2 * self.shared_inter, H, std=std, gen=gen)
                self.w_sd[i] = self._alloc(H, self.shared_inter, std=std / math.sqrt(2 * self.cfg.num_layers), gen=gen)
        return self

    def _load_mlp(self, i: int, p: dict, put) -> None:
        if i not in self.moe_layers:
            return super()._load_mlp(i, p, put)
        tp, E, I, H = self.tp, self.E, self.moe_inter, self.cfg.hidden_size
        ex = slice(self.e0, self.e0 + self.E_local)   # this rank's experts under EP (all otherwise)
        full = self.cfg.moe_intermediate_size
        self.w_router[i] = put(p["router.weight"])
        if "router.bias" in p:
            self.b_router[i] = p["router.bias"].reshape(-1).to(device=self.device, dtype=torch.float32).contiguous()

        def rows(t, n):  # this rank's slice of an intermediate dim stored in rows
            return t.narrow(0, tp.rank * n, min(n, t.shape[0] - tp.rank * n))

        if "experts.gate_up" in p:  # fused per layer: [E, 2I, H] gate rows then up rows, [E, H, I]
            g, u = p["experts.gate_up"].chunk(2, 1)
            dn = p["experts.down"]
            w13 = torch.cat([g[ex, tp.rank * I:(tp.rank + 1) * I], u[ex, tp.rank * I:(tp.rank + 1) * I]], 1)
            w2 = dn[ex, :, tp.rank * I:(tp.rank + 1) * I]
        elif "experts.dbrx_w1" in p:  # DBRX: w1 (gate) / v1 (up) / w2 (down, transposed) as [E*I, H]
            g = p["experts.dbrx_w1"].reshape(E, full, H)
            u = p["experts.dbrx_v1"].reshape(E, full, H)
            d = p["experts.dbrx_w2"].reshape(E, full, H)
            sl = slice(tp.rank * I, (tp.rank + 1) * I)
            w13 = torch.cat([g[ex, sl], u[ex, sl]], 1)
            w2 = d[ex, sl].transpose(1, 2)
        else:  # per expert
            gs, ds = [], []
            for e in range(ex.start, ex.stop):
                gw = p.get(f"experts.{e}.gate", p.get(f"experts.{e}.w1"))
                uw = p.get(f"experts.{e}.up", p.get(f"experts.{e}.w3"))
                dw = p.get(f"experts.{e}.down", p.get(f"experts.{e}.w2"))
                if gw is None or uw is None or dw is None:
                    raise ValueError(f"layer {i} expert {e}: missing weights")
                gs.append(torch.cat([rows(gw, I), rows(uw, I)], 0))
                ds.append(dw.narrow(1, tp.rank * I, min(I, dw.shape[1] - tp.rank * I)))
            w13, w2 = torch.stack(gs), torch.stack(ds)
        self.w13[i], self.w2[i] = put(w13), put(w2)
        if "shared.gate" in p:
            SI = self.shared_inter
            self.w_sgu[i] = put(torch.cat([rows(p["shared.gate"], SI), rows(p["shared.up"], SI)], 0))
            sd = p["shared.down"]
            self.w_sd[i] = put(sd.narrow(1, tp.rank * SI, min(SI, sd.shape[1] - tp.rank * SI)))

    def weight_bytes(self) -> int:
        n = super().weight_bytes()
        for lst in (self.w_router, self.b_router, self.w13, self.w2, self.w_sgu, self.w_sd):
            n += sum(t.numel() * t.element_size() for t in lst if t is not None)
        return n

    # ------------------------------------------------------------------ forward
    def _mlp(self, i: int, x: torch.Tensor) -> torch.Tensor:
        if i not in self.moe_layers:
            return super()._mlp(i, x)
        logits = linear(x, self.w_router[i])
        tw, tid = ops.moe_route(logits, self.k, self.renorm, self.scoring, bias=self.b_router[i],
                                group_mode=2 if self.b_router[i] is not None else 0)
        if self.ep > 1:
            from ome_amd.parallel.ep import moe_ep

            out = moe_ep(x, tw, tid, self.w13[i], self.w2[i], self.act, 1.0, self.E)
            if self.w_sgu[i] is not None:
                out = out + linear(ops.act_and_mul(linear(x, self.w_sgu[i]), self.act), self.w_sd[i])
            return out
        sh = None
        if self.w_sgu[i] is not None:   # the routed sum lands on the shared expert's output in the combine
            sh = linear(ops.act_and_mul(linear(x, self.w_sgu[i]), self.act), self.w_sd[i]).contiguous()
        return ops.fused_moe(x, tw, tid, self.w13[i], self.w2[i], self.act, add=sh)
