"""Expert-parallel load balancing with redundant experts (EPLB; SURVEY.md §2.7 EP row: the
reference's DeepSeek runtimes pass ``--enable-eplb --eplb-algorithm deepseek
--ep-num-redundant-experts $(PARALLELISM_SIZE)``, config/runtimes/srt/deepseek-rdma-pd-rt.yaml:
83-126).

Physical layout: every EP rank holds ``slots = (E + R) / ep`` expert slots; a placement maps each
slot to a logical expert, so hot experts can live on several ranks (R redundant replicas in
total).  Token dispatch picks a replica per (token, k-slot) assignment by round-robin over the
replicas of its expert, which splits a hot expert's rows evenly across its copies.

Rebalancing (per MoE layer, from the per-expert token counts recorded since the last round):
  1. replicate: hand out the R extra slots one at a time to the expert with the highest
     load-per-replica (greedy water-filling);
  2. pack: place the E + R weighted replicas onto ep ranks with exactly ``slots`` each, heaviest
     first onto the currently lightest rank that has a free slot and does not already hold that
     expert (LPT bin-packing with capacity).
The DeepSeek algorithm adds a node level (expert groups to nodes first); on one 8x MI355X node
every rank pair is one xGMI hop, so the flat packing is the whole problem.
Weights then migrate with one all-to-all-v per tensor: each new slot is filled from a rank that
held that expert before (itself when possible).  All ranks compute the same placement from the
all-reduced load, so no placement is ever communicated.
"""
from __future__ import annotations

import heapq
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class ExpertPlacement:
    num_experts: int
    ep: int
    slots: int
    phys_to_log: list[list[int]]  # [ep][slots] -> logical expert id

    @classmethod
    def default(cls, num_experts: int, ep: int, redundant: int = 0) -> "ExpertPlacement":
        """Contiguous blocks of logical experts per rank (R = 0 reproduces ``e // (E/ep)``);
        the R extra slots replicate experts 0, 1, ... on the ranks that do not own them."""
        if (num_experts + redundant) % ep:
            raise ValueError(f"experts {num_experts} + redundant {redundant} must split over ep={ep}")
        if num_experts % ep:
            raise ValueError(f"{num_experts} experts do not split over ep={ep}")
        slots = (num_experts + redundant) // ep
        per = num_experts // ep
        p2l = [list(range(r * per, (r + 1) * per)) for r in range(ep)]
        extra = redundant // ep
        nxt = 0
        for r in range(ep):
            for _ in range(extra):
                while nxt // per == r:  # an expert the rank does not already own
                    nxt = (nxt + 1) % num_experts
                p2l[r].append(nxt)
                nxt = (nxt + 1) % num_experts
        return cls(num_experts, ep, slots, p2l)

    def replicas(self) -> dict[int, list[tuple[int, int]]]:
        out: dict[int, list[tuple[int, int]]] = {e: [] for e in range(self.num_experts)}
        for r, row in enumerate(self.phys_to_log):
            for s, e in enumerate(row):
                out[e].append((r, s))
        return out

    def tables(self, device, rmax: int | None = None) -> tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """(rep_rank [E, Rmax], rep_slot [E, Rmax], n_rep [E]) int64 dispatch tables (``rmax``:
        a fixed replica width, so re-placements can be copied into the same tensors)."""
        reps = self.replicas()
        rmax = max(rmax or 0, max(len(v) for v in reps.values()))
        rank = torch.zeros(self.num_experts, rmax, dtype=torch.int64)
        slot = torch.zeros(self.num_experts, rmax, dtype=torch.int64)
        n = torch.zeros(self.num_experts, dtype=torch.int64)
        for e, lst in reps.items():
            if not lst:
                raise ValueError(f"expert {e} has no replica")
            n[e] = len(lst)
            for j, (r, s) in enumerate(lst):
                rank[e, j], slot[e, j] = r, s
        return rank.to(device), slot.to(device), n.to(device)

    def imbalance(self, load: list[float]) -> float:
        """max rank load / mean rank load under round-robin replica splitting (1.0 = perfect)."""
        reps = self.replicas()
        per_rank = [0.0] * self.ep
        for e, lst in reps.items():
            for r, _ in lst:
                per_rank[r] += load[e] / len(lst)
        mean = sum(per_rank) / self.ep
        return max(per_rank) / mean if mean > 0 else 1.0


def balance(load: list[float], ep: int, slots: int) -> ExpertPlacement:
    """Replicate + pack (module docstring).  Deterministic for a given load vector."""
    E = len(load)
    R = ep * slots - E
    if R < 0:
        raise ValueError("fewer slots than experts")
    nrep = [1] * E
    # 1. water-filling: give each extra slot to the expert with the largest load per replica
    heap = [(-load[e], e) for e in range(E)]
    heapq.heapify(heap)
    for _ in range(R):
        _, e = heapq.heappop(heap)
        nrep[e] += 1
        heapq.heappush(heap, (-load[e] / nrep[e], e))
    # 2. LPT packing with capacity, never two copies of one expert on one rank when avoidable
    items = sorted(((load[e] / nrep[e], e) for e in range(E) for _ in range(nrep[e])), key=lambda t: (-t[0], t[1]))
    rank_load = [0.0] * ep
    rows: list[list[int]] = [[] for _ in range(ep)]
    for w, e in items:
        cands = [r for r in range(ep) if len(rows[r]) < slots and e not in rows[r]]
        if not cands:
            cands = [r for r in range(ep) if len(rows[r]) < slots]
        r = min(cands, key=lambda r: (rank_load[r], r))
        rows[r].append(e)
        rank_load[r] += w
    return ExpertPlacement(E, ep, slots, rows)


def migrate(old: ExpertPlacement, new: ExpertPlacement, w_local: torch.Tensor, rank: int, group,
            a2a=None) -> torch.Tensor:
    """Re-lay this rank's expert weights ``w_local`` [slots, ...] from ``old`` to ``new``: a slot
    whose expert this rank already holds is copied locally, every other slot arrives from the
    lowest-numbered rank that held the expert (one all-to-all-v)."""
    if a2a is None:
        from ome_amd.parallel.ep import _a2a as a2a
    ep = old.ep
    old_reps = old.replicas()
    # (dest rank, dest slot) -> (src rank, src slot), identical on every rank
    plan: dict[tuple[int, int], tuple[int, int]] = {}
    for r, row in enumerate(new.phys_to_log):
        for s, e in enumerate(row):
            mine = [x for x in old_reps[e] if x[0] == r]
            plan[(r, s)] = mine[0] if mine else min(old_reps[e])
    out = torch.empty_like(w_local)
    row_shape = w_local.shape[1:]
    flat = w_local.reshape(w_local.shape[0], -1)
    send_rows = {d: [] for d in range(ep)}
    recv_slots = {src: [] for src in range(ep)}
    for (d, s), (src, ss) in sorted(plan.items()):
        if src == rank and d == rank:
            out[s].copy_(w_local[ss])
        elif src == rank:
            send_rows[d].append(ss)
        elif d == rank:
            recv_slots[src].append(s)
    in_splits = [0 if d == rank else len(send_rows[d]) for d in range(ep)]
    out_splits = [0 if s == rank else len(recv_slots[s]) for s in range(ep)]
    send_idx = [i for d in range(ep) if d != rank for i in send_rows[d]]
    send = flat.index_select(0, torch.tensor(send_idx, dtype=torch.long, device=w_local.device)) if send_idx \
        else flat.new_empty(0, flat.shape[1])
    recv = flat.new_empty(sum(out_splits), flat.shape[1])
    a2a(recv, send, out_splits, in_splits, group)
    o = 0
    for src in range(ep):
        if src == rank:
            continue
        for s in recv_slots[src]:
            out[s].copy_(recv[o].view(row_shape))
            o += 1
    return out


class EPLBState:
    """Per-model EPLB bookkeeping: placement + dispatch tables + token counts per MoE layer."""

    def __init__(self, layers, num_experts: int, ep: int, rank: int, redundant: int, device):
        self.ep, self.rank, self.device = ep, rank, device
        self.placement = {i: ExpertPlacement.default(num_experts, ep, redundant) for i in layers}
        # fixed width (an expert never has more than 1 + redundant replicas): tables are updated in
        # place after a re-placement, so HIP graphs that captured them stay valid
        self.rmax = 1 + max(0, int(redundant))
        self.tables = {i: p.tables(device, self.rmax) for i, p in self.placement.items()}
        self.load = {i: torch.zeros(num_experts, dtype=torch.float64, device=device) for i in layers}
        self.rounds = 0

    @property
    def slots(self) -> int:
        return next(iter(self.placement.values())).slots

    def local_experts(self, layer: int) -> list[int]:
        return self.placement[layer].phys_to_log[self.rank]

    def record(self, layer: int, topk_ids: torch.Tensor) -> None:
        ids = topk_ids.reshape(-1).long()
        self.load[layer].index_add_(0, ids, torch.ones_like(ids, dtype=torch.float64))

    def rebalance(self, weights: dict[int, list[torch.Tensor]], group) -> dict[int, float]:
        """All-reduce the recorded loads, re-place every layer, migrate its weight tensors in
        place (``weights[layer]`` = the per-slot tensors, e.g. [w13, w2]).  Returns the per-layer
        imbalance after the move."""
        out = {}
        for i in sorted(self.placement):
            load = self.load[i].clone()
            if group is not None:
                dist.all_reduce(load, group=group)
            lv = load.cpu().tolist()
            old = self.placement[i]
            new = balance(lv, self.ep, old.slots)
            if new.phys_to_log != old.phys_to_log:
                ws = weights[i]
                for j, w in enumerate(ws):
                    moved = migrate(old, new, w, self.rank, group)
                    if moved.shape == w.shape:
                        w.copy_(moved)   # in place: captured graphs keep reading this tensor
                    else:
                        ws[j] = moved
                self.placement[i] = new
                for dst, src in zip(self.tables[i], new.tables(self.device, self.rmax)):
                    dst.copy_(src)
            out[i] = new.imbalance(lv)
            self.load[i].zero_()
        self.rounds += 1
        return out


def attach(model) -> None:
    """Give an MoE model (``E``, ``ep``, ``moe_layers`` set) its EPLB state: ``model.eplb`` (None
    without expert parallelism), ``E_local`` = slots per rank, ``local_experts(i)``.
    ``cfg.extra['ep_num_redundant_experts']`` (``--ep-num-redundant-experts``) sizes the slots."""
    from ome_amd.parallel import state as pstate

    st = pstate.get()
    red = int((model.cfg.extra or {}).get("ep_num_redundant_experts", 0) or 0)
    if model.ep <= 1 or not model.E:
        model.eplb = None
        if red:
            raise ValueError("--ep-num-redundant-experts needs expert parallelism (--enable-dp-attention --dp N)")
        return
    model.eplb = EPLBState(sorted(model.moe_layers), model.E, model.ep, st.ep_rank, red, model.device)
    model.E_local = model.eplb.slots


def local_experts(model, layer: int) -> list[int]:
    if getattr(model, "eplb", None) is not None:
        return model.eplb.local_experts(layer)
    return list(range(model.e0, model.e0 + model.E_local))


def rebalance_model(model) -> dict[int, float]:
    """Engine hook (DP-attention lockstep): re-place experts of every MoE layer from the loads
    recorded since the last call and migrate ``w13`` / ``w2``."""
    from ome_amd.parallel import state as pstate

    if getattr(model, "eplb", None) is None:
        return {}
    from ome_amd.models.quant import Fp8Experts

    def parts(w):   # fp8 experts migrate their codes and block scales slot by slot
        return [w.q, w.scale] if isinstance(w, Fp8Experts) else [w]

    ws = {i: parts(model.w13[i]) + parts(model.w2[i]) for i in model.eplb.placement}
    res = model.eplb.rebalance(ws, pstate.get().ep_group)
    for i, lst in ws.items():
        if isinstance(model.w13[i], Fp8Experts):
            model.w13[i] = Fp8Experts(lst[0], lst[1], model.w13[i].block)
            model.w2[i] = Fp8Experts(lst[2], lst[3], model.w2[i].block)
        else:
            model.w13[i], model.w2[i] = lst
    return res
