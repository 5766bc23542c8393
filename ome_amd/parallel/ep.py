"""Expert-parallel MoE with all-to-all token dispatch / combine (SURVEY.md §2.9 K17, §2.8 C4;
the reference's runtimes use DeepEP ``--moe-a2a-backend deepep`` for this).

Under DP attention every rank holds different tokens and 1/EP of the experts.  Per MoE layer:

  route locally -> sort the T*k (token, expert) assignments by owning rank ->
  all-to-all-v #1: counts, then the token rows and their local expert ids ->
  owner runs its experts as a k=1 grouped MoE (``ome_moe_*`` kernels) ->
  all-to-all-v #2: expert outputs travel back in the same order ->
  combine in the original (token, slot) order with the routing weights (fp32).

On one MI355X node the all-to-alls are RCCL over the xGMI mesh (every pair of GPUs has a direct
link, so an all-to-all is N-1 independent point-to-point transfers); on CPU they run on gloo.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ome_amd import ops
from ome_amd.parallel import state as pstate


def _a2a(out: torch.Tensor, inp: torch.Tensor, out_splits: list[int], in_splits: list[int], group) -> None:
    if inp.is_cuda or dist.get_backend(group) != "gloo":
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=group)
        return
    # gloo has no all_to_all: N-1 pairwise exchanges (CPU tests only)
    st = pstate.get()
    ws, me = dist.get_world_size(group), dist.get_rank(group)
    ioff = [0]
    for s in in_splits:
        ioff.append(ioff[-1] + s)
    ooff = [0]
    for s in out_splits:
        ooff.append(ooff[-1] + s)
    out[ooff[me]:ooff[me + 1]].copy_(inp[ioff[me]:ioff[me + 1]])
    for step in range(1, ws):
        dst, src = (me + step) % ws, (me - step) % ws
        reqs = []
        if in_splits[dst]:
            reqs.append(dist.isend(inp[ioff[dst]:ioff[dst + 1]].contiguous(), dst, group=group))
        buf = None
        if out_splits[src]:
            buf = torch.empty_like(out[ooff[src]:ooff[src + 1]])
            reqs.append(dist.irecv(buf, src, group=group))
        for r in reqs:
            r.wait()
        if buf is not None:
            out[ooff[src]:ooff[src + 1]].copy_(buf)
    del st


def moe_ep_forward(x: torch.Tensor, topk_w: torch.Tensor, topk_ids: torch.Tensor, w13_local: torch.Tensor,
                   w2_local: torch.Tensor, act: int, scale: float, num_experts: int,
                   tables: tuple[torch.Tensor, torch.Tensor, torch.Tensor] | None = None,
                   b13_local: torch.Tensor | None = None, b2_local: torch.Tensor | None = None) -> torch.Tensor:
    """x [T, H] (this rank's tokens), routing [T, k] over the global (logical) experts; w13/w2
    hold this rank's expert slots.  Without ``tables`` rank r owns experts [r*E/ep, (r+1)*E/ep);
    with EPLB tables (``ome_amd.parallel.eplb``: rep_rank / rep_slot [E, Rmax], n_rep [E]) each
    (token, k-slot) assignment goes to replica ``(t*k + j) mod n_rep[e]`` of its expert, which
    spreads a replicated hot expert's rows evenly over its copies.  ``b13_local`` / ``b2_local``:
    per-expert biases of the owner's slots (GPT-OSS).  Returns [T, H]."""
    st = pstate.get()
    group, ep, me = st.ep_group, st.ep_size, st.ep_rank
    T, H = x.shape
    k = topk_ids.shape[1]
    flat_ids = topk_ids.reshape(-1).long()
    if tables is None:
        e_local = num_experts // ep
        owner = flat_ids // e_local
        local_slot = flat_ids - owner * e_local
    else:
        rep_rank, rep_slot, n_rep = tables
        j = torch.arange(flat_ids.shape[0], device=flat_ids.device) % n_rep.index_select(0, flat_ids)
        owner = rep_rank[flat_ids, j]
        local_slot = rep_slot[flat_ids, j]
    order = torch.argsort(owner, stable=True)
    send_counts = torch.bincount(owner, minlength=ep)
    recv_counts = torch.empty_like(send_counts)
    _a2a(recv_counts, send_counts, [1] * ep, [1] * ep, group)
    sc, rc = send_counts.tolist(), recv_counts.tolist()
    tok = order // k
    send_x = x.index_select(0, tok)
    send_e = local_slot.index_select(0, order).to(torch.int32)
    R = sum(rc)
    recv_x = x.new_empty(R, H)
    recv_e = torch.empty(R, dtype=torch.int32, device=x.device)
    _a2a(recv_x, send_x, rc, sc, group)
    _a2a(recv_e, send_e, rc, sc, group)
    if R:
        ones = torch.ones(R, 1, dtype=torch.float32, device=x.device)
        y = ops.fused_moe(recv_x, ones, recv_e.view(R, 1), w13_local, w2_local, act, 1.0, b13_local, b2_local)
    else:
        y = x.new_empty(0, H)
    back = x.new_empty(T * k, H)
    _a2a(back, y, sc, rc, group)
    unsorted = torch.empty_like(back)
    unsorted.index_copy_(0, order, back)
    out = (unsorted.view(T, k, H).float() * topk_w.float().view(T, k, 1)).sum(1) * scale
    return out.to(x.dtype)


def _a2a_async(out, inp, out_splits, in_splits, group):
    """Issue an all-to-all-v; returns a waitable (RCCL: runs on the communicator's stream, so
    the compute stream keeps going until ``wait()``).  gloo (CPU tests) completes inline."""
    if inp.is_cuda or dist.get_backend(group) != "gloo":
        return dist.all_to_all_single(out, inp, out_splits, in_splits, group=group, async_op=True)
    _a2a(out, inp, out_splits, in_splits, group)
    return None


def moe_ep_forward_tbo(x: torch.Tensor, topk_w: torch.Tensor, topk_ids: torch.Tensor, w13_local: torch.Tensor,
                       w2_local: torch.Tensor, act: int, scale: float, num_experts: int,
                       tables: tuple[torch.Tensor, torch.Tensor, torch.Tensor] | None = None,
                       b13_local: torch.Tensor | None = None, b2_local: torch.Tensor | None = None) -> torch.Tensor:
    """Two-batch overlap of the expert-parallel MoE block (SGLang ``--enable-two-batch-overlap``,
    reference deepseek-rdma-pd-rt.yaml:89): the token rows are split into two micro-batches;
    their dispatches are issued back to back, then micro-batch A's experts run while B's
    dispatch is still on the wire, and B's experts run while A's combine is on the wire:

        comm stream   | dispatch A | dispatch B | combine A | combine B |
        compute       |            | experts A  | experts B |   sum     |

    Every rank always runs exactly two micro-batches (an empty half still takes part in the
    collectives), so the collective sequence is identical across ranks.  Math is identical to
    :func:`moe_ep_forward` (each row's experts and weights are unchanged; the combine is in
    fp32 in (token, slot) order)."""
    st = pstate.get()
    group, ep = st.ep_group, st.ep_size
    T, H = x.shape
    k = topk_ids.shape[1]
    flat_ids = topk_ids.reshape(-1).long()
    if tables is None:
        e_local = num_experts // ep
        owner = flat_ids // e_local
        local_slot = flat_ids - owner * e_local
    else:
        rep_rank, rep_slot, n_rep = tables
        j = torch.arange(flat_ids.shape[0], device=flat_ids.device) % n_rep.index_select(0, flat_ids)
        owner = rep_rank[flat_ids, j]
        local_slot = rep_slot[flat_ids, j]
    half = (T + 1) // 2
    bounds = [(0, half * k), (half * k, T * k)]  # assignment ranges of micro-batches A and B
    mbs = []
    counts = []
    for a0, a1 in bounds:
        own = owner[a0:a1]
        order = torch.argsort(own, stable=True) + a0
        counts.append(torch.bincount(own, minlength=ep))
        mbs.append({"order": order})
    send_counts = torch.stack(counts, 1).reshape(-1)  # [ep, 2]: one exchange for both halves
    recv_counts = torch.empty_like(send_counts)
    _a2a(recv_counts, send_counts, [2] * ep, [2] * ep, group)
    sc, rc = send_counts.view(ep, 2).tolist(), recv_counts.view(ep, 2).tolist()
    for m, mb in enumerate(mbs):
        mb["sc"] = [r[m] for r in sc]
        mb["rc"] = [r[m] for r in rc]
        order = mb["order"]
        send_x = x.index_select(0, order // k)
        send_e = local_slot.index_select(0, order).to(torch.int32)
        R = sum(mb["rc"])
        mb["rx"] = x.new_empty(R, H)
        mb["re"] = torch.empty(R, dtype=torch.int32, device=x.device)
        mb["keep"] = (send_x, send_e)  # alive until the transfer completes
        mb["h"] = [_a2a_async(mb["rx"], send_x, mb["rc"], mb["sc"], group),
                   _a2a_async(mb["re"], send_e, mb["rc"], mb["sc"], group)]
    for mb in mbs:
        for h in mb["h"]:
            if h is not None:
                h.wait()
        R = mb["rx"].shape[0]
        if R:
            ones = torch.ones(R, 1, dtype=torch.float32, device=x.device)
            y = ops.fused_moe(mb["rx"], ones, mb["re"].view(R, 1), w13_local, w2_local, act, 1.0, b13_local,
                              b2_local)
        else:
            y = x.new_empty(0, H)
        mb["y"] = y
        mb["back"] = x.new_empty(sum(mb["sc"]), H)
        mb["hc"] = _a2a_async(mb["back"], y, mb["sc"], mb["rc"], group)
    unsorted = x.new_empty(T * k, H)
    for mb in mbs:
        if mb["hc"] is not None:
            mb["hc"].wait()
        unsorted.index_copy_(0, mb["order"], mb["back"])
    out = (unsorted.view(T, k, H).float() * topk_w.float().view(T, k, 1)).sum(1) * scale
    return out.to(x.dtype)


def moe_ep(x: torch.Tensor, topk_w: torch.Tensor, topk_ids: torch.Tensor, w13_local, w2_local, act: int,
           scale: float, num_experts: int, tables=None, b13_local=None, b2_local=None) -> torch.Tensor:
    """Expert-parallel MoE block: the device-only low-latency exchange
    (:mod:`ome_amd.parallel.ep_ll`) when this lockstep step allows it (``state.ep_ll_ok``: every
    rank's batch fits the fixed buckets; set per step by the engine, so all ranks pick the same
    mode), the RCCL all-to-all (normal / two-batch-overlap) otherwise.  EPLB replica tables are
    honoured by both.  Expert biases (GPT-OSS) take the RCCL path (the low-latency exchange is
    not attached for such models)."""
    st = pstate.get()
    ll = getattr(st, "ep_ll_cur", None) or getattr(st, "ep_ll", None)
    if ll is not None and x.is_cuda and st.ep_ll_ok and b13_local is None and b2_local is None:
        e_local = w13_local.shape[0]   # expert slots per rank (redundant replicas included)
        return ll.forward(x, topk_w, topk_ids, w13_local, w2_local, act, scale, e_local, tables)
    fwd = moe_ep_forward_tbo if st.tbo else moe_ep_forward
    return fwd(x, topk_w, topk_ids, w13_local, w2_local, act, scale, num_experts, tables, b13_local, b2_local)


def attach_low_latency(model, max_tokens: int) -> bool:
    """Create the low-latency EP exchange for an MoE model under DP attention on GPU (one node):
    buckets of ``max_tokens`` x top-k rows per peer.  Collective over the EP group (every rank
    calls it at model build).  Returns True when installed."""
    import os

    st = pstate.get()
    if st.ep_size <= 1 or not torch.cuda.is_available() or os.environ.get("OME_EP_LL", "1") == "0":
        return False
    k = getattr(model, "k", 0)
    if not k or getattr(model, "E", 0) % st.ep_size or getattr(model, "expert_biases", False):
        return False
    from ome_amd.parallel.ep_ll import LowLatencyEP

    st.ep_ll = LowLatencyEP(st.ep_group, model.cfg.hidden_size, max_tokens, k, cpu_group=st.cpu_group)
    if st.tbo:   # two-batch overlap: micro-batch B exchanges through its own buffers and epochs
        st.ep_ll_b = LowLatencyEP(st.ep_group, model.cfg.hidden_size, max_tokens, k, cpu_group=st.cpu_group)
    st.ep_ll_cap = max_tokens
    st.ep_ll_ok = True
    return True


def ep_idle_layers(model, ll) -> None:
    """This rank's part of one forward's worth of exchanges on ``ll`` with NO local tokens: every
    MoE layer in order dispatches nothing and computes the experts for the rows its peers send.
    Two-batch overlap: a rank whose step is not a split decode (prefill / mixed) still runs
    micro-batch B's exchanges, so every exchange keeps all participants."""
    H = model.cfg.hidden_size
    dev = model.device
    x = torch.empty(0, H, dtype=model.dtype, device=dev)
    k = model.k
    tw = torch.empty(0, k, dtype=torch.float32, device=dev)
    tid = torch.empty(0, k, dtype=torch.int32, device=dev)
    for i in model.layers:
        if i not in model.moe_layers:
            continue
        tables = model.eplb.tables[i] if getattr(model, "eplb", None) is not None else None
        w13 = model.w13[i]
        ll.forward(x, tw, tid, w13, model.w2[i], model.act, getattr(model, "routed_scale", 1.0), w13.shape[0],
                   tables)
