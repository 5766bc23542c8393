"""Process-group state for the runtime: one process per GPU, ``torch.distributed`` over RCCL.

Parallel layout of an engine "group" of ``world = tp * pp`` ranks:
  rank = pp_rank * tp + tp_rank.
Rendezvous follows the reference's multi-pod contract (``--dist-init-addr
$(LWS_LEADER_ADDRESS):5757 --nnodes $(LWS_GROUP_SIZE) --node-rank $(LWS_WORKER_INDEX)``,
``config/runtimes/srt/deepseek-rdma-pd-rt.yaml:105-110``): a TCP store at the leader.
On a single 8xMI355X node every pair of GPUs has a direct xGMI link, so the TP all-reduce
goes through :mod:`ome_amd.parallel.comm` (one-shot P2P for small decode messages, RCCL
otherwise).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.distributed as dist


@dataclass
class ParallelState:
    tp_size: int = 1
    tp_rank: int = 0
    pp_size: int = 1
    pp_rank: int = 0
    dp_size: int = 1
    dp_rank: int = 0
    ep_size: int = 1
    ep_rank: int = 0
    world_size: int = 1
    rank: int = 0
    tp_group: object | None = None
    pp_group: object | None = None
    ep_group: object | None = None
    backend: str = "nccl"
    comm: object | None = None  # ome_amd.parallel.comm.TPCommunicator
    tbo: bool = False           # two-batch overlap of the EP MoE all-to-alls (parallel/ep.py)
    cpu_group: object | None = None  # gloo group of this engine group (control-plane broadcasts)
    tp_cpu_group: object | None = None  # gloo group of this rank's TP group (host-side exchanges)
    global_rank: int = 0        # rank in the whole job (several engine replicas per job)
    replica: int = 0
    replicas: int = 1
    base: int = 0               # global rank of this group's rank 0
    ep_ll: object | None = None # ome_amd.parallel.ep_ll.LowLatencyEP (DP attention on one node)
    ep_ll_ok: bool = False      # this lockstep step may use it (every rank's batch fits the buckets)
    ep_ll_cap: int = 0          # tokens per rank the low-latency buckets hold
    ep_ll_b: object | None = None   # two-batch overlap: micro-batch B's own exchange (buffers + epochs)
    ep_ll_cur: object | None = None  # the exchange the MoE layers use right now (None: ep_ll)
    pp_prev: object | None = None   # CustomAllReduce over (previous stage, this stage): IPC hand-off
    pp_next: object | None = None   # CustomAllReduce over (this stage, next stage)
    pp_bcast: object | None = None  # CustomAllReduce over the pipeline group: sampled tokens from the last stage

    def to_global(self, r: int) -> int:
        return self.base + r

    @property
    def is_first_pp(self) -> bool:
        return self.pp_rank == 0

    @property
    def is_last_pp(self) -> bool:
        return self.pp_rank == self.pp_size - 1


_STATE = ParallelState()


def get() -> ParallelState:
    return _STATE


def init(tp_size: int = 1, pp_size: int = 1, ep_size: int | None = None, dist_init_addr: str | None = None,
         rank: int | None = None, world_size: int | None = None, backend: str | None = None,
         local_rank: int | None = None, dp_size: int = 1) -> ParallelState:
    """Initialise torch.distributed (if world > 1) and build TP / PP / EP groups.

    ``dp_size > 1`` is DP attention (SGLang ``--tp N --dp N --enable-dp-attention``): every rank
    runs attention and dense layers for its OWN requests with full weights (attention TP = 1),
    while MoE experts are partitioned over all N ranks (EP = N) and tokens travel to their
    experts by all-to-all (:mod:`ome_amd.parallel.ep`).

    A world larger than one engine group (``tp * pp * dp`` ranks) holds several independent
    engine REPLICAS (e.g. ``bench.py --gpus 8 --tp 2``: four TP=2 engines): ranks
    ``[r * g, (r + 1) * g)`` form replica ``r``; ``rank`` / ``world_size`` of the returned state
    are the group-local ones, ``global_rank`` / ``replica`` locate the process in the job."""
    global _STATE
    if dp_size > 1:
        if tp_size not in (1, dp_size) or pp_size != 1:
            raise ValueError("DP attention needs tp_size == dp_size and pp_size == 1")
        tp_size = 1
    gsize = tp_size * pp_size * dp_size
    world = world_size if world_size is not None else int(os.environ.get("WORLD_SIZE", gsize))
    grk = rank if rank is not None else int(os.environ.get("RANK", 0))
    if world % gsize:
        raise ValueError(f"world_size {world} is not a multiple of tp {tp_size} * pp {pp_size} * dp {dp_size}")
    replicas = world // gsize
    base = (grk // gsize) * gsize
    rk = grk - base
    if backend is None:
        # OME_DIST_BACKEND=gloo: several ranks sharing one GPU (tests on a 1-GPU box; RCCL refuses
        # two ranks on one device) -- the TP collectives then run on the xGMI/IPC peer kernels
        backend = os.environ.get("OME_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    st = ParallelState(tp_size=tp_size, pp_size=pp_size, world_size=gsize, rank=rk, backend=backend)
    st.global_rank, st.replica, st.replicas, st.base = grk, grk // gsize, replicas, base
    st.dp_size, st.dp_rank = dp_size, (rk if dp_size > 1 else 0)
    st.tp_rank, st.pp_rank = rk % tp_size, (rk // tp_size) % pp_size
    st.ep_size = dp_size if dp_size > 1 else 1
    st.ep_rank = st.dp_rank
    if world > 1:
        if not dist.is_initialized():
            init_method = f"tcp://{dist_init_addr}" if dist_init_addr else None
            kw = {}
            if torch.cuda.is_available():
                lr = local_rank if local_rank is not None else int(os.environ.get("LOCAL_RANK", grk % max(1, torch.cuda.device_count())))
                lr = lr if lr < torch.cuda.device_count() else 0
                torch.cuda.set_device(lr)
                if backend == "nccl":
                    kw["device_id"] = torch.device("cuda", lr)
            dist.init_process_group(backend=backend, init_method=init_method, rank=grk, world_size=world, **kw)
        tp_cpu = None
        pp_groups: dict = {}
        # new_group is collective over the whole job: every rank creates every replica's groups
        for rep in range(replicas):
            b = rep * gsize
            mine = rep == st.replica
            grp = list(range(b, b + gsize))
            cg = dist.new_group(grp, backend="gloo") if gsize > 1 else None
            eg = (dist.group.WORLD if replicas == 1 else dist.new_group(grp)) if dp_size > 1 else None
            if mine:
                st.cpu_group, st.ep_group = cg, eg
            for p in range(pp_size):
                ranks = [b + r for r in range(p * tp_size, (p + 1) * tp_size)]
                g = dist.new_group(ranks) if tp_size > 1 else None
                gc = dist.new_group(ranks, backend="gloo") if tp_size > 1 else None
                if mine and p == st.pp_rank:
                    st.tp_group, tp_cpu = g, gc
            pp_cpu = {}
            for t in range(tp_size):
                ranks = [b + p * tp_size + t for p in range(pp_size)]
                g = dist.new_group(ranks) if pp_size > 1 else None
                if mine and t == st.tp_rank:
                    st.pp_group = g
                if pp_size > 1 and torch.cuda.is_available():   # gloo groups for the IPC hand-off handles
                    pp_cpu[(t, "all")] = dist.new_group(ranks, backend="gloo")
                    for p in range(pp_size - 1):
                        pp_cpu[(t, p)] = dist.new_group(ranks[p:p + 2], backend="gloo")
            if mine:
                pp_groups = pp_cpu
        single_node = int(os.environ.get("LOCAL_WORLD_SIZE", world)) >= world
        if torch.cuda.is_available() and pp_size > 1 and single_node and pp_size in (2, 4, 8) and \
                os.environ.get("OME_PP_IPC", "1") != "0" and os.environ.get("OME_CUSTOM_AR", "1") != "0":
            _pp_ipc_init(st, pp_groups)
        if torch.cuda.is_available() and tp_size in (2, 4, 8) and single_node and \
                os.environ.get("OME_CUSTOM_AR", "1") != "0":
            from ome_amd.parallel.comm import TPCommunicator

            st.comm = TPCommunicator(st.tp_group, cpu_group=tp_cpu)
        st.tp_cpu_group = tp_cpu
    _STATE = st
    return st


def set_state(st: ParallelState) -> None:
    global _STATE
    _STATE = st


def tp_all_reduce(x: torch.Tensor) -> torch.Tensor:
    st = _STATE
    if st.tp_size == 1:
        return x
    if st.comm is not None and x.is_cuda:
        return st.comm.all_reduce(x)
    dist.all_reduce(x, group=st.tp_group)
    return x


def tp_ar_staging(shape, dtype: torch.dtype, device) -> torch.Tensor | None:
    """A buffer a row-parallel projection can write its partial sums into so that the following
    :func:`tp_all_reduce` needs no staging copy (None: allocate normally)."""
    st = _STATE
    if st.tp_size == 1 or st.comm is None or not torch.device(device).type == "cuda":
        return None
    return st.comm.staging(shape, dtype, device)


def tp_all_reduce_add_rmsnorm(x: torch.Tensor, residual: torch.Tensor, weight: torch.Tensor,
                              eps: float) -> torch.Tensor | None:
    """``residual += allreduce(x); return rmsnorm(residual) * weight`` fused into the all-reduce
    kernel.  None when not applicable (the caller then all-reduces and norms separately)."""
    st = _STATE
    if st.tp_size == 1 or st.comm is None or not x.is_cuda:
        return None
    return st.comm.all_reduce_add_rmsnorm(x, residual, weight, eps)


def tp_all_gather(x: torch.Tensor, dim: int = -1) -> torch.Tensor:
    st = _STATE
    if st.tp_size == 1:
        return x
    if st.comm is not None and x.is_cuda and x.dim() == 2 and dim in (-1, 1):
        return st.comm.all_gather_last(x.contiguous())
    parts = [torch.empty_like(x) for _ in range(st.tp_size)]
    dist.all_gather(parts, x.contiguous(), group=st.tp_group)
    return torch.cat(parts, dim=dim)


def stage_layers(num_layers: int, pp_size: int, pp_rank: int) -> list[int]:
    """Contiguous, balanced split of the decoder layers over pipeline stages."""
    return list(range(pp_rank * num_layers // pp_size, (pp_rank + 1) * num_layers // pp_size))


def _pp_peer(stage: int) -> int:
    st = _STATE
    return st.base + stage * st.tp_size + st.tp_rank


# ------------------------------------------------------------------ pipeline hand-offs
# On one node every stage pair has a direct xGMI link, so the stage-to-stage activations and the
# last stage's sampled tokens move through the IPC peer kernels of ome_amd.parallel.comm (a
# 2-rank gather per adjacent stage pair, a pp-wide gather for the tokens) instead of RCCL p2p:
# stream-ordered device-side hand-offs with no host round trip, which is what lets a pipeline
# stage's decode step -- receive, layers, send, token broadcast -- be ONE captured HIP graph.
# RCCL p2p / broadcast remain for multi-node pipelines and CPU (gloo) runs.
PP_IPC_BYTES = 64 << 20


def _pp_ipc_init(st: ParallelState, groups: dict) -> None:
    """Build the pipeline's IPC hand-off comms, then AGREE on the outcome over the engine group:
    IPC is kept only if every rank built every comm it needs.  A rank that fell back on its own
    would run RCCL ``send``/``recv`` against a peer still in ``all_gather_last`` -- both hang."""
    import logging

    from ome_amd.parallel.comm import CustomAllReduce

    t, p = st.tp_rank, st.pp_rank
    err = None
    try:
        # every rank builds its comms in stage order, so each pair's two members meet in the
        # same collective (handle exchange over that pair's gloo group)
        for q in range(st.pp_size - 1):
            if q == p - 1:
                st.pp_prev = CustomAllReduce(groups[(t, q)], max_bytes=PP_IPC_BYTES, cpu_group=groups[(t, q)])
            elif q == p:
                st.pp_next = CustomAllReduce(groups[(t, q)], max_bytes=PP_IPC_BYTES, cpu_group=groups[(t, q)])
        st.pp_bcast = CustomAllReduce(groups[(t, "all")], max_bytes=4 << 20, cpu_group=groups[(t, "all")])
    except Exception as e:  # noqa: BLE001 -- e.g. peers not IPC-reachable
        err = e
    if not _all_ranks_ok(err is None, st.cpu_group):
        logging.getLogger("ome_amd.parallel").warning(
            "pipeline IPC hand-off unavailable (%s); every rank uses RCCL p2p",
            err if err is not None else "failed on another rank")
        for c in (st.pp_prev, st.pp_next, st.pp_bcast):
            if c is not None:
                try:
                    c.close()
                except Exception:  # noqa: BLE001 -- best effort: the fallback does not use it
                    pass
        st.pp_prev = st.pp_next = st.pp_bcast = None


def _all_ranks_ok(ok: bool, group) -> bool:
    """MIN-reduce of a per-rank success flag over a (gloo) group: True only if every rank is ok."""
    if group is None:
        return ok
    flag = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
    return bool(flag.item())


def pp_graph_ok() -> bool:
    """Every hand-off of a decode step is a device-side IPC kernel (HIP-graph capturable)."""
    st = _STATE
    return st.pp_size > 1 and st.pp_bcast is not None and (st.is_first_pp or st.pp_prev is not None) and \
        (st.is_last_pp or st.pp_next is not None)


def _pp_ipc_cols(comm, rows: int, shapes, dtype) -> int | None:
    """Columns of the packed [rows, cols] hand-off, or None when the IPC path does not apply
    (sender and receiver evaluate this on the same shapes, so they always agree)."""
    if comm is None or dtype != torch.bfloat16 or rows <= 0:
        return None
    cols = 0
    for shp in shapes:
        if len(shp) < 1 or shp[0] != rows:
            return None
        n = 1
        for d in shp[1:]:
            n *= int(d)
        cols += n
    if (cols * 2) % 16 or rows * cols * 2 > comm.max_bytes:
        return None
    return cols


def pp_send(*tensors: torch.Tensor) -> None:
    """Activations to the next pipeline stage (same TP rank): the IPC pair gather on one node,
    RCCL p2p across nodes, gloo on CPU."""
    st = _STATE
    comm = st.pp_next if tensors and tensors[0].is_cuda else None
    rows = tensors[0].shape[0] if tensors else 0
    dts = {t.dtype for t in tensors}
    cols = _pp_ipc_cols(comm, rows, [tuple(t.shape) for t in tensors], dts.pop() if len(dts) == 1 else None)
    if cols is not None:
        packed = torch.cat([t.reshape(rows, -1) for t in tensors], dim=1) if len(tensors) > 1 else \
            tensors[0].reshape(rows, -1).contiguous()
        comm.all_gather_last(packed)   # the receiver takes the sender's (first) half
        return
    dst = _pp_peer(st.pp_rank + 1)
    for t in tensors:
        dist.send(t.contiguous(), dst=dst)


def pp_recv(*like: tuple[tuple, torch.dtype, torch.device]) -> list[torch.Tensor]:
    st = _STATE
    dev = torch.device(like[0][2]) if like else torch.device("cpu")
    comm = st.pp_prev if dev.type == "cuda" else None
    rows = like[0][0][0] if like and like[0][0] else 0
    dts = {dt for _, dt, _ in like}
    cols = _pp_ipc_cols(comm, rows, [tuple(s) for s, _, _ in like], dts.pop() if len(dts) == 1 else None)
    if cols is not None:
        dummy = torch.empty(rows, cols, dtype=torch.bfloat16, device=dev)
        got = comm.all_gather_last(dummy)[:, :cols]
        out, c0 = [], 0
        for shape, _dt, _d in like:
            n = 1
            for d in shape[1:]:
                n *= int(d)
            out.append(got[:, c0:c0 + n].contiguous().view(*shape))
            c0 += n
        return out
    src = _pp_peer(st.pp_rank - 1)
    out = []
    for shape, dtype, device in like:
        t = torch.empty(shape, dtype=dtype, device=device)
        dist.recv(t, src=src)
        out.append(t)
    return out


def pp_broadcast_from_last(t: torch.Tensor) -> torch.Tensor:
    """The last stage samples; every stage needs the tokens (identical scheduler state)."""
    st = _STATE
    if st.pp_size > 1:
        dist.broadcast(t, src=_pp_peer(st.pp_size - 1), group=st.pp_group)
    return t


def pp_broadcast_tokens(ids: torch.Tensor, logprobs: torch.Tensor) -> None:
    """Sampled ids (int32) and log-probs (fp32) of the last stage -> every stage, in place.  On
    the IPC path both ride one pp-wide gather of 16-B rows (id, logprob bits, 2 pad words)."""
    st = _STATE
    if st.pp_size == 1:
        return
    n = ids.shape[0]
    if st.pp_bcast is not None and ids.is_cuda and n and n * 16 <= st.pp_bcast.max_bytes:
        row = torch.zeros(n, 4, dtype=torch.int32, device=ids.device)
        row[:, 0] = ids
        row[:, 1] = logprobs.float().view(torch.int32)
        g = st.pp_bcast.all_gather_last(row.view(torch.bfloat16)).view(torch.int32)   # [n, 4 * pp]
        last = g[:, 4 * (st.pp_size - 1):4 * (st.pp_size - 1) + 2]
        ids.copy_(last[:, 0])
        logprobs.copy_(last[:, 1].contiguous().view(torch.float32))
        return
    pp_broadcast_from_last(ids)
    pp_broadcast_from_last(logprobs)


def destroy() -> None:
    global _STATE
    if dist.is_initialized():
        dist.destroy_process_group()
    _STATE = ParallelState()
