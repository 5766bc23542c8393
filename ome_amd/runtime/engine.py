"""The serving engine: scheduler + model runner + request lifecycle + metrics.

Tensor parallelism follows the one-process-per-GPU model: every TP rank owns a scheduler
replica; rank 0 (the one behind the HTTP server) broadcasts newly arrived requests/aborts
each step over a CPU (gloo) group, so all ranks schedule identical batches, run the same
forward (RCCL/xGMI collectives inside), and sample identical tokens from the all-gathered
logits with the same counter-based seeds.
"""
from __future__ import annotations

import logging
import os
import threading
import time
from dataclasses import asdict, dataclass, field

import torch

from ome_amd.models.config import ModelConfig, preset
from ome_amd.runtime.metrics import EngineMetrics
from ome_amd.runtime.request import ReqState, Request, SamplingParams
from ome_amd.runtime.scheduler import Scheduler
from ome_amd.runtime.tokenizer import get_tokenizer

log = logging.getLogger("ome_amd.engine")


_REASONS = ["stop", "length", "abort", "abort:error", "abort:kv_capacity", "abort:kv_layout_mismatch",
            "abort:kv_transfer"]
_REASON_CODE = {r: i for i, r in enumerate(_REASONS)}


def _unknown_code(reason) -> int:
    """Code of a finish reason missing from the table: "abort" for any abort:* (or other) reason."""
    return _REASON_CODE["stop"] if reason in (None, "stop") else _REASON_CODE["abort"]


def _unpack_updates(v: list[float]):
    """Inverse of the DP-attention update packing in :meth:`Engine._dp_step`."""
    n, i, out, heads = int(v[0]), 1, [], []
    for _ in range(n):
        h, nt, fin, code = int(v[i]), int(v[i + 1]), bool(v[i + 2]), int(v[i + 3])
        toks = [int(t) for t in v[i + 4:i + 4 + nt]]
        i += 4 + nt
        # a reason outside the table is still a failure, never a normal completion
        heads.append((h, toks, fin, _REASONS[code] if 0 <= code < len(_REASONS) else "abort"))
    for h, toks, fin, reason in heads:   # log-probs follow all headers, in the same order
        lps = v[i:i + len(toks)]
        i += len(toks)
        out.append((h, toks, lps, fin, reason))
    return out


@dataclass
class EngineArgs:
    model_path: str | None = None
    model: str | None = None               # preset name when no model_path (random-init)
    served_model_name: str | None = None
    tp_size: int = 1
    pp_size: int = 1
    pp_microbatches: int = 0               # micro-batches per pipeline step (0 = pp_size)
    dp_size: int = 1
    mem_fraction_static: float = 0.9
    max_running_requests: int = 256
    max_total_tokens: int | None = None
    chunked_prefill_size: int = 8192
    context_length: int | None = None
    page_size: int = 16
    cuda_graph: bool = True
    cuda_graph_max_bs: int | None = None
    load_format: str = "auto"
    dtype: str = "bfloat16"
    device: str = "cuda"
    seed: int = 0
    enable_mixed_chunk: bool = True        # decodes ride along prefill steps (one weight pass)
    disable_radix_cache: bool = False
    is_embedding: bool = False
    kv_cache_dtype: str = "auto"
    quantization: str | None = None        # "fp8": W8A8 projections (online quant of bf16 weights)
    dist_init_addr: str | None = None
    nnodes: int = 1
    node_rank: int = 0
    disaggregation_mode: str = "null"      # null | prefill | decode
    enable_dp_attention: bool = False      # --dp N --enable-dp-attention: per-rank batches + EP MoE
    ep_num_redundant_experts: int = 0      # EPLB: extra expert slots (replicas of hot experts) over the EP ranks
    eplb_rebalance_steps: int = 0          # EPLB: re-place experts from recorded loads every N lockstep steps
    enable_two_batch_overlap: bool = False # EP MoE: two micro-batches, all-to-alls overlapped with experts
    overlap_schedule: bool | None = None   # enqueue step k+1 before step k's tokens reach the host
    watchdog_timeout: float = 300.0        # --watchdog-timeout: a loop phase older than this ends the
                                           # process non-zero (0 disables; runtime/watchdog.py)
    cuda_graph_bs: list | None = None      # --cuda-graph-bs: exact decode batch sizes to capture
    tokenizer_path: str | None = None      # --tokenizer-path
    dp_balance: str = "shortest_queue"     # --load-balance-method / --prefill-round-robin-balance
    deepep_mode: str = "auto"              # --deepep-mode: normal = RCCL all_to_all only
    decode_log_interval: int = 0           # --decode-log-interval: log decode throughput every N steps
                                           # (None = on for GPU engines)
    num_layers_override: int | None = None
    extra: dict = field(default_factory=dict)

    def model_config(self) -> ModelConfig:
        if self.model_path and os.path.exists(os.path.join(self.model_path, "config.json")):
            cfg = ModelConfig.from_path(self.model_path)
        else:
            cfg = preset(self.model or "llama-3-8b")
        if self.num_layers_override:
            cfg = cfg.shrink(self.num_layers_override)
        if self.is_embedding:
            cfg.is_embedding = True
        if self.quantization:
            cfg.quantization = self.quantization
        if self.ep_num_redundant_experts:
            cfg.extra = {**(cfg.extra or {}), "ep_num_redundant_experts": int(self.ep_num_redundant_experts)}
        return cfg


class Engine:
    def __init__(self, args: EngineArgs):
        from ome_amd.parallel import state as pstate
        from ome_amd.runtime.model_runner import ModelRunner

        self.args = args
        self.cfg = args.model_config()
        dp = args.dp_size if args.enable_dp_attention else 1
        if args.deepep_mode == "normal":   # RCCL all_to_all for every MoE exchange
            os.environ["OME_EP_LL"] = "0"
        if args.tp_size > 1 or args.pp_size > 1 or dp > 1:
            pstate.init(args.tp_size, args.pp_size, dist_init_addr=args.dist_init_addr, dp_size=dp)
        self.pstate = pstate.get()
        self.pstate.tbo = bool(args.enable_two_batch_overlap and self.pstate.ep_size > 1)
        self.dp = self.pstate.dp_size > 1
        self._remote: dict[str, Request] = {}   # DP attention, rank 0: requests served by other ranks
        self._remote_h: dict[int, Request] = {}  # ... by the integer handle all ranks agree on
        self._dp_seq = 0
        self._dp_pending: list[float] = []   # this rank's token updates awaiting the next relay
        # relay capacity: one token (+ header and log-prob) per running request, in float64s
        self._dp_cap = 8 + 6 * (args.max_running_requests + 1)
        self._dp_next = 0
        device = args.device
        if device == "cuda" and torch.cuda.is_available():
            device = f"cuda:{torch.cuda.current_device()}"
        elif device == "cuda":
            device = "cpu"
        self.max_context = min(args.context_length or self.cfg.max_position_embeddings,
                               self.cfg.max_position_embeddings)
        dtype = {"bfloat16": torch.bfloat16, "float16": torch.float16, "float32": torch.float32,
                 "auto": torch.bfloat16}.get(str(args.dtype), torch.bfloat16)
        self.runner = ModelRunner(self.cfg, device=device, dtype=dtype, model_path=args.model_path,
                                  load_format=args.load_format,
                                  page_size=args.page_size, mem_fraction_static=args.mem_fraction_static,
                                  max_total_tokens=args.max_total_tokens, max_running=args.max_running_requests,
                                  max_context=self.max_context, cuda_graph=args.cuda_graph,
                                  cuda_graph_max_bs=args.cuda_graph_max_bs, seed=args.seed,
                                  cuda_graph_bs=args.cuda_graph_bs,
                                  kv_cache_dtype_name=args.kv_cache_dtype)
        self.runner.pp_microbatches = args.pp_microbatches
        prefix = None
        m = self.runner.model
        if not args.disable_radix_cache and not getattr(m, "stateful", False) and not getattr(m, "encoder_only", False):
            from ome_amd.runtime.prefix_cache import PrefixCache

            prefix = PrefixCache(self.runner.pages, args.page_size)
        self.scheduler = Scheduler(self.runner.pages, self.runner.slots, args.page_size, args.max_running_requests,
                                   args.chunked_prefill_size, self.max_context, args.enable_mixed_chunk, prefix)
        # TP / PP ranks schedule in lockstep on broadcast requests: no wall-clock decisions
        self.scheduler.lockstep = self.pstate.world_size > 1 and not self.dp
        if args.enable_mixed_chunk and os.environ.get("OME_STEP_COST", "0") == "1":
            self._init_step_cost(args)
        self.tokenizer = get_tokenizer(args.tokenizer_path or args.model_path, self.cfg.vocab_size)
        eos = getattr(self.tokenizer, "eos_token_id", None)
        self.eos_ids = {eos} if eos is not None else set()
        self.metrics = EngineMetrics()
        self.served_model_name = args.served_model_name or (args.model_path or args.model or "model")
        self._lock = threading.Lock()
        self._inbox: list[Request] = []
        self._aborts: list[str] = []
        self._wake = threading.Event()
        self._stop = False
        self._stop_pending = False
        self.step_count = 0
        self.kv_transfer = None  # PD disaggregation hook (ome_amd.runtime.disagg)
        # what a failed lockstep step does to a multi-rank group (tests replace it)
        self.on_fatal = lambda: os._exit(70)
        # engine watchdog (--watchdog-timeout) + collective expiry / fault-injection hooks
        from ome_amd.runtime import watchdog as _wd

        self._wd_mod = _wd
        self.watchdog = _wd.Watchdog(args.watchdog_timeout, self.pstate.rank) if args.watchdog_timeout > 0 else None
        self._fault = _wd.parse_fault()
        # overlapped scheduling: (batch, handle, launch time) of the step whose tokens are in flight
        self._inflight = None
        # host-side time split of the serving loop (seconds, cumulative): schedule / launch
        # (input packing + kernel / graph enqueue) / wait (blocked on the GPU) / commit
        self.host_times = {"schedule": 0.0, "launch": 0.0, "wait": 0.0, "commit": 0.0, "steps": 0}
        self.host_trace: list | None = None   # per-call (kind, rows, t_a, t_b) when profiling
        self.metrics.host_times = self.host_times
        ov = self.runner.is_cuda if args.overlap_schedule is None else bool(args.overlap_schedule)
        self.overlap = ov and not self.cfg.is_embedding and self.pstate.pp_size == 1 and not self.dp
        # DP attention overlaps too: step k+1 (this rank's part of the lockstep forward) is enqueued
        # before step k's tokens are read back; the relay then carries step k's tokens
        self.dp_overlap = ov and self.dp and not self.cfg.is_embedding

    # ------------------------------------------------------------------ API
    def make_request(self, prompt_ids: list[int], params: SamplingParams | None = None, **kw) -> Request:
        params = params or SamplingParams()
        params.validate()
        if len(prompt_ids) == 0:
            raise ValueError("empty prompt")
        if len(prompt_ids) + 1 > self.max_context:
            raise ValueError(f"prompt of {len(prompt_ids)} tokens exceeds context length {self.max_context}")
        params.max_new_tokens = min(params.max_new_tokens, self.max_context - len(prompt_ids))
        return Request(prompt_ids=list(prompt_ids), params=params, **kw)

    def make_mm_request(self, prompt_ids: list[int], images: list, params: SamplingParams | None = None,
                        **kw) -> Request:
        """A prompt with one image placeholder token per image (the model's ``image_token_id``) and
        the images (data URL / path / bytes / PIL, or a preprocessed ``(pixel_values, (t, h, w))``).
        Placeholders are expanded to one token per merged vision patch (content-hash ids, so the
        prefix cache only matches identical images) and the M-RoPE positions are precomputed."""
        import torch

        from ome_amd.multimodal import MMInput, expand_image_tokens, mrope_positions
        from ome_amd.multimodal.inputs import preprocess_image

        m = self.runner.model
        if not getattr(m, "is_multimodal", False):
            raise ValueError(f"{self.cfg.architecture} does not accept image inputs")
        if hasattr(m, "make_mm_input"):  # model-specific inputs (Mllama: tiles + cross-attention ranges)
            ids, mm = m.make_mm_input(list(prompt_ids), images)
            return self.make_request(ids, params, mm=mm, **kw)
        pvs, grids = [], []
        for im in images:
            if isinstance(im, tuple):
                pv, g = im
            else:
                pv, g = preprocess_image(im, patch=m.visual.patch, merge=m.merge, temporal=m.visual.temporal,
                                         **getattr(m, "image_processor_kwargs", {}))
            pvs.append(torch.as_tensor(pv, dtype=torch.float32))
            grids.append(tuple(int(v) for v in g))
        ids, spans = expand_image_tokens(list(prompt_ids), m.image_token_id, grids, m.merge, pvs,
                                         self.cfg.vocab_size)
        pos, delta = mrope_positions(len(ids), spans, grids, m.merge)
        mm = MMInput(torch.cat(pvs, 0), grids, spans, pos, delta)
        return self.make_request(ids, params, mm=mm, **kw)

    def add_request(self, req: Request) -> Request:
        with self._lock:
            self._inbox.append(req)
        self._wake.set()
        return req

    def abort(self, rid: str) -> None:
        with self._lock:
            self._aborts.append(rid)
        self._wake.set()

    def _drain_inbox(self) -> None:
        with self._lock:
            new, aborts = self._inbox, self._aborts
            self._inbox, self._aborts = [], []
        if self.pstate.world_size > 1:
            new, aborts = self._broadcast_control(new, aborts)
        kt = self.kv_transfer
        for r in new:
            if self.dp:   # every rank sees the same new requests in the same order: same handles
                r.dp_handle = self._dp_seq
                self._dp_seq += 1
            if self.dp and getattr(r, "dp_rank", 0) != self.pstate.rank:
                if self.pstate.rank == 0:
                    self._remote[r.rid] = r  # proxy: tokens arrive from the owning rank
                    self._remote_h[r.dp_handle] = r
                    self.metrics.on_arrival(r)
                continue
            r.arrival_time = r.arrival_time or time.perf_counter()
            if kt is not None and kt.mode == "decode" and (r.bootstrap or {}).get("disagg_role") == "decode":
                kt.hold(r)  # its KV comes from a prefill engine (ome_amd.runtime.disagg)
                continue
            self.scheduler.add(r)
            self.metrics.on_arrival(r)
        for rid in aborts:
            if kt is not None:
                for room, w in list(kt.waiting.items()):
                    if w.rid == rid:
                        kt.waiting.pop(room)
                        w.state, w.finish_reason = ReqState.FINISHED, "abort"
            r = self.scheduler.abort(rid)
            if r is None and rid in self._remote:  # DP proxy: the owning rank aborts its copy
                r = self._remote.pop(rid)
                self._remote_h.pop(getattr(r, "dp_handle", -1), None)
                r.state, r.finish_reason = ReqState.FINISHED, "abort"
            if r is not None and r.on_token:
                r.on_token(r, [], True)

    def _broadcast_control(self, new, aborts, stop: bool = False):
        """Rank 0 -> all TP ranks, once per step: new requests, aborts, and the group stop flag
        (followers leave ``run_forever`` when the leader shuts down)."""
        import torch.distributed as dist

        if self.dp and self.pstate.rank == 0:
            for r in new:  # DP attention: least-loaded rank owns the request
                r.dp_rank = self._dp_assign()
        leader = self.pstate.to_global(0)
        stop = bool(stop or self._stop_pending)
        # fixed-size header first: the common step with nothing new costs one small broadcast,
        # not a pickle round trip
        hdr = torch.tensor([len(new), len(aborts), int(stop)] if self.pstate.rank == 0 else [0, 0, 0],
                           dtype=torch.int64)
        dist.broadcast(hdr, src=leader, group=self._cpu_group())
        if not int(hdr[0]) and not int(hdr[1]):
            if int(hdr[2]):
                self._stop = True
            return (new, aborts) if self.pstate.rank == 0 else ([], [])
        payload = [[(r.rid, r.prompt_ids, asdict(r.params), r.bootstrap, getattr(r, "dp_rank", 0)) for r in new],
                   aborts, stop]
        obj = [payload if self.pstate.rank == 0 else None]
        dist.broadcast_object_list(obj, src=leader, group=self._cpu_group())
        if obj[0][2]:
            self._stop = True
        if self.pstate.rank == 0:
            return new, aborts
        reqs = []
        for rid, p, sp, b, dr in obj[0][0]:
            r = Request(prompt_ids=p, params=SamplingParams(**sp), rid=rid, bootstrap=b)
            r.dp_rank = dr
            reqs.append(r)
        return reqs, obj[0][1]

    def _log_decode(self, rows: int, now: float) -> None:
        """--decode-log-interval: one SGLang-style throughput line every N decode steps."""
        st = self.__dict__.setdefault("_dlog", {"n": 0, "tok": 0, "t": now})
        st["n"] += 1
        st["tok"] += rows
        if st["n"] < self.args.decode_log_interval:
            return
        dt = max(now - st["t"], 1e-9)
        log.info("Decode batch. #running-req: %d, #token: %d, token usage: %.2f, gen throughput (token/s): %.2f, "
                 "#queue-req: %d", self.scheduler.num_running,
                 (self.runner.pages.num_pages - 1 - self.runner.pages.num_free) * self.args.page_size,
                 self.runner.pages.usage(), st["tok"] / dt, self.scheduler.num_waiting)
        st.update(n=0, tok=0, t=now)

    def _dp_assign(self, req=None) -> int:
        """Rank 0: the DP rank that serves a new request (``--load-balance-method``):
        shortest_queue (default) = fewest outstanding requests, minimum_tokens = fewest outstanding
        prompt + output tokens, round_robin (also ``--prefill-round-robin-balance``) = strict
        rotation.  Ties rotate."""
        n = self.pstate.dp_size
        how = self.args.dp_balance
        if how == "round_robin":
            best = self._dp_next
            self._dp_next = (best + 1) % n
            return best
        load = [0] * n
        mine = list(self.scheduler.running) + list(self.scheduler.waiting)
        if how == "minimum_tokens":
            load[0] = sum(r.seq_len + r.params.max_new_tokens for r in mine)
            for r in self._remote.values():
                load[r.dp_rank] += len(r.prompt_ids) + r.params.max_new_tokens
        else:
            load[0] = len(mine)
            for r in self._remote.values():
                load[r.dp_rank] += 1
        best = min(range(n), key=lambda i: (load[i], (i - self._dp_next) % n))
        self._dp_next = (best + 1) % n
        return best

    def stop_group(self) -> None:
        """Leader: tell every follower rank to exit its step loop (one final control broadcast)."""
        if self.pstate.world_size > 1 and self.pstate.rank == 0:
            self._broadcast_control([], [], stop=True)
        self._stop = True

    def _init_step_cost(self, args) -> None:
        """Measure this model's GEMM staircase (runtime/step_cost.py) and give it to the
        scheduler.  Lockstep ranks (TP / PP) all measure, then take rank 0's table, so every rank
        cuts its mixed steps identically."""
        max_rows = min(args.chunked_prefill_size + args.max_running_requests,
                       int(os.environ.get("OME_STEP_COST_MAX_ROWS", "4096")))
        cost = self.runner.measure_step_cost(max_rows)
        if self.scheduler.lockstep:
            import torch.distributed as dist

            from ome_amd.runtime.step_cost import StepCost

            n = -(-max_rows // StepCost.G)
            ok = torch.tensor([1 if cost is not None else 0], dtype=torch.int64)
            dist.broadcast(ok, src=self.pstate.to_global(0), group=self._cpu_group())
            if not int(ok[0]):
                cost = None
            else:
                buf = torch.tensor(cost.to_list() if cost is not None else [0.0] * n, dtype=torch.float64)
                dist.broadcast(buf, src=self.pstate.to_global(0), group=self._cpu_group())
                cost = StepCost(buf.tolist())
        dump = os.environ.get("OME_STEP_COST_DUMP")
        if dump and cost is not None and self.pstate.rank == 0:
            import json

            with open(dump, "w") as f:
                json.dump({"grid": cost.G, "us_per_layer": [round(v, 2) for v in cost.to_list()]}, f)
        self.scheduler.cost = cost

    def _cpu_group(self):
        import torch.distributed as dist

        if not hasattr(self, "_gloo"):
            self._gloo = self.pstate.cpu_group if self.pstate.cpu_group is not None else dist.new_group(backend="gloo")
        return self._gloo

    def step(self) -> list[Request]:
        """One scheduler iteration: enqueue one step.  Returns requests that finished.

        Overlapped mode (default on GPU): step k+1 is scheduled and enqueued *before* step k's
        sampled tokens are copied back — its decode rows take their input ids from step k's
        device output (``ModelRunner.launch(prev=...)``) — so host-side scheduling, input packing
        and detokenisation hide behind the GPU.  Returned requests are those finished by step k.
        """
        wd = self.watchdog
        if wd is not None:
            wd.enter("control")
        if self._fault is not None:
            self._wd_mod.maybe_inject(self.pstate.rank, self.step_count, self._fault)
        try:
            return self._step(wd)
        finally:
            if wd is not None:
                wd.idle()

    def _step(self, wd) -> list[Request]:
        self._drain_inbox()
        if self._stop and self.pstate.world_size > 1:
            return []   # the leader's stop broadcast: it runs no further lockstep step
        if wd is not None:
            wd.enter("schedule")
        if self.kv_transfer is not None and self.kv_transfer.mode == "decode":
            self.kv_transfer.poll()
        if self.cfg.is_embedding:
            return self._embed_step()
        if self.dp:
            return self._dp_step()
        prev = self._inflight
        ht = self.host_times
        idle0 = None
        if self.host_trace is not None and prev and prev[1].event is not None:
            idle0 = bool(prev[1].event.query())
        ts = time.perf_counter()
        batch = self.scheduler.schedule()
        launched = None
        if batch is not None:
            t0 = time.perf_counter()
            if wd is not None:
                wd.enter("launch")
            handle = self.runner.launch(batch, prev[1] if prev else None)
            self.scheduler.launch_commit(batch)
            launched = (batch, handle, t0)
            ht["schedule"] += t0 - ts
            ht["launch"] += time.perf_counter() - t0
            if self.host_trace is not None:
                # did the GPU run dry before / while this step was enqueued (previous step done)?
                ev = prev[1].event if prev else None
                self.host_trace.append((batch.mode, len(batch.chunks), t0 - ts, time.perf_counter() - t0,
                                        idle0, bool(ev.query()) if ev is not None else None))
        done: list[Request] = []
        if not self.overlap:
            if launched:
                done = self._complete(*launched)
            return done
        if prev is not None:
            done = self._complete(*prev)
        self._inflight = launched
        return done

    def _complete(self, batch, handle, t0) -> list[Request]:
        ht = self.host_times
        tw = time.perf_counter()
        wd = self.watchdog
        if wd is not None:
            wd.enter(f"wait ({batch.mode}, {len(batch.chunks)} rows)")
        ids, lps = handle.result()
        if self.pstate.world_size > 1:
            # a bounded collective wait that expired leaves the step's output garbage: fail loudly
            # (run_forever turns this into a non-zero exit of the whole lockstep group)
            self._wd_mod.check_comms()
        if wd is not None:
            wd.enter("commit")
        now = time.perf_counter()
        done = self.scheduler.final_commit(batch, ids, lps, now, self.eos_ids)
        self.step_count += 1
        self.metrics.on_step(batch, now - t0, done, self.scheduler, self.runner.pages)
        if self.args.decode_log_interval > 0 and batch.mode == "decode":
            self._log_decode(len(batch.chunks), now)
        ht["wait"] += now - tw
        if self.host_trace is not None:
            self.host_trace.append(("wait", 0, now - tw, time.perf_counter() - now))
        ht["commit"] += time.perf_counter() - now
        ht["steps"] += 1
        return done

    def _dp_step(self) -> list[Request]:
        """DP attention: every rank schedules its own requests, all ranks run the forward in
        lockstep (a rank without work runs one dummy token so the MoE all-to-alls are complete),
        and the followers report their new tokens to rank 0, which owns the HTTP streams.

        ONE CPU collective per step (besides the leader's control header): a fixed-capacity
        all-gather of [this step's token count, payload length, the PREVIOUS step's packed token
        updates].  Every rank learns every batch size (same MoE exchange mode everywhere) and rank
        0 receives the relayed tokens, one step after they were sampled.  The capacity covers one
        token per running request; a larger payload (never in steady state) falls back to a
        sizes all-gather + gather for that step, decided identically on every rank."""
        import torch.distributed as dist

        batch = self.scheduler.schedule()
        n_tok = 0 if batch is None else sum(c.length for c in batch.chunks)
        pend = self._dp_pending
        self._dp_pending = []
        cap = self._dp_cap
        over = len(pend) > cap - 2
        buf = torch.zeros(cap, dtype=torch.float64)
        buf[0] = n_tok
        buf[1] = -1.0 if over else len(pend)
        if pend and not over:
            buf[2:2 + len(pend)] = torch.tensor(pend, dtype=torch.float64)
        bufs = [torch.empty(cap, dtype=torch.float64) for _ in range(self.pstate.world_size)]
        dist.all_gather(bufs, buf, group=self._cpu_group())
        allw = [int(b[0]) for b in bufs]
        done: list[Request] = []
        if any(int(b[1]) < 0 for b in bufs):   # overflow somewhere: two-phase exchange, all ranks
            # every rank re-sends its update: a rank that fit the capacity has already taken it
            # out of _dp_pending, so the fixed-capacity copy above is discarded with `bufs`
            payloads = self._dp_gather_updates(pend)
            bufs = [torch.cat([torch.tensor([0.0, float(len(pl))], dtype=torch.float64), pl]) for pl in payloads]
        if self.pstate.rank == 0:
            done += self._dp_apply_updates(bufs)
        prev = self._inflight if self.dp_overlap else None
        completed = None
        if not any(allw):
            if prev is not None:   # nothing new anywhere: drain the step still in flight
                done += self._complete(*prev)
                completed, self._inflight = prev[0], None
            self._dp_relay(completed)
            return done
        # every rank sees the same token counts, so all pick the same MoE exchange mode: the
        # device-only low-latency buckets when every rank's batch fits, RCCL all-to-all otherwise
        st = self.pstate
        st.ep_ll_ok = st.ep_ll is not None and max(allw) <= st.ep_ll_cap
        launched = None
        if batch is not None:
            t0 = time.perf_counter()
            handle = self.runner.launch(batch, prev[1] if prev is not None else None, allow_graph=st.ep_ll_ok)
            self.scheduler.launch_commit(batch)
            launched = (batch, handle, t0)
        elif st.ep_ll_ok:
            self.runner.idle_decode()
        else:
            self.runner.idle_forward()
        if self.dp_overlap:
            if prev is not None:
                done += self._complete(*prev)
                completed = prev[0]
            self._inflight = launched
        elif launched is not None:
            done += self._complete(*launched)
            completed = batch
        self._dp_relay(completed)
        self._dp_steps = getattr(self, "_dp_steps", 0) + 1
        n = self.args.eplb_rebalance_steps
        if n and self._dp_steps % n == 0:  # every rank reaches this point in the same lockstep step
            from ome_amd.parallel.eplb import rebalance_model

            imb = rebalance_model(self.runner.model)
            if imb:
                log.info("EPLB round: max/mean expert load per rank %.3f", max(imb.values()))
        return done

    def _dp_relay(self, completed) -> None:
        """Follower: pack the tokens ``completed`` (the step whose ids just reached the host)
        gave this rank's requests, for the next step's all-gather: [n_updates, then per update
        handle, n_tokens, finished, reason code, and the tokens; then all log-probs].  Only
        resolved tokens travel -- under overlap the rows of the step in flight are PENDING."""
        if self.pstate.rank == 0 or completed is None:
            return
        touched = list({id(c.req): c.req for c in completed.chunks}.values())
        if not touched:
            return
        packed: list[float] = [0.0]
        lps_all: list[float] = []
        for r in touched:
            k = getattr(r, "_reported", 0)
            end = len(r.output_ids) - r.n_pending
            toks = r.output_ids[k:end]
            fin = r.state == ReqState.FINISHED
            if (not toks and not fin) or getattr(r, "_fin_reported", False):
                continue   # (a finished request can sit in the next in-flight step as a dead row)
            r._fin_reported = fin
            packed += [float(getattr(r, "dp_handle", -1)), float(len(toks)), float(fin),
                       float(_REASON_CODE.get(r.finish_reason, _unknown_code(r.finish_reason)) if fin else -1)]
            packed += [float(t) for t in toks]
            lps_all += [float(x) for x in r.output_logprobs[k:end]]
            r._reported = end
            packed[0] += 1
        if packed[0]:
            self._dp_pending = packed + lps_all

    def _dp_gather_updates(self, mine_list: list[float]) -> list[torch.Tensor]:
        """Two-phase fallback of the update relay (sizes all-gather, then a padded gather to rank
        0); returns every rank's payload on rank 0 (empty tensors elsewhere)."""
        import torch.distributed as dist

        mine = torch.tensor(mine_list, dtype=torch.float64)
        sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(self.pstate.world_size)]
        dist.all_gather(sizes, torch.tensor([mine.numel()], dtype=torch.int64), group=self._cpu_group())
        cap = max(1, max(int(x) for x in sizes))
        buf = torch.zeros(cap, dtype=torch.float64)
        buf[:mine.numel()] = mine
        bufs = [torch.zeros(cap, dtype=torch.float64) for _ in range(self.pstate.world_size)] \
            if self.pstate.rank == 0 else None
        dist.gather(buf, bufs, dst=self.pstate.to_global(0), group=self._cpu_group())
        if self.pstate.rank != 0:
            return [torch.zeros(0, dtype=torch.float64)] * self.pstate.world_size
        return [b[:int(n)] for b, n in zip(bufs, sizes)]

    def _dp_apply_updates(self, bufs) -> list[Request]:
        """Rank 0: apply the followers' relayed token updates to the proxy requests."""
        done: list[Request] = []
        now = time.perf_counter()
        for b in bufs[1:]:
            n = int(b[1])
            if n <= 0:
                continue
            for handle, toks, lps, fin, reason in _unpack_updates(b[2:2 + n].tolist()):
                p = self._remote_h.get(handle)
                if p is None:
                    continue
                if toks and p.first_token_time is None:
                    p.first_token_time = now
                p.output_ids.extend(toks)
                p.output_logprobs.extend(lps)
                p.token_times.extend([now] * len(toks))
                if fin:
                    p.state, p.finish_reason = ReqState.FINISHED, reason
                    self._remote.pop(p.rid, None)
                    self._remote_h.pop(handle, None)
                    done.append(p)
                if p.on_token is not None and (toks or fin):
                    p.on_token(p, list(toks), fin)
        return done

    def flush(self) -> list[Request]:
        """Wait for the in-flight step (if any) and commit it."""
        prev, self._inflight = self._inflight, None
        return self._complete(*prev) if prev else []

    def _embed_step(self) -> list[Request]:
        batch = self.scheduler.schedule()
        if batch is None:
            return []
        embs = self.runner.embed(batch)
        now = time.perf_counter()
        done = []
        for c, e in zip(batch.chunks, embs):
            c.req.embedding = e
            c.req.num_cached = c.start + c.length
            if c.req.num_cached >= len(c.req.prompt_ids):
                c.req.first_token_time = now
                self.scheduler.finish(c.req, "stop")
                done.append(c.req)
                if c.req.on_token:
                    c.req.on_token(c.req, [], True)
        return done

    def has_work(self) -> bool:
        return (self.scheduler.has_work() or bool(self._inbox) or self._inflight is not None or bool(self._remote)
                or bool(self.kv_transfer is not None and self.kv_transfer.waiting))

    def generate(self, prompts: list[list[int]], params: SamplingParams | list[SamplingParams] | None = None) -> list[Request]:
        plist = params if isinstance(params, list) else [params] * len(prompts)
        reqs = [self.add_request(self.make_request(p, SamplingParams(**asdict(sp)) if sp else None))
                for p, sp in zip(prompts, plist)]
        while any(not r.finished for r in reqs):
            self.step()
        return reqs

    # ------------------------------------------------------------------ background loop
    def run_forever(self) -> None:
        while not self._stop:
            if not self.has_work():
                self._wake.wait(timeout=0.05)
                self._wake.clear()
                if self.pstate.world_size == 1:
                    continue
            try:
                self.step()
            except Exception:  # noqa: BLE001 — surface; single engines keep serving other requests
                log.exception("engine step failed")
                for r in list(self.scheduler.running):
                    self.scheduler.finish(r, "abort:error")
                    if r.on_token:
                        r.on_token(r, [], True)
                if self.pstate.world_size > 1:
                    # a multi-rank group runs in lockstep: a rank that skips a step would leave
                    # its peers blocked in the next collective.  Fail the whole group instead
                    # (non-zero exit -> the LeaderWorkerSet RecreateGroupOnPodRestart policy).
                    log.critical("rank %d of a %d-rank engine group failed a step; exiting",
                                 self.pstate.rank, self.pstate.world_size)
                    self.on_fatal()
                    return

    def start(self) -> threading.Thread:
        t = threading.Thread(target=self.run_forever, name="ome-engine", daemon=True)
        t.start()
        return t

    def shutdown(self) -> None:
        if self.watchdog is not None:
            self.watchdog.stop()
        if self.pstate.world_size > 1 and self.pstate.rank == 0:
            self._stop_pending = True  # the loop broadcasts it on its next step, then exits
        else:
            self._stop = True
        self._wake.set()

    def health(self) -> dict:
        return {"running": self.scheduler.num_running, "waiting": self.scheduler.num_waiting,
                "kv_usage": self.runner.pages.usage(), "steps": self.step_count}


__all__ = ["Engine", "EngineArgs", "Request", "ReqState", "SamplingParams"]
