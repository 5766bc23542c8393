"""Continuous-batching scheduler with chunked prefill and paged-KV admission control.

Policy (SGLang-style, which is what the reference's runtime catalog configures through
``--chunked-prefill-size`` / ``--max-running-requests`` / ``--mem-frac``):
  * prefill-priority: when requests are waiting and KV pages are available, the step is a
    prefill step packing up to ``chunked_prefill_size`` prompt tokens (a long prompt is split
    into chunks across steps; partially-prefilled requests are continued first);
  * otherwise a decode step over every decode-ready running request;
  * if a decode step cannot get a page, the most recently admitted requests are preempted
    (pages freed, recomputed later) — never a deadlock, never an OOM;
  * optional mixed steps (``enable_mixed_chunk``): running decodes ride along a prefill step
    as 1-token rows so prefills never stall decode (lower TPOT at some TTFT cost).
"""
from __future__ import annotations

import collections
import time
import os
from dataclasses import dataclass, field

from ome_amd.runtime.page_pool import PagePool, ReqSlotPool
from ome_amd.runtime.request import PENDING, ReqState, Request


@dataclass
class ScheduledChunk:
    req: Request
    start: int      # first token index computed this step
    length: int     # tokens computed this step
    sample: bool    # last row produces a new token
    out_index: int = -1   # index in req.output_ids the sampled token lands at (set at launch)


@dataclass
class StepBatch:
    mode: str                                   # "prefill" | "decode"
    chunks: list[ScheduledChunk] = field(default_factory=list)

    @property
    def reqs(self) -> list[Request]:
        return [c.req for c in self.chunks]

    @property
    def num_tokens(self) -> int:
        return sum(c.length for c in self.chunks)


def _mm_salt(req) -> tuple[bytes, int]:
    """Prefix-cache salt of a multimodal request (image digest, first image position)."""
    key = getattr(req.mm, "cache_key", None)
    return key() if key is not None else (b"", 0)


class Scheduler:
    def __init__(self, pages: PagePool, slots: ReqSlotPool, page_size: int, max_running: int = 256,
                 chunked_prefill_size: int = 8192, max_context: int = 8192, enable_mixed_chunk: bool = False,
                 prefix_cache=None):
        self.pages, self.slots, self.P = pages, slots, page_size
        self.max_running = max_running
        self.chunk = chunked_prefill_size
        self.max_context = max_context
        self.mixed = enable_mixed_chunk
        self.prefix_cache = prefix_cache
        self.waiting: collections.deque[Request] = collections.deque()
        self.running: list[Request] = []
        self.num_preemptions = 0
        self.on_finish = None  # hook(req) before a finished request's pages are released (PD prefill)
        # prefill batching (throughput knob, off by default): while decodes are running, hold new
        # requests until their prompts add up to ``prefill_batch_tokens`` or the oldest has waited
        # ``prefill_max_wait_s`` -- fewer, larger prefill chunks run their GEMMs at higher MFMA
        # efficiency, at the cost of queueing delay (TTFT)
        self.prefill_batch_tokens = int(os.environ.get("OME_PREFILL_BATCH_TOKENS", "0"))
        self.prefill_max_wait_s = float(os.environ.get("OME_PREFILL_MAX_WAIT_MS", "50")) / 1000.0
        # admission order: "sjf" (default) admits the waiting request with the fewest prompt tokens
        # left, so a burst's short prompts reach their first token without queueing behind long
        # ones (lower p50 TTFT at the same throughput); a request that has waited ``sjf_age_s``
        # (and any preempted one) goes first, so long prompts cannot starve.  "fifo" = arrival order.
        self.policy = os.environ.get("OME_SCHED_POLICY", "sjf")
        self.sjf_age_s = float(os.environ.get("OME_SJF_AGE_MS", "500")) / 1000.0
        # Lockstep mode (TP / PP: every rank runs its own copy of this scheduler on the requests
        # rank 0 broadcasts, and all ranks must pick the SAME batch): every time-based decision
        # (SJF aging, prefill batching hold) counts schedule() calls since the request was
        # enqueued instead of reading the wall clock -- followers rebuild a request later than the
        # leader and read their clocks at different moments, so a time test can flip between ranks
        # and desynchronise the collectives.  ~30 steps ~ the 500 ms default at 16 ms per step.
        self.lockstep = False
        self.n_sched = 0
        self.sjf_age_steps = int(os.environ.get("OME_SJF_AGE_STEPS", "32"))
        self.prefill_max_wait_steps = int(os.environ.get("OME_PREFILL_MAX_WAIT_STEPS", "3"))
        # row-count-aware chunk sizing of mixed steps (runtime/step_cost.py): set by the engine
        # when the model runner measured its GEMM staircase; None = plain chunked_prefill_size
        self.cost = None
        self._pf_deferred = 0

    # ------------------------------------------------------------------ queue ops
    def add(self, req: Request) -> None:
        req.state = ReqState.WAITING
        req.enq_step = self.n_sched
        self.waiting.append(req)

    def _waited(self, req: Request, seconds: float, steps: int) -> bool:
        """Has ``req`` waited longer than the bound?  Step-counted in lockstep mode (identical on
        every rank), wall clock otherwise."""
        if self.lockstep:
            return self.n_sched - getattr(req, "enq_step", self.n_sched) > steps
        return time.perf_counter() - req.arrival_time > seconds

    def abort(self, rid: str) -> Request | None:
        for q in (self.waiting, self.running):
            for r in list(q):
                if r.rid == rid:
                    q.remove(r)
                    self._release(r)
                    r.state, r.finish_reason = ReqState.FINISHED, "abort"
                    return r
        return None

    @property
    def num_waiting(self) -> int:
        return len(self.waiting)

    @property
    def num_running(self) -> int:
        return len(self.running)

    def has_work(self) -> bool:
        return bool(self.waiting or self.running)

    # ------------------------------------------------------------------ pages
    def _pages_needed(self, req: Request, upto_tokens: int) -> int:
        return max(0, -(-upto_tokens // self.P) - len(req.pages))

    def _grow(self, req: Request, upto_tokens: int) -> bool:
        need = self._pages_needed(req, upto_tokens)
        if need == 0:
            return True
        got = self.pages.alloc(need)
        if got is None and self.prefix_cache is not None:
            self.prefix_cache.evict(need - self.pages.num_free)
            got = self.pages.alloc(need)
        if got is None:
            return False
        start = len(req.pages)
        req.pages.extend(got)
        self.slots.set_pages(req.req_slot, start, got)
        return True

    def _release(self, req: Request, cache_prefix: bool = False) -> None:
        if req.pages:
            if cache_prefix and self.prefix_cache is not None:
                kept = self.prefix_cache.insert(req.all_ids[: req.num_cached], req.pages, *_mm_salt(req))
                rest = [p for p in req.pages if p not in kept]
                self.pages.free(rest)
            else:
                if self.prefix_cache is not None:
                    self.prefix_cache.release(req.pages)
                self.pages.free([p for p in req.pages if self.prefix_cache is None or not self.prefix_cache.owns(p)])
            req.pages = []
        if req.req_slot >= 0:
            rel = getattr(req.mm, "release", None)
            if rel is not None:  # model-owned per-request state (Mllama vision-token cache)
                rel()
                req.mm.release = None
            self.slots.free(req.req_slot)
            req.req_slot = -1
        req.pen_init = False

    def finish(self, req: Request, reason: str) -> None:
        if req in self.running:
            self.running.remove(req)
        req.state, req.finish_reason = ReqState.FINISHED, reason
        if self.on_finish is not None and req.bootstrap:
            self.on_finish(req)
        self._release(req, cache_prefix=True)

    def _preempt_one(self, keep: Request | None = None) -> bool:
        # newest admitted first (LIFO), never the request we are trying to serve, never one whose
        # sampled token is still in flight (its recompute would need that token)
        for r in reversed(self.running):
            if r is keep or r.n_pending:
                continue
            self.running.remove(r)
            self._release(r)
            r.num_cached = 0
            r.num_prefix_hit = 0
            r.state = ReqState.WAITING
            r.preempted += 1
            self.waiting.appendleft(r)
            self.num_preemptions += 1
            return True
        return False

    # ------------------------------------------------------------------ schedule
    def schedule(self) -> StepBatch | None:
        self.n_sched += 1
        batch = self._schedule_prefill()
        if batch is not None:
            if self.mixed:
                self._add_decodes(batch)
            return batch
        return self._schedule_decode()

    @staticmethod
    def _span_safe(r, n: int) -> int:
        """Chunk length that does not end inside an atomic multimodal span (bidirectional image
        blocks): cut before the span, or take the whole span when the chunk starts inside it."""
        mm = r.mm
        if mm is None or not getattr(mm, "atomic", False):
            return n
        a, end = r.num_cached, r.num_cached + n
        for s, k in mm.spans:
            if s < end < s + k:
                end = s if s > a else s + k
                break
        return max(1, min(end, r.seq_len) - a)

    def _next_waiting(self) -> Request:
        head = self.waiting[0]
        if self.policy != "sjf" or len(self.waiting) == 1 or head.preempted or \
                self._waited(head, self.sjf_age_s, self.sjf_age_steps):
            return head
        return min(self.waiting, key=lambda r: (not r.preempted, r.seq_len - r.num_cached))

    def _decode_rows(self) -> int:
        """Running requests that will ride the next mixed step as 1-token decode rows."""
        return sum(1 for r in self.running if r.prefill_done and not self._exhausted(r))

    def _prefill_avail(self) -> tuple[int, list[int]]:
        """Prompt tokens a prefill step could take now -- the rest of every partially prefilled
        running request plus the prompts of as many waiting requests as there are free slots --
        and the cumulative counts at which each of those prompts ends, in admission order."""
        rest = [r.seq_len - r.num_cached for r in self.running if r.num_cached < r.seq_len - 1]
        free = self.max_running - len(self.running)
        if free > 0 and self.waiting:
            w = [r.seq_len - r.num_cached for r in self.waiting]
            if self.policy == "sjf":
                w = [w[0]] + sorted(w[1:]) if self._waited(self.waiting[0], self.sjf_age_s, self.sjf_age_steps) \
                    else sorted(w)
            rest += w[:free]
        bounds, n = [], 0
        for k in rest:
            n += k
            bounds.append(n)
        return n, bounds

    def _sized_budget(self) -> int:
        """The chunked-prefill budget of this step: ``chunk``, or (with a step-cost table and
        decodes riding along) the chunk that lands M on the cheap side of the GEMM staircase;
        0 = defer the prefill one step."""
        if self.cost is None or not self.mixed:
            return self.chunk
        d = self._decode_rows()
        avail, bounds = self._prefill_avail() if d else (0, [])
        if avail == 0:
            return self.chunk
        p = self.cost.choose(d, avail, self.chunk, self._pf_deferred, bounds)
        self._pf_deferred = self._pf_deferred + 1 if p == 0 else 0
        return p

    def _schedule_prefill(self) -> StepBatch | None:
        budget = self._sized_budget()
        if budget <= 0:
            return None
        chunks: list[ScheduledChunk] = []
        # 1) continue partially prefilled running requests
        for r in self.running:
            if budget <= 0:
                break
            if r.num_cached < r.seq_len - 1:
                n = self._span_safe(r, min(r.seq_len - r.num_cached, budget))
                if not self._grow(r, r.num_cached + n):
                    break
                chunks.append(ScheduledChunk(r, r.num_cached, n, r.num_cached + n == r.seq_len))
                budget -= n
        # 2) admit new requests
        if self.prefill_batch_tokens and not chunks and self.running and self.waiting:
            pending = sum(r.seq_len - r.num_cached for r in self.waiting)
            if pending < min(self.prefill_batch_tokens, budget) and \
                    not self._waited(self.waiting[0], self.prefill_max_wait_s, self.prefill_max_wait_steps):
                return None
        while self.waiting and budget > 0 and len(self.running) < self.max_running:
            r = self._next_waiting()
            if r.req_slot < 0:
                slot = self.slots.alloc()
                if slot is None:
                    break
                r.req_slot = slot
            if self.prefix_cache is not None and r.num_cached == 0 and not r.pages:
                hit_pages = self.prefix_cache.match(r.all_ids[: r.seq_len - 1], *_mm_salt(r))
                if hit_pages:
                    r.pages = list(hit_pages)
                    self.slots.set_pages(r.req_slot, 0, hit_pages)
                    r.num_cached = r.num_prefix_hit = len(hit_pages) * self.P
            n = self._span_safe(r, min(r.seq_len - r.num_cached, budget))
            if not self._grow(r, r.num_cached + n):
                if not self.running and not chunks:
                    # cannot fit even alone: fail the request instead of spinning
                    self.waiting.remove(r)
                    self._release(r)
                    r.state, r.finish_reason = ReqState.FINISHED, "abort:kv_capacity"
                    continue
                break
            self.waiting.remove(r)
            r.state = ReqState.RUNNING
            self.running.append(r)
            chunks.append(ScheduledChunk(r, r.num_cached, n, r.num_cached + n == r.seq_len))
            budget -= n
        return StepBatch("prefill", chunks) if chunks else None

    def _add_decodes(self, batch: StepBatch) -> None:
        inb = {id(c.req) for c in batch.chunks}
        for r in self.running:
            if id(r) in inb or not r.prefill_done or self._exhausted(r):
                continue
            if self._grow(r, r.seq_len):
                batch.chunks.append(ScheduledChunk(r, r.seq_len - 1, 1, True))

    def _exhausted(self, r: Request) -> bool:
        """Every token this request may produce is already scheduled (incl. in-flight ones)."""
        return len(r.output_ids) >= r.params.max_new_tokens or r.seq_len >= self.max_context

    def _schedule_decode(self) -> StepBatch | None:
        chunks = []
        for r in list(self.running):
            if r.state != ReqState.RUNNING or not r.prefill_done or self._exhausted(r):
                continue
            while not self._grow(r, r.seq_len):
                if not self._preempt_one(keep=r):
                    break
            if r.state != ReqState.RUNNING or len(r.pages) * self.P < r.seq_len:
                continue
            chunks.append(ScheduledChunk(r, r.seq_len - 1, 1, True))
        # a later request's page growth may have preempted one already picked (LIFO victim)
        chunks = [c for c in chunks if c.req.state == ReqState.RUNNING and len(c.req.pages) * self.P >= c.req.seq_len]
        return StepBatch("decode", chunks) if chunks else None

    # ------------------------------------------------------------------ post-step
    def launch_commit(self, batch: StepBatch) -> None:
        """Phase 1, right after the step is enqueued on the GPU: advance the KV watermark and
        reserve a PENDING output slot for every sampled row, so the next step can be scheduled
        (and enqueued) before this step's tokens reach the host."""
        for i, c in enumerate(batch.chunks):
            r = c.req
            r.num_cached = c.start + c.length
            if c.sample and r.state == ReqState.RUNNING:
                c.out_index = len(r.output_ids)
                r.output_ids.append(PENDING)
                r.n_pending += 1
                r.pending_row = i

    def final_commit(self, batch: StepBatch, next_ids: list[int], logprobs: list[float] | None, now: float,
                     eos_ids: set[int]) -> list[Request]:
        """Phase 2, once the step's sampled ids are on the host: fill the PENDING slots, stream
        tokens, finish requests.  A request that finishes here may already sit in the next
        in-flight step as a dead row; its trailing placeholders are dropped and its pages are
        released — safe, because everything that could reuse them is enqueued later on the
        same stream."""
        done = []
        for i, c in enumerate(batch.chunks):
            r = c.req
            if c.out_index < 0 or r.state != ReqState.RUNNING:
                continue
            r.n_pending -= 1
            tok = int(next_ids[i])
            r.output_ids[c.out_index] = tok
            if logprobs is not None:
                r.output_logprobs.append(float(logprobs[i]))
            r.token_times.append(now)
            if r.first_token_time is None:
                r.first_token_time = now
            reason = None
            p = r.params
            n_out = c.out_index + 1
            if n_out >= p.max_new_tokens:
                reason = "length"
            elif not p.ignore_eos and (tok in eos_ids or tok in p.stop_token_ids):
                reason = "stop"
            elif len(r.prompt_ids) + n_out >= self.max_context:
                reason = "length"
            if reason:
                if len(r.output_ids) > n_out:  # speculative rows already launched past the end
                    del r.output_ids[n_out:]
                    r.n_pending = 0
                    r.num_cached = min(r.num_cached, r.seq_len)
                self.finish(r, reason)
                done.append(r)
            if r.on_token is not None:
                r.on_token(r, [tok], reason is not None)
        return done

    def commit(self, batch: StepBatch, next_ids: list[int], logprobs: list[float] | None, now: float,
               eos_ids: set[int]) -> list[Request]:
        """Synchronous (non-overlapped) commit: both phases at once."""
        self.launch_commit(batch)
        return self.final_commit(batch, next_ids, logprobs, now, eos_ids)
