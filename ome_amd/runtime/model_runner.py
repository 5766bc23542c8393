"""ModelRunner: owns the model, the paged KV cache, and the decode HIP graphs.

Step inputs are packed host-side into ONE pinned int32 buffer and sent with ONE
``hipMemcpyAsync`` per step; decode steps replay a HIP graph captured per batch-size bucket
(``--cuda-graph-max-bs``, reference runtimes use e.g. ``--cuda-graph-bs 128``), so the
steady-state decode loop costs one H2D copy + one graph launch + one D2H copy of the
sampled ids.  Prefill / mixed steps run eagerly (their GPU time dwarfs launch overhead).
"""
from __future__ import annotations

import collections
import contextlib

import logging
import math
import os
import time
import zlib
from pathlib import Path

import numpy as np
import torch

from ome_amd import ops
from ome_amd.models import build_model
from ome_amd.models.common import AttnMeta, PagedKVCache, kv_cache_dtype
from ome_amd.models.config import ModelConfig
from ome_amd.parallel import state as pstate
from ome_amd.runtime.page_pool import PagePool, ReqSlotPool
from ome_amd.runtime.request import PENDING
from ome_amd.runtime.scheduler import StepBatch
from ome_amd.runtime.staging import copy_d2h, copy_h2d

log = logging.getLogger("ome_amd.runtime")

_MASK64 = (1 << 64) - 1


def _mix(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & _MASK64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _MASK64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _MASK64
    return x ^ (x >> 31)


def default_buckets(max_bs: int) -> list[int]:
    b = [1, 2, 4, 8, 12, 16, 24, 32, 40, 48, 56, 64, 80, 96, 112, 128, 144, 160, 176, 192, 208, 224, 240, 256]
    b += list(range(288, max_bs + 1, 32))
    return [x for x in b if x <= max_bs] or [max_bs]


class _DecodeBuffers:
    FIELDS_I = ("ids", "pos", "slots", "seq_lens", "req_idx", "top_k", "src", "order")
    FIELDS_F = ("temp", "top_p", "min_p", "rep", "freq", "pres")

    def __init__(self, bmax: int, device):
        self.bmax = bmax
        n = (len(self.FIELDS_I) + len(self.FIELDS_F) + 2) * bmax
        self.dev = torch.zeros(n, dtype=torch.int32, device=device)
        # two pinned host images, alternated per step: with overlapped scheduling the host fills
        # step n+1's fields while step n's copy kernel (which reads the mapped host pages when it
        # runs) may still be queued; each image is refilled only after the event of the copy that
        # last read it
        self.cuda = device.type == "cuda"
        self.hosts = [torch.zeros(n, dtype=torch.int32, pin_memory=self.cuda) for _ in range(2)]
        self.events: list = [None, None]
        self.k = 0
        self._bind()
        self.off = {}
        o = 0
        for f in self.FIELDS_I + self.FIELDS_F:
            self.off[f] = o
            o += bmax
        self.off["seeds"] = o  # 2*bmax int32 words, 8-byte aligned (bmax even or o even)

    def _bind(self) -> None:
        self.host = self.hosts[self.k]
        self.hnp = self.host.numpy()
        self.hf = self.hnp.view(np.float32)

    def next_host(self) -> None:
        """Switch to the other host image, waiting for the copy that last read it."""
        self.k ^= 1
        ev = self.events[self.k]
        if ev is not None:
            ev.synchronize()
        self._bind()

    def copied(self) -> None:
        """Call right after enqueueing the copy of the current image."""
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record()
            self.events[self.k] = ev

    def sync_images(self) -> None:
        """Make the other image equal to the current one (after a full re-initialisation)."""
        self.hosts[self.k ^ 1].numpy()[:] = self.hnp

    def view(self, name: str, bs: int) -> torch.Tensor:
        o = self.off[name]
        if name in self.FIELDS_F:
            return self.dev[o:o + bs].view(torch.float32)
        if name == "seeds":
            return self.dev[o:o + 2 * bs].view(torch.int64)
        return self.dev[o:o + bs]


class StepHandle:
    """An enqueued step: device outputs (for the next step's pending-token gather) plus the
    pinned host copies that ``result()`` waits for."""

    __slots__ = ("ids_dev", "n", "host_ids", "host_lp", "event")

    def __init__(self, ids_dev, n, host_ids, host_lp, event):
        self.ids_dev, self.n, self.host_ids, self.host_lp, self.event = ids_dev, n, host_ids, host_lp, event

    def result(self) -> tuple[list[int], list[float]]:
        if self.event is not None:
            self.event.synchronize()
        return self.host_ids[:self.n].tolist(), self.host_lp[:self.n].tolist()


def _split_balanced(chunks: list, m: int) -> list[list]:
    """Contiguous split of ``chunks`` into at most ``m`` non-empty groups of similar token count
    (chunk order kept: the concatenated outputs stay in ``chunks`` order)."""
    m = min(m, len(chunks))
    total = sum(c.length for c in chunks)
    groups, cur, acc = [], [], 0
    for i, c in enumerate(chunks):
        cur.append(c)
        acc += c.length
        left_groups = m - len(groups) - 1
        left_chunks = len(chunks) - i - 1
        if left_groups > 0 and (acc >= total * (len(groups) + 1) / m or left_chunks == left_groups):
            groups.append(cur)
            cur = []
    if cur:
        groups.append(cur)
    return groups


class ModelRunner:
    def __init__(self, cfg: ModelConfig, device: str | torch.device = "cuda", dtype=torch.bfloat16,
                 model_path: str | None = None, load_format: str = "auto", page_size: int = 16,
                 mem_fraction_static: float = 0.9, max_total_tokens: int | None = None, max_running: int = 256,
                 max_context: int = 8192, cuda_graph: bool = True, cuda_graph_max_bs: int | None = None,
                 seed: int = 0, kv_cache_dtype_name: str = "auto", cuda_graph_bs: list | None = None):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.P = page_size
        self.max_context = max_context
        self.max_running = max_running
        self.is_cuda = self.device.type == "cuda"
        t0 = time.perf_counter()
        self.model = build_model(cfg, self.device, dtype, max_positions=max_context + page_size,
                                 model_path=model_path, load_format=load_format, seed=seed)
        self.load_time = time.perf_counter() - t0
        # DP attention + expert parallelism on GPU: the device-only low-latency EP exchange makes
        # the MoE layers capturable, so the decode graphs stay on (ome_amd.parallel.ep_ll)
        self.ep_ll = False
        if pstate.get().ep_size > 1 and self.device.type == "cuda":
            from ome_amd.parallel.ep import attach_low_latency

            self.ep_ll = attach_low_latency(self.model, max(max_running, 8))
        # two-batch overlap (--enable-two-batch-overlap) on the low-latency exchange: a decode step
        # runs as two half batches on two streams, each through its own exchange, so one half's
        # dispatch / combine waits overlap the other half's attention and expert GEMMs
        self.tbo = bool(self.ep_ll and pstate.get().tbo and pstate.get().ep_ll_b is not None)
        self._tbo_stream = torch.cuda.Stream(self.device) if self.tbo else None
        self._tbo_keep: dict = {}
        self.launch_stats = collections.Counter()
        self.stateful = bool(getattr(self.model, "stateful", False))
        if self.stateful:  # recurrent (SSM) state per request slot, the padding slot included; before
            # the KV sizing below so the page budget sees it
            self.model.alloc_state(max_running + 1)
            self._ssm_cu = torch.arange(max_running + 2, dtype=torch.int32, device=self.device)
            self._ssm_zero = torch.zeros(max_running + 1, dtype=torch.int32, device=self.device)
        # ---- KV cache sizing (reference: --mem-frac 0.9, llama-3-8b-instruct-rt.yaml:59-60) ----
        tp = self.model.tp
        kv_heads, k_dim, v_dim = getattr(self.model, "kv_layout", (tp.hkv, cfg.head_dim, cfg.head_dim))
        kv_layers = getattr(self.model, "kv_layers", None)  # hybrid models: only attention layers own KV
        n_local = len(self.model.layers if kv_layers is None else kv_layers)
        if getattr(self.model, "kv_heads_per_layer", None):   # per-layer GQA (DeciLM): {layer: local heads}
            kv_heads = dict(self.model.kv_heads_per_layer)
        kv_dtype = kv_cache_dtype(kv_cache_dtype_name, dtype)
        if kv_dtype != dtype and getattr(self.model, "kv_layout", None) is not None:
            # MLA's latent cache (mla.hip) keeps the model dtype
            log.warning("--kv-cache-dtype %s is not supported by the MLA latent cache; using %s",
                        kv_cache_dtype_name, dtype)
            kv_dtype = dtype
        self.kv_dtype = kv_dtype
        # encoders own no KV at all (page bookkeeping only)
        page_bytes = max(1, PagedKVCache.bytes_per_page(n_local, kv_heads, k_dim, page_size, kv_dtype, v_dim))
        if self.is_cuda:
            # per-stream GEMM workspaces exist before the budget is read (a lazily
            # created TBO-stream workspace used to come out of the KV headroom)
            ops.reserve_stream_workspaces(self.device, [None, self._tbo_stream])
            free, total = torch.cuda.mem_get_info(self.device)
            used_by_others = total - free
            if os.environ.get("OME_KV_BUDGET_OWN") == "1":
                # several engines share this device (1-GPU rehearsals of multi-rank runs): each
                # sizes its KV from its own allocations, the fraction being its share of the device
                used_by_others = torch.cuda.memory_reserved(self.device)
            budget = total * mem_fraction_static - used_by_others - 2 * (1 << 30)
            num_pages = int(max(budget, 0) // page_bytes)
        else:
            num_pages = 4096
        max_pages_per_seq = -(-max_context // page_size) + 1
        want = max_running * max_pages_per_seq + 2
        if max_total_tokens:
            want = min(want, -(-max_total_tokens // page_size) + 2)
        num_pages = max(min(num_pages, want), max_pages_per_seq + 2)
        self.kv = PagedKVCache(cfg.num_layers, num_pages, kv_heads, k_dim, page_size, kv_dtype, self.device, v_dim,
                               layers=self.model.layers if kv_layers is None else kv_layers)
        if self.kv.is_fp8:
            self.kv.set_scales(getattr(self.model, "kv_scales", None) or {})
        self.pp = pstate.get().pp_size > 1
        self.pages = PagePool(num_pages)
        self.slots = ReqSlotPool(max_running + 1, max_pages_per_seq, self.device)
        from ome_amd.runtime.staging import H2DStaging

        self.staging = H2DStaging(self.device)
        if self.is_cuda:
            self.slots.staging = self.staging
        log.info("KV cache: %d pages x %d tokens (%.1f GiB), weights %.1f GiB", num_pages, page_size,
                 num_pages * page_bytes / 2**30, self.model.weight_bytes() / 2**30)
        # ---- decode graphs ----
        if cuda_graph_bs:   # --cuda-graph-bs: exactly these decode batch sizes get graphs
            self.bmax = max(2, min(max(cuda_graph_bs), max_running))
            self.bmax += self.bmax % 2
            self.buckets = sorted({min(int(b), self.bmax) for b in cuda_graph_bs})
        else:
            self.bmax = max(2, cuda_graph_max_bs or max_running)
            self.bmax += self.bmax % 2
            self.buckets = default_buckets(self.bmax)
        if self.buckets[-1] < self.bmax:
            self.buckets.append(self.bmax)
        if self.tbo:   # every graph splits into two non-empty halves
            self.buckets = [b for b in self.buckets if b >= 2 and b % 2 == 0]
        self.dbuf = _DecodeBuffers(self.bmax, self.device)
        self.out_ids = torch.zeros(self.bmax, dtype=torch.int32, device=self.device)
        self.out_lp = torch.zeros(self.bmax, dtype=torch.float32, device=self.device)
        # pipeline stages decode in micro-batches (stage s works on micro-batch i while stage s+1
        # works on i-1); each micro-batch slot has its own input / output buffers and graphs
        self.dbufs = [self.dbuf]
        self.mb_out = [(self.out_ids, self.out_lp)]
        # pinned landing zone for sampled ids / logprobs, double-buffered so step k+1 can be
        # enqueued while the host still reads step k (overlapped scheduling)
        nout = max(self.bmax, max_running + 8)
        self._host_out = [(torch.zeros(nout, dtype=torch.int32, pin_memory=self.is_cuda),
                           torch.zeros(nout, dtype=torch.float32, pin_memory=self.is_cuda)) for _ in range(2)]
        self._ring = 0
        self._ws_cache: dict[int, ops.DecodeWorkspace] = {}
        # penalty bookkeeping: per request slot, output-token counts | prompt/output "seen" bit
        self.counts = torch.zeros(max_running + 1, cfg.vocab_size, dtype=torch.int32, device=self.device)
        self.graphs: dict[int, torch.cuda.CUDAGraph] = {}
        self.graph_pool = None
        # pipeline stages capture their decode step when every hand-off is an IPC peer kernel
        # (pstate.pp_graph_ok: one node); across nodes they run eagerly over RCCL p2p.  DP
        # attention replays graphs only with the low-latency EP exchange (cuda_graph=None: "if possible")
        dp_ok = pstate.get().ep_size <= 1 or self.ep_ll
        # on by default since round 5 (OME_PP_GRAPHS=0: eager micro-batched steps): the r04
        # rehearsal's 25 % graph regression is gone -- graphs 10.24k vs eager 10.17k tok/s,
        # decode steps 15.9 vs 16.9 ms, interleaved on one GPU (profiles/r05_pp_graphs.md).
        # UNVERIFIED on distinct GPUs: no 2-GPU PP graphs-vs-eager run has been recorded (only the
        # 1-GPU interleaved rehearsal); OME_PP_GRAPHS=0 is the fallback if a real node disagrees
        pp_ok = not self.pp or (pstate.pp_graph_ok() and os.environ.get("OME_PP_GRAPHS", "1") == "1"
                                and not self.stateful)
        self.use_graph = bool(cuda_graph) and self.is_cuda and pp_ok and dp_ok and \
            not getattr(self.model, "encoder_only", False)
        self.mb_graphs: list[dict[int, torch.cuda.CUDAGraph]] = [self.graphs]
        if self.use_graph and self.pp:
            for _ in range(pstate.get().pp_size - 1):
                self.dbufs.append(_DecodeBuffers(self.bmax, self.device))
                self.mb_out.append((torch.zeros(self.bmax, dtype=torch.int32, device=self.device),
                                    torch.zeros(self.bmax, dtype=torch.float32, device=self.device)))
                self.mb_graphs.append({})
        if self.use_graph:
            self.capture_graphs()

    # ------------------------------------------------------------------ step-cost table
    def measure_step_cost(self, max_rows: int, grid: int = 16, reps: int = 3):
        """GEMM time of one decoder layer at M = grid, 2 grid, ... max_rows rows, routed exactly as
        the forward routes it (``model.gemm_probe``), alternating two layers so the weights come
        from HBM as in a layer stack.  Returns a :class:`~ome_amd.runtime.step_cost.StepCost`, or
        None when the model has no probe or this is not a GPU run."""
        m = self.model
        probe = getattr(m, "gemm_probe", None)
        layers = [i for i in getattr(m, "layers", range(getattr(self.cfg, "num_layers", 0)))][:2]
        widths = m.gemm_probe_widths() if probe is not None and self.is_cuda and layers else None
        if widths is None:
            return None
        try:
            return self._measure_step_cost(probe, layers, widths, max_rows, grid, reps)
        except Exception as e:  # noqa: BLE001 -- a failed probe must not take serving down
            log.warning("step-cost probe failed (%s); mixed steps use the fixed chunk size", e)
            return None

    def _measure_step_cost(self, probe, layers, widths, max_rows: int, grid: int, reps: int):
        from ome_amd.runtime.step_cost import StepCost

        h, wo = widths
        x = torch.randn(max_rows, h, device=self.device, dtype=self.dtype) * 0.5
        a = torch.randn(max_rows, wo, device=self.device, dtype=self.dtype) * 0.5
        rows, us = [], []
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        with torch.no_grad():
            for M in range(grid, max_rows + 1, grid):
                for i in layers:   # warm-up: routing plans, hipBLASLt heuristics
                    probe(i, x[:M], a[:M])
                best = float("inf")
                for _ in range(reps):
                    s.record()
                    for i in layers:
                        probe(i, x[:M], a[:M])
                    e.record()
                    e.synchronize()
                    best = min(best, s.elapsed_time(e) * 1000.0 / len(layers))
                rows.append(M)
                us.append(best)
        log.info("step-cost table: %d row counts up to %d measured in %.1fs (t(256) %.0f us, t(%d) %.0f us per layer)",
                 len(rows), max_rows, time.perf_counter() - t0, us[min(len(us), 256 // grid) - 1], rows[-1], us[-1])
        return StepCost.from_measurements(rows, us, max_rows)

    # ------------------------------------------------------------------ helpers
    def decode_ws(self, bs: int, half: int = 0) -> ops.DecodeWorkspace | None:
        """Split-K partitioning chosen so a decode launch has >= ~1024 active workgroups.
        ``half``: the two-batch-overlap halves run concurrently, so each owns a workspace."""
        if getattr(self.model, "kv_layout", None) is not None:
            return None  # MLA models carry their own workspace
        key = bs if not half else (bs, half)
        ws = self._ws_cache.get(key)
        if ws is None:
            hkv = self.model.tp.hkv
            parts = max(1, math.ceil(1024 / max(1, bs * hkv)))
            span = self.max_context + self.P  # seq_lens never exceed this: one part covers it all
            if parts > 1 and os.environ.get("OME_DECODE_DYN_PARTS", "1") == "1":
                # split each sequence by its own length (short contexts fill every partition)
                ws = ops.DecodeWorkspace(bs, self.model.tp.hq, self.cfg.head_dim, span, 0, self.device, parts=parts)
            else:
                part = max(256, -(-span // parts))
                part = -(-part // 128) * 128
                ws = ops.DecodeWorkspace(bs, self.model.tp.hq, self.cfg.head_dim, span, part, self.device)
            self._ws_cache[key] = ws
        return ws

    def _tbo_forward(self, d: "_DecodeBuffers", bs: int, bt: torch.Tensor) -> torch.Tensor:
        """Two-batch overlap of a decode step (SGLang ``--enable-two-batch-overlap``, reference
        deepseek-rdma-pd-rt.yaml:89): rows [0, h) run on the current stream through exchange A,
        rows [h, bs) on a side stream through exchange B -- attention, routing, dispatch, experts
        and combine of every layer for each half.  The halves share nothing but the (disjoint) KV
        rows they write, so whatever one half waits on (a peer's dispatch / combine flag) the
        other half's kernels fill.  In a captured graph both chains are replayed concurrently.
        Every rank runs both exchanges in every step (``ep_idle_layers`` for eager steps)."""
        st = pstate.get()
        h = bs // 2
        main = torch.cuda.current_stream(self.device)
        side = self._tbo_stream
        outs = []
        for half, (a, b) in enumerate(((0, h), (h, bs))):
            ctx = torch.cuda.stream(side) if half else contextlib.nullcontext()
            if half:
                side.wait_stream(main)
            with ctx:
                meta = AttnMeta("decode", d.view("pos", bs)[a:b], d.view("slots", bs)[a:b], bt[a:b],
                                seq_lens=d.view("seq_lens", bs)[a:b], decode_ws=self.decode_ws(b - a, half),
                                order=None)
                st.ep_ll_cur = st.ep_ll_b if half else st.ep_ll
                try:
                    outs.append(self.model.forward(d.view("ids", bs)[a:b], meta, self.kv))
                finally:
                    st.ep_ll_cur = None
        main.wait_stream(side)
        if torch.cuda.is_current_stream_capturing():
            self._tbo_keep[bs] = outs   # graph-pool memory: kept for the graph's lifetime
        else:
            outs[1].record_stream(main)
        return torch.cat(outs, 0)

    def _decode_forward(self, bs: int, m: int = 0) -> None:
        d = self.dbufs[m]
        out_ids, out_lp = self.mb_out[m]
        bt = self.slots.table.index_select(0, d.view("req_idx", bs))
        if self.tbo and bs >= 2 and not self.stateful and pstate.get().ep_ll_ok:
            hidden = self._tbo_forward(d, bs, bt)
        else:
            meta = AttnMeta("decode", d.view("pos", bs), d.view("slots", bs), bt, seq_lens=d.view("seq_lens", bs),
                            decode_ws=self.decode_ws(bs), order=d.view("order", bs))
            if self.stateful:  # one-row sequences continuing each request slot's state
                meta.extra["ssm"] = (self._ssm_cu[:bs + 1], d.view("req_idx", bs), self._ssm_zero[:bs])
            hidden = self.model.forward(d.view("ids", bs), meta, self.kv)
        if hidden is not None:   # (an earlier pipeline stage returns None: it samples nothing)
            logits = self.model.compute_logits(hidden)
            pen = (d.view("rep", bs), d.view("freq", bs), d.view("pres", bs))
            ops.apply_penalties(logits, self.counts, d.view("req_idx", bs), *pen)
            ops.sample(logits, d.view("temp", bs), d.view("top_k", bs), d.view("top_p", bs), d.view("min_p", bs),
                       d.view("seeds", bs), 0, out_ids=out_ids[:bs], out_logprob=out_lp[:bs])
            ops.update_counts(self.counts, d.view("req_idx", bs), out_ids[:bs], *pen)
        # (pipeline stages: the last stage's tokens reach every stage in ONE broadcast after all
        # micro-batches, _launch_decode -- a per-micro-batch broadcast would hold stage 0 inside
        # micro-batch i until the last stage had sampled it, serialising the pipeline)

    # ------------------------------------------------------------------ GEMM tuning
    TUNED_DIR = Path(__file__).resolve().parent.parent / "_tuned"

    def _tuning_begin(self) -> bool:
        """PyTorch TunableOp over the decode GEMM shapes: benchmarks every hipBLASLt / rocBLAS
        solution for each (M=bucket, N, K) once and persists the winners in-tree
        (``ome_amd/_tuned/tunableop_gfx950.csv``) so later starts skip tuning.  Tuning is only
        ON during the eager pre-capture pass; prefill shapes use the tuned table when present and
        the library heuristic otherwise (never tuned inside serving)."""
        if os.environ.get("OME_TUNE_GEMM", "1") != "1" or not hasattr(torch.cuda, "tunable"):
            return False
        if not getattr(self.model, "tune_gemms", True):
            return False
        tun = torch.cuda.tunable
        self.TUNED_DIR.mkdir(parents=True, exist_ok=True)
        arch = torch.cuda.get_device_properties(self.device).gcnArchName.split(":")[0]
        fname = os.environ.get("OME_TUNE_FILE") or str(self.TUNED_DIR / f"tunableop_{arch}.csv")
        tun.enable(True)
        tun.tuning_enable(True)
        tun.set_max_tuning_duration(int(os.environ.get("OME_TUNE_MS", "40")))
        tun.set_max_tuning_iterations(int(os.environ.get("OME_TUNE_ITERS", "30")))
        # decode GEMMs stream cold weights (a layer stack is far larger than the 256 MB Infinity
        # Cache): OME_TUNE_ROTATING_MB > 256 times every candidate on rotating operand copies
        rot = int(os.environ.get("OME_TUNE_ROTATING_MB", "0"))
        if rot > 0:
            tun.set_rotating_buffer_size(rot)
        if os.path.exists(fname):
            tun.read_file(fname)
        # one writer for the in-tree table: other ranks of a multi-GPU job keep their results in
        # a private file (torch writes the table at process exit)
        if int(os.environ.get("LOCAL_RANK", "0")) != 0:
            fname = os.path.join("/tmp", f"tunableop_{arch}_rank{os.environ.get('LOCAL_RANK')}_{os.getpid()}.csv")
        tun.set_filename(fname, insert_device_ordinal=False)
        self._tune_file = fname
        return True

    def _tuning_end(self) -> None:
        tun = torch.cuda.tunable
        tun.tuning_enable(False)
        # torch writes the table to the configured filename at process exit (newer releases
        # also expose write_file for an explicit flush)
        if hasattr(tun, "write_file"):
            try:
                tun.write_file(self._tune_file)
            except Exception as e:  # noqa: BLE001 — read-only tree: keep the in-memory table
                log.warning("could not persist tuned GEMM table: %s", e)

    def capture_graphs(self) -> None:
        t0 = time.perf_counter()
        tuning = self._tuning_begin()
        for d in self.dbufs:
            d.hnp[:] = 0
            d.hnp[d.off["slots"]:d.off["slots"] + d.bmax] = -1
            for name, v in (("rep", 1.0), ("top_p", 1.0)):   # neutral sampling params for the warm-up rows
                d.hf[d.off[name]:d.off[name] + d.bmax] = v
            d.hnp[d.off["top_k"]:d.off["top_k"] + d.bmax] = -1
            d.sync_images()
            d.dev.copy_(d.host)
        torch.cuda.synchronize(self.device)
        stream = torch.cuda.Stream(self.device)
        stream.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(stream), ops.decode_gemm_tuning():
            for bs in reversed(self.buckets):
                self._decode_forward(bs)  # warm-up (allocations, hipBLASLt heuristics / tuning, GEMM routing)
                log.info("decode warm-up bs=%d done at %.1fs", bs, time.perf_counter() - t0)
        torch.cuda.current_stream(self.device).wait_stream(stream)
        torch.cuda.synchronize(self.device)
        if tuning:
            self._tuning_end()
            log.info("GEMM tuning pass done in %.1fs", time.perf_counter() - t0)
        for m, graphs in enumerate(self.mb_graphs):   # (one slot unless this is a pipeline stage)
            for bs in reversed(self.buckets):
                g = torch.cuda.CUDAGraph()
                # captured on the warm-up stream: per-stream state made there (the stream-K GEMM
                # workspace) already exists, so nothing is allocated or zeroed inside the capture
                with torch.cuda.graph(g, pool=self.graph_pool, stream=stream):
                    self._decode_forward(bs, m)
                if self.graph_pool is None:
                    self.graph_pool = g.pool()
                graphs[bs] = g
        torch.cuda.synchronize(self.device)
        log.info("captured %d decode graphs in %.1fs", sum(len(g) for g in self.mb_graphs), time.perf_counter() - t0)

    @staticmethod
    def _seed(req, pos: int) -> int:
        # stable across processes (TP ranks must draw identical tokens): no str hash()
        base = req.params.seed if req.params.seed is not None else zlib.crc32(req.rid.encode())
        return _mix((base * 1000003 + pos) & _MASK64)

    # ------------------------------------------------------------------ steps
    def run(self, batch: StepBatch) -> tuple[list[int], list[float]]:
        """Synchronous step: enqueue + wait."""
        return self.launch(batch).result()

    def launch(self, batch: StepBatch, prev: "StepHandle | None" = None, allow_graph: bool = True) -> "StepHandle":
        """Enqueue one step.  Rows whose input token is PENDING (sampled by ``prev``, still in
        flight) get it on the device from ``prev``'s output — no host round trip.
        ``allow_graph=False``: run eagerly even for a decode batch (DP attention steps whose MoE
        exchange must take the normal RCCL mode on every rank)."""
        self.probe = None
        if self.probe_log is not None:
            self.probe = (time.perf_counter(), prev.event if prev is not None else None)
        self.slots.flush()
        if batch.mode == "decode" and (not self.pp or self.use_graph) and all(c.length == 1 for c in batch.chunks):
            bs = next((b for b in self.buckets if b >= len(batch.chunks)), None)
            if bs is not None:
                self.launch_stats["decode-graph" if allow_graph and self.use_graph else "decode-eager"] += 1
                return self._launch_decode(batch, bs, prev, graph=allow_graph)
        self.launch_stats[f"{batch.mode}-eager"] += 1
        return self._launch_eager(batch, prev)

    probe_log: list | None = None   # (mode, host ms from launch start to the input copy, prev step done?)
    launch_stats: "collections.Counter"   # steps launched per path (decode-graph / decode-eager / <mode>-eager)

    def _probe_mark(self, mode: str) -> None:
        if self.probe is not None:
            t0, ev = self.probe
            self.probe_log.append((mode, 1000 * (time.perf_counter() - t0), bool(ev.query()) if ev is not None else None))

    def idle_decode(self) -> None:
        """DP attention, low-latency EP: this rank has nothing scheduled while its peers decode --
        replay the smallest decode graph on one padding row (scratch slot, sequence length 0) so
        every MoE exchange has all participants."""
        d, bs = self.dbuf, self.buckets[0]
        d.next_host()
        h, off = d.hnp, d.off
        for name, v in (("ids", 0), ("slots", -1), ("seq_lens", 0), ("pos", 0), ("src", -1), ("order", 0),
                        ("top_k", -1)):
            h[off[name]:off[name] + bs] = v
        h[off["req_idx"]:off["req_idx"] + bs] = self.slots.max_reqs - 1
        for name, v in (("temp", 0.0), ("top_p", 1.0), ("min_p", 0.0), ("rep", 1.0), ("freq", 0.0), ("pres", 0.0)):
            d.hf[off[name]:off[name] + bs] = v
        copy_h2d(d.dev, d.host) if self.is_cuda else d.dev.copy_(d.host)
        d.copied()
        if self.use_graph:
            self.graphs[bs].replay()
        else:
            self._decode_forward(bs)

    def _finish_launch(self, ids_dev: torch.Tensor, lp_dev: torch.Tensor, n: int) -> "StepHandle":
        hi, hl = self._host_out[self._ring]
        self._ring ^= 1
        if n and self.is_cuda:
            copy_d2h(hi[:n], ids_dev[:n].contiguous())
            copy_d2h(hl[:n], lp_dev[:n].float().contiguous())
        elif n:
            hi[:n].copy_(ids_dev[:n])
            hl[:n].copy_(lp_dev[:n])
        ev = None
        if self.is_cuda:
            ev = torch.cuda.Event()
            ev.record()
        return StepHandle(ids_dev, n, hi, hl, ev)

    def _init_penalty_rows(self, chunks) -> None:
        """First time a penalised request runs in its slot: zero the slot's count row, mark the
        prompt (and any already-generated tokens, e.g. after a preemption) as seen."""
        for c in chunks:
            r = c.req
            if r.pen_init or not r.params.has_penalties or r.req_slot < 0:
                continue
            row = self.counts[r.req_slot]
            row.zero_()
            seen = [t for t in r.prompt_ids]
            outs = [t for t in r.output_ids if t != PENDING]
            if seen:
                row[torch.tensor(seen, dtype=torch.long, device=self.device)] = ops.reference.SEEN_BIT
            if outs:
                oc = np.bincount(np.asarray(outs), minlength=self.cfg.vocab_size)
                nz = np.nonzero(oc)[0]
                idx = torch.from_numpy(nz).to(self.device)
                row[idx] = torch.from_numpy(oc[nz].astype(np.int32)).to(self.device) | ops.reference.SEEN_BIT
            r.pen_init = True

    @staticmethod
    def _src_row(r, pos: int, prev: "StepHandle | None") -> int:
        """Row of ``prev``'s sampled output holding the token at ``pos`` if it is pending."""
        if prev is None or not r.n_pending or pos != r.seq_len - 1 or r.token_at(pos) != PENDING:
            return -1
        return r.pending_row

    def _launch_decode(self, batch: StepBatch, bs: int, prev: "StepHandle | None",
                       graph: bool = True) -> "StepHandle":
        B = len(batch.chunks)
        n_mb = min(self.pp_microbatches or len(self.mb_graphs), len(self.mb_graphs), B) if self.pp else 1
        if n_mb > 1 and self.use_graph and graph:
            # pipeline stage: micro-batch i's graph (receive, layers, send, token broadcast) runs
            # while the next stage still works on micro-batch i-1
            ids, lps = [], []
            for m, part in enumerate(_split_balanced(batch.chunks, n_mb)):
                bs_m = next(b for b in self.buckets if b >= len(part))
                self._fill_decode(self.dbufs[m], part, bs_m, prev)
                self.mb_graphs[m][bs_m].replay()
                ids.append(self.mb_out[m][0][:len(part)])
                lps.append(self.mb_out[m][1][:len(part)])
            out_ids, out_lp = torch.cat(ids), torch.cat(lps)
            pstate.pp_broadcast_tokens(out_ids, out_lp)
            return self._finish_launch(out_ids, out_lp, B)
        self._fill_decode(self.dbuf, batch.chunks, bs, prev)
        if self.use_graph and graph:
            self.graphs[bs].replay()
        else:
            self._decode_forward(bs)
        if self.pp:
            pstate.pp_broadcast_tokens(self.out_ids[:B], self.out_lp[:B])
        return self._finish_launch(self.out_ids, self.out_lp, B)

    def _fill_decode(self, d: "_DecodeBuffers", chunks, bs: int, prev: "StepHandle | None") -> None:
        """Host-side fields of a decode (micro-)batch -> ``d``'s pinned image -> one H2D copy."""
        B = len(chunks)
        d.next_host()
        h, hf, off = d.hnp, d.hf, d.off
        h[off["ids"]:off["ids"] + bs] = 0
        h[off["slots"]:off["slots"] + bs] = -1
        h[off["seq_lens"]:off["seq_lens"] + bs] = 0
        h[off["req_idx"]:off["req_idx"] + bs] = self.slots.max_reqs - 1
        h[off["pos"]:off["pos"] + bs] = 0
        h[off["src"]:off["src"] + bs] = -1
        seeds = h[off["seeds"]:off["seeds"] + 2 * bs].view(np.uint64)
        any_pending = False
        P = self.P
        toks, poss, slots, lens, rsl, srcs, sds = [], [], [], [], [], [], []
        tk, tmp, tp, mp, rep, frq, prs = [], [], [], [], [], [], []
        for c in chunks:  # python lists, one numpy store per field (not per element)
            r = c.req
            pos = c.start
            src = self._src_row(r, pos, prev)
            if src >= 0:
                any_pending = True
                toks.append(0)
            else:
                toks.append(r.token_at(pos))
            srcs.append(src)
            poss.append(pos + (r.mm.rope_delta if r.mm is not None else 0))  # M-RoPE text offset
            slots.append(r.pages[pos // P] * P + pos % P)
            lens.append(pos + 1)
            rsl.append(r.req_slot)
            p = r.params
            tk.append(p.top_k)
            tmp.append(p.temperature)
            tp.append(p.top_p)
            mp.append(p.min_p)
            rep.append(p.repetition_penalty)
            frq.append(p.frequency_penalty)
            prs.append(p.presence_penalty)
            sds.append(self._seed(r, pos + 1))  # keyed by the position of the token being drawn
        for name, vals in (("ids", toks), ("src", srcs), ("pos", poss), ("slots", slots), ("seq_lens", lens),
                           ("req_idx", rsl), ("top_k", tk)):
            h[off[name]:off[name] + B] = vals
        for name, vals in (("temp", tmp), ("top_p", tp), ("min_p", mp), ("rep", rep), ("freq", frq),
                           ("pres", prs)):
            hf[off[name]:off[name] + B] = vals
        seeds[:B] = np.asarray(sds, dtype=np.uint64)
        if bs > B:  # neutral sampling parameters on the padding rows
            for name, v in (("temp", 0.0), ("top_p", 1.0), ("rep", 1.0), ("freq", 0.0), ("pres", 0.0)):
                hf[off[name] + B:off[name] + bs] = v
            h[off["top_k"] + B:off["top_k"] + bs] = -1
        # attention visits sequences longest-first (padding rows, seq_len 0, last)
        h[off["order"]:off["order"] + bs] = np.argsort(-h[off["seq_lens"]:off["seq_lens"] + bs], kind="stable")
        self._init_penalty_rows(chunks)
        self._probe_mark("decode")
        copy_h2d(d.dev, d.host) if self.is_cuda else d.dev.copy_(d.host)
        d.copied()
        if any_pending:
            ops.fill_pending(d.view("ids", bs), d.view("src", bs), prev.ids_dev)

    pp_microbatches = 0   # pipeline parallel: micro-batches per step (0 = one per stage)

    def _launch_eager(self, batch: StepBatch, prev: "StepHandle | None") -> "StepHandle":
        """Eager step for prefill / mixed batches (and every step of a pipeline-parallel engine).

        Pipeline parallel: the step's chunks are cut into token-balanced micro-batches that run
        through the stages back to back -- each stage's stream holds [forward mb0, send mb0,
        forward mb1, send mb1, ...] and the stage-to-stage hand-offs are stream-ordered RCCL
        p2p, so stage s works on micro-batch i while stage s+1 works on micro-batch i-1.  The
        sampled tokens of all micro-batches return in ONE broadcast from the last stage, issued
        after every micro-batch (a per-micro-batch broadcast would stall stage 0 on the last
        stage's sampling of micro-batch 0 and serialise the pipeline)."""
        chunks = batch.chunks
        m = self.pp_microbatches or pstate.get().pp_size
        if self.pp and m > 1 and len(chunks) > 1:
            outs = [self._eager_forward(g, prev, batch.mode) for g in _split_balanced(chunks, m)]
            out_ids = torch.cat([o[0] for o in outs])
            out_lp = torch.cat([o[1].float() for o in outs])
        else:
            out_ids, out_lp = self._eager_forward(chunks, prev, batch.mode)
        if self.pp:
            pstate.pp_broadcast_tokens(out_ids, out_lp)
        return self._finish_launch(out_ids, out_lp, len(chunks))

    def _eager_forward(self, chunks, prev: "StepHandle | None", mode: str) -> tuple[torch.Tensor, torch.Tensor]:
        """One eager forward over ``chunks``: (sampled ids int32, log-probs fp32) in chunk order;
        on an earlier pipeline stage, empty tensors the last stage's broadcast fills.  Token rows
        are laid out prefill chunks first, then single-token rows (decodes riding along, or
        1-token prompt tails), which attention routes to the decode kernel."""
        P = self.P
        pre = [i for i, c in enumerate(chunks) if c.length > 1]
        dec = [i for i, c in enumerate(chunks) if c.length == 1]
        ids, pos, slots, q_lens, kv_lens, req_idx, src = [], [], [], [], [], [], []
        dec_lens, dec_req = [], []
        last_row = [0] * len(chunks)
        any_pending = False
        for i in pre + dec:
            c = chunks[i]
            r = c.req
            t0 = len(ids)
            a, n = c.start, c.length
            pages = r.pages
            if n > 1:
                ids.extend(r.ids_range(a, a + n))
                src.extend([-1] * n)
                pp = np.arange(a, a + n, dtype=np.int64)
                pos.append(pp)
                slots.append(np.asarray(pages, np.int64)[pp // P] * P + pp % P)
                q_lens.append(n)
                kv_lens.append(a + n)
                req_idx.append(r.req_slot)
            else:
                ids.append(r.token_at(a))
                src.append(-1)
                pos.append(a)
                slots.append(pages[a // P] * P + a % P)
                dec_lens.append(a + 1)
                dec_req.append(r.req_slot)
            s_row = self._src_row(r, a + n - 1, prev)
            if s_row >= 0:
                src[t0 + n - 1] = s_row
                ids[t0 + n - 1] = 0
                any_pending = True
            last_row[i] = len(ids) - 1
        tp_ = self.model.tp
        # 64-row items only when EVERY attention layer has the qualifying shape (DeciLM varies
        # its kv heads per layer; the plan is shared by all layers)
        hkvs = set(getattr(self.model, "kv_heads_per_layer", {}).values()) | {tp_.hkv}
        rows = ops.prefill_rows(tp_.hq, tp_.hkv, self.cfg.head_dim, P) if len(hkvs) == 1 else 32
        items, split, comb, chunk, parts = ops.prefill_plan(q_lens, kv_lens, tile=rows, kv_heads=tp_.hkv) if q_lens \
            else ([], [], [], 0, 0)
        T, S, n_it, nd, B = len(ids), len(q_lens), len(items), len(dec_lens), len(chunks)
        n_sp, n_cb = len(split), len(comb)
        cu = np.zeros(S + 1, dtype=np.int32)
        cu[1:] = np.cumsum(q_lens)
        dec_order = np.argsort(-np.asarray(dec_lens, np.int64), kind="stable").astype(np.int32) if nd else \
            np.zeros(0, np.int32)

        def flat(parts):  # per-chunk numpy arrays (prefill) and scalars (single-token rows)
            return np.concatenate([np.atleast_1d(np.asarray(x)).astype(np.int32) for x in parts]) if parts else \
                np.zeros(0, np.int32)

        # sampling parameters ride in the same pinned H2D copy: int64 seeds first (8-B aligned),
        # then fp32 fields as raw 32-bit words
        sv = [self._seed(c.req, c.start + c.length) for c in chunks]
        seeds = np.asarray([v - (1 << 64) if v >= (1 << 63) else v for v in sv], np.int64).view(np.int32)
        fp = np.asarray([[c.req.params.temperature, c.req.params.top_p, c.req.params.min_p] for c in chunks],
                        np.float32).T.copy().view(np.int32).reshape(-1)
        top_k = np.asarray([c.req.params.top_k for c in chunks], np.int32)
        packed = np.concatenate([seeds, fp, top_k, np.asarray(ids, np.int32), flat(pos), flat(slots),
                                 cu, np.asarray(kv_lens, np.int32), np.asarray(req_idx, np.int32),
                                 np.asarray(last_row, np.int32), np.asarray(src, np.int32),
                                 np.asarray(dec_lens, np.int32), np.asarray(dec_req, np.int32), dec_order,
                                 np.asarray(items, np.int32).reshape(-1) if n_it else np.zeros(0, np.int32),
                                 np.asarray(split, np.int32).reshape(-1) if n_sp else np.zeros(0, np.int32),
                                 np.asarray(comb, np.int32).reshape(-1) if n_cb else np.zeros(0, np.int32)])
        self._probe_mark(mode)
        dev = self.staging.to_device(packed)
        o = 0

        def take(n):
            nonlocal o
            t = dev[o:o + n]
            o += n
            return t

        t_seeds = take(2 * B).view(torch.int64)
        t_temp, t_top_p, t_min_p = (take(B).view(torch.float32) for _ in range(3))
        t_top_k = take(B)
        t_ids, t_pos, t_slots = take(T), take(T), take(T)
        t_cu, t_kv, t_req, t_rows = take(S + 1), take(S), take(S), take(B)
        t_src = take(T)
        t_dlen, t_dreq, t_dord = take(nd), take(nd), take(nd)
        t_items = take(2 * n_it).view(n_it, 2)
        if n_sp:   # split-KV prefill attention (ops.prefill_plan)
            t_items = ops.PrefillPlan(t_items, take(4 * n_sp).view(n_sp, 4), take(4 * n_cb).view(n_cb, 4), chunk,
                                      parts, rows)
        elif rows != 32 and n_it:   # 64-row classic items (the 8-wave kernel)
            t_items = ops.PrefillPlan(t_items, t_items[:0], t_items[:0], 0, 0, rows)
        if any_pending:
            ops.fill_pending(t_ids, t_src, prev.ids_dev)
        ws = None
        if nd:
            bucket = next((b for b in self.buckets if b >= nd), None)
            ws = self.decode_ws(bucket if bucket is not None else nd)
        if S and nd:
            meta = AttnMeta("mixed", t_pos, t_slots, self.slots.table.index_select(0, t_req), seq_lens=t_dlen,
                            cu_q=t_cu, kv_lens=t_kv, items=t_items, decode_ws=ws, order=t_dord,
                            num_prefill=int(cu[-1]), dec_block_tables=self.slots.table.index_select(0, t_dreq))
        elif S:
            meta = AttnMeta("prefill", t_pos, t_slots, self.slots.table.index_select(0, t_req), cu_q=t_cu,
                            kv_lens=t_kv, items=t_items)
        else:
            meta = AttnMeta("decode", t_pos, t_slots, self.slots.table.index_select(0, t_dreq), seq_lens=t_dlen,
                            decode_ws=ws, order=t_dord)
        self._init_penalty_rows(chunks)
        if self.stateful:  # sequences in row order: prefill chunks, then single-token rows
            lens = [chunks[i].length for i in pre + dec]
            cu_s = np.zeros(len(lens) + 1, dtype=np.int32)
            cu_s[1:] = np.cumsum(lens)
            sl = np.asarray([chunks[i].req.req_slot for i in pre + dec], np.int32)
            rs = np.asarray([int(chunks[i].start == 0) for i in pre + dec], np.int32)
            pk = torch.from_numpy(np.concatenate([cu_s, sl, rs])).to(self.device, non_blocking=True)
            S_ = len(lens)
            meta.extra["ssm"] = (pk[:S_ + 1], pk[S_ + 1:2 * S_ + 1], pk[2 * S_ + 1:])
        embeds = None
        if hasattr(self.model, "prepare_chunks"):  # e.g. Mllama: vision tower + vision-token cache at first chunks
            self.model.prepare_chunks([chunks[i] for i in pre + dec])
        if getattr(self.model, "is_multimodal", False) and not getattr(self.model, "mm_cross", False) and \
                any(chunks[i].req.mm is not None for i in pre + dec):
            embeds = self._mm_prepare(chunks, pre + dec, T, t_ids, meta)
        hidden = self.model.forward(t_ids, meta, self.kv, embeds)
        self._tbo_idle()
        if hidden is None:  # an earlier pipeline stage: tokens arrive from the last stage
            return (torch.empty(len(chunks), dtype=torch.int32, device=self.device),
                    torch.empty(len(chunks), dtype=torch.float32, device=self.device))
        logits = self.model.compute_logits(hidden.index_select(0, t_rows))
        pen = None
        if any(c.req.params.has_penalties for c in chunks):
            pen = [torch.tensor([getattr(c.req.params, f) for c in chunks], dtype=torch.float32)
                   for f in ("repetition_penalty", "frequency_penalty", "presence_penalty")]
            pslot = torch.tensor([c.req.req_slot for c in chunks], dtype=torch.int32)
            if self.is_cuda:
                pen = [x.to(self.device, non_blocking=True) for x in pen]
                pslot = pslot.to(self.device, non_blocking=True)
            # only rows that sample a token this step are penalised/counted
            sample_mask = torch.tensor([c.sample for c in chunks], dtype=torch.bool)
            if not bool(sample_mask.all()):
                keep = sample_mask.to(pen[0].device)
                pen[0] = torch.where(keep, pen[0], torch.ones_like(pen[0]))
                pen[1] = torch.where(keep, pen[1], torch.zeros_like(pen[1]))
                pen[2] = torch.where(keep, pen[2], torch.zeros_like(pen[2]))
            ops.apply_penalties(logits, self.counts, pslot, *pen)
        out_ids, out_lp = ops.sample(logits, t_temp, t_top_k, t_top_p, t_min_p, t_seeds, 0)
        out_ids = out_ids.to(torch.int32)
        if pen is not None:
            ops.update_counts(self.counts, pslot, out_ids, *pen)
        return out_ids, out_lp.float().contiguous()

    def _mm_prepare(self, chunks, order, T: int, t_ids: torch.Tensor, meta: AttnMeta):
        """Multimodal rows of an eager step: per-row 3D M-RoPE positions -> a row-indexed cos/sin
        table (``meta.extra['rope']``), and the input embeddings with every image-placeholder row
        replaced by its vision feature (vision tower run once per request, at the first chunk
        that reaches one of its images; freed once the prompt is fully cached)."""
        m = self.model
        p3 = np.empty((3, T), dtype=np.int64)
        bidir = getattr(m, "bidirectional_images", False)
        hi_rows = np.full(T, -1, dtype=np.int32) if bidir else None   # last visible key per row (image blocks)
        rows, feats, row = [], [], 0
        deep: list[list[torch.Tensor]] = []
        for i in order:
            c = chunks[i]
            r, L = c.req, c.length
            xs = np.arange(c.start, c.start + L)
            mm = r.mm
            if mm is None:
                p3[:, row:row + L] = xs
            else:
                plen = len(r.prompt_ids)
                if mm.mrope_pos is None:  # plain 1D positions (Llama 4)
                    p3[:, row:row + L] = xs
                else:
                    blk = np.empty((3, L), dtype=np.int64)
                    inside = xs < plen
                    blk[:, inside] = mm.mrope_pos[:, xs[inside]]
                    blk[:, ~inside] = xs[~inside] + mm.rope_delta
                    p3[:, row:row + L] = blk
                off = 0
                for s, n in mm.spans:
                    lo, hi = max(s, c.start), min(s + n, c.start + L)
                    if lo < hi:
                        if mm.features is None:
                            mm.features = m.encode_images(mm.pixel_values, mm.grid_thw)
                        rows.extend(range(row + lo - c.start, row + hi - c.start))
                        main = mm.features[0] if isinstance(mm.features, tuple) else mm.features
                        feats.append(main[off + lo - s: off + hi - s])
                        if isinstance(mm.features, tuple):   # (main, [deepstack level features]) -- Qwen3-VL
                            for lvl, d in enumerate(mm.features[1]):
                                if len(deep) <= lvl:
                                    deep.append([])
                                deep[lvl].append(d[off + lo - s: off + hi - s])
                        if bidir:
                            hi_rows[row + lo - c.start:row + hi - c.start] = s + n - 1
                    off += n
                if c.start + L >= plen:
                    mm.features = None  # prompt fully scheduled: image features no longer needed
            row += L
        dv = self.device
        if bidir:
            meta.extra["row_hi"] = torch.from_numpy(hi_rows).to(dv)
        if any(chunks[i].req.mm is not None and chunks[i].req.mm.mrope_pos is not None for i in order):
            meta.extra["rope"] = (torch.arange(T, dtype=torch.int32, device=dv), m.mrope_table(torch.from_numpy(p3)))
        r_dev = torch.tensor(rows, dtype=torch.long, device=dv)
        if deep:
            meta.extra["deepstack"] = (r_dev, [torch.cat(d, 0) for d in deep])
        f = torch.cat(feats, 0) if feats else torch.zeros(0, m.cfg.hidden_size, dtype=m.dtype, device=dv)
        return m.embed_with_images(t_ids, r_dev, f)

    def idle_forward(self) -> None:
        """DP attention: this rank has nothing scheduled but its peers do -- run one dummy token
        (scratch page 0) through the model so every MoE all-to-all has all participants."""
        dv = self.device
        z = torch.zeros(1, dtype=torch.int32, device=dv)
        meta = AttnMeta("prefill", z, z.clone(), torch.zeros(1, 1, dtype=torch.int32, device=dv),
                        cu_q=torch.tensor([0, 1], dtype=torch.int32, device=dv),
                        kv_lens=torch.ones(1, dtype=torch.int32, device=dv),
                        items=torch.zeros(1, 2, dtype=torch.int32, device=dv))
        if self.stateful:
            pad = self.slots.max_reqs - 1
            meta.extra["ssm"] = (self._ssm_cu[:2], torch.full((1,), pad, dtype=torch.int32, device=dv),
                                 torch.ones(1, dtype=torch.int32, device=dv))
        self.model.forward(z, meta, self.kv)
        self._tbo_idle()

    def _tbo_idle(self) -> None:
        """Two-batch overlap, eager (prefill / mixed / idle) step on the low-latency exchange: the
        peers that decode split their rows over exchanges A and B, so this rank takes part in B's
        exchanges too (no tokens of its own; it still computes the experts for rows sent to it)."""
        st = pstate.get()
        if self.tbo and st.ep_ll_ok:
            from ome_amd.parallel.ep import ep_idle_layers

            ep_idle_layers(self.model, st.ep_ll_b)

    def embed(self, batch: StepBatch) -> list[list[float]]:
        """Embedding models (``--is-embedding``): last-token pooling + L2 norm over full prompts
        (model-specific pooling / heads via ``model.pool``; image requests of models with
        ``embed_images``, e.g. CLIP, go through the vision side in one batch)."""
        self.slots.flush()  # block-table rows of the newly admitted requests
        m = self.model
        if hasattr(m, "embed_images") and any(c.req.mm is not None for c in batch.chunks):
            img = [k for k, c in enumerate(batch.chunks) if c.req.mm is not None]
            txt = [k for k, c in enumerate(batch.chunks) if c.req.mm is None]
            res: list = [None] * len(batch.chunks)
            e = m.embed_images(torch.cat([batch.chunks[k].req.mm.pixel_values for k in img]))
            for k, v in zip(img, e.cpu().tolist()):
                res[k] = v
            if txt:
                for k, v in zip(txt, self.embed(StepBatch(batch.mode, [batch.chunks[k] for k in txt]))):
                    res[k] = v
            return res
        P = self.P
        ids, pos, slots, q_lens, req_idx = [], [], [], [], []
        for c in batch.chunks:
            r = c.req
            ids.extend(r.prompt_ids)
            pos.extend(range(len(r.prompt_ids)))
            slots.extend(r.pages[x // P] * P + x % P for x in range(len(r.prompt_ids)))
            q_lens.append(len(r.prompt_ids))
            req_idx.append(r.req_slot)
        cu = [0]
        for q in q_lens:
            cu.append(cu[-1] + q)
        items = ops.prefill_work_items(q_lens, q_lens)
        dv = self.device
        t = lambda a: torch.tensor(a, dtype=torch.int32, device=dv)  # noqa: E731
        bt = self.slots.table.index_select(0, t(req_idx))
        meta = AttnMeta("prefill", t(pos), t(slots), bt, cu_q=t(cu), kv_lens=t(q_lens),
                        items=t(items).view(-1, 2) if items else torch.zeros(0, 2, dtype=torch.int32, device=dv))
        meta.extra["lengths"] = q_lens  # host copy (encoders' varlen attention work items)
        t_ids = t(ids)
        embeds = None
        if getattr(m, "is_multimodal", False) and not getattr(m, "mm_cross", False) and \
                any(c.req.mm is not None for c in batch.chunks):
            # VLM embedders (GME-Qwen2-VL): image features + M-RoPE positions of whole prompts
            from types import SimpleNamespace

            whole = [SimpleNamespace(req=c.req, start=0, length=len(c.req.prompt_ids)) for c in batch.chunks]
            embeds = self._mm_prepare(whole, list(range(len(whole))), len(ids), t_ids, meta)
        hidden = self.model.forward(t_ids, meta, self.kv, embeds) if embeds is not None else \
            self.model.forward(t_ids, meta, self.kv)
        pool = getattr(self.model, "pool", None)  # classification / reward heads (models/decoder.py)
        out = pool(hidden, t(cu)) if pool is not None else ops.pool(hidden, t(cu), 0, True)
        return out.cpu().tolist()
