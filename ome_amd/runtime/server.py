"""OpenAI-compatible HTTP server of the first-party runtime (the engine container of an ISVC).

Endpoints (the contract the reference's runtime catalog and probes rely on,
``config/runtimes/srt/meta/llama-3-8b-instruct-rt.yaml:76-102``): ``/v1/chat/completions``,
``/v1/completions``, ``/v1/embeddings``, ``/v1/models``, ``/generate``, ``/health``,
``/health_generate`` (a real 1-token generation), ``/metrics`` (SGLang + vLLM metric names),
``/get_model_info``, ``/get_server_info``; plus the PD-disaggregation KV bootstrap routes.

CLI flags follow SGLang's names so ServingRuntime YAML and the operator's TP/PP rewrite
keep working: ``--model-path --served-model-name --tp-size --pp-size --dp-size --mem-frac
--context-length --chunked-prefill-size --page-size --max-running-requests --port --host
--enable-metrics --is-embedding --disable-radix-cache --disable-cuda-graph --cuda-graph-max-bs
--dist-init-addr --nnodes --node-rank --disaggregation-mode ...``; unknown flags are logged and
ignored.  Tensor parallelism: one process per GPU (rank 0 serves HTTP, other ranks run the
engine loop in lockstep), torch.distributed over RCCL.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import logging
import os
import sys
import threading
import time
import uuid

from fastapi import Request  # noqa: E402  (module level: FastAPI resolves string annotations here)

log = logging.getLogger("ome_amd.server")


_IMG_SENTINEL = "\x00<ome-image>\x00"  # stands in for an image content part while the chat template renders


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser("ome_amd.runtime.server")
    a = ap.add_argument
    a("--model-path", "--model", dest="model_path", default=os.environ.get("MODEL_PATH"))
    a("--model-preset", default=None, help="random-init architecture preset when model-path has no config")
    a("--served-model-name", default=os.environ.get("SERVED_MODEL_NAME"))
    a("--tp-size", "--tp", "--tensor-parallel-size", dest="tp_size", type=int, default=1)
    a("--pp-size", "--pp", "--pipeline-parallel-size", dest="pp_size", type=int, default=1)
    a("--pp-microbatches", type=int, default=0,
      help="pipeline parallel: micro-batches per step that flow through the stages back to back (0 = pp size)")
    a("--dp-size", "--dp", "--data-parallel-size", dest="dp_size", type=int, default=1)
    a("--mem-frac", "--mem-fraction-static", "--gpu-memory-utilization", dest="mem_frac", type=float, default=0.88)
    a("--context-length", "--max-model-len", dest="context_length", type=int, default=None)
    a("--chunked-prefill-size", type=int, default=8192)
    a("--page-size", type=int, default=16)
    a("--max-running-requests", "--max-num-seqs", dest="max_running_requests", type=int, default=256)
    a("--max-total-tokens", type=int, default=None)
    a("--host", default="0.0.0.0")
    a("--port", type=int, default=8080)
    a("--enable-metrics", action="store_true")
    a("--is-embedding", action="store_true")
    a("--disable-radix-cache", action="store_true")
    a("--disable-cuda-graph", action="store_true")
    a("--disable-overlap-schedule", action="store_true")
    a("--cuda-graph-max-bs", type=int, default=None)
    a("--enable-mixed-chunk", action="store_true", default=True)
    a("--disable-mixed-chunk", dest="enable_mixed_chunk", action="store_false")
    a("--load-format", default="auto")
    a("--dtype", default="bfloat16")
    a("--kv-cache-dtype", default="auto")
    a("--enable-dp-attention", action="store_true",
      help="--dp N with --tp N: attention/dense layers data-parallel per rank, MoE experts expert-parallel")
    a("--moe-a2a-backend", default="rccl", help="expert-parallel dispatch backend (rccl all-to-all over xGMI)")
    a("--enable-two-batch-overlap", action="store_true",
      help="EP MoE: split tokens into two micro-batches, overlap their all-to-alls with expert compute")
    a("--enable-eplb", action="store_true", help="expert-parallel load balancing (re-place experts from loads)")
    a("--ep-num-redundant-experts", type=int, default=0, help="EPLB: replicas of hot experts across EP ranks")
    a("--eplb-rebalance-num-iterations", type=int, default=1000, help="EPLB: lockstep steps between rebalances")
    a("--eplb-algorithm", default="deepseek", help="accepted for SGLang runtime compatibility (one algorithm)")
    a("--ep-dispatch-algorithm", default="dynamic", help="accepted for SGLang runtime compatibility")
    a("--quantization", default=None, help="fp8: W8A8 projections (per-channel online, or the checkpoint's blocks)")
    a("--random-seed", type=int, default=0)
    a("--device", default="cuda")
    a("--dist-init-addr", "--nccl-init", dest="dist_init_addr", default=None)
    a("--nnodes", type=int, default=1)
    a("--distributed-executor-backend", dest="distributed_executor_backend", default=None,
      help="vLLM spelling; 'ray': the group spans the nodes of a RayCluster (ome_amd.raylet)")
    a("--node-rank", type=int, default=0)
    a("--disaggregation-mode", default="null", choices=["null", "prefill", "decode"])
    a("--disaggregation-bootstrap-port", type=int, default=8998)
    a("--log-requests", action="store_true")
    a("--num-layers", type=int, default=None, help="debug: truncate the model")
    a("--tool-call-parser", default=None,
      help="llama3_json | pythonic | qwen3_coder | hermes | qwen25 | nano_v3 | gpt-oss | mistral")
    a("--reasoning-parser", default=None, help="deepseek-r1 | qwen3 | nano_v3 | gpt-oss")
    a("--enable-auto-tool-choice", action="store_true", help="accepted (tool_choice=auto is the default)")
    a("--chat-template", default=None, help="path of a Jinja chat template replacing the tokenizer's")
    # ---- the rest of the reference runtimes' flags (ome_amd/runtime/flags.py has the table)
    a("--tokenizer-path", default=None, help="tokenizer directory / file (default: the model's)")
    a("--grpc-mode", action="store_true",
      help="serve sglang.grpc.scheduler.SglangScheduler + grpc.health.v1 over gRPC on --port (no HTTP)")
    a("--watchdog-timeout", type=float, default=300.0,
      help="seconds an engine phase may take before the process exits non-zero (0 disables)")
    a("--log-requests-level", type=int, default=0, choices=[0, 1, 2, 3])
    a("--max-log-len", type=int, default=None, help="truncate logged request text to this many characters")
    a("--log-level", default="info")
    a("--middleware", action="append", default=[], help="vllm...middleware.log_opc_header only")
    a("--cuda-graph-bs", nargs="+", type=int, default=None, help="decode batch sizes captured as HIP graphs")
    a("--cuda-graph-sizes", nargs="+", type=int, default=None, help="vLLM spelling of --cuda-graph-bs")
    a("--enforce-eager", action="store_true", help="vLLM spelling of --disable-cuda-graph")
    a("--enable-dp-lm-head", action="store_true", help="requires --enable-dp-attention (per-rank LM head)")
    a("--moe-dense-tp-size", type=int, default=None, help="only 1, with --enable-dp-attention")
    a("--load-balance-method", default="shortest_queue", choices=["round_robin", "shortest_queue", "minimum_tokens"])
    a("--prefill-round-robin-balance", action="store_true")
    a("--preemption-mode", default="recompute", choices=["recompute", "swap"])
    a("--limit-mm-per-prompt", default=None, help="image=N (or JSON {\"image\": N})")
    a("--deepep-mode", default="auto", choices=["auto", "normal", "low_latency"])
    a("--enable-deepep-moe", action="store_true", help="older spelling of --moe-a2a-backend deepep")
    a("--decode-log-interval", type=int, default=0, help="log decode throughput every N decode steps (0: off)")
    # accepted with no effect on purpose (reasons: ome_amd/runtime/flags.py)
    a("--trust-remote-code", action="store_true")
    a("--skip-server-warmup", action="store_true")
    a("--enable-chunked-prefill", action="store_true")
    a("--enable-multimodal", action="store_true")
    a("--disable-fast-image-processor", action="store_true")
    a("--attention-backend", default=None)
    a("--mm-attention-backend", default=None)
    a("--enable-torch-compile", action="store_true")
    a("--torch-compile-max-bs", type=int, default=None)
    a("--disable-shared-experts-fusion", action="store_true")
    a("--disaggregation-ib-device", default=None)
    return ap


def validate_args(ns, ap: argparse.ArgumentParser | None = None) -> None:
    """Reject reference flag values this framework cannot honour (instead of silently serving
    something else); normalise aliases.  ``ap.error`` exits 2 like any argparse error."""
    def bad(msg):
        if ap is not None:
            ap.error(msg)
        raise ValueError(msg)

    if ns.enable_dp_lm_head and not ns.enable_dp_attention:
        bad("--enable-dp-lm-head requires --enable-dp-attention")
    if ns.moe_dense_tp_size not in (None, 1):
        bad(f"--moe-dense-tp-size {ns.moe_dense_tp_size}: only 1 is supported (dense MLPs data-parallel)")
    if ns.moe_dense_tp_size == 1 and not ns.enable_dp_attention and ns.tp_size > 1:
        bad("--moe-dense-tp-size 1 requires --enable-dp-attention (dense layers are tensor-parallel otherwise)")
    for m in ns.middleware:
        if not m.endswith("log_opc_header"):
            bad(f"--middleware {m}: only the opc-request-id logging middleware is available")
    if ns.enable_deepep_moe:
        ns.moe_a2a_backend = "deepep"
    if ns.enforce_eager:
        ns.disable_cuda_graph = True
    if ns.cuda_graph_bs is None and ns.cuda_graph_sizes:
        ns.cuda_graph_bs = ns.cuda_graph_sizes
    if ns.cuda_graph_bs and min(ns.cuda_graph_bs) <= 0:
        bad("--cuda-graph-bs: batch sizes must be positive")
    if ns.limit_mm_per_prompt is not None:
        ns.mm_limit = parse_mm_limit(ns.limit_mm_per_prompt)
        if ns.mm_limit is None:
            bad(f"--limit-mm-per-prompt {ns.limit_mm_per_prompt!r}: expected image=N or JSON")
    else:
        ns.mm_limit = None
    if ns.preemption_mode == "swap":
        log.info("--preemption-mode swap: preempted requests recompute (KV swap to host is not implemented; "
                 "288 GB of HBM keeps preemption rare)")


def parse_mm_limit(v: str) -> int | None:
    """``image=4`` / ``{"image": 4}`` -> 4 (max images per prompt)."""
    v = v.strip()
    try:
        if v.startswith("{"):
            d = json.loads(v)
            return int(d.get("image", d.get("images")))
        k, _, n = v.partition("=")
        if k.strip() in ("image", "images"):
            return int(n)
    except (ValueError, TypeError, json.JSONDecodeError):
        return None
    return None


def engine_args_from(ns, rank_tp: int | None = None):
    from ome_amd.runtime.engine import EngineArgs

    mp = ns.model_path
    preset = ns.model_preset
    load_fmt = ns.load_format
    if mp and mp.startswith("random://"):
        preset, mp, load_fmt = mp[len("random://"):].split("?")[0], None, "dummy"
    elif mp and not os.path.exists(os.path.join(mp, "config.json")) and preset is None:
        # a model directory without a config (synthetic benchmark nodes): fall back to a preset
        preset = os.environ.get("OME_MODEL_PRESET", "llama-3-8b")
    return EngineArgs(model_path=mp, model=preset, served_model_name=ns.served_model_name, tp_size=ns.tp_size,
                      pp_size=ns.pp_size, pp_microbatches=ns.pp_microbatches, dp_size=ns.dp_size,
                      mem_fraction_static=ns.mem_frac,
                      max_running_requests=ns.max_running_requests, max_total_tokens=ns.max_total_tokens,
                      chunked_prefill_size=ns.chunked_prefill_size, context_length=ns.context_length,
                      page_size=ns.page_size, cuda_graph=not ns.disable_cuda_graph,
                      cuda_graph_max_bs=ns.cuda_graph_max_bs, load_format=load_fmt, dtype=ns.dtype,
                      device=ns.device, seed=ns.random_seed, enable_mixed_chunk=ns.enable_mixed_chunk,
                      disable_radix_cache=ns.disable_radix_cache, is_embedding=ns.is_embedding,
                      kv_cache_dtype=ns.kv_cache_dtype, quantization=ns.quantization,
                      enable_dp_attention=ns.enable_dp_attention,
                      ep_num_redundant_experts=ns.ep_num_redundant_experts,
                      enable_two_batch_overlap=ns.enable_two_batch_overlap,
                      eplb_rebalance_steps=ns.eplb_rebalance_num_iterations if ns.enable_eplb else 0,
                      dist_init_addr=ns.dist_init_addr, nnodes=ns.nnodes,
                      node_rank=ns.node_rank, disaggregation_mode=ns.disaggregation_mode,
                      num_layers_override=ns.num_layers,
                      overlap_schedule=False if ns.disable_overlap_schedule else None,
                      watchdog_timeout=getattr(ns, "watchdog_timeout", 300.0),
                      cuda_graph_bs=getattr(ns, "cuda_graph_bs", None),
                      tokenizer_path=getattr(ns, "tokenizer_path", None),
                      dp_balance=("round_robin" if getattr(ns, "prefill_round_robin_balance", False)
                                  else getattr(ns, "load_balance_method", "shortest_queue")),
                      deepep_mode=getattr(ns, "deepep_mode", "auto"),
                      decode_log_interval=getattr(ns, "decode_log_interval", 0))


# ------------------------------------------------------------------ request plumbing
class _Delivery:
    """Engine thread -> event loop hand-off for ALL streams of one loop: an engine step that
    produces tokens for N requests wakes the loop once (one ``call_soon_threadsafe``, one
    self-pipe write) instead of N times; the loop then fans the batch out to the per-request
    queues.  At 256 streams x ~60 steps/s that is ~15k fewer wake-ups (and GIL hand-offs) per
    second on the thread that also launches the GPU steps."""

    _by_loop: dict = {}

    def __init__(self, loop):
        self.loop = loop
        self.pending: list = []
        self.scheduled = False
        self.lock = threading.Lock()

    @classmethod
    def of(cls, loop) -> "_Delivery":
        d = cls._by_loop.get(id(loop))
        if d is None or d.loop is not loop:
            d = cls._by_loop[id(loop)] = cls(loop)
        return d

    def push(self, q, item) -> None:
        with self.lock:
            self.pending.append((q, item))
            if self.scheduled:
                return
            self.scheduled = True
        self.loop.call_soon_threadsafe(self._flush)

    def _flush(self) -> None:
        with self.lock:
            items, self.pending = self.pending, []
            self.scheduled = False
        for q, item in items:
            q.put_nowait(item)


class _Stream:
    """Thread-safe bridge: engine thread -> asyncio queue of (new_token_ids, finished)."""

    def __init__(self, loop):
        self.loop = loop
        self.q: asyncio.Queue = asyncio.Queue()
        self.delivery = _Delivery.of(loop)

    def __call__(self, req, toks, finished):
        if _BATCHED_DELIVERY:
            self.delivery.push(self.q, (list(toks), finished))
        else:
            self.loop.call_soon_threadsafe(self.q.put_nowait, (list(toks), finished))


_BATCHED_DELIVERY = os.environ.get("OME_BATCHED_DELIVERY", "1") == "1"


def _sampling_from(body: dict, default_max: int):
    from ome_amd.runtime.request import SamplingParams

    stop = body.get("stop")
    if isinstance(stop, str):
        stop = [stop]
    max_tokens = body.get("max_completion_tokens") or body.get("max_tokens") or body.get("max_new_tokens")
    return SamplingParams(
        max_new_tokens=int(max_tokens) if max_tokens is not None else default_max,
        temperature=float(body.get("temperature", 1.0) if body.get("temperature") is not None else 1.0),
        top_p=float(body.get("top_p") or 1.0), top_k=int(body.get("top_k") or -1),
        min_p=float(body.get("min_p") or 0.0), stop=list(stop or []),
        stop_token_ids=list(body.get("stop_token_ids") or []), ignore_eos=bool(body.get("ignore_eos", False)),
        seed=body.get("seed"), presence_penalty=float(body.get("presence_penalty") or 0.0),
        frequency_penalty=float(body.get("frequency_penalty") or 0.0),
        repetition_penalty=float(body.get("repetition_penalty") or 1.0), logprobs=bool(body.get("logprobs")),
        n=int(body.get("n") or 1))


def create_app(engine, ns=None):
    from fastapi import FastAPI
    from fastapi.responses import JSONResponse, PlainTextResponse, StreamingResponse

    app = FastAPI(title="ome_amd runtime")
    tok = engine.tokenizer
    model_name = engine.served_model_name
    from ome_amd.runtime.detok import IncrementalDetokenizer, StopMatcher, special_strings, strip_special
    from ome_amd.runtime.parsers import ReasoningParser, ToolParser

    tool_kind = getattr(ns, "tool_call_parser", None) if ns is not None else None
    reason_kind = getattr(ns, "reasoning_parser", None) if ns is not None else None
    if tool_kind:
        ToolParser(tool_kind)  # validate the name at startup
    tpl = getattr(ns, "chat_template", None) if ns is not None else None
    if tpl and os.path.exists(tpl) and hasattr(tok, "chat_template"):
        with open(tpl) as f:
            tok.chat_template = f.read()
    encoder = bool(getattr(getattr(engine, "runner", None), "model", None) is not None and
                   getattr(engine.runner.model, "encoder_only", False))

    def encode_text(text: str) -> list[int]:  # encoders take [CLS] ... [SEP]
        return tok.encode_special(text) if encoder else tok.encode(text)
    created = int(time.time())
    default_max = 128
    app.state.engine = engine
    # --log-requests (+ --log-requests-level / --max-log-len), --limit-mm-per-prompt, --middleware
    log_req = bool(getattr(ns, "log_requests", False)) if ns is not None else False
    log_level = int(getattr(ns, "log_requests_level", 0) or 0) if ns is not None else 0
    log_len = getattr(ns, "max_log_len", None) if ns is not None else None
    mm_limit = getattr(ns, "mm_limit", None) if ns is not None else None
    rlog = logging.getLogger("ome_amd.requests")

    def _clip(text: str) -> str:
        return text if log_len is None or len(text) <= log_len else text[:log_len] + f"...(+{len(text) - log_len})"

    def _log_in(req) -> None:
        msg = f"request {req.rid}: prompt_tokens={len(req.prompt_ids)} max_new_tokens={req.params.max_new_tokens}"
        if log_level >= 1:
            msg += f" params={req.params}"
        if log_level >= 2:
            msg += f" prompt={_clip(tok.decode(req.prompt_ids))!r}"
        rlog.info(msg)

    def _log_out(req) -> None:
        msg = (f"finished {req.rid}: output_tokens={len(req.output_ids)} reason={req.finish_reason} "
               f"ttft={req.ttft}")
        if log_level >= 2:
            msg += f" output={_clip(tok.decode(req.output_ids))!r}"
        rlog.info(msg)

    for mw in (getattr(ns, "middleware", None) or []) if ns is not None else []:
        if mw.endswith("log_opc_header"):   # vLLM's OCI middleware: log the opc-request-id header
            @app.middleware("http")
            async def _opc(request, call_next):
                oid = request.headers.get("opc-request-id")
                if oid:
                    rlog.info("opc-request-id %s %s %s", oid, request.method, request.url.path)
                resp = await call_next(request)
                if oid:
                    resp.headers["opc-request-id"] = oid
                return resp

    def err(code: int, msg: str, typ: str = "invalid_request_error"):
        return JSONResponse({"error": {"message": msg, "type": typ, "code": code}}, status_code=code)

    async def run_request(prompt_ids, params, bootstrap=None, images=None):
        loop = asyncio.get_running_loop()
        stream = _Stream(loop)
        if bootstrap and bootstrap.get("disagg_role") == "prefill":
            params.max_new_tokens = 1  # the prefill engine only produces the first token + KV
        if images and mm_limit is not None and len(images) > mm_limit:
            raise ValueError(f"{len(images)} images in the prompt; this server accepts at most {mm_limit} "
                             f"(--limit-mm-per-prompt)")
        if images:
            req = engine.make_mm_request(prompt_ids, images, params, on_token=stream, bootstrap=bootstrap)
        else:
            req = engine.make_request(prompt_ids, params, on_token=stream, bootstrap=bootstrap)
        if log_req:
            _log_in(req)
            inner = req.on_token

            def on_token(r, toks, fin, _inner=inner):
                if fin:
                    _log_out(r)
                return _inner(r, toks, fin)
            req.on_token = on_token
        engine.add_request(req)
        return req, stream

    def _bootstrap_of(body: dict):
        if body.get("bootstrap_room") is None:
            return None
        return {k: body.get(k) for k in ("bootstrap_room", "bootstrap_host", "bootstrap_port", "disagg_role",
                                         "bootstrap_prefill")} | {"room": int(body["bootstrap_room"])}

    @app.get("/health")
    @app.get("/HealthCheck")   # the reference routers' --health-check-endpoint spelling
    async def health():
        return {"status": "ok", **engine.health()}

    @app.get("/health_generate")
    async def health_generate():
        from ome_amd.runtime.request import SamplingParams

        try:
            req, stream = await run_request([tok.bos_token_id or 1, 3 + 72, 3 + 105], SamplingParams(max_new_tokens=1))
            while True:
                _, fin = await asyncio.wait_for(stream.q.get(), timeout=120)
                if fin:
                    break
            if req.finish_reason and req.finish_reason.startswith("abort"):
                return err(503, f"generation failed: {req.finish_reason}", "service_unavailable")
            return {"status": "ok"}
        except asyncio.TimeoutError:
            return err(503, "health generation timed out", "service_unavailable")

    @app.get("/v1/models")
    async def models():
        return {"object": "list", "data": [{"id": model_name, "object": "model", "created": created,
                                            "owned_by": "ome_amd", "max_model_len": engine.max_context}]}

    @app.get("/get_model_info")
    async def model_info():
        c = engine.cfg
        return {"model_path": engine.args.model_path, "served_model_name": model_name,
                "architecture": c.architecture, "is_generation": not c.is_embedding,
                "num_layers": c.num_layers, "hidden_size": c.hidden_size, "vocab_size": c.vocab_size,
                "context_length": engine.max_context}

    @app.get("/get_server_info")
    @app.get("/server_info")
    async def server_info():
        a = engine.args
        return {"tp_size": a.tp_size, "pp_size": a.pp_size, "page_size": a.page_size,
                "max_running_requests": a.max_running_requests, "chunked_prefill_size": a.chunked_prefill_size,
                "kv_pages": engine.runner.kv.num_pages, "cuda_graph_buckets": engine.runner.buckets,
                "disaggregation_mode": a.disaggregation_mode,
                "disaggregation_bootstrap_port": getattr(engine.kv_transfer, "port", None),
                "kv_transfer": engine.kv_transfer.stats() if engine.kv_transfer is not None else None,
                **engine.health()}

    @app.get("/metrics")
    async def metrics():
        engine.metrics.model_name = model_name
        return PlainTextResponse(engine.metrics.render(), media_type="text/plain; version=0.0.4")

    def _chat_images(msgs: list) -> tuple[list, list]:
        """OpenAI ``image_url`` / ``image`` content parts -> (messages with a sentinel text part in
        their place, image sources in order)."""
        images, out = [], []
        for m in msgs:
            content = m.get("content") if isinstance(m, dict) else None
            if not isinstance(content, list):
                out.append(m)
                continue
            parts = []
            for c in content:
                if isinstance(c, dict) and c.get("type") in ("image_url", "image"):
                    src = c.get("image_url", c.get("image"))
                    images.append(src.get("url") if isinstance(src, dict) else src)
                    parts.append({"type": "text", "text": _IMG_SENTINEL})
                else:
                    parts.append(c)
            out.append({**m, "content": parts})
        return out, images

    def _encode(body: dict, chat: bool):
        """-> (prompt ids, images); image prompts carry one ``image_token_id`` per image, wrapped
        in the model's vision start / end tokens."""
        if chat:
            msgs = body.get("messages")
            if not isinstance(msgs, list) or not msgs:
                raise ValueError("messages must be a non-empty list")
            msgs, images = _chat_images(msgs)
            tools = body.get("tools") if body.get("tool_choice", "auto") != "none" else None
            text = tok.apply_chat_template(msgs, add_generation_prompt=True, tools=tools)
            if not images:
                return tok.encode(text), []
            m = engine.runner.model
            if not getattr(m, "is_multimodal", False):
                raise ValueError(f"model {model_name} does not accept image inputs")
            segs = text.split(_IMG_SENTINEL)
            ids = []
            for k, seg in enumerate(segs):
                ids.extend(tok.encode(seg) if seg else [])
                if k + 1 < len(segs):
                    ids.extend(m.image_prompt_ids() if hasattr(m, "image_prompt_ids") else
                               [m.vision_start_id, m.image_token_id, m.vision_end_id])
            return ids, images
        p = body.get("prompt", body.get("text"))
        images = list(body.get("image_data") or [])  # SGLang /generate spelling
        if isinstance(p, list) and p and isinstance(p[0], int):
            return list(p), images
        if isinstance(p, list):
            p = p[0] if p else ""
        if body.get("input_ids"):
            return list(body["input_ids"]), images
        if not isinstance(p, str):
            raise ValueError("prompt must be a string or a list of token ids")
        return tok.encode(p), images

    def _logprobs(req, chat: bool):
        toks = [tok.decode([t], skip_special=False) for t in req.output_ids]
        if chat:
            return {"content": [{"token": t, "logprob": lp, "bytes": list(t.encode("utf-8")), "top_logprobs": []}
                                for t, lp in zip(toks, req.output_logprobs)]}
        offs, o = [], 0
        for t in toks:
            offs.append(o)
            o += len(t)
        return {"tokens": toks, "token_logprobs": list(req.output_logprobs), "top_logprobs": None,
                "text_offset": offs}

    async def _complete(body: dict, chat: bool):
        n = int(body.get("n") or 1)
        if n > 1:   # n choices = n independent requests (distinct seeds), one batched engine run
            if body.get("stream"):
                return err(400, "n > 1 is not supported with stream=true")
            seed = body.get("seed")
            subs = await asyncio.gather(*[_complete({**body, "n": 1, "seed": None if seed is None else seed + i},
                                                    chat) for i in range(n)])
            for s_ in subs:
                if not isinstance(s_, dict):
                    return s_
            out = subs[0]
            out["choices"] = [{**s_["choices"][0], "index": i} for i, s_ in enumerate(subs)]
            ct = sum(s_["usage"]["completion_tokens"] for s_ in subs)
            out["usage"] = {**out["usage"], "completion_tokens": ct, "total_tokens": out["usage"]["prompt_tokens"] + ct}
            return out
        try:
            ids, images = _encode(body, chat)
            params = _sampling_from(body, default_max)
            req, stream = await run_request(ids, params, _bootstrap_of(body), images)
            ids = req.prompt_ids  # image placeholders expanded
        except (ValueError, OSError) as e:  # OSError: undecodable image data
            return err(400, str(e))
        rid = f"{'chatcmpl' if chat else 'cmpl'}-{uuid.uuid4().hex[:24]}"
        obj = "chat.completion" if chat else "text_completion"
        stops = params.stop

        def usage():
            return {"prompt_tokens": len(ids), "completion_tokens": len(req.output_ids),
                    "total_tokens": len(ids) + len(req.output_ids)}

        # streamed text-completion chunk template: {"id","object","created","model","choices"[,"usage"]}
        text_pre = f'data: {{"id":{json.dumps(rid)},"object":"text_completion","created":'
        text_mid = f',"model":{json.dumps(model_name)},"choices":[{{"index":0,"text":'

        use_tools = bool(chat and tool_kind and body.get("tools") and body.get("tool_choice", "auto") != "none")
        use_reason = bool(chat and reason_kind and body.get("separate_reasoning", True))
        # parsers look for special-token markers (harmony <|channel|>/<|call|>, [TOOL_CALLS]):
        # decode with them kept, strip them from what the client sees
        raw_mode = use_tools or use_reason
        specials = special_strings(tok) if raw_mode else []
        harmony_tools = use_tools and tool_kind == "gpt-oss"
        det = IncrementalDetokenizer(tok, skip_special=not raw_mode)
        stopm = StopMatcher(stops)

        def pull(fin: bool) -> tuple[str, bool]:
            """New text since the last call (incremental, O(new tokens)), cut at a stop string."""
            delta = det.push(req.output_ids[len(det.ids):])
            if fin:
                delta += det.flush()
            cut = stopm.find(det.text, len(delta))
            if cut is not None:
                delta = delta[:max(0, cut - (len(det.text) - len(delta)))]
                return delta, True
            return delta, False

        if body.get("stream"):
            async def gen():
                first = True
                rp = ReasoningParser(reason_kind) if use_reason else None
                tp = ToolParser(tool_kind) if use_tools else None
                content_all, content_sent, calls_started, raw_all = "", 0, False, ""
                every_usage = bool((body.get("stream_options") or {}).get("continuous_usage_stats"))
                try:
                    async for chunk in body_chunks(first, rp, tp, content_all, content_sent, calls_started, raw_all,
                                                   every_usage):
                        yield chunk
                finally:
                    # client gone (generator closed mid-stream): stop generating for it
                    if req.finish_reason is None:
                        engine.abort(req.rid)

            async def body_chunks(first, rp, tp, content_all, content_sent, calls_started, raw_all, every_usage):
                while True:
                    _, fin = await stream.q.get()
                    while not fin and not stream.q.empty():   # coalesce steps the loop fell behind on
                        _, fin = stream.q.get_nowait()
                    delta, stopped = pull(fin)
                    if stopped:
                        fin = True
                        engine.abort(req.rid)
                    raw_all += delta
                    if chat:
                        d: dict = {}
                        if rp is not None:
                            rd, cd = rp.feed(delta)
                            if fin:
                                fr, fc = rp.flush()
                                rd, cd = rd + fr, cd + fc
                            rd = strip_special(rd, specials)
                            if rd:
                                d["reasoning_content"] = rd
                        else:
                            cd = delta
                        content_all += cd
                        if tp is not None and not calls_started:
                            i = tp.start_index(raw_all if harmony_tools else content_all)
                            if i >= 0:
                                calls_started = True
                                cd = content_all[content_sent:] if harmony_tools else content_all[content_sent:i]
                            elif harmony_tools:   # harmony content is already channel-filtered
                                cd = content_all[content_sent:]
                            else:   # hold back a suffix that may still become a call marker
                                cd = content_all[content_sent:len(content_all) if fin else tp.safe_len(content_all)]
                        elif tp is not None:
                            cd = content_all[content_sent:] if harmony_tools else ""
                        content_sent += len(cd)
                        cd = strip_special(cd, specials)
                        if cd or not d:
                            d["content"] = cd
                        if first:
                            d["role"] = "assistant"
                        finish = None
                        if fin and calls_started:
                            _, calls = tp.parse(raw_all if harmony_tools else content_all)
                            if calls:
                                d["tool_calls"] = [{"index": k, **c} for k, c in enumerate(calls)]
                                finish = "tool_calls"
                            elif content_all[content_sent:]:   # not a call after all: release the text
                                d["content"] = d.get("content", "") + strip_special(content_all[content_sent:],
                                                                                    specials)
                        choice = {"index": 0, "delta": d, "finish_reason": None}
                        chunk_obj = "chat.completion.chunk"
                        if finish:
                            choice["_finish"] = finish
                    else:
                        # text completion: the chunk is formatted from a template -- one small
                        # json.dumps of the text instead of the whole nested dict (~1.5 vs ~7.7 us per
                        # chunk; 256 streams x one chunk per engine step run on the server's event-loop
                        # thread, which shares the GIL with the engine loop)
                        first = False
                        fr = ("stop" if stopped else _finish(req)) if fin else None
                        chunk = (f'{text_pre}{int(time.time())}{text_mid}{json.dumps(strip_special(delta, specials))}'
                                 f',"finish_reason":{"null" if fr is None else json.dumps(fr)}}}]')
                        if every_usage or (fin and (body.get("stream_options") or {}).get("include_usage", True)):
                            n_out = len(req.output_ids)
                            chunk += (f',"usage":{{"prompt_tokens":{len(ids)},"completion_tokens":{n_out},'
                                      f'"total_tokens":{len(ids) + n_out}}}')
                        yield f"{chunk}}}\n\n"
                        if fin:
                            break
                        continue
                    first = False
                    forced = choice.pop("_finish", None)
                    if fin:
                        choice["finish_reason"] = forced or ("stop" if stopped else _finish(req))
                    out = {"id": rid, "object": chunk_obj, "created": int(time.time()), "model": model_name,
                           "choices": [choice]}
                    if every_usage or (fin and (body.get("stream_options") or {}).get("include_usage", True)):
                        out["usage"] = usage()
                    yield f"data: {json.dumps(out)}\n\n"
                    if fin:
                        break
                yield "data: [DONE]\n\n"

            return StreamingResponse(gen(), media_type="text/event-stream")
        stopped = False
        while True:
            _, fin = await stream.q.get()
            if stopm.stops:
                _, stopped = pull(fin)
                if stopped:
                    engine.abort(req.rid)
                    break
            if fin:
                break
        text = tok.decode(req.output_ids, skip_special=not raw_mode)
        cut = stopm.find(text, len(text))
        reason = _finish(req)
        if cut is not None:
            text, reason = text[:cut], "stop"
        if chat:
            msg: dict = {"role": "assistant", "content": text}
            if use_reason:
                r, msg["content"] = ReasoningParser(reason_kind).split(text)
                msg["reasoning_content"] = strip_special(r, specials)
            if use_tools:
                # the tool parser sees the raw output: harmony calls live in the commentary
                # channel, which the reasoning split above does not keep
                content, calls = ToolParser(tool_kind).parse(text if harmony_tools else msg["content"])
                if calls:
                    msg["content"], msg["tool_calls"], reason = content or None, calls, "tool_calls"
            msg["content"] = strip_special(msg["content"], specials)
            choice = {"index": 0, "message": msg, "finish_reason": reason}
        else:
            choice = {"index": 0, "text": strip_special(text, specials), "finish_reason": reason, "logprobs": None}
        if params.logprobs:
            choice["logprobs"] = _logprobs(req, chat)
        return {"id": rid, "object": obj, "created": int(time.time()), "model": model_name, "choices": [choice],
                "usage": usage()}

    def _finish(req):
        r = req.finish_reason or "stop"
        return "length" if r == "length" else ("stop" if not r.startswith("abort") else "abort")

    @app.post("/v1/chat/completions")
    async def chat(request: Request):
        return await _complete(await request.json(), True)

    @app.post("/v1/responses")
    async def responses(request: Request):
        """OpenAI Responses API (``OPENAI_V1_RESPONSES`` in the API capabilities), mapped onto the
        chat path: ``input`` (string or message list) + ``instructions`` -> messages; the reply
        becomes ``output`` items (reasoning, message with ``output_text``, function calls)."""
        body = await request.json()
        inp = body.get("input")
        msgs = [{"role": "system", "content": body["instructions"]}] if body.get("instructions") else []
        if isinstance(inp, str):
            msgs.append({"role": "user", "content": inp})
        elif isinstance(inp, list):
            for m in inp:
                c = m.get("content")
                if isinstance(c, list):   # input_text / input_image parts -> chat parts
                    c = [{"type": "text", "text": p.get("text", "")} if p.get("type") in ("input_text", "text")
                         else {"type": "image_url", "image_url": {"url": p.get("image_url")}} for p in c]
                msgs.append({"role": m.get("role", "user"), "content": c})
        else:
            return err(400, "input must be a string or a list of messages")
        tools = [{"type": "function", "function": {k: t[k] for k in ("name", "description", "parameters") if k in t}}
                 if "function" not in t else t for t in (body.get("tools") or [])]
        chat_body = {"messages": msgs, "max_tokens": body.get("max_output_tokens"), "temperature": body.get("temperature"),
                     "top_p": body.get("top_p"), "tools": tools or None, "tool_choice": body.get("tool_choice", "auto")}
        res = await _complete({k: v for k, v in chat_body.items() if v is not None}, True)
        if not isinstance(res, dict):
            return res
        m = res["choices"][0]["message"]
        out = []
        if m.get("reasoning_content"):
            out.append({"type": "reasoning", "id": f"rs_{uuid.uuid4().hex[:16]}",
                        "summary": [{"type": "summary_text", "text": m["reasoning_content"]}]})
        for c in m.get("tool_calls") or []:
            out.append({"type": "function_call", "id": f"fc_{uuid.uuid4().hex[:16]}", "call_id": c["id"],
                        "name": c["function"]["name"], "arguments": c["function"]["arguments"], "status": "completed"})
        if m.get("content"):
            out.append({"type": "message", "id": f"msg_{uuid.uuid4().hex[:16]}", "role": "assistant",
                        "status": "completed", "content": [{"type": "output_text", "text": m["content"],
                                                            "annotations": []}]})
        u = res["usage"]
        done = res["choices"][0]["finish_reason"] != "length"
        return {"id": f"resp_{uuid.uuid4().hex[:24]}", "object": "response", "created_at": int(time.time()),
                "model": model_name, "status": "completed" if done else "incomplete",
                "incomplete_details": None if done else {"reason": "max_output_tokens"}, "output": out,
                "output_text": m.get("content") or "",
                "usage": {"input_tokens": u["prompt_tokens"], "output_tokens": u["completion_tokens"],
                          "total_tokens": u["total_tokens"]}}

    @app.post("/v1/completions")
    async def completions(request: Request):
        return await _complete(await request.json(), False)

    @app.post("/generate")
    async def generate(request: Request):
        body = await request.json()
        sp = body.get("sampling_params") or {}
        merged = {**sp, "prompt": body.get("text"), "input_ids": body.get("input_ids"),
                  "image_data": body.get("image_data"),
                  "max_tokens": sp.get("max_new_tokens"), "stream": body.get("stream", False)}
        res = await _complete(merged, False)
        if isinstance(res, dict):
            c = res["choices"][0]
            return {"text": c["text"], "meta_info": {"finish_reason": c["finish_reason"], **res["usage"]}}
        return res

    @app.post("/v1/embeddings")
    async def embeddings(request: Request):
        body = await request.json()
        inp = body.get("input")
        items = inp if isinstance(inp, list) and (not inp or not isinstance(inp[0], int)) else [inp]
        out, total = [], 0
        from ome_amd.runtime.request import SamplingParams

        for i, x in enumerate(items):
            if isinstance(x, dict) and ("image" in x or "image_url" in x):
                im = x.get("image") or (x.get("image_url") or {}).get("url")
                m = engine.runner.model
                if hasattr(m, "image_prompt_ids") or hasattr(m, "image_token_id"):
                    # VLM embedder (GME-Qwen2-VL style): the image (+ text) as one user turn of the
                    # chat template, last-token pooling over the language model
                    content = [{"type": "image_url", "image_url": {"url": im}}]
                    if x.get("text"):
                        content.append({"type": "text", "text": str(x["text"])})
                    ids, ims = _encode({"messages": [{"role": "user", "content": content}]}, True)
                    total += len(ids)
                    emb = await _embed_ids(ids, images=ims)
                else:   # CLIP-style image tower embedding
                    emb = await _embed_ids([], images=[im])
            else:
                if isinstance(x, dict):
                    x = x.get("text", "")
                ids = list(x) if isinstance(x, list) else encode_text(str(x))
                total += len(ids)
                emb = await _embed_ids(ids)
            out.append({"object": "embedding", "index": i, "embedding": emb})
        return {"object": "list", "data": out, "model": model_name,
                "usage": {"prompt_tokens": total, "total_tokens": total}}

    async def _embed_ids(ids: list[int], images=None) -> list[float]:
        from ome_amd.runtime.request import SamplingParams

        req, stream = await run_request(ids, SamplingParams(max_new_tokens=0), images=images)
        req.is_embedding = True
        while True:
            _, fin = await stream.q.get()
            if fin:
                break
        return req.embedding or []

    @app.post("/v1/rerank")
    async def rerank(request: Request):
        """Cross-encoder reranking (SGLang's ``/v1/rerank``): score every (query, document) pair with
        a sequence-classification encoder; results sorted by relevance (the head's first logit)."""
        body = await request.json()
        if not encoder:
            return JSONResponse({"error": {"message": "rerank needs a cross-encoder model",
                                           "type": "invalid_request_error"}}, status_code=400)
        query, docs = body.get("query"), body.get("documents") or []
        if not isinstance(query, str) or not isinstance(docs, list):
            return JSONResponse({"error": {"message": "query (str) and documents (list) are required",
                                           "type": "invalid_request_error"}}, status_code=400)
        texts = [d if isinstance(d, str) else (d or {}).get("text", "") for d in docs]
        pairs = [tok.encode_special(query, text) for text in texts]
        total = sum(len(ids) for ids in pairs)
        scores = await asyncio.gather(*[_embed_ids(ids) for ids in pairs])  # one batched engine step
        res = []
        for i, (text, score) in enumerate(zip(texts, scores)):
            item = {"index": i, "relevance_score": float(score[0]) if score else 0.0}
            if body.get("return_documents", True):
                item["document"] = {"text": text}
            res.append(item)
        res.sort(key=lambda r: -r["relevance_score"])
        top_n = body.get("top_n")
        if top_n:
            res = res[:int(top_n)]
        return {"id": f"rerank-{uuid.uuid4().hex[:12]}", "model": model_name, "results": res,
                "usage": {"prompt_tokens": total, "total_tokens": total}}

    return app


def _worker_main(rank: int, world: int, ns_dict: dict, addr: str, local_rank: int) -> None:
    os.environ.update({"RANK": str(rank), "WORLD_SIZE": str(world), "LOCAL_RANK": str(local_rank)})
    ns = argparse.Namespace(**ns_dict)
    ns.dist_init_addr = addr
    from ome_amd.runtime.engine import Engine

    eng = Engine(engine_args_from(ns))
    eng.run_forever()


_RAY_STORE = None   # the head's rendezvous store client / host, alive as long as the server


def _ray_group(ns, argv: list[str], world: int) -> None:
    """``--distributed-executor-backend ray`` (MultiNodeRayVLLM): the TP x PP group spans the
    RayCluster's nodes -- publish this launch for the workers' ``ome_amd.raylet`` agents and run
    as node 0 (``ome_amd.raylet`` module doc)."""
    global _RAY_STORE
    from ome_amd import raylet

    gpn = int(os.environ.get("OME_RAY_GPUS_PER_NODE") or 0)
    if gpn <= 0:
        import torch

        gpn = torch.cuda.device_count() or 8   # does not initialise the GPU on this stack
    nnodes = max(1, -(-world // gpn))
    if nnodes == 1:
        return
    addr = raylet.head_address()
    _RAY_STORE = raylet.connect_or_host(addr)
    drop = {"--distributed-executor-backend"}
    wargv, skip = [], False
    for a in argv:
        if skip:
            skip = False
            continue
        if a in drop:
            skip = True
            continue
        if a.split("=", 1)[0] in drop:
            continue
        wargv.append(a)
    port = raylet.publish_launch(_RAY_STORE, wargv, nnodes)
    ns.nnodes, ns.node_rank = nnodes, 0
    ns.dist_init_addr = f"{addr.rpartition(':')[0] or '127.0.0.1'}:{port}"
    log.info("ray backend: %d nodes x %d ranks, rendezvous %s", nnodes, world // nnodes, ns.dist_init_addr)


def main(argv=None) -> int:
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    # the engine thread shares the GIL with the asyncio HTTP loop: a shorter switch interval than
    # CPython's 5 ms default bounds how long the engine waits to launch the next step while the
    # loop formats SSE chunks for hundreds of streams
    sw = float(os.environ.get("OME_GIL_SWITCH_S", "0") or 0)
    if sw > 0:
        import sys as _sys

        _sys.setswitchinterval(sw)
    ap = build_parser()
    ns, unknown = ap.parse_known_args(argv)
    if unknown:
        # every flag of the reference runtimes is either implemented or an explicit no-op
        # (ome_amd/runtime/flags.py); anything else would silently change what was asked for
        if os.environ.get("OME_ALLOW_UNKNOWN_FLAGS", "0") == "1":
            log.warning("ignoring unsupported flags: %s", " ".join(unknown))
        else:
            ap.error(f"unsupported flags: {' '.join(unknown)} (OME_ALLOW_UNKNOWN_FLAGS=1 to ignore)")
    validate_args(ns, ap)
    logging.getLogger().setLevel(getattr(logging, str(ns.log_level).upper(), logging.INFO))
    world = (ns.dp_size if ns.enable_dp_attention and ns.tp_size == 1 else ns.tp_size) * ns.pp_size
    if ns.distributed_executor_backend == "ray" and world > 1 and ns.nnodes == 1:
        _ray_group(ns, argv if argv is not None else sys.argv[1:], world)
    per_node = max(1, world // max(1, ns.nnodes))
    base_rank = ns.node_rank * per_node
    procs = []
    if world > 1:
        import multiprocessing as mp

        addr = ns.dist_init_addr or f"127.0.0.1:{29500 + (os.getpid() % 1000)}"
        ns.dist_init_addr = addr
        ctx = mp.get_context("spawn")
        for i in range(1, per_node):
            p = ctx.Process(target=_worker_main, args=(base_rank + i, world, vars(ns), addr, i), daemon=True)
            p.start()
            procs.append(p)
        os.environ.update({"RANK": str(base_rank), "WORLD_SIZE": str(world), "LOCAL_RANK": "0"})
    from ome_amd.runtime.engine import Engine

    if world > 1 and base_rank != 0:
        # worker pod of a multi-node group: serve probes only, run the engine loop in lockstep
        eng = Engine(engine_args_from(ns))
        threading.Thread(target=eng.run_forever, daemon=True).start()
        from fastapi import FastAPI
        import uvicorn

        app = FastAPI()

        @app.get("/health")
        async def h():
            return {"status": "ok", "rank": base_rank}

        if ns.grpc_mode:   # worker pods of a gRPC runtime answer the same grpc.health.v1 probes
            from ome_amd.runtime import grpc_server

            asyncio.run(grpc_server.serve(app, eng, ns.host, ns.port))
            return 0
        uvicorn.run(app, host=ns.host, port=ns.port, log_level="warning")
        return 0
    eng = Engine(engine_args_from(ns))
    if ns.disaggregation_mode != "null":
        from ome_amd.runtime.disagg import attach_kv_transfer

        attach_kv_transfer(eng, ns.disaggregation_mode, ns.disaggregation_bootstrap_port)
    eng.start()
    app = create_app(eng, ns)
    if ns.grpc_mode:
        from ome_amd.runtime import grpc_server

        log.info("serving %s over gRPC on %s:%d (tp=%d)", eng.served_model_name, ns.host, ns.port, ns.tp_size)
        try:
            asyncio.run(grpc_server.serve(app, eng, ns.host, ns.port))
        except KeyboardInterrupt:
            pass
    else:
        import uvicorn

        log.info("serving %s on %s:%d (tp=%d)", eng.served_model_name, ns.host, ns.port, ns.tp_size)
        uvicorn.run(app, host=ns.host, port=ns.port, log_level="warning")
    eng.shutdown()
    for p in procs:
        p.terminate()
    return 0


if __name__ == "__main__":
    sys.exit(main())
