"""Load generator behind BenchmarkJob (genai-bench compatible CLI; the reference runs the external
``genai-bench`` image, ``pkg/controller/v1beta1/benchmark/utils/benchmark.go:95-167``).

    python -m ome_amd.bench.loadgen benchmark --api-backend openai --api-base http://svc:8080 \
        --api-model-name M --task text-to-text --traffic-scenario "N(480,240)/(300,150)" \
        --num-concurrency 1 --num-concurrency 64 --max-time-per-run 15 --max-requests-per-run 300 \
        --experiment-base-dir /tmp/results
    python -m ome_amd.bench.loadgen report /tmp/results/<experiment>

Closed-loop: for every (scenario, concurrency) pair ``C`` asyncio workers each keep one
streaming request in flight until the run's request or time budget is spent.  Per request we
record TTFT (first content chunk), end-to-end latency, output/input tokens (server ``usage``),
and TPOT = (e2e - TTFT) / (out - 1).  Each run writes one JSON with per-request samples and
aggregates (mean / p50 / p90 / p99, output and total token throughput, RPS, error rate) under
``<base>/<experiment>/``; ``experiment_metadata.json`` records the command and server info.
Hostnames ``*.svc.cluster.local`` resolve through the local executor's service proxies.
"""
from __future__ import annotations

import argparse
import asyncio
import json
import math
import os
import random
import statistics
import sys
import time
from dataclasses import asdict, dataclass, field
from pathlib import Path

from ome_amd.bench.scenarios import DEFAULT_CONCURRENCY, DEFAULT_SCENARIOS, Scenario, validate
from ome_amd.executor.dns import resolve_url

WORDS = ("the of and to in is that for it as was with be by on not he this are or his from at which but have an "
         "they you were her she there one all we their been has when who will more no if out so said what up its "
         "about into than them can only other new some could time these two may then do first any my now such "
         "like our over man me even most made after also did many before must through back years where much your "
         "way well down should because each just those people how too little state good very make world still "
         "own see men work long get here between both life being under never day same another know while last").split()


@dataclass
class Sample:
    ok: bool
    input_tokens: int
    output_tokens: int
    ttft: float = 0.0
    e2e: float = 0.0
    tpot: float = 0.0
    start: float = 0.0
    error: str = ""


@dataclass
class RunResult:
    scenario: str
    task: str
    concurrency: int
    duration_s: float
    samples: list = field(default_factory=list)
    aggregates: dict = field(default_factory=dict)


class PromptFactory:
    """Builds prompts of a target token length with the model's tokenizer when available."""

    def __init__(self, tokenizer_path: str | None, seed: int = 0):
        self.rng = random.Random(seed)
        self.tok = None
        if tokenizer_path and os.path.isdir(tokenizer_path) and any(
                os.path.exists(os.path.join(tokenizer_path, f)) for f in ("tokenizer.json", "tokenizer.model")):
            try:
                from transformers import AutoTokenizer

                self.tok = AutoTokenizer.from_pretrained(tokenizer_path)
            except Exception:  # noqa: BLE001 — fall back to the word-count approximation
                self.tok = None

        # without a local tokenizer: server tokens ~= a * words + b, fitted by calibrate()
        self.tok_per_word, self.overhead = 1.0, 0.0

    def calibrate(self, counts: list[tuple[int, int]]) -> None:
        """Fit the server's prompt tokens per word from (words, prompt_tokens) probes, so an
        N(480, 240) scenario sends ~480-token prompts whatever the server's tokenizer (a byte-level
        fallback turns one word into ~4.6 tokens)."""
        (w0, t0), (w1, t1) = counts[0], counts[-1]
        if w1 != w0 and t1 > t0:
            self.tok_per_word = (t1 - t0) / (w1 - w0)
            self.overhead = max(0.0, t0 - self.tok_per_word * w0)

    def make(self, n_tokens: int, rng: random.Random | None = None) -> str:
        rng = rng or self.rng
        n_words = n_tokens if self.tok is not None else \
            int(round((n_tokens - self.overhead) / self.tok_per_word))
        words = [rng.choice(WORDS) for _ in range(max(1, n_words))]
        if self.tok is None:
            return " ".join(words)
        ids = self.tok(" ".join(words), add_special_tokens=False)["input_ids"][:n_tokens]
        return self.tok.decode(ids)


def pct(xs: list[float], p: float) -> float:
    if not xs:
        return 0.0
    s = sorted(xs)
    k = (len(s) - 1) * p / 100.0
    lo, hi = math.floor(k), math.ceil(k)
    return s[lo] + (s[hi] - s[lo]) * (k - lo)


def aggregate(samples: list[Sample], duration: float) -> dict:
    ok = [s for s in samples if s.ok]
    out = {"num_requests": len(samples), "num_completed": len(ok), "num_errors": len(samples) - len(ok),
           "error_rate": (len(samples) - len(ok)) / max(1, len(samples)), "duration_s": duration}
    for name, xs in (("ttft_s", [s.ttft for s in ok]), ("e2e_latency_s", [s.e2e for s in ok]),
                     ("tpot_s", [s.tpot for s in ok if s.output_tokens > 1]),
                     ("output_tokens", [s.output_tokens for s in ok]), ("input_tokens", [s.input_tokens for s in ok])):
        out[name] = {"mean": statistics.fmean(xs) if xs else 0.0, "p50": pct(xs, 50), "p90": pct(xs, 90),
                     "p99": pct(xs, 99), "min": min(xs) if xs else 0.0, "max": max(xs) if xs else 0.0}
    otoks = sum(s.output_tokens for s in ok)
    itoks = sum(s.input_tokens for s in ok)
    out["output_throughput_tokens_per_s"] = otoks / duration if duration > 0 else 0.0
    out["input_throughput_tokens_per_s"] = itoks / duration if duration > 0 else 0.0
    out["total_throughput_tokens_per_s"] = (otoks + itoks) / duration if duration > 0 else 0.0
    out["requests_per_s"] = len(ok) / duration if duration > 0 else 0.0
    return out


async def _one_request(session, args, base: str, scen: Scenario, pf: PromptFactory, rng: random.Random,
                       extra: dict) -> Sample:
    n_in, n_out = scen.sample(rng)
    t0 = time.perf_counter()
    headers = {"Authorization": f"Bearer {args.api_key}"} if args.api_key else {}
    try:
        if args.task in ("text-to-embeddings", "text-to-rerank"):
            body = {"model": args.api_model_name, "input": pf.make(n_in, rng), **extra}
            async with session.post(f"{base}/v1/embeddings", json=body, headers=headers) as r:
                data = await r.json()
                if r.status != 200:
                    return Sample(False, n_in, 0, start=t0, error=str(data)[:200])
                e2e = time.perf_counter() - t0
                itok = int((data.get("usage") or {}).get("prompt_tokens", n_in))
                return Sample(True, itok, 0, ttft=e2e, e2e=e2e, start=t0)
        body = {"model": args.api_model_name, "messages": [{"role": "user", "content": pf.make(n_in, rng)}],
                "max_tokens": n_out, "stream": True, "ignore_eos": True, "temperature": 0.0,
                "stream_options": {"include_usage": True}, **extra}
        ttft, usage, n_chunks = None, None, 0
        async with session.post(f"{base}/v1/chat/completions", json=body, headers=headers) as r:
            if r.status != 200:
                return Sample(False, n_in, 0, start=t0, error=(await r.text())[:200])
            async for raw in r.content:
                line = raw.decode(errors="ignore").strip()
                if not line.startswith("data:"):
                    continue
                payload = line[5:].strip()
                if payload == "[DONE]":
                    break
                try:
                    ev = json.loads(payload)
                except json.JSONDecodeError:
                    continue
                if ev.get("usage"):
                    usage = ev["usage"]
                for ch in ev.get("choices") or []:
                    if (ch.get("delta") or {}).get("content"):
                        n_chunks += 1
                        if ttft is None:
                            ttft = time.perf_counter() - t0
        e2e = time.perf_counter() - t0
        out_t = int((usage or {}).get("completion_tokens", n_chunks))
        in_t = int((usage or {}).get("prompt_tokens", n_in))
        ttft = ttft if ttft is not None else e2e
        return Sample(True, in_t, out_t, ttft=ttft, e2e=e2e,
                      tpot=(e2e - ttft) / (out_t - 1) if out_t > 1 else 0.0, start=t0)
    except Exception as e:  # noqa: BLE001 — count as an error sample
        return Sample(False, n_in, 0, start=t0, error=f"{type(e).__name__}: {e}"[:200])


async def _calibrate(session, args, base: str, pf: PromptFactory) -> None:
    """Two 1-token chat requests (50 and 400 words) -> server prompt tokens per word."""
    headers = {"Authorization": f"Bearer {args.api_key}"} if args.api_key else {}
    counts = []
    rng = random.Random(12345)
    for n in (50, 400):
        body = {"model": args.api_model_name, "max_tokens": 1, "temperature": 0.0,
                "messages": [{"role": "user", "content": " ".join(rng.choice(WORDS) for _ in range(n))}]}
        try:
            async with session.post(f"{base}/v1/chat/completions", json=body, headers=headers) as r:
                if r.status != 200:
                    return
                usage = (await r.json()).get("usage") or {}
        except Exception:  # noqa: BLE001 — keep the 1 token / word approximation
            return
        if "prompt_tokens" not in usage:
            return
        counts.append((n, int(usage["prompt_tokens"])))
    pf.calibrate(counts)


async def run_one(args, scen_text: str, conc: int, seed: int) -> RunResult:
    import aiohttp

    base = resolve_url(args.api_base.rstrip("/"))
    scen = Scenario.parse(scen_text)
    pf = PromptFactory(args.model_tokenizer, seed)
    extra = {}
    for kv in args.additional_request_params or []:
        k, _, v = kv.partition("=")
        try:
            extra[k] = json.loads(v)
        except json.JSONDecodeError:
            extra[k] = v
    samples: list[Sample] = []
    budget = {"left": args.max_requests_per_run}
    deadline = time.perf_counter() + args.max_time_per_run * 60.0 if args.time_unit == "min" else \
        time.perf_counter() + args.max_time_per_run
    timeout = aiohttp.ClientTimeout(total=args.request_timeout)

    async with aiohttp.ClientSession(timeout=timeout,
                                     connector=aiohttp.TCPConnector(limit=max(conc, 1) * 2)) as session:
        if pf.tok is None and args.task not in ("text-to-embeddings", "text-to-rerank"):
            await _calibrate(session, args, base, pf)

        async def worker(wid: int):
            # per (run seed, concurrency, worker) streams: a sweep's levels do not replay each
            # other's prompts (the server's prefix cache would turn later levels into cache hits)
            rng = random.Random((seed * 1000003 + conc) * 1000003 + wid)
            while time.perf_counter() < deadline and budget["left"] > 0:
                budget["left"] -= 1
                samples.append(await _one_request(session, args, base, scen, pf, rng, extra))

        t0 = time.perf_counter()
        await asyncio.gather(*(worker(i) for i in range(conc)))
        dur = time.perf_counter() - t0
    return RunResult(scen_text, args.task, conc, dur, samples, aggregate(samples, dur))


def _fmt_row(r: RunResult) -> str:
    a = r.aggregates
    return (f"{r.scenario:<24} {r.concurrency:>5} {a['num_completed']:>6} {a['error_rate']:>6.1%} "
            f"{a['output_throughput_tokens_per_s']:>10.1f} {a['ttft_s']['p50'] * 1e3:>9.1f} "
            f"{a['ttft_s']['p99'] * 1e3:>9.1f} {a['tpot_s']['p50'] * 1e3:>8.2f} {a['e2e_latency_s']['p50']:>8.2f}")


HEADER = (f"{'scenario':<24} {'conc':>5} {'done':>6} {'err':>6} {'out tok/s':>10} {'TTFT p50':>9} "
          f"{'TTFT p99':>9} {'TPOT p50':>8} {'E2E p50':>8}")


def cmd_benchmark(args) -> int:
    scenarios = args.traffic_scenario or DEFAULT_SCENARIOS.get(args.task, [])
    for s in scenarios:
        if not validate(s, args.task):
            print(f"invalid traffic scenario {s!r} for task {args.task}", file=sys.stderr)
            return 2
    concs = args.num_concurrency or DEFAULT_CONCURRENCY
    folder = args.experiment_folder_name or (
        f"{args.api_backend}_{args.task}_{args.api_model_name.replace('/', '_')}_{time.strftime('%Y%m%d_%H%M%S')}")
    outdir = Path(args.experiment_base_dir) / folder
    outdir.mkdir(parents=True, exist_ok=True)
    meta = {"cmd": " ".join(sys.argv), "api_backend": args.api_backend, "api_base": args.api_base,
            "model": args.api_model_name, "task": args.task, "traffic_scenario": scenarios,
            "num_concurrency": concs, "max_time_per_run": args.max_time_per_run,
            "max_requests_per_run": args.max_requests_per_run, "server_engine": args.server_engine,
            "server_gpu_type": args.server_gpu_type, "server_version": args.server_version,
            "server_gpu_count": args.server_gpu_count, "start_time": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())}
    (outdir / "experiment_metadata.json").write_text(json.dumps(meta, indent=2))
    print(HEADER, flush=True)
    summary = []
    for si, s in enumerate(scenarios):
        for c in concs:
            r = asyncio.run(run_one(args, s, c, seed=args.seed + si))
            safe = s.replace("/", "_").replace("(", "").replace(")", "").replace(",", "_")
            (outdir / f"{safe}_{args.task}_num_concurrency_{c}.json").write_text(
                json.dumps({"scenario": r.scenario, "task": r.task, "concurrency": r.concurrency,
                            "aggregates": r.aggregates, "samples": [asdict(x) for x in r.samples]}, indent=1))
            print(_fmt_row(r), flush=True)
            summary.append({"scenario": s, "concurrency": c, **r.aggregates})
    (outdir / "summary.json").write_text(json.dumps(summary, indent=2))
    _upload(args, outdir)
    errs = sum(x["num_errors"] for x in summary)
    total = sum(x["num_requests"] for x in summary)
    print(f"results: {outdir}  ({total - errs}/{total} requests ok)", flush=True)
    return 0 if total and errs < total else 1


def _upload(args, outdir: Path) -> None:
    """Object-store upload (filesystem-backed, see ``ome_amd.storage.backends``)."""
    if not args.storage_provider:
        return
    from ome_amd.storage.backends import object_store_root, write_manifest
    import shutil

    write_manifest(outdir)
    dest = object_store_root() / args.storage_provider / (args.namespace or "") / (args.storage_bucket or "") / (
        args.storage_prefix or "") / outdir.name
    shutil.copytree(outdir, dest, dirs_exist_ok=True)


def cmd_report(args) -> int:
    d = Path(args.experiment_dir)
    rows = json.loads((d / "summary.json").read_text())
    lines = ["| scenario | concurrency | completed | out tok/s | TTFT p50 ms | TTFT p99 ms | TPOT p50 ms | E2E p50 s |",
             "|---|---:|---:|---:|---:|---:|---:|---:|"]
    for r in rows:
        lines.append(f"| {r['scenario']} | {r['concurrency']} | {r['num_completed']} | "
                     f"{r['output_throughput_tokens_per_s']:.1f} | {r['ttft_s']['p50'] * 1e3:.1f} | "
                     f"{r['ttft_s']['p99'] * 1e3:.1f} | {r['tpot_s']['p50'] * 1e3:.2f} | {r['e2e_latency_s']['p50']:.2f} |")
    text = "\n".join(lines)
    (d / "report.md").write_text(text + "\n")
    print(text)
    return 0


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser("ome_amd.bench.loadgen")
    sub = ap.add_subparsers(dest="cmd", required=True)
    b = sub.add_parser("benchmark")
    a = b.add_argument
    a("--api-backend", default="openai")
    a("--api-base", required=True)
    a("--api-key", default=os.environ.get("OPENAI_API_KEY", ""))
    a("--api-model-name", required=True)
    a("--model-tokenizer", default=None)
    a("--task", default="text-to-text")
    a("--traffic-scenario", action="append")
    a("--num-concurrency", action="append", type=int)
    a("--max-time-per-run", type=float, default=15.0, help="minutes (genai-bench unit); see --time-unit")
    a("--time-unit", choices=["min", "s"], default="min")
    a("--max-requests-per-run", type=int, default=300)
    a("--additional-request-params", action="append")
    a("--experiment-folder-name", default=None)
    a("--experiment-base-dir", default="./experiments")
    a("--server-engine", default=None)
    a("--server-gpu-type", default=None)
    a("--server-version", default=None)
    a("--server-gpu-count", default=None)
    a("--storage-provider", default=None)
    a("--storage-bucket", default=None)
    a("--storage-prefix", default=None)
    a("--storage-region", default=None)
    a("--storage-account", default=None)
    a("--storage-auth-type", default=None)
    a("--storage-auth-config-file", default=None)
    a("--storage-auth-profile", default=None)
    a("--namespace", default=None)
    a("--github-owner", default=None)
    a("--github-repo", default=None)
    a("--request-timeout", type=float, default=600.0)
    a("--seed", type=int, default=42)
    r = sub.add_parser("report")
    r.add_argument("experiment_dir")
    return ap


def main(argv=None) -> int:
    args = build_parser().parse_args(argv)
    if args.cmd == "benchmark":
        return cmd_benchmark(args)
    return cmd_report(args)


if __name__ == "__main__":
    raise SystemExit(main())
