"""End-to-end serving benchmark: the HTTP path a BenchmarkJob exercises (``bench.py --e2e``).

A ``ome_amd.runtime.server`` child process serves random-init Llama-3-8B on one GPU; a
closed-loop asyncio client keeps ``concurrency`` streaming ``/v1/completions`` requests in flight
(prompt = token ids of the scenario's input length, ``ignore_eos``, temperature 0 -- the
genai-bench defaults of the reference's BenchmarkJob, ``benchmark_webhook.go:84-89`` and
``config/samples/benchmark/llama3-1-70b-instruct.yaml:16-35``).  Every SSE chunk carries the
running ``usage`` (``stream_options.continuous_usage_stats``), so tokens are counted exactly as
they arrive at the client.  A "step" is ``step_s`` seconds of wall time: W warm-up steps, then K
timed steps; output tok/s = tokens streamed inside the timed window / its length; TTFT = time
from request send to the first content chunk, for requests whose first chunk lands in the window.
"""
from __future__ import annotations

import asyncio
import json
import os
import random
import signal
import socket
import subprocess
import sys
import time

from ome_amd.bench.scenarios import Scenario


_REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child_env(extra: dict | None = None) -> dict:
    """Environment for server / router children: the repo importable from any working directory
    (e.g. under ``cd /tmp && rocprofv3 ... -- python3 /path/bench.py``)."""
    env = dict(os.environ)
    env["PYTHONPATH"] = _REPO + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    env.update(extra or {})
    return env


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def start_server(model: str, concurrency: int, context_length: int, extra: list[str] | None = None,
                 log_path: str | None = None) -> tuple[subprocess.Popen, str]:
    port = _free_port()
    cmd = [sys.executable, "-m", "ome_amd.runtime.server", "--model-path", f"random://{model}", "--host",
           "127.0.0.1", "--port", str(port), "--max-running-requests", str(concurrency), "--context-length",
           str(context_length), *(extra or [])]
    out = open(log_path, "w") if log_path else subprocess.DEVNULL
    p = subprocess.Popen(cmd, stdout=out, stderr=subprocess.STDOUT, start_new_session=True, env=child_env())
    return p, f"http://127.0.0.1:{port}"


def wait_ready(base: str, proc: subprocess.Popen, timeout: float = 900.0) -> None:
    import urllib.request

    t0 = time.time()
    while time.time() - t0 < timeout:
        if proc.poll() is not None:
            raise RuntimeError(f"server exited with {proc.returncode} during start-up")
        try:
            with urllib.request.urlopen(base + "/health", timeout=2) as r:
                if r.status == 200:
                    return
        except OSError:
            pass
        time.sleep(1.0)
    raise TimeoutError("server did not become ready")


def stop_server(proc: subprocess.Popen) -> None:
    if proc.poll() is None:
        try:
            os.killpg(proc.pid, signal.SIGTERM)   # the child's own session: nothing else is in it
            proc.wait(timeout=30)
        except (ProcessLookupError, subprocess.TimeoutExpired):
            try:
                os.killpg(proc.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass


async def _client(base: str, scen: Scenario, concurrency: int, vocab: int, max_in: int, warm_s: float,
                  timed_s: float, seed: int) -> dict:
    import aiohttp

    events: list[tuple[float, int]] = []      # (arrival time, new output tokens)
    firsts: list[tuple[float, float]] = []    # (first-chunk time, ttft)
    t_start = time.perf_counter()
    t0, t1 = t_start + warm_s, t_start + warm_s + timed_s
    stop = asyncio.Event()

    async def one(session, rng):
        n_in, n_out = scen.sample(rng, max_in=max_in)
        n_out = max(1, min(n_out, max_in + 1 - n_in))
        ids = [rng.randrange(3, vocab) for _ in range(n_in)]
        body = {"model": "m", "prompt": ids, "max_tokens": n_out, "temperature": 0.0, "ignore_eos": True,
                "stream": True, "stream_options": {"include_usage": True, "continuous_usage_stats": True}}
        ts = time.perf_counter()
        seen = 0
        first = True
        async with session.post(base + "/v1/completions", json=body) as r:
            if r.status != 200:
                raise RuntimeError(f"HTTP {r.status}: {(await r.text())[:200]}")
            async for raw in r.content:
                line = raw.strip()
                if not line.startswith(b"data: {"):
                    continue
                ev = json.loads(line[6:])
                n = int((ev.get("usage") or {}).get("completion_tokens", seen))
                now = time.perf_counter()
                if n > seen:
                    events.append((now, n - seen))
                    if first:
                        firsts.append((now, now - ts))
                        first = False
                    seen = n

    errors: list[str] = []

    async def worker(wid):
        rng = random.Random(seed * 7919 + wid)
        async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=3600)) as session:
            while not stop.is_set():
                try:
                    await one(session, rng)
                except asyncio.CancelledError:
                    raise
                except Exception as e:  # noqa: BLE001 — counted and reported, the loop keeps its load
                    errors.append(f"{type(e).__name__}: {e}")
                    await asyncio.sleep(0.05)

    tasks = [asyncio.create_task(worker(i)) for i in range(concurrency)]
    await asyncio.sleep(max(0.0, t1 - time.perf_counter()))
    stop.set()
    for t in tasks:
        t.cancel()
    await asyncio.gather(*tasks, return_exceptions=True)
    toks = sum(n for ts, n in events if t0 <= ts < t1)
    ttfts = sorted(tt for ts, tt in firsts if t0 <= ts < t1)
    return {"tokens": toks, "window_s": timed_s, "p50_ttft_ms": 1000 * ttfts[len(ttfts) // 2] if ttfts else None,
            "requests_started_in_window": len(ttfts), "errors": len(errors), "first_error": errors[0] if errors else None}


def run(model: str, scenario: str, concurrency: int, context_length: int, steps: int, warmup: int,
        step_s: float, vocab: int = 128256, server_args: list[str] | None = None, log_path: str | None = None,
        seed: int = 1234) -> dict:
    proc, base = start_server(model, concurrency, context_length, server_args, log_path)
    try:
        wait_ready(base, proc)
        scen = Scenario.parse(scenario)
        res = asyncio.run(_client(base, scen, concurrency, vocab, context_length - 2, warmup * step_s,
                                  steps * step_s, seed))
    finally:
        stop_server(proc)
    res["value"] = res["tokens"] / res["window_s"] if res["window_s"] > 0 else 0.0
    return res
