"""Prefill-decode disaggregated serving benchmark (``bench.py --pd P+D``; BASELINE config 4,
reference ``config/runtimes/srt/meta/llama-3-1-70b-instruct-pd-rt.yaml:67-70,153-156,213-224``).

P prefill servers (``--disaggregation-mode prefill``) and D decode servers
(``--disaggregation-mode decode``, each with its own KV bootstrap port) run as separate
processes, with the PD router (``ome_amd.router --pd-disaggregation``) in front; the closed-loop
streaming client of :mod:`ome_amd.bench.e2e` drives the router, so every request takes the real
path: router -> prefill engine (prompt + first token) -> KV pages to the decode engine (the
same-node IPC fast path, csrc/comm/kvlink.hip) -> decode engine streams the rest.
With at least P + D GPUs every server gets its own device (prefill i -> GPU i, decode j -> GPU
P + j); on a smaller box they share the visible devices round-robin, each bounded by
``--max-total-tokens`` so the co-located engines fit side by side.  A prefill engine only holds
the prompts in flight (64K tokens of KV); a decode engine holds every running request's whole
context (512K tokens: 256 requests x ~800 tokens without preemption).
"""
from __future__ import annotations

import asyncio
import os
import subprocess
import sys
import time

from ome_amd.bench import e2e
from ome_amd.bench.scenarios import Scenario


def _gpu_count() -> int:
    import torch

    return torch.cuda.device_count()   # does not initialise the GPU on this stack


def _server_info(url: str) -> dict:
    import json
    import urllib.request

    try:
        with urllib.request.urlopen(url + "/get_server_info", timeout=10) as r:
            return json.loads(r.read())
    except OSError:
        return {}


def run(model: str, scenario: str, concurrency: int, context_length: int, steps: int, warmup: int, step_s: float,
        n_prefill: int = 1, n_decode: int = 1, max_total_tokens: int = 65536, decode_total_tokens: int = 524288,
        log_dir: str | None = None,
        extra: list[str] | None = None) -> dict:
    ngpu = max(1, _gpu_count())
    procs: list[subprocess.Popen] = []
    prefill_urls, decode_urls = [], []
    try:
        roles = [("prefill", i) for i in range(n_prefill)] + [("decode", j) for j in range(n_decode)]
        for idx, (role, i) in enumerate(roles):
            env = e2e.child_env({"HIP_VISIBLE_DEVICES": str(idx % ngpu)})
            port = e2e._free_port()
            args = [sys.executable, "-m", "ome_amd.runtime.server", "--model-path", f"random://{model}", "--host",
                    "127.0.0.1", "--port", str(port), "--max-running-requests", str(concurrency),
                    "--context-length", str(context_length), "--disaggregation-mode", role,
                    "--max-total-tokens", str(max_total_tokens if role == "prefill" else decode_total_tokens),
                    "--mem-frac", "0.95", *(extra or [])]
            if role == "decode":
                args += ["--disaggregation-bootstrap-port", str(e2e._free_port())]
            out = open(os.path.join(log_dir, f"{role}{i}.log"), "w") if log_dir else subprocess.DEVNULL
            p = subprocess.Popen(args, stdout=out, stderr=subprocess.STDOUT, env=env, start_new_session=True)
            procs.append(p)
            (prefill_urls if role == "prefill" else decode_urls).append(f"http://127.0.0.1:{port}")
            e2e.wait_ready(f"http://127.0.0.1:{port}", p)   # one at a time: co-located engines size KV in turn
        rport = e2e._free_port()
        rargs = [sys.executable, "-m", "ome_amd.router", "--host", "127.0.0.1", "--port", str(rport),
                 "--pd-disaggregation", "--health-check-interval-secs", "1"]
        for u in prefill_urls:
            rargs += ["--prefill", u]
        for u in decode_urls:
            rargs += ["--decode", u]
        out = open(os.path.join(log_dir, "router.log"), "w") if log_dir else subprocess.DEVNULL
        rp = subprocess.Popen(rargs, stdout=out, stderr=subprocess.STDOUT, start_new_session=True, env=e2e.child_env())
        procs.append(rp)
        base = f"http://127.0.0.1:{rport}"
        e2e.wait_ready(base, rp, timeout=120)
        time.sleep(2.0)   # first health sweep marks the workers ready
        from ome_amd.models.config import preset

        scen = Scenario.parse(scenario)
        res = asyncio.run(e2e._client(base, scen, concurrency, preset(model).vocab_size, context_length - 2, warmup * step_s,
                                      steps * step_s, 4321))
        res["kv_transfer"] = [_server_info(u).get("kv_transfer") for u in prefill_urls]
    finally:
        for p in reversed(procs):
            e2e.stop_server(p)
    res["value"] = res["tokens"] / res["window_s"] if res["window_s"] > 0 else 0.0
    res["gpus"] = min(ngpu, n_prefill + n_decode)
    return res
