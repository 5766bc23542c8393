#!/usr/bin/env python3
"""Serving sweep over HTTP/SSE (verdict r02 item 3): one ome_amd.runtime.server (random-init
Llama-3-8B, bf16, --context-length 8192) driven by the closed-loop streaming client of
ome_amd.bench.e2e at several concurrencies for the five default BenchmarkJob scenarios.
Writes one JSON line per point to gpurun_out/e2e_sweep.jsonl."""
import argparse
import asyncio
import json
import os
import sys
import time
import urllib.request

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd.bench import e2e  # noqa: E402
from ome_amd.bench.scenarios import Scenario  # noqa: E402

SCENARIOS = ["N(480,240)/(300,150)", "D(100,100)", "D(100,1000)", "D(2000,200)", "D(7800,200)"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--concurrency", default="1,8,32,128,256")
    ap.add_argument("--scenarios", default="|".join(SCENARIOS))
    ap.add_argument("--warm-s", type=float, default=4.0)
    ap.add_argument("--window-s", type=float, default=8.0)
    ap.add_argument("--context-length", type=int, default=8192)
    ap.add_argument("--out", default="gpurun_out/e2e_sweep.jsonl")
    a = ap.parse_args()
    cs = [int(c) for c in a.concurrency.split(",")]
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    proc, base = e2e.start_server("llama-3-8b", max(cs), a.context_length, ["--chunked-prefill-size", "8192"],
                                  log_path=os.path.join(os.path.dirname(a.out) or ".", "e2e_sweep_server.log"))
    try:
        e2e.wait_ready(base, proc)
        with open(a.out, "w") as f:
            for sc in a.scenarios.split("|"):
                for c in cs:
                    t0 = time.time()
                    r = asyncio.run(e2e._client(base, Scenario.parse(sc), c, 128256, a.context_length - 2, a.warm_s,
                                                a.window_s, 99))
                    row = {"scenario": sc, "concurrency": c, "output_tok_s": round(r["tokens"] / r["window_s"], 1),
                           "p50_ttft_ms": round(r["p50_ttft_ms"], 1) if r["p50_ttft_ms"] is not None else None,
                           "requests_started": r["requests_started_in_window"], "errors": r["errors"],
                           "wall_s": round(time.time() - t0, 1)}
                    f.write(json.dumps(row) + "\n")
                    f.flush()
                    print(json.dumps(row), flush=True)
                    # drain: the client's cancelled streams abort their requests server-side;
                    # wait until the engine is idle before the next point
                    t1 = time.time()
                    while time.time() - t1 < 60:
                        try:
                            with urllib.request.urlopen(base + "/get_server_info", timeout=5) as resp:
                                info = json.loads(resp.read())
                            if info.get("running", 0) == 0 and info.get("waiting", 0) == 0:
                                break
                        except OSError:
                            pass
                        time.sleep(0.5)
    finally:
        e2e.stop_server(proc)


if __name__ == "__main__":
    main()
