#!/usr/bin/env python3
"""BenchmarkJob protocol sweep through the operator slice on the GPU box (SURVEY §7.3,
BASELINE.md "Measurement protocol"): random-init Llama-3-8B InferenceService on 1 GPU, the
headline scenario N(480,240)/(300,150) (or --scenario), concurrency 1..256, 15 s / 100 requests per
iteration, temperature 0 -- driven by a BenchmarkJob through ome_amd.bench.loadgen.  Writes the
summary table to --out (JSON + markdown)."""
import argparse
import json
import os
import sys
import tempfile
from pathlib import Path

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd.bench import operator_slice  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenario", default="N(480,240)/(300,150)")
    ap.add_argument("--concurrency", default="1,2,4,8,16,32,64,128,256")
    ap.add_argument("--max-time", type=int, default=15)
    ap.add_argument("--max-requests", type=int, default=100)
    ap.add_argument("--preset", default="llama-3-8b")
    ap.add_argument("--out", default="gpurun_out/operator_sweep")
    a = ap.parse_args()
    work = Path(tempfile.mkdtemp(prefix="ome_slice_"))
    res = operator_slice.run(work, preset=a.preset, scenarios=(a.scenario,),
                             concurrency=[int(c) for c in a.concurrency.split(",")],
                             max_time=a.max_time, max_requests=a.max_requests,
                             extra_args=["--max-running-requests", "256"],
                             log=lambda m: print(m, flush=True), bench_timeout=3000)
    out = Path(a.out)
    out.mkdir(parents=True, exist_ok=True)
    (out / "summary.json").write_text(json.dumps(res["summary"], indent=1))
    lines = [f"# BenchmarkJob sweep via the operator slice: {a.preset} (random init), scenario {a.scenario}, "
             f"{a.max_time} s / {a.max_requests} requests per iteration, 1 GPU",
             f"# timings: {res['timings']}", "",
             "| concurrency | completed | output tok/s | req/s | TTFT p50 ms | TTFT p99 ms | TPOT p50 ms | e2e p50 s |",
             "|---:|---:|---:|---:|---:|---:|---:|---:|"]
    for s in res["summary"]:
        lines.append(f"| {s['concurrency']} | {s['num_completed']} | {s['output_throughput_tokens_per_s']:.1f} | "
                     f"{s.get('requests_per_s', 0):.2f} | {s['ttft_s']['p50'] * 1e3:.1f} | {s['ttft_s']['p99'] * 1e3:.1f} | "
                     f"{s['tpot_s']['p50'] * 1e3:.2f} | {s['e2e_latency_s']['p50']:.2f} |")
    (out / "summary.md").write_text("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
