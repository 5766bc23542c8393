"""How much does per-shape hipBLASLt / rocBLAS solution search buy on the headline's projections?

Times ``F.linear`` (bf16, Llama-3-8B qkv / o / gate_up / down) at the M values the serving
loop produces, first with the library's default heuristic, then with PyTorch's TunableOp
(which benchmarks every hipBLASLt + rocBLAS solution for the exact shape).  The tuned
solution table is written to gpurun_out/tunableop_results.csv so the winning algorithm
indices can be inspected.  Experiment only: nothing here is on the serving path.
"""
import argparse
import os
import time

import torch
import torch.nn.functional as F

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def timeit(fn, iters=30):
    """fn(i) for rotating weight copies i: every call reads its weight cold from HBM, as in serving."""
    for i in range(3):
        fn(i)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for i in range(iters):
        fn(i)
    ev[1].record()
    torch.cuda.synchronize()
    return ev[0].elapsed_time(ev[1]) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="256,512,1024,1280,2048,2304")
    ap.add_argument("--out", default="gpurun_out/tunableop_results.csv")
    a = ap.parse_args()
    ms = [int(m) for m in a.ms.split(",")]
    dev = torch.device("cuda")
    # enough copies of each weight that a rotation exceeds the caches (>= 1 GiB per shape)
    ws = {k: [torch.randn(n, kk, device=dev, dtype=torch.bfloat16) * 0.02
              for _ in range(max(2, (1 << 30) // (n * kk * 2) + 1))] for k, (n, kk) in SHAPES.items()}
    xs = {(m, k): torch.randn(m, SHAPES[k][1], device=dev, dtype=torch.bfloat16) for m in ms for k in SHAPES}
    def run(key):
        w = ws[key[1]]
        return lambda i: F.linear(xs[key], w[i % len(w)])

    base = {key: timeit(run(key)) for key in xs}
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_max_tuning_duration(200)
    tun.set_rotating_buffer_size(1024)   # MiB: candidates are timed on cold operands
    tun.set_filename(a.out)
    t0 = time.time()
    for key in xs:      # the first call per shape tunes it
        F.linear(xs[key], ws[key[1]][0])
        torch.cuda.synchronize()
        print(f"tuned {key} ({time.time() - t0:.0f}s)", flush=True)
    tun.tuning_enable(False)
    tuned = {key: timeit(run(key)) for key in xs}
    pass  # TunableOp writes the results file itself at exit
    tot_b = tot_t = 0.0
    for (m, k) in xs:
        n, kk = SHAPES[k]
        tf = 2 * m * n * kk / 1e6
        b, t = base[(m, k)], tuned[(m, k)]
        tot_b += b
        tot_t += t
        print(f"M={m:5d} {k:8s} default {b:8.1f}us {tf / b:6.0f}TF  tuned {t:8.1f}us {tf / t:6.0f}TF  x{b / t:.2f}")
    print(f"sum default {tot_b:.0f}us tuned {tot_t:.0f}us  x{tot_b / tot_t:.3f}")


if __name__ == "__main__":
    main()
