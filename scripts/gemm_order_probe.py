"""Is hipBLASLt at large M limited by how often it re-reads the weight from HBM?

TunableOp (scripts/tunableop_probe.py) found no better library solution on cold weights, yet the
same solutions run 1.3-1.4x faster when the weight is already cache-resident.  If the tile order
re-reads each weight panel from HBM once per row tile, slicing the projection into column
blocks whose weight fits the 256 MB Infinity Cache (each slice written straight into its columns
of the output, ld = N) should recover most of that.  Prints cold-weight times for: one call,
N-slices, M-slices.  Experiment only.
"""
import argparse

import torch
import torch.nn.functional as F

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def timeit(fn, iters=20):
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
    ap.add_argument("--ms", default="1024,2048,2304")
    a = ap.parse_args()
    dev = torch.device("cuda")
    ws = {k: [torch.randn(n, kk, device=dev, dtype=torch.bfloat16) * 0.02
              for _ in range(max(2, (1 << 30) // (n * kk * 2) + 1))] for k, (n, kk) in SHAPES.items()}
    for m in [int(v) for v in a.ms.split(",")]:
        for k, (n, kk) in SHAPES.items():
            x = torch.randn(m, kk, device=dev, dtype=torch.bfloat16)
            out = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
            w = ws[k]
            ref = F.linear(x, w[0])
            row = [f"M={m:5d} {k:8s}"]
            tf = 2 * m * n * kk / 1e6
            t0 = timeit(lambda i: torch.matmul(x, w[i % len(w)].t(), out=out))
            row.append(f"one {t0:7.1f}us {tf / t0:5.0f}TF")
            for s in (2, 4, 8):
                if n % (s * 256):
                    continue
                c = n // s

                def nsl(i, c=c, s=s):
                    wi = w[i % len(w)]
                    for j in range(s):
                        torch.matmul(x, wi[j * c:(j + 1) * c].t(), out=out[:, j * c:(j + 1) * c])

                t = timeit(nsl)
                nsl(0)
                err = (out.float() - ref.float()).abs().max().item()
                row.append(f"n/{s} {t:7.1f}us x{t0 / t:4.2f}{'' if err < 0.05 else ' BAD'}")
            for s in (2, 4):
                r = m // s

                def msl(i, r=r, s=s):
                    wi = w[i % len(w)]
                    for j in range(s):
                        torch.matmul(x[j * r:(j + 1) * r], wi.t(), out=out[j * r:(j + 1) * r])

                t = timeit(msl)
                row.append(f"m/{s} {t:7.1f}us x{t0 / t:4.2f}")
            tt = timeit(lambda i: torch.matmul(w[i % len(w)], x.t()))   # y^T = W x^T: the other tile order
            row.append(f"T {tt:7.1f}us x{t0 / tt:4.2f}")
            print("  ".join(row), flush=True)


if __name__ == "__main__":
    main()
