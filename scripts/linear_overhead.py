"""Host-side enqueue cost of one F.linear (bf16, hipBLASLt) with and without PyTorch TunableOp,
for decode- and prefill-sized GEMMs: the launch-bound budget of eager (prefill / mixed) steps."""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def enqueue_us(x, w, n=300):
    for _ in range(20):
        F.linear(x, w)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        F.linear(x, w)
    host = (time.perf_counter() - t) / n * 1e6
    torch.cuda.synchronize()
    dev = (time.perf_counter() - t) / n * 1e6
    return host, dev


shapes = [(256, 6144, 4096), (2048, 6144, 4096), (2048, 4096, 14336), (37, 4096, 4096)]
tensors = [(torch.randn(m, k, device="cuda").bfloat16(), torch.randn(n, k, device="cuda").bfloat16())
           for m, n, k in shapes]
for mode in ("plain", "tunableop"):
    if mode == "tunableop":
        tun = torch.cuda.tunable
        tun.enable(True)
        tun.tuning_enable(False)
        f = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ome_amd", "_tuned",
                         "tunableop_gfx950.csv")
        if os.path.exists(f):
            tun.read_file(f)
    for (m, n, k), (x, w) in zip(shapes, tensors):
        h, d = enqueue_us(x, w)
        print(f"{mode:10s} M={m:5d} N={n:5d} K={k:5d}: host enqueue {h:6.1f} us/call, wall {d:7.1f} us/call",
              flush=True)
