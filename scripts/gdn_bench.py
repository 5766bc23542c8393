"""Gated DeltaNet recurrence (``ome_gdn_scan``) at the Qwen3-Next-80B shape (Hk 16, Hv 32,
dk = dv = 128): long single prefills, batched prefills, decode batches.  Prints time per launch,
ns per row (sequence-serial latency) and the error against the fp32 reference on a small case."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import ops  # noqa: E402
from ome_amd.ops import reference as ref  # noqa: E402

Hk, Hv, dk, dv = 16, 32, 128, 128
kd, vd = Hk * dk, Hv * dv


def case(lens, iters=10, v1=False):
    T, S = sum(lens), len(lens)
    torch.manual_seed(0)
    proj = torch.randn(T, 2 * kd + vd + 2 * Hv, device="cuda").bfloat16()
    q, k, v = proj[:, :kd], proj[:, kd:2 * kd], proj[:, 2 * kd:2 * kd + vd]
    b, a = proj[:, 2 * kd + vd:2 * kd + vd + Hv], proj[:, 2 * kd + vd + Hv:]
    A_log, dtb = torch.rand(Hv, device="cuda"), torch.randn(Hv, device="cuda")
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device="cuda")
    slot = torch.arange(S, dtype=torch.int32, device="cuda")
    reset = torch.ones(S, dtype=torch.int32, device="cuda")
    st = torch.zeros(S, Hv, dv, dk, device="cuda")
    out = torch.empty(T, vd, dtype=torch.bfloat16, device="cuda")
    fn = lambda: ops.gdn_scan(q, k, v, a, b, A_log, dtb, st, cu, slot, reset, Hv, Hk, out=out, v1=v1)  # noqa: E731
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    us = (time.perf_counter() - t0) / iters * 1e6
    err = None
    if T <= 64:
        c = lambda x: x.cpu()  # noqa: E731
        st_r = torch.zeros(S, Hv, dv, dk)
        want = ref.gdn_scan(c(q), c(k), c(v), c(a), c(b), c(A_log), c(dtb), st_r, c(cu), c(slot), c(reset), Hv, Hk,
                            torch.empty(T, vd, dtype=torch.bfloat16))
        err = (out.float().cpu() - want.float()).abs().max().item()
    return us, err


for name, lens in [("prefill 1x4096", [4096]), ("prefill 1x1024", [1024]), ("prefill 8x512", [512] * 8),
                   ("prefill 32x128", [128] * 32), ("decode 1", [1]), ("decode 64", [1] * 64),
                   ("decode 256", [1] * 256), ("check 3 seqs", [5, 1, 20])]:
    for v1 in ((False,) if os.environ.get("OME_GDN_NC") else (False, True)):   # NC sweeps: v3 only
        us, err = case(lens, v1=v1)
        tag = "v1" if v1 else "v3/nc" + os.environ.get("OME_GDN_NC", "auto")
        print(f"{name:16s} {tag:9s} {us:9.1f} us  {us * 1e3 / max(lens):8.1f} ns/row" +
              (f"  max|err| {err:.3g}" if err is not None else ""), flush=True)
