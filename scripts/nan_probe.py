#!/usr/bin/env python3
"""Where do non-finite values appear in a decode warm-up forward (padding rows, seq_len 0)?
Runs tiny-moe (bf16 and fp8) through ModelRunner._decode_forward with hooks on every op's output."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("OME_TUNE_GEMM", "0")
from ome_amd import ops  # noqa: E402
from ome_amd.runtime.engine import Engine, EngineArgs  # noqa: E402

for quant in (None, "fp8"):
    eng = Engine(EngineArgs(model="tiny-moe", device="cuda", max_running_requests=8, context_length=256,
                            cuda_graph=False, quantization=quant, max_total_tokens=4096))
    bad = []
    for name in ("linear", "fp8_linear", "fused_moe", "paged_decode", "fused_add_rmsnorm", "rmsnorm", "act_and_mul",
                 "moe_route", "embedding", "fp8_quant"):
        fn = getattr(ops, name, None)
        if fn is None:
            continue

        def wrap(f, nm):
            def g(*a, **k):
                r = f(*a, **k)
                outs = r if isinstance(r, tuple) else (r,)
                for o in outs:
                    if isinstance(o, torch.Tensor) and o.is_floating_point() and not torch.isfinite(o.float()).all():
                        bad.append(nm)
                for t in a:
                    if isinstance(t, torch.Tensor) and t.is_floating_point() and not torch.isfinite(t.float()).all():
                        bad.append(nm + ":in")
                return r
            return g
        setattr(ops, name, wrap(fn, name))
    r = eng.runner
    d = r.dbuf
    d.hnp[:] = 0
    d.hnp[d.off["slots"]:d.off["slots"] + d.bmax] = -1
    d.hnp[d.off["req_idx"]:d.off["req_idx"] + d.bmax] = r.slots.max_reqs - 1
    d.dev.copy_(d.host)
    r._decode_forward(4)
    torch.cuda.synchronize()
    print(quant, "non-finite at:", sorted(set(bad))[:20], flush=True)
