#!/usr/bin/env python3
"""Small-shape correctness sweep of ome_gemm_xl: where (rows / columns / K extent) a result goes wrong."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import ops  # noqa: E402

DEV = torch.device("cuda")
torch.manual_seed(0)


def case(M, N, K, bn, nwg, probe=0, epi=0):
    x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / K ** 0.5
    ref = F.linear(x.float(), w.float())
    wi = w
    if epi == 2:
        wi = ops.interleave_gate_up(w)
        ref = F.silu(ref[:, :N // 2]) * ref[:, N // 2:]
    out = torch.full((M, N // 2 if epi else N), float("nan"), device=DEV, dtype=torch.bfloat16)
    y = ops.gemm_xl(x, wi, out=out, epi=epi, bn=bn, nwg=nwg, probe=probe).float()
    torch.cuda.synchronize()
    d = (y - ref).abs()
    bad = d > 0.05 * ref.abs().max() + 1e-2
    err = (d.nan_to_num(1e9).max() / ref.abs().max()).item()
    msg = f"M={M} N={N} K={K} bn={bn} nwg={nwg} probe={probe} epi={epi}: err {err:.3g}"
    if bad.any():
        rows = bad.any(1).nonzero().flatten()
        cols = bad.any(0).nonzero().flatten()
        msg += (f"  bad {bad.sum().item()}/{bad.numel()} rows[{rows.min().item()}..{rows.max().item()}] n={rows.numel()}"
                f" cols[{cols.min().item()}..{cols.max().item()}] n={cols.numel()}")
        # pattern of bad columns mod 64 and rows mod 64
        cm = torch.zeros(64, dtype=torch.int64)
        for c in cols.tolist():
            cm[c % 64] += 1
        rm = torch.zeros(64, dtype=torch.int64)
        for r in rows.tolist():
            rm[r % 64] += 1
        msg += f"\n   cols%64 {cm.tolist()}\n   rows%64 {rm.tolist()}"
    print(msg, flush=True)


PROBE = int(os.environ.get("XL_DEBUG_PROBE", "0"))
for bn in ((128,) if PROBE == 5 else (256, 128)):
    case(256, bn, 32, bn, 8, 1)
    case(256, bn, 128, bn, 8, 1)
    case(256, bn, 32, bn, 8, PROBE)
    case(256, bn, 64, bn, 8, PROBE)
    case(256, bn, 128, bn, 8, PROBE)
    case(256, bn, 256, bn, 8, PROBE)
    case(256, bn, 1024, bn, 8, PROBE)
    case(256, 2 * bn, 1024, bn, 8, PROBE)
    case(512, 2 * bn, 1024, bn, 8, PROBE)
    case(200, bn, 256, bn, 8, PROBE)
    case(256, bn, 256, bn, 8, PROBE, 2)
    case(512, 2048, 1024, bn, 16, PROBE)
    case(512, 2048, 1024, bn, 32, PROBE)
    case(512, 2048, 1024, bn, 64, PROBE)
    case(1024, 4096, 4096, bn, 256, PROBE)
    case(1000, 4096, 4096, bn, 248, PROBE)
    case(1024, 4096, 4096, bn, 256, PROBE, 2)
