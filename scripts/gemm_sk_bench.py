#!/usr/bin/env python3
"""ome_gemm_sk (csrc/kernels/gemm_sk.hip) vs hipBLASLt (F.linear) on the Llama-3-8B projections.

Cold weights: every call uses the next of several weight copies (> 256 MiB Infinity Cache in
total), as in a layer stack; activations stay warm.  gate_up is timed as the serving path runs
it: hipBLASLt GEMM + act_and_mul against the fused SiLU*mul epilogue (interleaved weight).
Every stream-K configuration is checked against an fp32 reference before it is timed.
Prints one line per (shape, M); --json PATH writes the best configuration per (shape, M), and
--table PATH the planner table of ``ops.gemm_sk_plan`` (``ome_amd/_tuned/gemm_sk_gfx950.json``).
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ome_amd import ops  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
          "lm_head": (128256, 4096),
          # Llama-3-70B at TP = 1 (BASELINE config 3 on one 288 GB MI355X)
          "qkv70": (10240, 8192), "o70": (8192, 8192), "gate_up70": (57344, 8192), "down70": (8192, 28672),
          "lm_head70": (128256, 8192)}
DEV = torch.device("cuda")


def bench(fn, n_w, iters=30):
    for i in range(4):
        fn(i % n_w)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(i % n_w)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1000 / iters


TILES = ((256, 128), (256, 256), (128, 256), (128, 128))   # (bm, bn)


def nwg_cands(M, N, K, bn, bm):
    T = ops.gemm_sk_tiles(M, N, bn, bm)
    c = {256, 240, 224, 192}
    for k in (1, 2, 3, 4, 6, 8):
        if T % k == 0 and (T // k) % 8 == 0 and T // k <= 256:
            c.add(T // k)
    return sorted(x for x in c if ops.gemm_sk_ok(M, N, K, bn, x, bm))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="128,192,256,384,512,768,1024,1280,1536,1792,2048,2304")
    ap.add_argument("--shapes", default=",".join(SHAPES))
    ap.add_argument("--json", default=None)
    ap.add_argument("--table", default=None, help="write the ops.gemm_sk_plan table here")
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--merge", action="store_true", help="--table: update the existing table's shapes")
    a = ap.parse_args()
    ms = [int(v) for v in a.m.split(",")]
    table, plan = {}, {}
    for name in a.shapes.split(","):
        N, K = SHAPES[name]
        epi = 2 if name.startswith("gate_up") else 0
        n_w = max(2, -(-(600 << 20) // (N * K * 2)))
        ws = [torch.randn(N, K, device=DEV, dtype=torch.bfloat16) / K ** 0.5 for _ in range(n_w)]
        wi = [ops.interleave_gate_up(w) for w in ws] if epi == 2 else ws
        for M in ms:
            if name.startswith("lm_head") and M > 512:
                continue
            x = torch.randn(M, K, device=DEV, dtype=torch.bfloat16)
            ref = F.linear(x, ws[0]).float()
            if epi == 2:
                ref = F.silu(ref[:, :N // 2]) * ref[:, N // 2:]
            fl = 2 * M * N * K
            if epi == 2:   # the serving fallback: hipBLASLt on the interleaved weight + interleaved act
                t_lib = bench(lambda i: ops.act_and_mul(F.linear(x, wi[i]), interleaved=True), n_w, a.iters)
            else:
                t_lib = bench(lambda i: F.linear(x, ws[i]), n_w, a.iters)
            row = [f"M={M:5d} {name:8s} hipblaslt{'+act' if epi else ''} {t_lib:7.1f}us {fl / t_lib / 1e6:5.0f}TF"]
            best = None
            res = []
            out = torch.empty(M, N // 2 if epi else N, device=DEV, dtype=torch.bfloat16)
            for bm, bn in TILES:
                for nwg in nwg_cands(M, N, K, bn, bm):
                    y = ops.gemm_sk(x, wi[0], out=out, epi=epi, bn=bn, nwg=nwg, bm=bm)
                    err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
                    if not err < 2e-2:
                        row.append(f"{bm}x{bn}/w{nwg} ERR {err:.3g}")
                        continue
                    t = bench(lambda i: ops.gemm_sk(x, wi[i], out=out, epi=epi, bn=bn, nwg=nwg, bm=bm), n_w, a.iters)
                    res.append((t, bm, bn, nwg))
                    if best is None or t < best[0]:
                        best = (t, bm, bn, nwg)
            res.sort()
            row.append(" ".join(f"{m}x{b}/w{n} {t:6.1f}" for t, m, b, n in res[:4]))
            if best:
                row.append(f"BEST {best[0]:6.1f}us {fl / best[0] / 1e6:5.0f}TF x{t_lib / best[0]:.2f}")
                table.setdefault(name, {})[str(M)] = {"bm": best[1], "bn": best[2], "nwg": best[3],
                                                      "us": round(best[0], 1), "lib_us": round(t_lib, 1)}
                plan.setdefault(f"{N},{K},{epi}", {})[str(M)] = table[name][str(M)]
            print("  ".join(row), flush=True)
        del ws, wi
        torch.cuda.empty_cache()
    if a.json:
        with open(a.json, "w") as f:
            json.dump(table, f, indent=1)
    if a.table:
        if a.merge and os.path.exists(a.table):
            with open(a.table) as f:
                old = json.load(f).get("shapes", {})
            for k, v in plan.items():
                old.setdefault(k, {}).update(v)
            plan = old
        with open(a.table, "w") as f:
            json.dump({"device": torch.cuda.get_device_name(), "method": "scripts/gemm_sk_bench.py, cold weights",
                       "shapes": plan}, f, indent=1)


if __name__ == "__main__":
    main()
