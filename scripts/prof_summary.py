#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace run (CSV) into markdown: top kernels, per-category
time per engine step (one sample kernel launch == one step), and GEMM shapes by grid."""
import collections
import csv
import sys
from pathlib import Path

CATS = [("attn_mla", ("mla_attn", "mla_reduce")), ("mla_prep", ("mla_prep",)), ("moe", ("moe_",)),
        ("gemm", ("Cijk_", "Custom_Cijk", "gemm", "Gemm")), ("attn_decode", ("paged_decode",)),
        ("attn_prefill", ("paged_prefill",)), ("rope_kv", ("rope_qkv", "kv_cache_write")),
        ("norm", ("rmsnorm",)), ("act", ("act_and_mul",)), ("sample", ("sample_kernel",)),
        ("embed", ("embedding_kernel",)), ("copy", ("copyBuffer", "fill_pending", "Fill", "index")),
        ("comm", ("rccl", "nccl", "allreduce", "AllReduce"))]


def cat_of(name: str) -> str:
    for c, keys in CATS:
        if any(k in name for k in keys):
            return c
    return "other"


def short(name: str, n: int = 90) -> str:
    return name if len(name) <= n else name[:n] + "…"


def main(d: str, last_steps: int = 0) -> None:
    d = Path(d)
    trace = next(d.rglob("*kernel_trace.csv"))
    rows = list(csv.DictReader(open(trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if last_steps:  # keep only the window covering the last N engine steps (the timed region)
        marks = [i for i, r in enumerate(rows) if "sample_kernel" in r["Kernel_Name"]]
        if len(marks) > last_steps:
            rows = rows[marks[-last_steps - 1] + 1:]
    tot = collections.Counter()
    cnt = collections.Counter()
    cat = collections.Counter()
    grids = collections.Counter()
    gcnt = collections.Counter()
    steps = 0
    t_first, t_last = None, None
    for r in rows:
        name = r["Kernel_Name"]
        dt = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        t_first = s if t_first is None else min(t_first, s)
        t_last = e if t_last is None else max(t_last, e)
        tot[name] += dt
        cnt[name] += 1
        c = cat_of(name)
        cat[c] += dt
        if c == "gemm":
            key = f"{short(name, 60)} grid=({r['Grid_Size_X']},{r['Grid_Size_Y']},{r['Grid_Size_Z']})"
            grids[key] += dt
            gcnt[key] += 1
        if "sample_kernel" in name:
            steps += 1
    busy = sum(tot.values())
    print(f"# Kernel summary: {trace.parent.name}\n")
    print(f"kernels: {len(rows)}, busy {busy / 1e6:.1f} ms over {(t_last - t_first) / 1e6:.1f} ms wall "
          f"({100 * busy / max(1, t_last - t_first):.0f}% GPU busy), engine steps (sample launches): {steps}\n")
    print("## By category (per step = total / steps)\n\n| category | total ms | % | per step us |\n|---|---:|---:|---:|")
    for c, v in cat.most_common():
        print(f"| {c} | {v / 1e6:.2f} | {100 * v / busy:.1f} | {v / 1e3 / max(1, steps):.1f} |")
    print("\n## Top kernels\n\n| total ms | % | calls | avg us | kernel |\n|---:|---:|---:|---:|---|")
    for n, v in tot.most_common(25):
        print(f"| {v / 1e6:.2f} | {100 * v / busy:.1f} | {cnt[n]} | {v / cnt[n] / 1e3:.1f} | `{short(n)}` |")
    # ---- per step type: a step ends at its sample kernel; "mixed" if it ran prefill attention
    kinds = {"decode": collections.Counter(), "mixed": collections.Counter()}
    nk = {"decode": 0, "mixed": 0}
    span = {"decode": 0, "mixed": 0}
    cur = collections.Counter()
    has_pf = False
    s0 = None
    for r in rows:
        name = r["Kernel_Name"]
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        s0 = st if s0 is None else s0
        cur[cat_of(name)] += en - st
        has_pf |= "paged_prefill" in name
        if "sample_kernel" in name:
            k = "mixed" if has_pf else "decode"
            kinds[k].update(cur)
            nk[k] += 1
            span[k] += en - s0
            cur, has_pf, s0 = collections.Counter(), False, None
    print("\n## Per step type (us per step; span = first kernel start to sample end)\n")
    print("| category | decode-only | mixed (prefill + decodes) |\n|---|---:|---:|")
    for c in sorted(set(kinds["decode"]) | set(kinds["mixed"]), key=lambda c: -(kinds["decode"][c] + kinds["mixed"][c])):
        print(f"| {c} | {kinds['decode'][c] / 1e3 / max(1, nk['decode']):.0f} | "
              f"{kinds['mixed'][c] / 1e3 / max(1, nk['mixed']):.0f} |")
    print(f"| **busy total** | {sum(kinds['decode'].values()) / 1e3 / max(1, nk['decode']):.0f} | "
          f"{sum(kinds['mixed'].values()) / 1e3 / max(1, nk['mixed']):.0f} |")
    print(f"| **span** | {span['decode'] / 1e3 / max(1, nk['decode']):.0f} | {span['mixed'] / 1e3 / max(1, nk['mixed']):.0f} |")
    print(f"| steps | {nk['decode']} | {nk['mixed']} |")
    # ---- idle time: gaps between consecutive kernels (the device is serial here), split into the
    # gap before a step's first kernel (host scheduling / launch latency between steps) and gaps
    # inside a step, attributed to the kernel that started late
    inter = {"decode": 0, "mixed": 0}
    intra = {"decode": collections.Counter(), "mixed": collections.Counter()}
    step_rows, prev_end, pending_inter = [], None, 0
    pairs, pair_n, prev_name = collections.Counter(), collections.Counter(), None
    for r in rows:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if prev_end is not None:
            gap = max(0, st - prev_end)
            if not step_rows:
                pending_inter = gap
            elif gap > 2000:
                step_rows.append(("gap", cat_of(r["Kernel_Name"]), gap))
            if gap > 2000:
                key = f"{short(prev_name, 48)}` -> `{short(r['Kernel_Name'], 48)}"
                pairs[key] += gap
                pair_n[key] += 1
        prev_name = r["Kernel_Name"]
        step_rows.append(("k", r["Kernel_Name"], 0))
        prev_end = en if prev_end is None else max(prev_end, en)
        if "sample_kernel" in r["Kernel_Name"]:
            k = "mixed" if any(t == "k" and "paged_prefill" in n for t, n, _ in step_rows) else "decode"
            inter[k] += pending_inter
            for t, n, g in step_rows:
                if t == "gap":
                    intra[k][n] += g
            step_rows, pending_inter = [], 0
    print("\n## Idle gaps (us per step)\n\n| | decode-only | mixed |\n|---|---:|---:|")
    print(f"| before the step's first kernel | {inter['decode'] / 1e3 / max(1, nk['decode']):.0f} | "
          f"{inter['mixed'] / 1e3 / max(1, nk['mixed']):.0f} |")
    for c in sorted(set(intra["decode"]) | set(intra["mixed"]), key=lambda c: -(intra["decode"][c] + intra["mixed"][c])):
        print(f"| inside, before a {c} kernel (gaps > 2 us) | {intra['decode'][c] / 1e3 / max(1, nk['decode']):.0f} | "
              f"{intra['mixed'][c] / 1e3 / max(1, nk['mixed']):.0f} |")
    print("\n## Largest idle gaps by (kernel before -> kernel after), gaps > 2 us\n")
    print("| total ms | count | avg us | previous kernel -> next kernel |\n|---:|---:|---:|---|")
    for k, v in pairs.most_common(12):
        print(f"| {v / 1e6:.2f} | {pair_n[k]} | {v / pair_n[k] / 1e3:.1f} | `{k}` |")
    dump = int(__import__("os").environ.get("PROF_DUMP_GAPS", "0"))
    if dump:   # kernel sequences around the first few gaps > 300 us (timestamps relative, us)
        print("\n## Kernel sequences around large gaps\n")
        shown, prev_end = 0, None
        for j, r in enumerate(rows):
            st = int(r["Start_Timestamp"])
            if prev_end is not None and st - prev_end > 300_000 and j > 8:
                base = int(rows[j - 8]["Start_Timestamp"])
                print("```")
                for q in rows[j - 8:j + 6]:
                    print(f"{(int(q['Start_Timestamp']) - base) / 1e3:9.1f} {(int(q['End_Timestamp']) - base) / 1e3:9.1f} "
                          f"{short(q['Kernel_Name'], 70)}")
                print("```")
                shown += 1
                if shown >= dump:
                    break
            prev_end = int(r["End_Timestamp"]) if prev_end is None else max(prev_end, int(r["End_Timestamp"]))
    print("\n## GEMMs by kernel+grid\n\n| total ms | calls | avg us | kernel / grid |\n|---:|---:|---:|---|")
    for n, v in grids.most_common(20):
        print(f"| {v / 1e6:.2f} | {gcnt[n]} | {v / gcnt[n] / 1e3:.1f} | `{n}` |")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 0)
