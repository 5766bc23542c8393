#!/usr/bin/env python3
"""Largest GPU idle gaps in a rocprofv3 kernel + memory-copy trace: which op precedes and which
follows each gap (is the device waiting for the host, or for a DMA?).
usage: gap_probe.py <rocprof output dir> [top N] [tail ms: only the last ms of the trace]"""
import csv
import glob
import os
import sys
from collections import Counter


def load(d):
    ops = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K:" + r["Kernel_Name"][:90]))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                        "C:" + r.get("Direction", "?") + ":" + r.get("Bytes", r.get("Size", "?"))))
    ops.sort()
    return ops


def main():
    d, top = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25
    ops = load(d)
    if len(sys.argv) > 3:
        t_end = max(e for _, e, _ in ops)
        ops = [o for o in ops if o[0] >= t_end - float(sys.argv[3]) * 1e6]
    gaps = []
    end = ops[0][1]
    prev = ops[0][2]
    for s, e, n in ops[1:]:
        if s > end:
            gaps.append((s - end, prev, n))
        if e > end:
            end, prev = e, n
    tot = sum(g for g, _, _ in gaps)
    span = ops[-1][1] - ops[0][0]
    print(f"ops {len(ops)} span {span / 1e6:.1f} ms idle {tot / 1e6:.1f} ms ({100 * tot / span:.1f}%)")
    by_next = Counter()
    by_pair = Counter()
    for g, p, n in gaps:
        if g > 20000:
            by_next[n[:60]] += g
            by_pair[(p[:50], n[:50])] += g
    print("\nidle (gaps > 20 us) by following op, ms:")
    for k, v in by_next.most_common(15):
        print(f"  {v / 1e6:8.2f}  {k}")
    print("\nidle (gaps > 20 us) by (previous, following), ms:")
    for k, v in by_pair.most_common(15):
        print(f"  {v / 1e6:8.2f}  {k[0]}  ->  {k[1]}")
    # context of the three largest gaps: the ops around each (start relative to the gap, duration)
    idx = sorted(range(1, len(ops)), key=lambda i: ops[i][0] - max(o[1] for o in ops[max(0, i - 8):i]), reverse=True)
    for i in idx[:3]:
        g0 = max(o[1] for o in ops[max(0, i - 8):i])
        print(f"\ncontext of a {(ops[i][0] - g0) / 1e3:.1f} us gap:")
        for s_, e_, n_ in ops[max(0, i - 10):i + 4]:
            print(f"  {(s_ - g0) / 1e3:10.1f} us  dur {(e_ - s_) / 1e3:8.1f}  {n_[:90]}")
    print(f"\ntop {top} gaps:")
    for g, p, n in sorted(gaps, reverse=True)[:top]:
        print(f"  {g / 1e3:9.1f} us  {p[:60]}  ->  {n[:60]}")


if __name__ == "__main__":
    main()
