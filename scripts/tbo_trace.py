#!/usr/bin/env python3
"""Where does two-batch overlap lose time?  Reads a rocprofv3 --kernel-trace directory of
``scripts/tbo_bench.py --modes on`` (or off) -- one kernel_trace.csv per process -- and prints,
per process: busy time, the kernels with the largest total and the longest single instances,
the exchange wait kernels' share (a spinning wait kernel is time a rank spent waiting for its
peer), and how many kernels ran concurrently (overlap) on the device per queue."""
import collections
import csv
import sys
from pathlib import Path


def short(n, k=80):
    return n if len(n) <= k else n[:k] + "..."


def main(d):
    files = sorted(Path(d).rglob("*kernel_trace.csv"))
    if not files:
        sys.exit(f"no kernel_trace.csv under {d}")
    for f in files:
        rows = list(csv.DictReader(open(f)))
        if not rows:
            continue
        by_pid = collections.defaultdict(list)
        for r in rows:
            by_pid[r.get("Process_Id", "?")].append(r)
        for pid, rs in by_pid.items():
            rs.sort(key=lambda r: int(r["Start_Timestamp"]))
            t0, t1 = int(rs[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in rs)
            tot, cnt, mx = collections.Counter(), collections.Counter(), {}
            queues = collections.Counter()
            for r in rs:
                dur = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                n = r["Kernel_Name"]
                tot[n] += dur
                cnt[n] += 1
                mx[n] = max(mx.get(n, 0), dur)
                queues[(r.get("Queue_Id", "?"), r.get("Stream_Id", "?"))] += 1
            busy = sum(tot.values())
            wait = sum(v for n, v in tot.items() if "wait" in n or "spin" in n or "ep_signal" in n)
            print(f"## {f.name} pid {pid}: {len(rs)} kernels over {(t1 - t0) / 1e6:.1f} ms, "
                  f"kernel time {busy / 1e6:.1f} ms, exchange wait / signal kernels {wait / 1e6:.1f} ms "
                  f"({100 * wait / max(busy, 1):.0f} %)")
            print("queues/streams:", dict(queues))
            print("| total ms | calls | avg us | max us | kernel |\n|---:|---:|---:|---:|---|")
            for n, v in tot.most_common(15):
                print(f"| {v / 1e6:.2f} | {cnt[n]} | {v / cnt[n] / 1e3:.1f} | {mx[n] / 1e3:.1f} | `{short(n)}` |")
            print()


if __name__ == "__main__":
    main(sys.argv[1])
