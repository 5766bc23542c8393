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
            # intra-process overlap: time covered by >= 2 of this process's kernels at once
            ev = []
            for r in rs:
                ev.append((int(r["Start_Timestamp"]), 1))
                ev.append((int(r["End_Timestamp"]), -1))
            ev.sort()
            depth, last, cover, multi = 0, None, 0, 0
            for t, dv in ev:
                if last is not None and depth > 0:
                    cover += t - last
                    if depth > 1:
                        multi += t - last
                depth += dv
                last = t
            print(f"kernel-covered time {cover / 1e6:.1f} ms, of which >= 2 kernels in flight {multi / 1e6:.1f} ms "
                  f"({100 * multi / max(cover, 1):.0f} %)")
            # the exchange kernels' longest instances: a wait that lasts milliseconds is a rank
            # waiting on a peer whose matching kernel is queued behind other work
            ex = sorted(((int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), r["Kernel_Name"]) for r in rs
                        if "ep_" in r["Kernel_Name"] or "wait" in r["Kernel_Name"]), reverse=True)[:8]
            if ex:
                print("longest exchange kernels (us):", ", ".join(f"{d / 1e3:.0f} {short(n, 40)}" for d, n in ex))
            print("| total ms | calls | avg us | max us | kernel |\n|---:|---:|---:|---:|---|")
            for n, v in tot.most_common(15):
                print(f"| {v / 1e6:.2f} | {cnt[n]} | {v / cnt[n] / 1e3:.1f} | {mx[n] / 1e3:.1f} | `{short(n)}` |")
            print()


if __name__ == "__main__":
    main(sys.argv[1])
