#!/usr/bin/env python3
"""Average rocprofv3 counter_collection.csv values per kernel name under a directory tree."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root):
    for path in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        agg = defaultdict(lambda: defaultdict(list))
        with open(path) as f:
            for row in csv.DictReader(f):
                k = row.get("Kernel_Name", "?")
                if "gemm" not in k and "Cijk" not in k:
                    continue
                agg[k[:90]][row["Counter_Name"]].append(float(row["Counter_Value"]))
        print(f"== {os.path.relpath(path, root)}")
        for k, cs in agg.items():
            vals = {c: sum(v) / len(v) for c, v in cs.items()}
            n = max(len(v) for v in cs.values())
            print(f"  {k}  (dispatches {n})")
            wc = vals.get("SQ_WAVE_CYCLES", 0) or 1
            for c, v in sorted(vals.items()):
                extra = f"  ({100 * v / wc:.1f}% of wave-cycles)" if c.startswith("SQ_WAIT") or c == "SQ_ACTIVE_INST_ANY" else ""
                print(f"    {c:28s} {v:16.0f}{extra}")


if __name__ == "__main__":
    main(sys.argv[1])
