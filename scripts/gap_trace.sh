set -o pipefail
cd "${GRAFT_REPO_ROOT}"
R=$(pwd)
mkdir -p gpurun_out/r04gap2
export TMPDIR=/tmp
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/r04gap2 -o run --output-format csv -- python3 $R/bench.py --steps 4 --warmup 2 --no-e2e-block --max-ramp-iters 200 > $R/gpurun_out/r04gap2_bench.log 2>&1
rc=$?
cd $R
[ $rc -eq 0 ] || exit $rc
PROF_DUMP_GAPS=4 python scripts/prof_summary.py gpurun_out/r04gap2 32 > gpurun_out/r04gap2/summary.md
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r04gap2/**/*memory_copy*.csv", recursive=True)
print("memcpy files", f)
for x in f:
    rows = list(csv.DictReader(open(x)))
    print(len(rows), "copies")
    import collections
    c = collections.Counter((r.get("Direction") or r.get("Operation") or "?", int(r.get("Bytes") or r.get("Size") or 0) // 1024) for r in rows)
    print(c.most_common(12))
    if rows: print(list(rows[0].keys()))
PY
find gpurun_out/r04gap2 -name "*kernel_trace.csv" -delete
exit 0
