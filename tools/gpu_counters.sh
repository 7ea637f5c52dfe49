#!/usr/bin/env bash
# Counter passes on one kernel of tools/kernel_bench.py (run via gpurun).
#   bash tools/gpu_counters.sh TAG KERNEL "CTR1 CTR2 ..." ["CTR ..." ...]
set -u
TAG=$1; K=$2; shift 2
OUT=$PWD/gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp; REPO=$PWD
timeout -k 10 300 python3 "$REPO/tools/kernel_bench.py" $K > "$OUT/time.txt" 2>&1 || exit $?
cat "$OUT/time.txt"
i=0
for set in "$@"; do
  i=$((i+1))
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $set -d "$OUT/pmc$i" -o run --output-format csv \
    -- python3 "$REPO/tools/kernel_bench.py" $K --reps 1 > "$OUT/pmc$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/pmc$i.log"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, re
out = sys.argv[1]
agg = {}
for f in sorted(glob.glob(out + "/pmc*/run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "mmb" not in r["Kernel_Name"]:
            continue
        k = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")[:50]
        agg.setdefault((k, r["Counter_Name"]), []).append(float(r["Counter_Value"]))
for (k, c), v in sorted(agg.items()):
    print(f"{k:50s} {c:28s} {sum(v)/len(v):.4g}")
PY
