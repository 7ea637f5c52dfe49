#!/usr/bin/env bash
# Round 6: G2 tiles per squaring workgroup, 2 vs 4 (tools/ab_libs/build_sq.sh),
# alternated: the solve alone and the dataset graphs.
set -u
OUT=$PWD/gpurun_out/${1:-r06sq2}; mkdir -p "$OUT"
ok() { local rc=$1; [ "$rc" -eq 0 ] || { echo "step failed rc=$rc"; exit "$rc"; }; }
for rep in 1 2; do
  for v in 2 4; do
    lib=tools/ab_libs/libmmb_sq$v.so
    timeout -k 10 120 python3 tools/pc_time.py --lib $lib --reps 100 > "$OUT/pc_time_sq${v}_$rep.json" 2>&1; ok $?
    timeout -k 10 200 python3 tools/pom_graph_ab.py --lib $lib --dataset mosi --variants split_fork --reps 40 > "$OUT/mosi_sq${v}_$rep.json" 2>&1; ok $?
    timeout -k 10 200 python3 tools/pom_graph_ab.py --lib $lib --dataset pom --variants split_fork --reps 40 > "$OUT/pom_sq${v}_$rep.json" 2>&1; ok $?
    echo "sq$v rep$rep: $(tail -1 "$OUT/pc_time_sq${v}_$rep.json" | cut -c1-60) | mosi $(tail -1 "$OUT/mosi_sq${v}_$rep.json") | pom $(tail -1 "$OUT/pom_sq${v}_$rep.json")"
  done
done
