#!/usr/bin/env bash
# Round 6: the split stream's text depth / text ranges (tools/ab_libs/build_split.sh),
# alternated twice: the stream alone (split_ab, auto plan) and POM's graph.
set -u
OUT=$PWD/gpurun_out/${1:-r06splitab}; mkdir -p "$OUT"
ok() { local rc=$1; [ "$rc" -eq 0 ] || { echo "step failed rc=$rc"; exit "$rc"; }; }
for rep in 1 2; do
  for v in ${VARIANTS:-tu8_x1 tu16_x1 tu8_x2 tu16_x2}; do
    lib=tools/ab_libs/libmmb_split_$v.so
    timeout -k 10 200 python3 tools/split_ab.py --lib $lib --parts 0 > "$OUT/split_${v}_$rep.json" 2>&1; ok $?
    timeout -k 10 200 python3 tools/pom_graph_ab.py --lib $lib --dataset pom --variants split_fork --reps 40 > "$OUT/pom_${v}_$rep.json" 2>&1; ok $?
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); e=json.loads(open(sys.argv[2]).read().strip().splitlines()[-1]); print(sys.argv[3], 'valid', d['split0_p0_ms'], 'test', d['split1_p0_ms'], 'pom graph', e['split_fork_concurrent'])" "$OUT/split_${v}_$rep.json" "$OUT/pom_${v}_$rep.json" "$v rep$rep"
  done
done
