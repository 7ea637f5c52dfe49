#!/usr/bin/env bash
# Round 6: the split stream's finish fused into its last-arriving workgroup
# -- tests, then alternated A/B against the two-launch library.
set -u
OUT=$PWD/gpurun_out/${1:-r06fin1}; mkdir -p "$OUT"
ok() { local rc=$1; [ "$rc" -eq 0 ] || { echo "step failed rc=$rc"; exit "$rc"; }; }
timeout -k 10 600 python3 -u -m pytest -q --timeout 180 --timeout-method thread -m gpu \
  tests/test_gpu_split.py tests/test_gpu_robustness.py \
  tests/test_gpu_mmb2.py -k "split or pom or drop_in or fused_id or graph or check" > "$OUT/pytest.log" 2>&1; ok $?
tail -1 "$OUT/pytest.log"
for rep in 1 2; do
  for lib in multimodal-baselines_amd/libmmb.so tools/ab_libs/libmmb_split2launch.so; do
    tag=$(basename $lib .so)
    timeout -k 10 200 python3 tools/split_ab.py --lib $lib --parts 0,1 > "$OUT/split_${tag}_$rep.json" 2>&1; ok $?
    timeout -k 10 200 python3 tools/pom_graph_ab.py --lib $lib --dataset pom --variants split_fork --reps 40 > "$OUT/pom_${tag}_$rep.json" 2>&1; ok $?
    echo "$tag rep$rep: $(tail -1 "$OUT/split_${tag}_$rep.json" | cut -c1-400) | pom $(tail -1 "$OUT/pom_${tag}_$rep.json")"
  done
done
