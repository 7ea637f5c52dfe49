#!/usr/bin/env bash
# Round 6 iteration: targeted GPU tests, the POM graph kernel trace, the
# dataset_splits leg.
set -u
OUT=$PWD/gpurun_out/${1:-r06iter}; mkdir -p "$OUT"; export TMPDIR=/tmp; REPO=$PWD
ok() { local rc=$1; [ "$rc" -eq 0 ] || { echo "step failed rc=$rc"; exit "$rc"; }; }
timeout -k 10 600 python3 -u -m pytest -q --timeout 180 --timeout-method thread -m gpu \
  tests/test_gpu_pc_solve.py tests/test_gpu_sif.py tests/test_gpu_robustness.py tests/test_gpu_split.py \
  "tests/test_gpu_variants.py::test_variants_agree[timeouts]" \
  tests/test_gpu_mmb2.py -k "pc or split or pom or mosi or full_size or graph or removal or status or check" > "$OUT/pytest.log" 2>&1; ok $?
tail -1 "$OUT/pytest.log"
timeout -k 10 120 python3 tools/pc_time.py > "$OUT/pc_time.json" 2> "$OUT/pc_time.err"; ok $?
cat "$OUT/pc_time.json"
(cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT/trace" -o run --output-format csv \
  -- python3 "$REPO/tools/pom_graph_ab.py" --reps 5 --variants split_fork,split_nofork > "$OUT/ab.json" 2> "$OUT/ab.err"); ok $?
cat "$OUT/ab.json"
timeout -k 10 300 python3 bench.py --only-leg dataset_splits > "$OUT/splits.json" 2> "$OUT/splits.err"; ok $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['dataset_splits']; [print(k, d[k]['all_splits_one_graph_concurrent_ms'], {s: (v['graph_ms'], v['phase_ms']) for s, v in d[k]['splits'].items()}) for k in ('mosi','pom')]" "$OUT/splits.json"
