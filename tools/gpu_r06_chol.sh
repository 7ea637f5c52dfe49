#!/usr/bin/env bash
# Round 6: the compact Cholesky -- PC tests, the solve warm / cold / in
# context, the dataset splits.
set -u
OUT=$PWD/gpurun_out/${1:-r06chol}; mkdir -p "$OUT"; export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || { echo "step failed rc=$rc"; exit "$rc"; }; }
timeout -k 10 600 python3 -u -m pytest -q --timeout 180 --timeout-method thread -m gpu \
  tests/test_gpu_pc_solve.py tests/test_gpu_sif.py tests/test_gpu_robustness.py tests/test_gpu_variants.py \
  tests/test_gpu_mmb2.py -k "pc or split or pom or mosi or full_size or graph or removal or status or check or variants or solve" > "$OUT/pytest.log" 2>&1; ok $?
tail -1 "$OUT/pytest.log"
timeout -k 10 60 tools/pc_probe/pc_probe_mc > "$OUT/pc_probe_warm.txt" 2>&1; ok $?
timeout -k 10 60 tools/pc_probe/pc_probe_mc cold > "$OUT/pc_probe_cold.txt" 2>&1; ok $?
grep "rep 4" "$OUT/pc_probe_warm.txt"; grep "rep 4" "$OUT/pc_probe_cold.txt"; tail -1 "$OUT/pc_probe_warm.txt"
timeout -k 10 120 python3 tools/pc_context.py > "$OUT/pc_context.json" 2> "$OUT/pc_context.err"; ok $?
cat "$OUT/pc_context.json"
timeout -k 10 120 python3 tools/pc_time.py > "$OUT/pc_time.json" 2> "$OUT/pc_time.err"; ok $?
cat "$OUT/pc_time.json"
timeout -k 10 300 python3 bench.py --only-leg dataset_splits > "$OUT/splits.json" 2> "$OUT/splits.err"; ok $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['dataset_splits']; [print(k, d[k]['all_splits_one_graph_concurrent_ms'], {s: (v['graph_ms'], v['phase_ms'].get('pc_solve')) for s, v in d[k]['splits'].items()}) for k in ('mosi','pom')]" "$OUT/splits.json"
