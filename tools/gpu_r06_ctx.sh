#!/usr/bin/env bash
# Round 6: the solve after different preceding work, alone, and its tests.
set -u
OUT=$PWD/gpurun_out/${1:-r06ctx}; mkdir -p "$OUT"; export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -eq 0 ] || { echo "step failed rc=$rc"; exit "$rc"; }; }
timeout -k 10 300 python3 -u -m pytest -q --timeout 180 --timeout-method thread -m gpu tests/test_gpu_pc_solve.py tests/test_gpu_robustness.py > "$OUT/pytest.log" 2>&1; ok $?
tail -1 "$OUT/pytest.log"
timeout -k 10 120 python3 tools/pc_context.py > "$OUT/pc_context.json" 2> "$OUT/pc_context.err"; ok $?
cat "$OUT/pc_context.json"
timeout -k 10 120 python3 tools/pc_time.py > "$OUT/pc_time.json" 2> "$OUT/pc_time.err"; ok $?
cat "$OUT/pc_time.json"
timeout -k 10 60 tools/pc_probe/pc_probe_mc > "$OUT/pc_probe.txt" 2>&1; ok $?
tail -6 "$OUT/pc_probe.txt" | head -2
timeout -k 10 300 python3 bench.py --only-leg dataset_splits > "$OUT/splits.json" 2> "$OUT/splits.err"; ok $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['dataset_splits']; [print(k, d[k]['all_splits_one_graph_concurrent_ms'], {s: (v['graph_ms'], v['phase_ms'], v['phase_ms_host_bound'].get('pc_solve')) for s, v in d[k]['splits'].items()}) for k in ('mosi','pom')]" "$OUT/splits.json"
