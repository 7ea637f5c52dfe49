#!/usr/bin/env bash
# Every -m gpu test, smoke(), then the default bench line.  Stops at the first failure.
set -u
TAG=${1:-check}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
ok() { local rc=$1; [ "$rc" -eq 0 ] || { echo "step failed rc=$rc"; exit "$rc"; }; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1; ok $?
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; ok $?
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"; ok $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['value'], d['ms_per_step'], d['phase_ms'], d['roofline']['frac'])" "$OUT/bench.json"
