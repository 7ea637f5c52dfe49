#!/usr/bin/env bash
# Round-2 check on the GPU box: every -m gpu test, smoke(), then the default
# bench line (headline + configs_measured + CPU legs).  Each GPU step has its
# own limit; the script stops at the first failure.
set -u
OUT=$PWD/gpurun_out/${1:-r02}; mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ "$rc" -eq 0 ] || exit "$rc"
[ -n "${SKIP_BENCH:-}" ] && exit 0
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 "$OUT/smoke.log"; [ "$rc" -eq 0 ] || exit "$rc"
timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; [ "$rc" -eq 0 ] || { tail -5 "$OUT/bench.err"; exit "$rc"; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['phase_ms'])" "$OUT/bench.json"
