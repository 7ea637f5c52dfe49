#!/usr/bin/env bash
# Quick GPU check: parity tests, smoke, then one bench line (run via gpurun).
set -u
TAG=${1:-quick}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 python3 -m pytest tests -m gpu -q --timeout 300 ${PYTEST_ARGS:-} > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"
[ "$rc" -le 1 ] || exit "$rc"
timeout -k 10 600 python3 bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -3 "$OUT/bench.err"
exit $rc
