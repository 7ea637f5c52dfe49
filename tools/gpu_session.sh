#!/usr/bin/env bash
# One GPU-box session (run via gpurun from the repo root): parity tests, the
# CU-mask bit -> XCD map, the profiled bench (tools/gpu_profile.sh) and the
# CU-partition sweep (tools/cu_sweep.sh).  Each GPU step has its own time
# limit; the session stops at the first failing step.
set -u
TAG=${1:-session}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python3 -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 "$OUT/pytest.log"; [ "$rc" -eq 0 ] || exit "$rc"
fi
if [ -x tools/cu_map/cu_map ] && [ -z "${SKIP_MAP:-}" ]; then
  timeout -k 10 120 tools/cu_map/cu_map > "$OUT/cu_map.txt" 2>&1 || { echo "cu_map failed"; exit 3; }
  echo "cu_map: $(wc -l < "$OUT/cu_map.txt") lines"
fi
if [ -z "${SKIP_PROFILE:-}" ]; then
  bash tools/gpu_profile.sh "$TAG" || exit $?
fi
if [ -z "${SKIP_SWEEP:-}" ]; then
  bash tools/cu_sweep.sh || exit $?
fi
echo "session done"
