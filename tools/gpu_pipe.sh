#!/usr/bin/env bash
# Pipelined fused streamer: bit-identity + fused-kernel tests, then the in-process A/B.
#   tools/gpu_pipe.sh TAG [DIAGS]
set -u
TAG=${1:-pipe}
DIAGS=${2:-1,0:8:1,1:8:1,0:4:1}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_mmb2.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -k "pipelined or stream_project" > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 "$OUT/pytest.log"
[ "$rc" -eq 0 ] || exit "$rc"
timeout -k 10 400 python3 -u tools/fused_ab.py --rounds 3 --diags "$DIAGS" > "$OUT/ab.txt" 2>&1
rc=$?; echo "ab rc=$rc"; cat "$OUT/ab.txt"
exit $rc
