#!/usr/bin/env bash
# Full GPU test suite, then the fused-kernel A/B with its timing ablations.
#   tools/gpu_check_ab.sh TAG [DIAGS]
set -u
TAG=${1:-check}
DIAGS=${2:-1,8,2,4,0:12,0:16,1:16}
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
  > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 "$OUT/pytest.log"
[ "$rc" -eq 0 ] || exit "$rc"
timeout -k 10 400 python3 -u tools/fused_ab.py --rounds 3 --diags "$DIAGS" > "$OUT/ab.txt" 2>&1
rc=$?; echo "ab rc=$rc"; cat "$OUT/ab.txt"
exit $rc
