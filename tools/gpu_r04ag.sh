#!/usr/bin/env bash
# headline-step A/B of two product builds (tools/nf_ab.py --workload synthetic)
set -o pipefail
OUT=gpurun_out/${1:-r04ag}; shift; mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_mmb2.py -x -q --timeout 300 --timeout-method thread \
  -k "stream_project or fused or int8" > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do for v in "$@"; do
  timeout -k 10 200 python3 -u tools/nf_ab.py --workload synthetic --lib tools/ab_libs/libmmb_nf_$v.so >> "$OUT/ab.txt" 2>>"$OUT/ab.err" || exit 1
done; done
cat "$OUT/ab.txt"
