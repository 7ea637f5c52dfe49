#!/usr/bin/env bash
# r04g: narrow fused kernel tests, then a same-box A/B of its knob builds on
# the MOSI workload (tools/nf_ab.py; libs from tools/ab_libs/build_nf.sh).
set -o pipefail
OUT=gpurun_out/${1:-r04g}; shift
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_mmb2.py -x -v --timeout 300 --timeout-method thread \
  -k "narrow or compensated or mosi" > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in "$@"; do
    chk=""; [ $rep -eq 1 ] && [[ $v != *_a* ]] && chk=--check
    timeout -k 10 120 python3 -u tools/nf_ab.py --lib tools/ab_libs/libmmb_nf_$v.so $chk >> "$OUT/ab.txt" 2>>"$OUT/ab.err" || exit $?
  done
done
cat "$OUT/ab.txt"
