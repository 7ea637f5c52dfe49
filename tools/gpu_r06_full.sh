#!/usr/bin/env bash
# Every -m gpu test, smoke(), the default bench line, then the 12-wave
# narrow-kernel variant measured once against the product library.
set -u
TAG=${1:-r06full}
OUT=$PWD/gpurun_out/$TAG; mkdir -p "$OUT"
ok() { local rc=$1; [ "$rc" -eq 0 ] || { echo "step failed rc=$rc"; exit "$rc"; }; }
timeout -k 10 900 python3 -u -m pytest tests -m gpu ${PYX--x} -v --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1; ok $?
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; ok $?
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"; ok $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'])" "$OUT/bench.json"
if [ -n "${NF_AB:-}" ]; then
  for lib in multimodal-baselines_amd/libmmb.so tools/ab_libs/libmmb_nf_w12_2_1_4_2.so multimodal-baselines_amd/libmmb.so tools/ab_libs/libmmb_nf_w12_2_1_4_2.so; do
    timeout -k 10 200 python3 tools/nf_ab.py --lib $lib --check >> "$OUT/nf_w12_ab.txt" 2>&1; ok $?
  done
  grep kernel_ms "$OUT/nf_w12_ab.txt"
fi
