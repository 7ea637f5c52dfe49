#!/usr/bin/env bash
# CU-partition sweep of the overlapped step (run via gpurun).
set -u
OUT=$PWD/gpurun_out/cu; mkdir -p "$OUT"
run() {
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 5 "$@" > "$OUT/b.json" 2> "$OUT/b.err" || { tail -5 "$OUT/b.err"; exit 3; }
  python3 -c "import json,sys;d=json.load(open('$OUT/b.json'));print(sys.argv[1:], round(d['value']/1e6,2), d['ms_per_step'], {k: round(v,2) for k,v in d['phase_ms'].items()})" "$@"
}
run --chunks 1
for s in ${CU_SET:-64 96 128}; do run --chunks 8 --side-cus $s --side-layout ${LAYOUT:-high}; done
run --chunks 8 --side-cus 96 --side-layout strided
