#!/usr/bin/env bash
# CU-partition sweep of the overlapped step (run via gpurun): one bench line
# per point; POINTS is a ';'-separated list of bench.py argument sets.
set -u
OUT=$PWD/gpurun_out/cu; mkdir -p "$OUT"
run() {
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 5 --warmup 2 "$@" > "$OUT/b.json" 2> "$OUT/b.err" || { tail -5 "$OUT/b.err"; exit 3; }
  python3 -c "import json,sys;d=json.load(open('$OUT/b.json'));print(sys.argv[1:], round(d['value']/1e6,2), d['ms_per_step'], {k: round(v,2) for k,v in d['phase_ms'].items()})" "$@"
}
POINTS=${POINTS:-"--chunks 1;--chunks 1 --no-tiled;--chunks 8 --side-cus 64;--chunks 8 --side-cus 96;--chunks 8 --side-cus 128;--chunks 8 --side-cus 96 --side-layout strided;--chunks 16 --side-cus 96"}
IFS=';' read -ra PTS <<< "$POINTS"
for p in "${PTS[@]}"; do run $p; done
