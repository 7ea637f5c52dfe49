#!/usr/bin/env bash
# MOSI step with the chunked / CU-masked overlap of FusedStep (bench.py --chunks / --side-cus)
set -o pipefail
mkdir -p gpurun_out/mosi_sweep
for cfg in "1 0" "4 0" "8 0" "4 32" "8 32" "8 64" "16 32"; do
  set -- $cfg
  timeout -k 10 180 python -u bench.py --workload mosi --only-main --no-cpu-baseline --steps 10 --warmup 3 \
    --chunks $1 --side-cus $2 > gpurun_out/mosi_sweep/c$1_s$2.json 2> gpurun_out/mosi_sweep/c$1_s$2.err || exit $?
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['ms_per_step'], d['phase_ms'])" gpurun_out/mosi_sweep/c$1_s$2.json $1 $2
done
