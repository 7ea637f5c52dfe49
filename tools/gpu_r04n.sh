#!/usr/bin/env bash
# r04n: 125k-row step (the 8-GPU rank's share of configs[3]) and the 1M MOSI
# step: bench lines + rocprofv3 kernel stats of each.
set -o pipefail
OUT=gpurun_out/${1:-r04n}
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --utts 125000 --only-main --no-cpu-baseline --steps 20 --warmup 3 \
  > "$OUT/b125k.json" 2> "$OUT/b125k.err" || exit $?
timeout -k 10 300 python3 -u bench.py --workload mosi --only-main --no-cpu-baseline --steps 10 --warmup 3 \
  > "$OUT/mosi.json" 2> "$OUT/mosi.err" || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof125k" -o run --output-format csv -- \
  python3 -u bench.py --utts 125000 --only-main --no-cpu-baseline --steps 20 --warmup 3 > "$OUT/prof125k.log" 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/profmosi" -o run --output-format csv -- \
  python3 -u bench.py --workload mosi --only-main --no-cpu-baseline --steps 10 --warmup 3 > "$OUT/profmosi.log" 2>&1 || exit $?
echo done
