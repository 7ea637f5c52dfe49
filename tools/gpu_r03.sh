#!/bin/bash
# Round-3 GPU session: `tools/gpu_r03.sh TAG STEP...` with steps
#   tests   the full -m gpu suite (one process)
#   sizes   bench.py per-rank sizes U = 125k / 250k / 500k / 1M (--only-main)
#   bench   the default bench line (N = 1, every configs_measured leg)
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
TAG=$1
shift
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 \
        --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || exit $?
      ;;
    sizes)
      for u in 125000 250000 500000 1000000; do
        timeout -k 10 240 python -u bench.py --utts-per-gpu $u --steps 10 --warmup 3 --only-main \
          --no-cpu-baseline > gpurun_out/${TAG}_u$u.json 2> gpurun_out/${TAG}_u$u.log || exit $?
      done
      ;;
    bench)
      timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json \
        2> gpurun_out/${TAG}_bench.log || exit $?
      ;;
    *)
      echo "unknown step $step" >&2
      exit 2
      ;;
  esac
done
