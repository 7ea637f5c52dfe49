#!/usr/bin/env bash
# latent-step GPU tests + the latent step bench (tools/latent_bench.py)
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-latent}
timeout -k 10 600 python -u -m pytest tests/test_gpu_latent.py tests/test_gpu_regressor.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -u tools/latent_bench.py --steps 100 --cpu-steps 1 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $?
cat gpurun_out/${TAG}_bench.json
