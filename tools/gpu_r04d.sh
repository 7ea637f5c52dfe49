set -o pipefail
mkdir -p gpurun_out/r04d
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_mmb2.py -x -v --timeout 300 --timeout-method thread -k "real_pom or mosi_splits or step_graph or int8_gram" > gpurun_out/r04d/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r04d/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --only-leg dataset_splits > gpurun_out/r04d/splits.json 2> gpurun_out/r04d/splits.err || exit $?
echo done
