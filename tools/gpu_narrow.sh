set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_mmb2.py -m gpu -x -q --timeout 120 --timeout-method thread -k "narrow_frame_stream_kernel and 3000" > gpurun_out/r03x_pytest.log 2>&1 || exit $?
tail -2 gpurun_out/r03x_pytest.log
timeout -k 10 300 python -u tools/narrow_ab.py --variants 0,10 > gpurun_out/r03x_narrow_ab.txt 2>&1 || exit $?
cat gpurun_out/r03x_narrow_ab.txt
