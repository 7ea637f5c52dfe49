set -u
OUT=$PWD/gpurun_out/lat1; mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_regressor.py tests/test_gpu_latent.py -x -v --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log; [ "$rc" -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/latent_bench.py > $OUT/latent.json 2> $OUT/latent.err
rc=$?; echo "latent rc=$rc"; cat $OUT/latent.json; tail -3 $OUT/latent.err; exit $rc
