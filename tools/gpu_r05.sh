#!/usr/bin/env bash
# Round-5 GPU session: `tools/gpu_r05.sh TAG STEP...` with steps
#   tests   the full -m gpu suite (one process), sha of the tree in the log
#   robust  tests/test_gpu_robustness.py + tests/test_gpu_variants.py only
#   smoke   __graft_entry__.smoke()
#   bench   the driver's bench line (N = 1, --steps 20 --warmup 5, every configs_measured leg)
#   main    bench.py --only-main (headline only, no CPU leg)
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
TAG=$1
shift
OUT=$PWD/gpurun_out/$TAG
mkdir -p "$OUT"
[ -f TREE_SHA ] && echo "tree: $(cat TREE_SHA)" | tee "$OUT/tree_sha.txt"
for step in "$@"; do
  case $step in
    tests)
      { [ -f TREE_SHA ] && echo "tree: $(cat TREE_SHA)"; } > "$OUT/pytest.log"
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 \
        --timeout-method thread >> "$OUT/pytest.log" 2>&1 || exit $?
      tail -1 "$OUT/pytest.log"
      ;;
    robust)
      timeout -k 10 600 python3 -u -m pytest tests/test_gpu_robustness.py tests/test_gpu_variants.py \
        -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/robust.log" 2>&1 || exit $?
      tail -1 "$OUT/robust.log"
      ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || exit $?
      tail -1 "$OUT/smoke.log"
      ;;
    bench)
      timeout -k 10 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
      ;;
    main)
      timeout -k 10 300 python3 -u bench.py --only-main --no-cpu-baseline --steps 10 --warmup 3 \
        > "$OUT/main.json" 2> "$OUT/main.err" || exit $?
      ;;
    pcprobe)  # phase marks of the multi-workgroup PC solve, r05 round and (V1) r04 round
      timeout -k 10 60 tools/pc_probe/pc_probe_mc > "$OUT/pc_probe.txt" 2>&1 || exit $?
      MMB_PC_SOLVE_V1=1 timeout -k 10 60 tools/pc_probe/pc_probe_mc_diag > "$OUT/pc_probe_v1.txt" 2>&1 || exit $?
      ;;
    splits)  # the dataset splits as one graph (tools/splits_ab.py)
      timeout -k 10 300 python3 -u tools/splits_ab.py > "$OUT/splits_ab.txt" 2>&1 || exit $?
      ;;
    *)
      echo "unknown step $step" >&2
      exit 2
      ;;
  esac
done
echo "session $TAG done"
