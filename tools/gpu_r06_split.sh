#!/usr/bin/env bash
# Round 6: the split stream path's tests, the deterministic timeout group, the
# POM-split tests, then the dataset_splits leg.
set -u
TAG=${1:-r06split}
OUT=$PWD/gpurun_out/$TAG; mkdir -p "$OUT"
ok() { local rc=$1; [ "$rc" -eq 0 ] || { echo "step failed rc=$rc"; exit "$rc"; }; }
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu \
  tests/test_gpu_split.py "tests/test_gpu_variants.py::test_variants_agree[timeouts]" \
  tests/test_gpu_mmb2.py -k "split or timeouts or pom or removal_matches or graph" > "$OUT/pytest.log" 2>&1; ok $?
tail -1 "$OUT/pytest.log"
timeout -k 10 300 python3 bench.py --only-leg dataset_splits > "$OUT/splits.json" 2> "$OUT/splits.err"; ok $?
python3 -c "import json,sys; d=json.load(open(sys.argv[1]))['dataset_splits']; [print(k, d[k]['all_splits_one_graph_concurrent_ms'], {s: (v['graph_ms'], v['phase_ms']) for s, v in d[k]['splits'].items()}) for k in ('mosi','pom')]" "$OUT/splits.json"
