#!/usr/bin/env bash
# Round-end check on the GPU box: every -m gpu test, smoke(), the POM-shaped
# bench line (configs[2]) and the latent-objective step bench.
set -u
OUT=$PWD/gpurun_out/${1:-final}; mkdir -p "$OUT"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$OUT/pytest.log"; [ "$rc" -eq 0 ] || exit "$rc"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 "$OUT/smoke.log"; [ "$rc" -eq 0 ] || exit "$rc"
timeout -k 10 300 python3 bench.py --workload pom --steps 5 --warmup 2 > "$OUT/pom.json" 2> "$OUT/pom.err"
rc=$?; echo "pom rc=$rc"; [ "$rc" -eq 0 ] || { tail -3 "$OUT/pom.err"; exit "$rc"; }
timeout -k 10 300 python3 tools/latent_bench.py > "$OUT/latent.json" 2> "$OUT/latent.err"
rc=$?; echo "latent rc=$rc"; tail -1 "$OUT/latent.json"; exit "$rc"
