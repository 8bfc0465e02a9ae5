#!/bin/bash
# Round-3 pass O: diagonal factor with the pivot chain one column ahead (v1) vs round 2 (v0), traced;
# TuRBO / GP-fit parity; config-6 bench.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_o}
mkdir -p "$O"
timeout -k 10 120 ./tools/ablate/ablate_chol_v0 512 3000 > "$O/ablate_chol_v0.txt" 2>&1
timeout -k 10 120 ./tools/ablate/ablate_chol 512 3000 > "$O/ablate_chol_v1.txt" 2>&1
timeout -k 10 500 python -u -m pytest tests/test_gpu_turbo.py tests/test_gpu_gpfit.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.txt" 2>&1
timeout -k 10 300 python -u bench.py --config 6 --steps 20 --warmup 3 --cpu-seconds 2 > "$O/bench_c6.json" 2> "$O/bench_c6.err"
echo pass-o-done
