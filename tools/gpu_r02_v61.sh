#!/bin/bash
# concurrent per-objective GP fits: fit parity, driver tests, config-1 bench, fit profile
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r02_v61}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_gpfit.py tests/test_gpu_surface.py tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.txt" 2>&1
timeout -k 10 300 python -u bench.py --config 1 > "$O/bench_c1.json" 2> "$O/bench_c1.err"
echo v61-done
