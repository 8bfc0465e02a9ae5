#!/bin/bash
# Round-3 pass F: fit kernel ablation, GP fit tests, README run, fit profile, config-1 bench.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_f}
mkdir -p "$O"
timeout -k 10 120 ./tools/ablate/ablate_gpfit > "$O/ablate_gpfit.txt" 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_gpfit.py tests/test_gpu_config1.py tests/test_gpu_surface.py -x -v --timeout 200 --timeout-method thread > "$O/gpu_tests_gpfit.txt" 2>&1
timeout -k 10 200 python -u tools/diag/fit_profile.py > "$O/fit_profile.txt" 2>&1
timeout -k 10 300 python -u bench.py --config 1 > "$O/bench_c1.json" 2> "$O/bench_c1.err"
echo pass-f-done
