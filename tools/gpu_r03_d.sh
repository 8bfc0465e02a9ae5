#!/bin/bash
# Round-3 pass D: GP-fit block sweep — GP fit tests first, then the whole suite, fit profile, config-1 bench.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_d}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_gpfit.py -x -v --timeout 120 --timeout-method thread > "$O/gpu_tests_gpfit.txt" 2>&1
OMB_TEST_RECORD=$O/c1_checked.json timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.txt" 2>&1
timeout -k 10 200 python -u tools/diag/fit_profile.py > "$O/fit_profile.txt" 2>&1
timeout -k 10 300 python -u bench.py --config 1 > "$O/bench_c1.json" 2> "$O/bench_c1.err"
echo pass-d-done
