#!/bin/bash
# Round-3 pass E: 512-thread fit kernel — GP fit tests, fit profile (+ rocprofv3 kernel stats of it), config 1.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_e}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_gpfit.py tests/test_gpu_config1.py -x -v --timeout 200 --timeout-method thread > "$O/gpu_tests_gpfit.txt" 2>&1
timeout -k 10 200 python -u tools/diag/fit_profile.py > "$O/fit_profile.txt" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o fit --output-format csv -- python3 tools/diag/fit_profile.py > "$O/fit_profile_prof.txt" 2>&1
timeout -k 10 300 python -u bench.py --config 1 > "$O/bench_c1.json" 2> "$O/bench_c1.err"
echo pass-e-done
