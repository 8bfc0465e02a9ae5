#!/bin/bash
# library with the 16-wave register-resident n ≤ 128 posterior: full GPU suite, config-2 bench and its profile
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r02_v50}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.txt" 2>&1
timeout -k 10 300 python -u bench.py --config 2 --steps 20 --warmup 5 > "$O/bench_c2.json" 2> "$O/bench_c2.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof_c2" -o run --output-format csv -- python3 bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench_c2_prof.json" 2> "$O/bench_c2_prof.err"
PMC_BENCH_ARGS="--config 2" bash tools/pmc_run.sh "$O/pmc_c2"
echo v50-done
