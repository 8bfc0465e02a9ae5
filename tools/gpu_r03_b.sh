#!/bin/bash
# Round-3 pass B: GPU suite (maximiser vs all DE fixtures, README run at full size), K-block ablation at
# configs 5 and 3, config 1 bench, PMC for configs 4 and 5.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_b}
mkdir -p "$O"
OMB_TEST_RECORD=$O/c1_checked.json timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.txt" 2>&1
timeout -k 10 120 ./tools/ablate/ablate_kblock3 1024 524288 30 > "$O/ablate_kblock3_c5.txt" 2>&1
timeout -k 10 120 ./tools/ablate/ablate_kblock3 512 1048576 6 > "$O/ablate_kblock3_c3.txt" 2>&1
timeout -k 10 300 python -u bench.py --config 1 > "$O/bench_c1.json" 2> "$O/bench_c1.err"
PMC_BENCH_ARGS="--config 4" bash tools/pmc_run.sh "$O/pmc_c4"
PMC_BENCH_ARGS="--config 5" bash tools/pmc_run.sh "$O/pmc_c5"
echo pass-b-done
