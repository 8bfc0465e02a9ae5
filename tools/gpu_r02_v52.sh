#!/bin/bash
# spill-free 16-wave n ≤ 128 posterior: ablation, new parity tests, config-2 bench + PMC
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r02_v52}
mkdir -p "$O"
timeout -k 10 120 ./tools/ablate/ablate_posterior 128 65536 6 2 > "$O/ablate_c2.txt" 2>&1
timeout -k 10 120 ./tools/ablate/ablate_posterior 128 262144 6 2 > "$O/ablate_c2_N18.txt" 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > "$O/gpu_tests.txt" 2>&1
timeout -k 10 300 python -u bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench_c2.json" 2> "$O/bench_c2.err"
PMC_BENCH_ARGS="--config 2" bash tools/pmc_run.sh "$O/pmc_c2"
echo v52-done
