#!/bin/bash
# Round-3 pass S: radix-select heads for the Thompson selection, Cholesky memsets folded into the first kernel;
# TuRBO / GP-fit parity; config-6 bench and rocprofv3 per-kernel times.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_s}
mkdir -p "$O"
timeout -k 10 500 python -u -m pytest tests/test_gpu_turbo.py tests/test_gpu_gpfit.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.txt" 2>&1
timeout -k 10 300 python -u bench.py --config 6 --steps 20 --warmup 3 --cpu-seconds 2 > "$O/bench_c6.json" 2> "$O/bench_c6.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run --output-format csv -- python3 bench.py --config 6 --steps 10 --warmup 2 --no-cpu-baseline > "$O/bench_c6_prof.json" 2> "$O/bench_c6_prof.err"
echo pass-s-done
