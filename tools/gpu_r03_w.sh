#!/bin/bash
# Round-3 pass W: lower-triangular V = L⁻¹K* GEMM; parity of every path that runs it, config-6 bench + profile.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_w}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_edges.py tests/test_gpu_turbo.py tests/test_gpu_gpfit.py tests/test_gpu_config1.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.txt" 2>&1
timeout -k 10 300 python -u bench.py --config 6 --steps 20 --warmup 3 --cpu-seconds 2 > "$O/bench_c6.json" 2> "$O/bench_c6.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_c6" -o c6 --output-format csv -- python -u bench.py --config 6 --steps 20 --warmup 3 --cpu-seconds 1 > "$O/prof_c6.log" 2>&1
echo pass-w-done
