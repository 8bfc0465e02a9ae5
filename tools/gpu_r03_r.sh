#!/bin/bash
# Round-3 pass R: EHVI-2D with L lanes per candidate for small batches; parity, config-2 stages and bench.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_r}
mkdir -p "$O"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bench_workloads.py tests/test_gpu_fused.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.txt" 2>&1
timeout -k 10 300 python -u bench.py --config 2 --steps 50 --warmup 10 --stage-timing --no-cpu-baseline --no-kblock > "$O/bench_c2_stages.json" 2> "$O/bench_c2_stages.err"
timeout -k 10 300 python -u bench.py --config 2 --steps 50 --warmup 10 --cpu-seconds 3 > "$O/bench_c2.json" 2> "$O/bench_c2.err"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 3 > "$O/bench.json" 2> "$O/bench.err"
echo pass-r-done
