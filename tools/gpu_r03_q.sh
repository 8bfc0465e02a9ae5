#!/bin/bash
# Round-3 pass Q: Cholesky wait-timeout test, TuRBO / GP-fit parity, stage timing of configs 2 and 3.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_q}
mkdir -p "$O"
timeout -k 10 500 python -u -m pytest tests/test_gpu_turbo.py tests/test_gpu_gpfit.py tests/test_gpu_edges.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.txt" 2>&1
timeout -k 10 300 python -u bench.py --config 2 --steps 50 --warmup 10 --stage-timing --no-cpu-baseline --no-kblock > "$O/bench_c2_stages.json" 2> "$O/bench_c2_stages.err"
timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --stage-timing --no-cpu-baseline --no-kblock > "$O/bench_c3_stages.json" 2> "$O/bench_c3_stages.err"
echo pass-q-done
