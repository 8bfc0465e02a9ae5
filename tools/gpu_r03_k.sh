#!/bin/bash
# Round-3 pass K: Cholesky (fused step with coherent W fragments vs two launches), GEMM-shape ablation
# with rocBLAS as a reference rate, TuRBO / GP-fit parity, config-6 bench.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_k}
mkdir -p "$O"
timeout -k 10 120 ./tools/ablate/ablate_chol 130 512 1024 3000 5000 > "$O/ablate_chol.txt" 2>&1
timeout -k 10 120 ./tools/ablate/ablate_gemm 3000 512 > "$O/ablate_gemm.txt" 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_turbo.py tests/test_gpu_gpfit.py -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.txt" 2>&1
timeout -k 10 300 python -u bench.py --config 6 --steps 20 --warmup 3 --cpu-seconds 2 > "$O/bench_c6.json" 2> "$O/bench_c6.err"
echo pass-k-done
