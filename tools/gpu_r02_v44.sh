#!/bin/bash
# n ≤ 128 register-resident posterior: ablation vs the tile kernel, parity tests, config-2 bench
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r02_v45}
mkdir -p "$O"
timeout -k 10 120 ./tools/ablate/ablate_posterior 128 65536 6 2 > "$O/ablate_c2.txt" 2>&1
timeout -k 10 120 ./tools/ablate/ablate_posterior 100 100000 6 3 > "$O/ablate_n100.txt" 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_edges.py -x -v --timeout 120 --timeout-method thread > "$O/gpu_tests.txt" 2>&1
timeout -k 10 300 python -u bench.py --config 2 --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench_c2.json" 2> "$O/bench_c2.err"
echo v44-done
