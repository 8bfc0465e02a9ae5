#!/bin/bash
# Round-3 pass L: K block at n_var > 8 with r² from the augmented MFMA (aug r²), parity, config-5 bench.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_l}
mkdir -p "$O"
timeout -k 10 150 ./tools/ablate/ablate_kblock3 1024 524288 30 > "$O/ablate_kblock3_c5.txt" 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_turbo.py -m gpu -x -q --timeout 300 --timeout-method thread -k "kernel_block or config5 or turbo or samples or cov" > "$O/gpu_tests.txt" 2>&1
timeout -k 10 300 python -u bench.py --config 5 --steps 20 --warmup 5 --cpu-seconds 2 > "$O/bench_c5.json" 2> "$O/bench_c5.err"
echo pass-l-done
