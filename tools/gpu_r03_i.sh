#!/bin/bash
# Round-3 pass I: config-2 posterior staging ablation (one-wait staging, ℓ in registers, prefetch), small-n parity.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_i}
mkdir -p "$O"
timeout -k 10 150 ./tools/ablate/ablate_posterior 128 65536 6 2 > "$O/ablate_c2.txt" 2>&1
timeout -k 10 150 ./tools/ablate/ablate_posterior 128 262144 6 2 > "$O/ablate_c2_N18.txt" 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -k "posterior or small or reg or config2" > "$O/gpu_tests.txt" 2>&1
timeout -k 10 300 python -u bench.py --config 2 --steps 20 --warmup 5 --cpu-seconds 2 > "$O/bench_c2.json" 2> "$O/bench_c2.err"
echo pass-i-done
