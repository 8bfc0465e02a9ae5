#!/bin/bash
# lockstep batched GP fits (exact parity): full GPU suite, config 1 twice
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r02_v69}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.txt" 2>&1
timeout -k 10 300 python -u bench.py --config 1 > "$O/bench_c1.json" 2> "$O/bench_c1.err"
timeout -k 10 300 python -u bench.py --config 1 > "$O/bench_c1_again.json" 2> "$O/bench_c1_again.err"
echo v69-done
