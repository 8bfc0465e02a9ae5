#!/bin/bash
# Round-3 pass A: GPU suite (EA alias fixtures, config-4 full-size tests, bench self-launch), smoke,
# config 4 in both modes with CPU baselines.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_a}
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.txt" 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1
timeout -k 10 300 python -u bench.py --config 4 --steps 20 --warmup 5 > "$O/bench_c4.json" 2> "$O/bench_c4.err"
timeout -k 10 300 python -u bench.py --config 4 --mode textbook --steps 20 --warmup 5 > "$O/bench_c4_exact.json" 2> "$O/bench_c4_exact.err"
echo pass-a-done
