#!/bin/bash
# Round-3 pass C: GPU suite, smoke, benches of configs 3 (default), 5, 6 (K block now persistent).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_c}
mkdir -p "$O"
OMB_TEST_RECORD=$O/c1_checked.json timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.txt" 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1
timeout -k 10 300 python -u bench.py > "$O/bench.json" 2> "$O/bench.err"
timeout -k 10 300 python -u bench.py --config 5 --steps 20 --warmup 5 > "$O/bench_c5.json" 2> "$O/bench_c5.err"
timeout -k 10 300 python -u bench.py --config 6 --steps 20 --warmup 3 --no-cpu-baseline > "$O/bench_c6.json" 2> "$O/bench_c6.err"
timeout -k 10 300 python -u bench.py --config 2 --steps 20 --warmup 5 > "$O/bench_c2.json" 2> "$O/bench_c2.err"
echo pass-c-done
