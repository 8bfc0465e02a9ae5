#!/bin/bash
# One GPU-box verification pass: GPU tests, smoke, default bench, rocprofv3 kernel stats.
# Every GPU step has its own time limit; the first failing step ends the script.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-verify}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.txt" 2>&1
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err"
echo verify-done
