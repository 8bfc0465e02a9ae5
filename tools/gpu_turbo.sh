#!/bin/bash
# GPU-box pass for the Thompson-sampling path: its tests, bench config 6, rocprofv3 kernel stats.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-turbo}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_turbo.py -x -q --timeout 120 --timeout-method thread > "$OUT/turbo_tests.txt" 2>&1
timeout -k 10 300 python -u bench.py --config 6 --steps 10 --warmup 2 ${BENCH_EXTRA:---no-cpu-baseline} > "$OUT/bench_c6.json" 2> "$OUT/bench_c6.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_c6" -o run --output-format csv -- python3 bench.py --config 6 --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/bench_c6_prof.json" 2> "$OUT/bench_c6_prof.err"
echo turbo-done
