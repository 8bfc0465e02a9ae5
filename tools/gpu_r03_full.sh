#!/bin/bash
# Round-3 verification pass on one GPU box: GPU suite, smoke, default bench, rocprofv3 kernel stats of it,
# the other BASELINE configs (1, 2, 4 in both modes, 5) and the TuRBO Thompson step (6).
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_full}
mkdir -p "$O"
OMB_TEST_RECORD=$O/c1_checked.json timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.txt" 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1
timeout -k 10 300 python -u bench.py > "$O/bench.json" 2> "$O/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$O/bench_prof.json" 2> "$O/bench_prof.err"
for c in 2 4 5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 > "$O/bench_c$c.json" 2> "$O/bench_c$c.err"
done
timeout -k 10 300 python -u bench.py --config 4 --mode textbook --steps 20 --warmup 5 > "$O/bench_c4_exact.json" 2> "$O/bench_c4_exact.err"
timeout -k 10 300 python -u bench.py --config 6 --steps 20 --warmup 3 > "$O/bench_c6.json" 2> "$O/bench_c6.err"
timeout -k 10 300 python -u bench.py --config 1 > "$O/bench_c1.json" 2> "$O/bench_c1.err"
echo full-done
