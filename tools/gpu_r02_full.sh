#!/bin/bash
# Round-2 verification pass on one GPU box: GPU tests, smoke, default bench (+ degenerate cache line),
# rocprofv3 kernel stats of the default bench, the other BASELINE configs, PMC passes for configs 2/3.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r02_full}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.txt" 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1
timeout -k 10 300 python -u bench.py > "$O/bench.json" 2> "$O/bench.err"
timeout -k 10 300 python -u bench.py --cache-seed 0 --no-cpu-baseline > "$O/bench_cache_seed0.json" 2> "$O/bench_cache_seed0.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > "$O/bench_prof.json" 2> "$O/bench_prof.err"
for c in 2 4 5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 > "$O/bench_c$c.json" 2> "$O/bench_c$c.err"
done
timeout -k 10 300 python -u bench.py --config 4 --mode textbook --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench_c4_exact.json" 2> "$O/bench_c4_exact.err"
timeout -k 10 300 python -u bench.py --config 6 --steps 20 --warmup 3 > "$O/bench_c6.json" 2> "$O/bench_c6.err"
timeout -k 10 300 python -u bench.py --config 1 > "$O/bench_c1.json" 2> "$O/bench_c1.err"
PMC_BENCH_ARGS="--config 2" bash tools/pmc_run.sh "$O/pmc_c2"
bash tools/pmc_run.sh "$O/pmc_c3"
echo full-done
