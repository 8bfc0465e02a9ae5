#!/bin/bash
# Round-3 pass H: the bench workloads' interior arg-max test, smoke, configs 2, 3 and 5 benches.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_h}
mkdir -p "$O"
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_workloads.py -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.txt" 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1
timeout -k 10 300 python -u bench.py --cpu-seconds 3 > "$O/bench.json" 2> "$O/bench.err"
for c in 2 5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 5 --cpu-seconds 3 > "$O/bench_c$c.json" 2> "$O/bench_c$c.err"
done
echo pass-h-done
