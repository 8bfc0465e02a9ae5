#!/bin/bash
# staged K block for every n_var: full GPU suite, configs 5 and 6
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r02_v55}
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.txt" 2>&1
timeout -k 10 300 python -u bench.py --config 5 --steps 20 --warmup 5 --no-cpu-baseline > "$O/bench_c5.json" 2> "$O/bench_c5.err"
timeout -k 10 300 python -u bench.py --config 6 --steps 20 --warmup 3 --no-cpu-baseline > "$O/bench_c6.json" 2> "$O/bench_c6.err"

timeout -k 10 200 ./tools/ablate/ablate_kblock2 512 1048576 6 > "$O/ablate_kblock_c3.txt" 2>&1
timeout -k 10 200 ./tools/ablate/ablate_kblock2_lc 512 1048576 6 > "$O/ablate_kblock_c3_lanecoords.txt" 2>&1
timeout -k 10 200 ./tools/ablate/ablate_kblock2 512 1048576 6 > "$O/ablate_kblock_c3_again.txt" 2>&1
echo v55-ablate-done
