#!/bin/bash
# Round-3 pass Z: GEMM slab loop without accumulator copies (VGPR-form MFMA for omb_linalg.hip) and
# running-pointer loads; GEMM/Cholesky ablations, every GPU test, smoke, config-6 bench + kernel stats.
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-r03_z}
mkdir -p "$O"
timeout -k 10 120 ./tools/ablate/ablate_gemm > "$O/ablate_gemm.txt" 2>&1
timeout -k 10 180 ./tools/ablate/ablate_chol 512 3000 5000 > "$O/ablate_chol.txt" 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/gpu_tests.txt" 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.txt" 2>&1
timeout -k 10 300 python -u bench.py --config 6 --steps 20 --warmup 3 --cpu-seconds 2 > "$O/bench_c6.json" 2> "$O/bench_c6.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_c6" -o c6 --output-format csv -- python -u bench.py --config 6 --steps 20 --warmup 3 --cpu-seconds 1 > "$O/prof_c6.log" 2>&1
echo pass-z-done
