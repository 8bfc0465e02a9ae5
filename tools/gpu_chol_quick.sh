# Cholesky iteration loop: phase trace + per-size timing, the Thompson/GP-fit GPU tests, config 6.
set -e
O=gpurun_out/${1:-chol_quick}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./tools/ablate/ablate_chol 64 65 130 512 1024 3000 5000 > $O/ablate_chol.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_turbo.py tests/test_gpu_gpfit.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
timeout -k 10 300 python -u bench.py --config 6 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c6.json 2>&1
echo done
