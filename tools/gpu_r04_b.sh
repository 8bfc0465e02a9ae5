# Round 4, call b: blocked diagonal Cholesky (ablation, traces, rocsolver bar), Thompson / GP-fit tests, RCCL tests,
# the table transform on the README states, config 6.
set -e
O=gpurun_out/${1:-r04_b}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 240 ./tools/ablate/ablate_chol 64 65 130 512 1024 3000 5000 > $O/ablate_chol.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_multirank.py -x -v -s --timeout 240 --timeout-method thread > $O/rccl_tests.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_turbo.py tests/test_gpu_gpfit.py tests/test_gpu_config1.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
timeout -k 10 300 python -u bench.py --config 6 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c6.json 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_cov_table.py -v -s --timeout 240 --timeout-method thread > $O/cov_table.txt 2>&1
echo done
