# Round 4, call g: the table transform in the covariance kernel (diagnostics), stage timing of config 2.
set -e
O=gpurun_out/${1:-r04_g}
mkdir -p $O
export TMPDIR=/tmp
OMB_TEST_RECORD=$O/cov_table_worst.npz timeout -k 10 300 python -u -m pytest tests/test_gpu_cov_table.py -q -s --timeout 240 --timeout-method thread > $O/cov_table.txt 2>&1 || true
timeout -k 10 200 python -u bench.py --config 2 --steps 200 --warmup 20 --no-cpu-baseline --one-launch 0 --stage-timing > $O/bench_c2_stages.json 2>&1
echo done
