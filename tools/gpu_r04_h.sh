# Round 4, call h: table-covariance install failure diagnosis; Cholesky (mov DPP) trace + stress; chain tests; configs.
set -e
O=gpurun_out/${1:-r04_h}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_cov_table.py -q -s -k diagnose --timeout 240 --timeout-method thread > $O/cov_diag.txt 2>&1
timeout -k 10 60 ./tools/microbench/mb_chol16 > $O/mb_chol16.txt 2>&1
timeout -k 10 240 ./tools/ablate/ablate_chol 512 3000 5000 > $O/ablate_chol.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_turbo.py tests/test_gpu_fused.py tests/test_gpu_gpfit.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
for v in 0 1; do
  timeout -k 10 200 python -u bench.py --config 2 --steps 200 --warmup 20 --no-cpu-baseline --one-launch $v --stage-timing > $O/bench_c2_ol$v.json 2>&1
done
timeout -k 10 200 python -u bench.py --config 3 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c3.json 2>&1
timeout -k 10 300 python -u bench.py --config 5 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_c5.json 2>&1
timeout -k 10 300 python -u bench.py --config 6 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c6.json 2>&1
echo done
