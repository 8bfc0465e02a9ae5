# Round 4, call i: table-covariance failure (full README run) dissected; EHVI+argmax one launch (cheap ticket).
set -e
O=gpurun_out/${1:-r04_i}
mkdir -p $O
export TMPDIR=/tmp
OMB_TEST_RECORD=$O/failing_state.npz timeout -k 10 300 python -u -m pytest tests/test_gpu_cov_table.py -q -s -k diagnose --timeout 240 --timeout-method thread > $O/cov_diag.txt 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 240 --timeout-method thread > $O/fused_tests.txt 2>&1
for v in 0 1; do
  timeout -k 10 200 python -u bench.py --config 2 --steps 200 --warmup 20 --no-cpu-baseline --one-launch $v > $O/bench_c2_ol$v.json 2>&1
  timeout -k 10 200 python -u bench.py --config 3 --steps 20 --warmup 5 --no-cpu-baseline --one-launch $v > $O/bench_c3_ol$v.json 2>&1
done
echo done
