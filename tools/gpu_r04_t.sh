# Round 4, call t: config 6 with the per-step (1) and persistent (2) Cholesky, interleaved twice; Cholesky-mode
# parity test.
set -e
O=gpurun_out/${1:-r04_t}
mkdir -p $O
export TMPDIR=/tmp
for r in a b; do
  for m in 1 2; do
    timeout -k 10 200 python -u bench.py --config 6 --steps 20 --warmup 5 --no-cpu-baseline --chol-mode $m > $O/bench_c6_m${m}_$r.json 2>&1
  done
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_turbo.py -x -q -k "chol" --timeout 240 --timeout-method thread > $O/chol_tests.txt 2>&1
echo done
