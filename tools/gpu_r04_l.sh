# Round 4, call l: persistent Cholesky check with a short spin bound (stuck waits named), line-buffered; one-launch
# arg-max tests and configs 2/3 with one / two arg-max launches.
set -e
O=gpurun_out/${1:-r04_l}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./tools/ablate/chol_persist_check 65536 64 65 130 200 1000 3000 > $O/check.txt 2>&1 || echo "check rc=$?" >> $O/check.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k argmax --timeout 240 --timeout-method thread > $O/argmax_tests.txt 2>&1
for p in 2 1; do
  timeout -k 10 200 python -u bench.py --config 2 --steps 200 --warmup 20 --no-cpu-baseline --argmax-passes $p > $O/bench_c2_p$p.json 2>&1
done
timeout -k 10 200 python -u bench.py --config 3 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c3.json 2>&1
echo done
