# Round 4, call u: persistent Cholesky with the walker's W from LDS and its panel flag deferred past the next D
# tiles: bitwise check, phases, Cholesky / TuRBO tests, config 6 both modes.
set -e
O=gpurun_out/${1:-r04_u}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 ./tools/ablate/chol_persist_check 65536 130 200 1000 2000 3000 3500 4000 5000 > $O/check.txt 2>&1
timeout -k 10 60 ./tools/ablate/chol_persist_check_nodbg 65536 3000 > $O/check_timed.txt 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_turbo.py -x -q --timeout 300 --timeout-method thread > $O/turbo_tests.txt 2>&1
for m in 1 2; do
  timeout -k 10 200 python -u bench.py --config 6 --steps 20 --warmup 5 --no-cpu-baseline --chol-mode $m > $O/bench_c6_m$m.json 2>&1
done
echo done
