# Round 4, call q: persistent Cholesky with epoch LDS flags (no barrier after D) as the default up to N = 3584:
# timing and bitwise check against the blocked path, phases, TuRBO tests through the default path, config 6.
set -e
O=gpurun_out/${1:-r04_q}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 ./tools/ablate/chol_persist_check 65536 130 200 1000 2000 3000 3500 4000 5000 > $O/check.txt 2>&1
timeout -k 10 60 ./tools/ablate/chol_persist_check_nodbg 65536 3000 > $O/check_timed.txt 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_turbo.py -x -q --timeout 300 --timeout-method thread > $O/turbo_tests.txt 2>&1
timeout -k 10 200 python -u bench.py --config 6 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c6.json 2>&1
echo done
