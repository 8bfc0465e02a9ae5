# Round 4, call r: persistent Cholesky at two workgroups per CU: timing + bitwise check, phases, TuRBO tests,
# config 6 with a kernel-trace summary.
set -e
O=gpurun_out/${1:-r04_r}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 ./tools/ablate/chol_persist_check 65536 130 200 1000 2000 3000 3500 4000 5000 > $O/check.txt 2>&1
timeout -k 10 60 ./tools/ablate/chol_persist_check_nodbg 65536 3000 5000 > $O/check_timed.txt 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_turbo.py -x -q --timeout 300 --timeout-method thread > $O/turbo_tests.txt 2>&1
timeout -k 10 200 python -u bench.py --config 6 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c6.json 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c6 -o c6 --output-format csv -- python3 bench.py --config 6 --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_c6.log 2>&1
echo done
