# Round 4, call s: config 6 with the persistent Cholesky (one workgroup per CU) — bench twice and a kernel trace.
set -e
O=gpurun_out/${1:-r04_s}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python -u bench.py --config 6 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c6.json 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c6 -o c6 --output-format csv -- python3 bench.py --config 6 --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_c6.log 2>&1
timeout -k 10 200 python -u bench.py --config 6 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c6_again.json 2>&1
echo done
