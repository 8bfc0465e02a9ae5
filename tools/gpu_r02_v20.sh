set -e
O=gpurun_out/r02_v20
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c6 -o c6 -- python -u bench.py --config 6 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c6.json 2>&1
echo done
