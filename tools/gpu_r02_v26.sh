set -e
O=gpurun_out/r02_v26
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_c3 -o c3 -- python -u bench.py --config 3 --steps 20 --warmup 3 --no-cpu-baseline > $O/bench_c3.json 2>&1
echo done
