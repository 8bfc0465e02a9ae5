set -e
O=gpurun_out/r02_v30
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./tools/ablate/ablate_chol 64 65 130 512 1024 3000 5000 > $O/ablate_chol.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_turbo.py tests/test_gpu_gpfit.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c6 -o c6 -- python -u bench.py --config 6 --steps 10 --warmup 2 --no-cpu-baseline > $O/bench_c6.json 2>&1
echo done
