set -e
mkdir -p gpurun_out/r02_v2
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_v2/parity.txt 2>&1
timeout -k 10 120 ./tools/ablate/ablate_posterior 128 65536 6 2 > gpurun_out/r02_v2/ablate_c2.txt 2>&1
timeout -k 10 120 ./tools/ablate/ablate_posterior 256 131072 6 3 > gpurun_out/r02_v2/ablate_c4.txt 2>&1
timeout -k 10 120 ./tools/microbench/mb_write > gpurun_out/r02_v2/mb_write.txt 2>&1
timeout -k 10 300 python -u bench.py --config 2 --steps 50 --warmup 10 > gpurun_out/r02_v2/bench_c2.json 2>&1
timeout -k 10 300 python -u bench.py --config 4 --steps 20 --warmup 5 > gpurun_out/r02_v2/bench_c4.json 2>&1
echo done
