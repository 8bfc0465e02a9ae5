set -e
O=gpurun_out/r02_v3
mkdir -p $O
timeout -k 10 120 ./tools/ablate/ablate_kblock2 512 1048576 6 > $O/ablate_kblock_c3.txt 2>&1
timeout -k 10 120 ./tools/ablate/ablate_kblock2 1024 524288 30 > $O/ablate_kblock_c5.txt 2>&1
timeout -k 10 120 ./tools/ablate/ablate_posterior 128 65536 6 2 > $O/ablate_c2.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread > $O/parity.txt 2>&1
timeout -k 10 300 python -u bench.py --config 2 --steps 50 --warmup 10 > $O/bench_c2.json 2>&1
echo done
