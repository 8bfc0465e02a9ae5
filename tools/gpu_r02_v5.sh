set -e
O=gpurun_out/r02_v5
mkdir -p $O
timeout -k 10 120 ./tools/ablate/ablate_kblock2 512 1048576 6 > $O/ablate_kblock_c3.txt 2>&1
timeout -k 10 120 ./tools/ablate/ablate_kblock2 128 65536 6 > $O/ablate_kblock_c2.txt 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_polish.py tests/test_gpu_multirank.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
timeout -k 10 300 python -u bench.py > $O/bench.json 2>&1
echo done
