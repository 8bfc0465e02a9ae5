set -e
O=gpurun_out/r02_v5
mkdir -p $O
timeout -k 10 120 ./tools/ablate/ablate_kblock2 512 1048576 6 > $O/ablate_kblock_c3.txt 2>&1
timeout -k 10 120 ./tools/ablate/ablate_kblock2 128 65536 6 > $O/ablate_kblock_c2.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "kernel_block or posterior_sizes" > $O/parity.txt 2>&1
echo done
