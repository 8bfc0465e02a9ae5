# Round 4, call a: RCCL one-rank group on the box (tests/test_gpu_rccl.py) + the multirank rehearsal.
set -e
O=gpurun_out/r04_a
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_rccl.py tests/test_gpu_multirank.py -x -v -s --timeout 240 --timeout-method thread > $O/rccl_tests.txt 2>&1
echo done
