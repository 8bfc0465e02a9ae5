# Round 4, call z: Cholesky tests over the hand-over sizes, every schedule.
set -e
O=gpurun_out/${1:-r04_z}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_turbo.py -x -q -k chol --timeout 300 --timeout-method thread > $O/chol_tests.txt 2>&1
echo done
