# Round 4, call w: hybrid Cholesky (k0 per-step launches, then the persistent launch): sweep k0 at N = 1000, 2000,
# 3000, 4000, 5000 (GPU-side times: a busy kernel ahead lets the host queue every launch); check tool; Cholesky tests.
set -e
O=gpurun_out/${1:-r04_w}
mkdir -p $O
export TMPDIR=/tmp
CHOL_K0S=0,2,4,8,12,16,24,32,48 timeout -k 10 200 ./tools/ablate/chol_hybrid_sweep 1000 2000 3000 4000 5000 > $O/sweep.txt 2>&1
timeout -k 10 60 ./tools/ablate/chol_persist_check 65536 130 1000 3000 > $O/check.txt 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_turbo.py -x -q -k chol --timeout 300 --timeout-method thread > $O/chol_tests.txt 2>&1
echo done
