# Round 4, call k: persistent one-launch Cholesky (kCholPersistent) against the per-step launches, edge sizes included.
set -e
O=gpurun_out/${1:-r04_k}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 ./tools/ablate/ablate_chol 63 64 65 130 512 1000 3000 5000 > $O/ablate_chol.txt 2>&1
echo done
