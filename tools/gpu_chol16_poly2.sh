#!/bin/bash
# Round 6: the Cholesky pivot's inverse square root with one second-order correction instead of two Newton steps
# (OMB_CHOL16_POLY2; the library keeps the Newton form): accuracy over 2^23 pivots, then the persistent factorisation timed with each form, alternated.
set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-poly2}
mkdir -p "$OUT"
H="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17"
timeout -k 10 300 $H -o tools/microbench/mb_rsq tools/microbench/mb_rsq.hip
timeout -k 10 400 $H -o tools/ablate/chol_hybrid_sweep tools/ablate/chol_hybrid_sweep.hip
timeout -k 10 400 $H -DOMB_CHOL16_POLY2 -o tools/ablate/chol_hybrid_sweep_poly2 tools/ablate/chol_hybrid_sweep.hip
timeout -k 10 120 ./tools/microbench/mb_rsq > "$OUT/mb_rsq.txt" 2>&1
for r in 1 2 3; do
  CHOL_K0S=0 CHOL_LS=2 timeout -k 10 200 ./tools/ablate/chol_hybrid_sweep 3000 2048 5000 > "$OUT/sweep_newton_$r.txt" 2>&1
  CHOL_K0S=0 CHOL_LS=2 timeout -k 10 200 ./tools/ablate/chol_hybrid_sweep_poly2 3000 2048 5000 > "$OUT/sweep_poly2_$r.txt" 2>&1
done
echo poly2-done
