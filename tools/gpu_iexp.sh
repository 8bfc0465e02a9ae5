set -e
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/r06_bb
mkdir -p $OUT
timeout -k 10 400 /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/ablate/ablate_posterior tools/ablate/ablate_posterior.hip
timeout -k 10 200 ./tools/ablate/ablate_posterior 512 1048576 6 2 > $OUT/ablate_c3_iexp.txt 2>&1
timeout -k 10 200 ./tools/ablate/ablate_posterior 256 131072 6 3 > $OUT/ablate_c4_iexp.txt 2>&1
echo done
