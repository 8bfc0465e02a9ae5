set -e
cd "$GRAFT_REPO_ROOT"
PMC_BENCH_ARGS="--config 2" bash tools/pmc_run.sh gpurun_out/r02_v6/pmc_c2
bash tools/pmc_run.sh gpurun_out/r02_v6/pmc_c3
echo done
