# Round 4, call n: full GPU suite; Cholesky ablation (delayed trailing workgroups, persistent mode); K-block PMC at
# config 5 (traffic after the XCD-aware grid).
set -e
O=gpurun_out/${1:-r04_n}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
timeout -k 10 400 ./tools/ablate/ablate_chol 512 3000 5000 > $O/ablate_chol.txt 2>&1
PMC_BENCH_ARGS="--config 5" bash tools/pmc_run.sh $O/pmc_c5 > $O/pmc_c5.log 2>&1
echo done
