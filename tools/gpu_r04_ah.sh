# Round 4, call ah: omb_thompson_step (draws + selection, one synchronisation): turbo tests (incl. the TuRBO
# (The --split-thompson flag and omb_thompson_step this call compared were not kept)
# drivers), config 6 A/B against the two calls.
set -e
O=gpurun_out/${1:-r04_ah}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_turbo.py -x -q --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
for r in a b; do
  timeout -k 10 200 python -u bench.py --config 6 --steps 100 --warmup 10 --no-cpu-baseline > $O/c6_step_$r.json 2>&1
  timeout -k 10 200 python -u bench.py --config 6 --steps 100 --warmup 10 --no-cpu-baseline --split-thompson > $O/c6_split_$r.json 2>&1
done
echo done
