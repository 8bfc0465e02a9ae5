# Round 4, call ai: config 2 over 400 timed steps (the final pass's 50-step line carries the loop's start-up),
# config 3 on the spec's uniform training set (--uniform-train) beside the default box, config 1 once more.
set -e
O=gpurun_out/${1:-r04_ai}
mkdir -p $O
export TMPDIR=/tmp
for r in a b; do
  timeout -k 10 200 python -u bench.py --config 2 --steps 400 --warmup 40 > $O/c2_400_$r.json 2>&1
done
timeout -k 10 200 python -u bench.py --config 3 --no-cpu-baseline --uniform-train > $O/c3_uniform.json 2>&1
timeout -k 10 200 python -u bench.py --config 3 --no-cpu-baseline > $O/c3_box.json 2>&1
timeout -k 10 400 python -u bench.py --config 1 > $O/c1.json 2>&1
echo done
