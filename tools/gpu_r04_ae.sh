# Round 4, call ae: the cost of the bench's in-loop timing events at config 2 (events on every step against every
# 8th / 64th), chain modes 0 and 2 at stride 8; the timing-stride test.
set -e
O=gpurun_out/${1:-r04_ae}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread > $O/tests.txt 2>&1
for r in a b; do
  for s in 1 8 64; do
    timeout -k 10 200 python -u bench.py --config 2 --steps 400 --warmup 40 --no-cpu-baseline --no-kblock --one-launch 0 --timing-stride $s > $O/c2_m0_s${s}_$r.json 2>&1
  done
  timeout -k 10 200 python -u bench.py --config 2 --steps 400 --warmup 40 --no-cpu-baseline --no-kblock --one-launch 2 --timing-stride 8 > $O/c2_m2_s8_$r.json 2>&1
done
echo done
