# Round 4, call ap: EHVI-2D lanes per candidate once more — varA: one lane from 2^16 (config 2 on one lane), varB:
# two lanes for every batch from 2^16 (config 3 on two lanes) — against the library (config 2 two lanes, config 3
# one), stage timings, libraries swapped on the box's copy only.
set -e
O=gpurun_out/${1:-r04_ap}
mkdir -p $O
export TMPDIR=/tmp
for r in a b; do
  for v in prev varA varB; do
    cp tools/ablate/$v/liboptimobo_hip.so optimobo_amd/liboptimobo_hip.so
    timeout -k 10 200 python -u bench.py --config 2 --steps 400 --warmup 40 --no-cpu-baseline --no-kblock --stage-timing > $O/c2_${v}_$r.json 2>&1
    timeout -k 10 200 python -u bench.py --config 3 --steps 20 --warmup 5 --no-cpu-baseline --no-kblock --stage-timing > $O/c3_${v}_$r.json 2>&1
  done
done
cp tools/ablate/prev/liboptimobo_hip.so optimobo_amd/liboptimobo_hip.so
echo done
