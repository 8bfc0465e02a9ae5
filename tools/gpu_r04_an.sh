# Round 4, call an: config 2 with two lanes per EHVI-2D candidate (tools/ablate/var: threshold 2^16) against four
# (Two lanes from 2^16 adopted)
# (the library), A/B/A/B on one box (libraries swapped on the box's copy only).
set -e
O=gpurun_out/${1:-r04_an}
mkdir -p $O
export TMPDIR=/tmp
for r in a b; do
  cp tools/ablate/var/liboptimobo_hip.so optimobo_amd/liboptimobo_hip.so
  timeout -k 10 200 python -u bench.py --config 2 --steps 400 --warmup 40 --no-cpu-baseline --no-kblock --stage-timing > $O/c2_l2_$r.json 2>&1
  cp tools/ablate/prev/liboptimobo_hip.so optimobo_amd/liboptimobo_hip.so
  timeout -k 10 200 python -u bench.py --config 2 --steps 400 --warmup 40 --no-cpu-baseline --no-kblock --stage-timing > $O/c2_l4_$r.json 2>&1
done
echo done
