# Round 4, call ao: K block at n_var 30 (config 5) with 8 (library), 4 or 2 candidate blocks per workgroup
# (CB = 8 kept)
# (tools/ablate/var{4,2}: the pick_cb threshold raised), A/B/C twice on one box (libraries swapped on the box's copy).
set -e
O=gpurun_out/${1:-r04_ao}
mkdir -p $O
export TMPDIR=/tmp
for r in a b; do
  for v in prev var4 var2; do
    cp tools/ablate/$v/liboptimobo_hip.so optimobo_amd/liboptimobo_hip.so
    timeout -k 10 200 python -u bench.py --config 5 --steps 10 --warmup 3 --no-cpu-baseline > $O/c5_${v}_$r.json 2>&1
  done
done
cp tools/ablate/prev/liboptimobo_hip.so optimobo_amd/liboptimobo_hip.so
echo done
