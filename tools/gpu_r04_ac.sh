# Round 4, call ac: config-2 chain variants after the EHVI-2D Φ/φ changes — separate (EHVI + two arg-max passes),
# one-pass arg-max, EHVI+arg-max in one launch — A/B/C twice, then kernel durations of each under rocprofv3.
set -e
O=gpurun_out/${1:-r04_ac}
mkdir -p $O
export TMPDIR=/tmp
for r in a b; do
  timeout -k 10 200 python -u bench.py --config 2 --steps 400 --warmup 40 --no-cpu-baseline --no-kblock --one-launch 0 > $O/c2_sep_$r.json 2>&1
  timeout -k 10 200 python -u bench.py --config 2 --steps 400 --warmup 40 --no-cpu-baseline --no-kblock --one-launch 0 --argmax-passes 1 > $O/c2_ap1_$r.json 2>&1
  timeout -k 10 200 python -u bench.py --config 2 --steps 400 --warmup 40 --no-cpu-baseline --no-kblock --one-launch 1 > $O/c2_ol1_$r.json 2>&1
done
for v in "sep --one-launch 0" "ap1 --one-launch 0 --argmax-passes 1" "ol1 --one-launch 1"; do
  set -- $v
  n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o run -- python3 bench.py --config 2 --steps 200 --warmup 20 --no-cpu-baseline --no-kblock "$@" > $O/prof_$n.log 2>&1
done
echo done
