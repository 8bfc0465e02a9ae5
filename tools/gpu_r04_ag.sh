# Round 4, call ag: config-6 kernel timeline (rocprofv3 kernel trace, csv) to find the GPU's idle gaps per
# Thompson step.
set -e
O=gpurun_out/${1:-r04_ag}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_c6 -o run -- python3 bench.py --config 6 --steps 30 --warmup 5 --no-cpu-baseline > $O/prof_c6.log 2>&1
echo done
