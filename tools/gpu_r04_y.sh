# Round 4, call y: config-4 posterior variants (n = 256, 3 objectives, 2^17 candidates): counter ring CT 2 / 4,
# 16-wave rings, tile kernel.
set -e
O=gpurun_out/${1:-r04_y}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 ./tools/ablate/ablate_posterior 256 131072 6 3 > $O/ablate_c4.txt 2>&1
echo done
