set -e
O=gpurun_out/r02_v4
mkdir -p $O
timeout -k 10 120 ./tools/ablate/ablate_kblock2 512 1048576 6 > $O/ablate_kblock_c3.txt 2>&1
timeout -k 10 120 ./tools/ablate/ablate_kblock2 1024 524288 30 > $O/ablate_kblock_c5.txt 2>&1
echo done
