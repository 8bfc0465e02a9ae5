# Round 4, call al: EHVI-2D chain with the batch in chunks, each chunk's EHVI on a second stream overlapping the
# next chunk's posterior (tools/ablate/overlap_chain.py), configs 3 and 2.
set -e
O=gpurun_out/${1:-r04_al}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ablate/overlap_chain.py 3 20 2,4,8 > $O/overlap_c3.txt 2>&1
timeout -k 10 200 python -u tools/ablate/overlap_chain.py 2 300 2,4 > $O/overlap_c2.txt 2>&1
echo done
