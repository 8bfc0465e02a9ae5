# Round 4, call o: the persistent Cholesky with wave-uniform waits/flags/ticket, without the progress words
# (the build that stalled before), then the Cholesky ablation (blocked with delayed trailing workgroups).
O=gpurun_out/${1:-r04_o}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 60 ./tools/ablate/chol_persist_check_nodbg 65536 130 200 1000 3000 5000 130 > $O/check_nodbg.txt 2>&1
rc=$?; echo "rc=$rc" >> $O/check_nodbg.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 ./tools/ablate/ablate_chol 512 3000 5000 > $O/ablate_chol.txt 2>&1
echo "rc=$?" >> $O/ablate_chol.txt
