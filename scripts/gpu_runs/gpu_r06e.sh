# Round 6, pass e: fc1_bwd regression bisection -- current kernels vs the library built with the
# round-start f32_bwd.hip (alt/k_oldbwd.so, swapped into this scratch copy only).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06e; mkdir -p $O
timeout -k 10 200 python scripts/kbench_f32.py --match "fc1_bwd|conv2_fwd|conv2_bwd" > $O/kbench_cur.txt 2>&1 || { tail -20 $O/kbench_cur.txt; exit 1; }
cat $O/kbench_cur.txt
cp alt/k_oldbwd.so mihvd/_native/libmihvd_kernels.so
timeout -k 10 200 python scripts/kbench_f32.py --match "fc1_bwd|conv2_bwd" > $O/kbench_oldbwd.txt 2>&1 || { tail -20 $O/kbench_oldbwd.txt; exit 1; }
cat $O/kbench_oldbwd.txt
echo ALLDONE
