# Round 6, pass q2: split conv2_bwd (both roles split) balance study: dgrad tiles per block x wgrad images.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06q2; mkdir -p $O
for cfg in "12 0" "11 0" "11 20" "10 0" "10 10"; do set -- $cfg; MIHVD_C2BX_TPB=$1 MIHVD_C2BX_SLACK=$2 timeout -k 10 120 python scripts/kbench_f32.py --match "x6 dgrad" > $O/k_$1_$2.txt 2>&1 || { tail -20 $O/k_$1_$2.txt; exit 1; }; echo "tpb $1 slack $2: $(grep x6 $O/k_$1_$2.txt)"; done
echo ALLDONE
