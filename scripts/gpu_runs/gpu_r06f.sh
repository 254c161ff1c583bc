# Round 6, pass f: split-bf16 conv2_fwd phase study (no MFMA / no LDS reads / LDS reads only).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r06f; mkdir -p $O
for s in 0 1 2 3; do MIHVD_X9_STUDY=$s timeout -k 10 120 python scripts/kbench_f32.py --match "conv2_fwd [split" > $O/k$s.txt 2>&1 || { tail -20 $O/k$s.txt; exit 1; }; echo "study $s: $(grep split $O/k$s.txt)"; done
echo ALLDONE
