# Round 4, pass ac: PMC counters at HEAD (8-wave conv2_fwd, fragment W2, fc1 kernels) + stamps.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04ac; mkdir -p $O
ONLY="conv2_fwd [W2 fragment copy],conv2_bwd [W2 fragment copy],conv2_bwd [W2 fragment copy]:dg,fc1_fwd,fc1_bwd+W3 adam,head,conv_reduce+adam,conv1_fwd [+ W2 fragment copies]" timeout -k 10 300 bash scripts/pmc_r04.sh $O/pmc > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
cat $O/pmc/pmc_summary.txt
echo ALLDONE
