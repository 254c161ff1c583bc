# Round 5, pass ai: PMC counters of the fp32 step's kernels at round-5 closing HEAD (after the
# load-order fixes), scripts/pmc_r05.sh.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
bash scripts/pmc_r05.sh gpurun_out/r05ai && echo ALLDONE
