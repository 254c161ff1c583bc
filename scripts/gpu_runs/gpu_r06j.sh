# Round 6, pass j: split-bf16 dot-product numerics probe (bench_native/mfma_split_numerics.hip).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06j
timeout -k 10 60 ./bench_native/msn > gpurun_out/r06j/msn.txt 2>&1; rc=$?; cat gpurun_out/r06j/msn.txt; exit $rc
