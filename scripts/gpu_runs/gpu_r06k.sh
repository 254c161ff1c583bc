cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
mkdir -p gpurun_out/r06k
timeout -k 10 60 ./bench_native/msn > gpurun_out/r06k/msn.txt 2>&1 && cat gpurun_out/r06k/msn.txt | grep -E "f32 |x6 |x6alt|x9fresh" &&
timeout -k 10 120 python scripts/debug/dgrad_split_probe.py 100 > gpurun_out/r06k/probe.txt 2>&1; rc=$?; cat gpurun_out/r06k/probe.txt; exit $rc
