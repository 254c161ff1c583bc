cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06p
timeout -k 10 60 ./bench_native/tr16 > gpurun_out/r06p/tr16.txt 2>&1; rc=$?; cat gpurun_out/r06p/tr16.txt; exit $rc
