# Round 5, pass g: BASELINE.json's stretch configs on one MI355X (benchmarks/stress_models.py):
# ResNet-50 bf16 and BERT-base seq 512 (fp16 compression), eager and whole-step HIP graph, with the
# DistributedOptimizer's buckets forced through the framework-owned RCCL bucket plane.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
export MIHVD_NO_AUTOBUILD=1
O=gpurun_out/r05g; mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  MIHVD_FORCE_COLLECTIVES=1 timeout -k 10 240 python benchmarks/stress_models.py "$@" > $O/$n.log 2>&1 || { echo "FAILED $n"; tail -15 $O/$n.log; exit 1; }
  grep '^{' $O/$n.log | python3 -c "import json,sys; d=json.loads(sys.stdin.readline()); print('$n', d['value'], d['unit'], d.get('ms_per_step'))"
}
run resnet50_eager --model resnet50 --steps 30 --warmup 10
run resnet50_graph --model resnet50 --steps 30 --warmup 10 --graph
run bert_eager --model bert-base --steps 20 --warmup 5
run bert_graph --model bert-base --steps 20 --warmup 5 --graph
echo ALLDONE
