#!/bin/bash
# One-GPU variants of the stress configurations (benchmarks/stress_models.py): engine overhead
# (--no-dp), whole-step HIP graph, BERT's MLM head on masked positions vs all positions.
set -u
run() { timeout -k 5 240 python benchmarks/stress_models.py "$@" 2>/dev/null | grep '^{' || return $?; }
for m in resnet50 bert-base; do
  for v in "" "--no-dp" "--graph"; do
    echo "== $m $v"; run --model $m $v || exit $?
  done
done
echo "== bert-base --mlm-all-positions"; run --model bert-base --mlm-all-positions || exit $?
