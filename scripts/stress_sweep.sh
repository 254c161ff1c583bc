#!/bin/bash
# One-GPU variants of the stress configurations (benchmarks/stress_models.py): engine overhead
# (--no-dp), whole-step HIP graph, BERT's MLM head on masked positions vs all positions.
set -u
run() { timeout -k 5 240 python benchmarks/stress_models.py "$@" 2>/dev/null | grep '^{' || return $?; }
# (bert-base has no --graph variant: see the note in benchmarks/stress_models.py)
for v in "" "--no-dp" "--graph"; do
  echo "== resnet50 $v"; run --model resnet50 $v || exit $?
done
for v in "" "--no-dp"; do
  echo "== bert-base $v"; run --model bert-base $v || exit $?
done
echo "== bert-base --mlm-all-positions"; run --model bert-base --mlm-all-positions || exit $?
