set -e
timeout -k 5 120 python scripts/kbench.py --only fc1_wgrad,fc1_wgrad_k8x,adam --iters 300
for cfg in "MIHVD_FORCE_COLLECTIVES=0" "MIHVD_FORCE_COLLECTIVES=1" "MIHVD_FORCE_COLLECTIVES=1 MIHVD_FC_GATHER=0" "MIHVD_FORCE_COLLECTIVES=1 MIHVD_OVERLAP=0"; do
  echo "== $cfg"
  env $cfg timeout -k 5 90 python bench.py --steps 400 --warmup 40 | grep -o '"ms_per_step": [0-9.]*'
done
