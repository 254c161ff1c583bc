set -e
timeout -k 5 120 python scripts/kbench.py --only "fc1_wgrad_k8x;fc1_wgrad_k8x_slice;adam;adam_w3_slice8;adam_small"
