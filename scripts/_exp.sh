set -e
timeout -k 5 120 python scripts/kbench.py --roles --phases --only "conv2_bwd,conv2_bwd[role0],conv2_bwd[role1],conv2_bwd[role0,exit1],conv2_bwd[role0,exit2],conv2_bwd[role0,exit3],fc1_wgrad[role0],fc1_wgrad[role1]"
