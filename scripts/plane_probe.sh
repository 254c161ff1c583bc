#!/bin/bash
# World-1 rehearsal of the N > 1 data planes (MIHVD_FORCE_COLLECTIVES=1: the collectives run over a
# process group of one, so the step's launch/stream structure is the multi-GPU one, minus the wire).
set -u
for cfg in "MIHVD_XGMI=off MIHVD_SHARD_W3=0" "MIHVD_XGMI=off MIHVD_SHARD_W3=1" "MIHVD_XGMI=on MIHVD_SHARD_W3=0" "MIHVD_XGMI=on MIHVD_SHARD_W3=1" "MIHVD_XGMI=auto"; do
  r=$(env $cfg MIHVD_FORCE_COLLECTIVES=1 timeout -k 5 90 python bench.py --steps 400 --warmup 40 2>/dev/null | grep '^{') || exit $?
  echo "$cfg: $(echo "$r" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); c=d["config"]; print(round(d["ms_per_step"]*1000,2), "us/step;", c.get("data_plane"))')"
done
