#!/bin/bash
# first-run-on-a-fresh-box effect: bench with a long warm-up first, then the
# default warm-up, then the default again.  Usage: bash tools/warm_probe.sh W
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/warm; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for W in $1 3 3; do
  timeout -k 10 200 python3 bench.py --cpu-budget 0 --e2e-steps 0 --steps 20 --warmup $W > $O/w$W.json 2> $O/w$W.err || { tail $O/w$W.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/w$W.json').read().strip().splitlines()[-1]); print('W=$W', round(d['value']), round(d['ms_per_step'],1), 'enqueue_s', round(d['detail']['host_enqueue_s'],3), 'roll_ms', round(d['detail']['rollout_kernel_ms'],1), 'coll_ms', round(d['detail']['collision_kernel_ms'],1))"
done
