#!/bin/bash
# First-process effect: on a fresh box, a long warm-up first, then the driver's
# command twice.  Usage: bash tools/gpu_warm_probe2.sh [tag]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-warm2}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for w in 60 5 5; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup $w --cpu-budget 0 --e2e-steps 0 > $O/w$w.json 2> $O/w$w.err || { tail -20 $O/w$w.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$O/w$w.json').read().strip().splitlines()[-1])
print('warmup $w', round(d['value']), 'ms/step', round(d['ms_per_step'], 2), 'roll ms', round(d['detail']['rollout_kernel_ms'], 2))"
done
