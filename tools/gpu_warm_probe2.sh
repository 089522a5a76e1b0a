#!/bin/bash
# First-process effect: on a fresh box, the driver's command with the default
# wall-time warm-up floor (2 s), then without it (--warmup-s 0) twice, then
# with it again.  Usage: bash tools/gpu_warm_probe2.sh [tag]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-warm2}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
i=0
for ws in 2 0 0 2; do
  i=$((i+1))
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --warmup-s $ws --cpu-budget 0 --e2e-steps 0 > $O/r$i.json 2> $O/r$i.err || { tail -20 $O/r$i.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$O/r$i.json').read().strip().splitlines()[-1])
print('run $i warmup-s $ws', round(d['value']), 'ms/step', round(d['ms_per_step'], 2), 'warm steps', d['detail']['warmup_steps_executed'])"
done
