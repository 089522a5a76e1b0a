#!/bin/bash
# Slot-packing probe of the headline pipeline (work-queue launches): streams in
# flight, batch size per launch, escalation machinery on/off.
# Usage: bash tools/gpu_pack_probe.sh [tag]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-pack}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
B="python3 bench.py --cpu-budget 0 --e2e-steps 0"
run() {
  local name=$1; shift
  timeout -k 10 300 $B "$@" > $O/$name.json 2> $O/$name.err || { tail -20 $O/$name.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$O/$name.json').read().strip().splitlines()[-1])
print('$name', '$*', round(d['value']), 'roll ms', round(d['detail']['rollout_kernel_ms'], 2), 'ms/step', round(d['ms_per_step'], 2))"
}
run s3 --steps 30 --streams 3
run s1_big --steps 4 --streams 1 --candidates 65536
run s2 --steps 30 --streams 2
run s4 --steps 30 --streams 4
run s6 --steps 30 --streams 6
run s3_noesc --steps 30 --streams 3 --no-escalate
run s3_big --steps 6 --streams 3 --candidates 32768
