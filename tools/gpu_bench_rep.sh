#!/bin/bash
# The driver's bench command repeated (run-to-run spread on one box), then a
# 60-step run.  Usage: bash tools/gpu_bench_rep.sh [tag]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-rep}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-budget 0 --e2e-steps 0 > $O/b$r.json 2> $O/b$r.err || { tail -20 $O/b$r.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$O/b$r.json').read().strip().splitlines()[-1])
print('run $r', round(d['value']), 'ms/step', round(d['ms_per_step'], 2), 'roll ms', round(d['detail']['rollout_kernel_ms'], 2))"
done
timeout -k 10 300 python3 bench.py --steps 60 --cpu-budget 0 --e2e-steps 0 > $O/b60.json 2> $O/b60.err || { tail -20 $O/b60.err; exit 1; }
python3 -c "
import json; d = json.loads(open('$O/b60.json').read().strip().splitlines()[-1])
print('60 steps', round(d['value']), 'ms/step', round(d['ms_per_step'], 2))"
