#!/bin/bash
# round-3 iteration on the GPU: suite, three short headline bench runs, stage
# timers (headline and Shadow pile).  Usage: bash tools/gpu_r03_step.sh tag [skip-tests]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/$1
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
for r in a b c; do
  timeout -k 10 120 python3 bench.py --cpu-budget 0 --e2e-steps 0 --steps 20 > $O/bench.$r.json 2> $O/bench.$r.err || { tail $O/bench.$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench.$r.json').read().strip().splitlines()[-1]); print('$r', round(d['value']), round(d['detail']['rollout_kernel_ms'],1), d['detail']['static_layout_kernel'])"
done
timeout -k 10 300 python3 tools/stage_profile.py 160 > $O/stages.txt 2>&1 || { tail $O/stages.txt; exit 1; }
tail -5 $O/stages.txt
timeout -k 10 400 python3 tools/stage_profile_clutter.py 300 > $O/stages_clutter.txt 2>&1 || { tail $O/stages_clutter.txt; exit 1; }
tail -5 $O/stages_clutter.txt
