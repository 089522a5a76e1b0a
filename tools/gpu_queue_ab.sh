#!/bin/bash
# Work-queue rollout launch: parity test first, then the GPU suite, then a bench
# A/B of the launch mode (0: one workgroup per candidate, 1: the work queue on
# the resident grid) at 1 and 3 pipelines, then the default bench line.
# Usage: bash tools/gpu_queue_ab.sh [tag] [skip-tests]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-queue}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 300 $T tests/test_gpu_parity.py -k work_queue > $O/queue_test.log 2>&1 || { tail -30 $O/queue_test.log; exit 1; }
  tail -2 $O/queue_test.log
  timeout -k 10 900 $T tests -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -2 $O/tests.log
fi
B="python3 bench.py --cpu-budget 0 --e2e-steps 0 --steps 20"
for s in 1 3; do
  for q in 0 1; do
    timeout -k 10 300 $B --streams $s --queue $q > $O/ab_s${s}_q${q}.json 2> $O/ab_s${s}_q${q}.err || { tail -20 $O/ab_s${s}_q${q}.err; exit 1; }
    python3 -c "
import json; d = json.loads(open('$O/ab_s${s}_q${q}.json').read().strip().splitlines()[-1])
print('streams $s queue $q', round(d['value']), 'grid', d['detail']['rollout_grid'], 'roll ms', round(d['detail']['rollout_kernel_ms'], 2))"
  done
done
timeout -k 10 600 python3 bench.py --steps 20 > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
python3 -c "
import json; d = json.loads(open('$O/bench_n1.json').read().strip().splitlines()[-1])
print('default', round(d['value']), d['detail']['end_to_end_api'], d['cpu_baseline']['value'] if d['cpu_baseline'] else None)"
