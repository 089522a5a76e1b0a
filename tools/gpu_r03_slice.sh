#!/bin/bash
# Time-sliced work-queue launches: queue / slice parity tests, GPU suite, smoke,
# bench A/B (slices on / off at 1 and 4 pipelines), the drop-in API line, C5 at
# the reference schedule.  Usage: bash tools/gpu_r03_slice.sh [tag] [skip-tests]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-slice}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 300 $T tests/test_gpu_parity.py -k "work_queue or sliced" > $O/queue_test.log 2>&1 || { tail -30 $O/queue_test.log; exit 1; }
  tail -1 $O/queue_test.log
  timeout -k 10 900 $T tests -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
B="python3 bench.py --cpu-budget 0 --e2e-steps 0 --steps 30"
for cfg in "1 1" "1 0" "4 1" "4 0" "4 1"; do
  set -- $cfg
  n=ab_s$1_sl$2
  timeout -k 10 300 $B --streams $1 --slice $2 > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$O/$n.json').read().strip().splitlines()[-1])
print('$n', round(d['value']), 'grid', d['detail']['rollout_grid'], 'slice', d['detail']['slice_steps'], 'roll ms', round(d['detail']['rollout_kernel_ms'], 2))"
done
timeout -k 10 600 python3 bench.py --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
python3 -c "
import json; d = json.loads(open('$O/bench_n1.json').read().strip().splitlines()[-1])
print('default', round(d['value']), 'e2e', round(d['detail']['end_to_end_api']['candidates_per_s']), round(d['detail']['end_to_end_api']['one_call_over_repeated_batch']['candidates_per_s']), 'cpu', d['cpu_baseline']['value'])"
timeout -k 10 600 python3 -u tools/bench_configs.py c5 --c5-steps 3000 --c5-per-object 2048 > $O/c5.jsonl 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python3 -c "
import json; d = json.loads(open('$O/c5.jsonl').read().strip().splitlines()[-1]); print('c5', round(d['value'], 1), d['rollout_kernel_ms'])"
