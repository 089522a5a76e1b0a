#!/bin/bash
# Round-3 closing pass: queue parity test, GPU suite, smoke, the driver's bench
# command, a launch-mode A/B, C3/C4/C5 configs (C5 at the reference schedule
# with its CPU baseline), then kernel-trace stats and PMC passes of the bench.
# Usage: bash tools/gpu_r03_final.sh [tag] [skip-tests]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-final}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 300 $T tests/test_gpu_parity.py -k work_queue > $O/queue_test.log 2>&1 || { tail -30 $O/queue_test.log; exit 1; }
  tail -1 $O/queue_test.log
  timeout -k 10 900 $T tests -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
python3 -c "
import json; d = json.loads(open('$O/bench_n1.json').read().strip().splitlines()[-1])
e = d['detail']['end_to_end_api']
print('bench', round(d['value']), 'grid', d['detail']['rollout_grid'], 'e2e', round(e['candidates_per_s']), round(e['one_call_over_repeated_batch']['candidates_per_s']), 'cpu', round(d['cpu_baseline']['value']), 'frac', d['roofline']['frac'])"
B="python3 bench.py --cpu-budget 0 --e2e-steps 0 --steps 30"
for q in 0 1; do
  timeout -k 10 300 $B --queue $q > $O/ab_q$q.json 2> $O/ab_q$q.err || { tail -20 $O/ab_q$q.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$O/ab_q$q.json').read().strip().splitlines()[-1])
print('queue $q', round(d['value']), 'grid', d['detail']['rollout_grid'], 'roll ms', round(d['detail']['rollout_kernel_ms'], 2))"
done
timeout -k 10 900 python3 -u tools/bench_configs.py c5 c3 c4 --c5-steps 3000 --c5-per-object 2048 --c5-cpu-sample 1024 > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 1; }
python3 -c "
import json
for l in open('$O/configs.jsonl'):
    d = json.loads(l); print(d['config'], round(d['value'], 1))"
bash tools/prof_r03.sh $1/prof nostages || exit 1
head -4 $O/prof/trace/bench_kernel_stats.csv | cut -c1-150
