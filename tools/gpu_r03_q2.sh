#!/bin/bash
# Queue counters without a per-launch fill + unrolled wide LDL loads: queue
# parity test, GPU suite, bench A/B of the launch mode at the default 4
# pipelines, the C5 configuration at the reference schedule, and the
# kernel-trace stats of the default bench.  Usage: bash tools/gpu_r03_q2.sh [tag]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-q2}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="python3 -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_parity.py -k work_queue > $O/queue_test.log 2>&1 || { tail -30 $O/queue_test.log; exit 1; }
tail -1 $O/queue_test.log
timeout -k 10 900 $T tests -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B="python3 bench.py --cpu-budget 0 --e2e-steps 0 --steps 30"
for q in 1 0 1; do
  timeout -k 10 300 $B --queue $q > $O/ab_q${q}.json 2> $O/ab_q${q}.err || { tail -20 $O/ab_q${q}.err; exit 1; }
  python3 -c "
import json; d = json.loads(open('$O/ab_q${q}.json').read().strip().splitlines()[-1])
print('queue $q', round(d['value']), 'grid', d['detail']['rollout_grid'], 'roll ms', round(d['detail']['rollout_kernel_ms'], 2))"
done
timeout -k 10 600 python3 -u tools/bench_configs.py c5 --c5-steps 3000 --c5-per-object 2048 > $O/c5.jsonl 2> $O/c5.err || { tail -20 $O/c5.err; exit 1; }
python3 -c "
import json; d = json.loads(open('$O/c5.jsonl').read().strip().splitlines()[-1]); print('c5', round(d['value'], 1), d['rollout_kernel_ms'])"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o bench -f csv -- python3 bench.py --cpu-budget 0 --e2e-steps 0 --steps 20 --warmup 5 > $O/trace.json 2> $O/trace.err || exit 1
head -4 $O/trace/bench_kernel_stats.csv | cut -c1-160
