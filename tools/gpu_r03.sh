#!/bin/bash
# round-3 GPU pass: GPU suite, smoke, 2-rank launcher check (ranks share the
# one GPU over gloo), the N=1 bench line.  Usage: bash tools/gpu_r03.sh [tag] [skip-tests]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r03}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
(cat /sys/fs/cgroup/cpu.max; nproc; python3 -c "import os; print(len(os.sched_getaffinity(0)))") > $O/host.txt 2>&1
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -3 $O/tests.log
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  cat $O/smoke.log
fi
timeout -k 10 300 python3 bench.py --gpus 2 --steps 3 --warmup 1 --cpu-budget 0 --e2e-steps 0 > $O/bench_n2.json 2> $O/bench_n2.err || { tail -20 $O/bench_n2.err; exit 1; }
timeout -k 10 600 python3 bench.py --steps 20 > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
python3 -c "
import json
for f in ['$O/bench_n2.json', '$O/bench_n1.json']:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, d['n_gpus'], round(d['value']), d['detail']['static_layout_kernel'], d['detail'].get('shard_check'), d.get('cpu_baseline'))
"
