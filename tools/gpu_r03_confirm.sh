#!/bin/bash
# Final-tree confirmation: GPU suite, smoke, the 2-rank launcher on one GPU
# (ranks share it over gloo), the driver's bench command.
# Usage: bash tools/gpu_r03_confirm.sh [tag]
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-confirm}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --gpus 2 --steps 3 --warmup 1 --cpu-budget 0 --e2e-steps 0 > $O/bench_n2.json 2> $O/bench_n2.err || { tail -20 $O/bench_n2.err; exit 1; }
python3 -c "
import json; d = json.loads(open('$O/bench_n2.json').read().strip().splitlines()[-1])
print('n2', d['n_gpus'], round(d['value']), d['detail']['shard_check']['labels_identical_to_single_rank'])"
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_n1.json 2> $O/bench_n1.err || { tail -20 $O/bench_n1.err; exit 1; }
python3 -c "
import json; d = json.loads(open('$O/bench_n1.json').read().strip().splitlines()[-1])
e = d['detail']['end_to_end_api']
print('n1', round(d['value']), 'e2e', round(e['candidates_per_s']), round(e['one_call_over_repeated_batch']['candidates_per_s']), 'cpu', round(d['cpu_baseline']['value']), 'one thread', round(d['cpu_baseline']['one_thread']['value']))"
