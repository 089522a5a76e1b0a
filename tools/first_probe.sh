set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/first; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
i=0
for S in $1; do i=$((i+1))
  timeout -k 10 200 python3 bench.py --cpu-budget 0 --e2e-steps 0 --steps 20 --streams $S $2 > $O/r$i.json 2> $O/r$i.err || { tail $O/r$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/r$i.json').read().strip().splitlines()[-1]); print('run $i S=$S', round(d['value']), round(d['ms_per_step'],1), 'roll_ms', round(d['detail']['rollout_kernel_ms'],1), 'coll_ms', round(d['detail']['collision_kernel_ms'],1))"
done
