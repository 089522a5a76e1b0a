set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/streams; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
for r in a b; do for S in 3 4 6; do
  timeout -k 10 150 python3 bench.py --cpu-budget 0 --e2e-steps 0 --steps 30 --streams $S > $O/s$S.$r.json 2> $O/s$S.$r.err || { tail $O/s$S.$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/s$S.$r.json').read().strip().splitlines()[-1]); print('S=$S $r', round(d['value']), round(d['ms_per_step'],1))"
done; done
