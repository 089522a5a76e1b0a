#!/bin/bash
# A/B of headline code-object variants (tools/ab_variant.py) on the driver's
# bench without CPU baseline / e2e: base (the cached object), then each
# NAME:ncon:nefc[:ESCOBJ[:ESCGRID]] (an object under mgs/_lib/ab, its capacity,
# optionally the escalation engine's object and the escalation grid), twice
# interleaved.
#   bash tools/ab_bench.sh <tag> NAME:NCON:NEFC[:ESC[:GRID]] ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/$1; shift
mkdir -p "$O"
B="python3 bench.py --steps 20 --warmup 5 --cpu-budget 0 --e2e-steps 0"
summ() { python3 -c "import json,sys; d=json.loads(open('$1').read().strip().splitlines()[-1]); x=d['detail']; print('$2', round(d['value']), 'ms', round(d['ms_per_step'],2), 'roll', round(x['rollout_kernel_ms'],1), 'free', x['collision_free'], 'stable', x['stable'], 'ovf', x['overflow_candidates'], 'capped', x['still_capped_after_escalation'], 'grid', x['rollout_grid'])"; }
for r in 1 2; do
  timeout -k 10 300 $B > $O/base$r.json 2> $O/base$r.err || { tail -20 $O/base$r.err; exit 1; }
  summ $O/base$r.json base$r
  for v in "$@"; do
    IFS=: read n nc ne esc eg <<< "$v"
    objs=$PWD/mj-grasp-sim_amd/mgs/_lib/ab/$n.hsaco
    [ -n "$esc" ] && objs=$objs:$PWD/mj-grasp-sim_amd/mgs/_lib/ab/$esc.hsaco
    MGS_SPECIAL_OBJECT=$objs timeout -k 10 300 $B --ncon-max $nc --nefc-max $ne ${eg:+--esc-grid $eg} \
      > $O/$n$r.json 2> $O/$n$r.err || { tail -20 $O/$n$r.err; exit 1; }
    summ $O/$n$r.json $n$r
  done
done
