#!/bin/bash
# A/B of the headline bench across specialised code objects of the headline
# model: MGS_SPECIAL_OBJECT=<each object> (built with tools/ab_build.py),
# interleaved over 3 rounds; AB_CALL=1 also times one API rollout launch
# (tools/probes/single_call.py).  Usage: bash tools/ab_special.sh obj1 obj2 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/ab
mkdir -p $O
for r in a b c; do for v in "$@"; do
  MGS_SPECIAL_OBJECT=$PWD/mj-grasp-sim_amd/mgs/_lib/ab/$v.hsaco timeout -k 10 120 python3 bench.py --cpu-budget 0 --e2e-steps 0 --steps 20 > $O/$v.$r.json 2>$O/$v.$r.err || { tail $O/$v.$r.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$v.$r.json').read().strip().splitlines()[-1]); print('$v.$r', round(d['value']), round(d['detail']['rollout_kernel_ms'],1), d['detail']['static_layout_kernel'], 'stable', d['detail']['stable'], 'free', d['detail']['collision_free'])"
  if [ -n "$AB_CALL" ]; then
    MGS_SPECIAL_OBJECT=$PWD/mj-grasp-sim_amd/mgs/_lib/ab/$v.hsaco timeout -k 10 120 python3 tools/probes/single_call.py \
      2>$O/$v.$r.call.err | sed "s/^/$v.$r /" || { tail $O/$v.$r.call.err; exit 1; }
  fi
done; done
