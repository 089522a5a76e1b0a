#!/bin/bash
# One GPU call (gpurun), any sequence of steps; each step has its own time
# limit, the chain stops at the first failure and prints what it left.
#
#   bash tools/gpu.sh <tag> <step> [<step> ...]
#
# steps:
#   tests     the GPU suite (pytest -m gpu)
#   tk:<expr> the GPU tests matching a pytest -k expression
#   smoke     __graft_entry__.smoke()
#   bench     the driver's command, `bench.py --gpus 1 --steps 20 --warmup 5`
#             (full line: e2e API, CPU baseline); first process of the call
#   rep       the driver's command without CPU baseline / e2e, 3 processes
#   api       the drop-in env API per call, one rollout launch vs 4 time slices
#   rot       in-launch rotation A/B (bench --yield-every, env API --e2e-yield)
#   streams   the driver's command with 2 / 6 / 8 pipelines in flight
#   n2        2-rank launcher rehearsal on one GPU (gloo) with the shard check
#   trace     rocprofv3 --kernel-trace --stats of the driver's command
#   pmc       PMC passes (FETCH / WRITE / SQ / VALU) on a one-pipeline bench
#   pmclds    PMC passes on LDS conflicts / waits and scalar work (one-pipeline bench)
#   stages    stage timers (MGS_PROFILE builds): headline and Shadow pile
#   heavy     stage timers over the 64 heaviest rollouts of the headline batch
#   configs   tools/bench_configs.py (C3, C4, C5)
#   c5big     C5 at 3000 + 3000 steps on 10 240 candidates, rotation on / off
#   c5cpu     the same (rotation on) with a same-run 16-thread CPU baseline
#   ghbm      G rows in HBM (MGS_G_HBM=1) vs LDS (=0: library kernels), driver's command x 2
#   c5ab:a,b  C5 (600 + 600) on the listed mgs/_lib/ab objects (MGS_SPECIAL_OBJECT)
#   py:<file> python3 <file> (a probe script under tools/)
# Outputs: gpurun_out/<tag>/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=$1
shift
O=gpurun_out/$TAG
mkdir -p "$O"
export HSA_ENABLE_IPC_MODE_LEGACY=0
DRIVER="bench.py --gpus 1 --steps 20 --warmup 5"
P1="bench.py --streams 1 --steps 1 --warmup 0 --cpu-budget 0 --e2e-steps 0 --no-escalate --fused 0"

summ() {   # one-line summary of a bench JSON line
  python3 - "$1" <<'EOF'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
x = d["detail"]
e = x.get("end_to_end_api") or {}
c = d.get("cpu_baseline") or {}
print(sys.argv[1], "value", round(d["value"]), "ms/step", round(d["ms_per_step"], 2),
      "roll ms", round(x["rollout_kernel_ms"], 2), "frac", round(d["roofline"]["frac"], 5),
      "e2e", round(e.get("candidates_per_s", 0)), "cpu", round(c.get("value", 0)),
      "shard", (x.get("shard_check") or {}).get("labels_identical_to_single_rank"))
EOF
}

fail() { echo "FAILED step $1"; tail -40 "$2"; exit 1; }

for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 1200 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > $O/tests.log 2>&1 || fail tests $O/tests.log
      tail -1 $O/tests.log ;;
    tk:*)
      # a subset of the GPU suite (pytest -k expression), before the whole suite
      k=${step#tk:}
      timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$k" \
        > $O/tk.log 2>&1 || fail "$step" $O/tk.log
      tail -1 $O/tk.log ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || fail smoke $O/smoke.log
      tail -1 $O/smoke.log ;;
    bench)
      timeout -k 10 600 python3 $DRIVER > $O/bench.json 2> $O/bench.err || fail bench $O/bench.err
      summ $O/bench.json ;;
    rep)
      for r in 1 2 3; do
        timeout -k 10 300 python3 $DRIVER --cpu-budget 0 --e2e-steps 0 > $O/rep$r.json 2> $O/rep$r.err || fail rep $O/rep$r.err
        summ $O/rep$r.json
      done ;;
    api)
      # the drop-in env API per 8192-candidate call: one rollout launch vs time slices
      for sl in 1 4; do
        timeout -k 10 300 python3 $DRIVER --cpu-budget 0 --e2e-steps 4 --e2e-slices $sl > $O/api$sl.json \
          2> $O/api$sl.err || fail api $O/api$sl.err
        summ $O/api$sl.json
      done ;;
    rot)
      # in-launch rotation A/B: the driver's command with --yield-every 0 / 16 / 32 / 64,
      # then the env API per call with its rotation off and on
      for y in 0 16 32 64; do
        timeout -k 10 300 python3 $DRIVER --cpu-budget 0 --e2e-steps 0 --yield-every $y > $O/rot$y.json \
          2> $O/rot$y.err || fail rot $O/rot$y.err
        summ $O/rot$y.json
      done
      for y in 0 32; do
        timeout -k 10 300 python3 $DRIVER --cpu-budget 0 --e2e-steps 4 --e2e-yield $y > $O/apiy$y.json \
          2> $O/apiy$y.err || fail rot $O/apiy$y.err
        summ $O/apiy$y.json
      done ;;
    streams)
      # pipelines in flight (bench --streams): 2, 6, 8 against the default 4
      for k in 2 6 8; do
        timeout -k 10 300 python3 $DRIVER --cpu-budget 0 --e2e-steps 0 --streams $k > $O/streams$k.json \
          2> $O/streams$k.err || fail streams $O/streams$k.err
        summ $O/streams$k.json
      done ;;
    n2)
      timeout -k 10 300 python3 bench.py --gpus 2 --steps 3 --warmup 1 --cpu-budget 0 --e2e-steps 0 \
        > $O/n2.json 2> $O/n2.err || fail n2 $O/n2.err
      summ $O/n2.json ;;
    trace)
      (cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
        timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o bench -f csv -- python3 $DRIVER \
          --cpu-budget 0 --e2e-steps 0 > $O/trace.json 2> $O/trace.err) || fail trace $O/trace.err
      summ $O/trace.json ;;
    pmc)
      export TMPDIR=/tmp
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_fetch -o pmc -f csv -- python3 $P1 \
        > $O/pmc_fetch.json 2> $O/pmc_fetch.err || fail pmc_fetch $O/pmc_fetch.err
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc_write -o pmc -f csv -- python3 $P1 \
        > $O/pmc_write.json 2> $O/pmc_write.err || fail pmc_write $O/pmc_write.err
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
        SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM -d $O/pmc_sq -o pmc -f csv -- python3 $P1 \
        > $O/pmc_sq.json 2> $O/pmc_sq.err || fail pmc_sq $O/pmc_sq.err
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_MFMA_F64 SQ_VALU_MFMA_BUSY_CYCLES \
        SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU \
        SQ_INSTS_SALU -d $O/pmc_valu -o pmc -f csv -- python3 $P1 > $O/pmc_valu.json 2> $O/pmc_valu.err \
        || fail pmc_valu $O/pmc_valu.err
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES \
        SQ_WAVES -d $O/pmc_lane -o pmc -f csv -- python3 $P1 > $O/pmc_lane.json 2> $O/pmc_lane.err \
        || fail pmc_lane $O/pmc_lane.err
      echo "pmc ok" ;;
    pmclds)
      # LDS pressure of the rollout kernel: bank / address conflicts, waits, in-flight level
      export TMPDIR=/tmp
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT \
        SQ_LDS_UNALIGNED_STALL SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_WAVE_CYCLES \
        -d $O/pmc_lds -o pmc -f csv -- python3 $P1 > $O/pmc_lds.json 2> $O/pmc_lds.err || fail pmc_lds $O/pmc_lds.err
      timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM \
        SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC \
        -d $O/pmc_sca -o pmc -f csv -- python3 $P1 > $O/pmc_sca.json 2> $O/pmc_sca.err || fail pmc_sca $O/pmc_sca.err
      echo "pmclds ok" ;;
    stages)
      timeout -k 10 300 python3 tools/stage_profile.py 160 > $O/stages.txt 2>&1 || fail stages $O/stages.txt
      tail -3 $O/stages.txt
      timeout -k 10 400 python3 tools/stage_profile_clutter.py 300 > $O/stages_clutter.txt 2>&1 \
        || fail stages_clutter $O/stages_clutter.txt
      tail -3 $O/stages_clutter.txt ;;
    heavy)
      # stage timers over the 64 heaviest rollouts of the headline batch (the single launch's critical path)
      timeout -k 10 300 python3 tools/stage_profile.py 64 --heavy > $O/stages_heavy.txt 2>&1 \
        || fail heavy $O/stages_heavy.txt
      tail -8 $O/stages_heavy.txt ;;
    configs)
      timeout -k 10 900 python3 tools/bench_configs.py > $O/configs.jsonl 2> $O/configs.err || fail configs $O/configs.err
      cat $O/configs.jsonl | cut -c1-300 ;;
    c5big)
      # C5 at the reference's schedule (3000 + 3000) on 10 240 candidates, rotation on and off
      for y in 32 0; do
        timeout -k 10 600 python3 tools/bench_configs.py c5 --c5-per-object 2048 --c5-steps 3000 --yield $y \
          > $O/c5big_y$y.jsonl 2> $O/c5big_y$y.err || fail c5big $O/c5big_y$y.err
        cut -c1-400 $O/c5big_y$y.jsonl
      done ;;
    ghbm)
      # G rows in HBM (mgs_model_desc.g_rows_hbm: five headline workgroups per CU,
      # <= 256 registers) against G in LDS on the driver's command, interleaved
      for r in 1 2; do for g in 0 1; do
        MGS_G_HBM=$g timeout -k 10 300 python3 $DRIVER --cpu-budget 0 --e2e-steps 0 > $O/ghbm$g.$r.json \
          2> $O/ghbm$g.$r.err || fail ghbm $O/ghbm$g.$r.err
        summ $O/ghbm$g.$r.json
      done; done ;;
    c5cpu)
      # C5 at the reference's schedule on 10 240 candidates with a same-run CPU
      # baseline (the C oracle, 16 threads, 400 evenly spaced candidates)
      timeout -k 10 900 python3 tools/bench_configs.py c5 --c5-per-object 2048 --c5-steps 3000 --c5-cpu-sample 400 \
        > $O/c5cpu.jsonl 2> $O/c5cpu.err || fail c5cpu $O/c5cpu.err
      cut -c1-600 $O/c5cpu.jsonl ;;
    c5ab:*)
      # C5 (600 + 600, 1280 candidates: one round of 48 rollouts, i.e. their latency) on
      # each listed object of mgs/_lib/ab (MGS_SPECIAL_OBJECT), interleaved twice
      objs=${step#c5ab:}
      for r in a b; do for v in ${objs//,/ }; do
        MGS_SPECIAL_OBJECT=$PWD/mj-grasp-sim_amd/mgs/_lib/ab/$v.hsaco timeout -k 10 300 python3 tools/bench_configs.py c5 \
          > $O/c5ab_$v.$r.jsonl 2> $O/c5ab_$v.$r.err || fail "$step" $O/c5ab_$v.$r.err
        python3 -c "import json; d=json.loads(open('$O/c5ab_$v.$r.jsonl').read().strip().splitlines()[-1]); print('$v.$r', round(d['value'],1), 'cand/s, rollout ms', round(d['rollout_kernel_ms'],1), 'stable', d['stable'], 'free', d['collision_free'])"
      done; done ;;
    py:*)
      f=${step#py:}
      b=$(basename "$f" .py)
      timeout -k 10 600 python3 -u "$f" > $O/$b.txt 2>&1 || fail "$step" $O/$b.txt
      tail -20 $O/$b.txt ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
