"""Headline benchmark: grasp candidates evaluated / s at a 200-step horizon,
Robotiq 2F-85 x YCB 003_cracker_box (BASELINE.json configs[1]: 8192 candidates
x 200 steps per MI355X).

One step = the reference's filter_to_stable pipeline (mgs/cli/filter_to_stable.py:
39-50) over one batch: collision mask of every candidate, then the close ->
lift -> shake rollout of the collision-free ones (h200 horizon).  Inputs are
host-prepared once (float32 SE3 processing, mocap schedule), uploaded, and
resident in HBM when the timed region starts; each step runs the fused mask +
rollout launch (mgs_mask_rollout_device, a work queue on the resident grid)
on its pipeline's HIP stream with no host round trip; the launch lists its
capacity overflows itself and the wider re-run of the listed candidates (the
env's escalation) follows on a side stream.  Steps rotate over
`--streams` pipelines (engine + stream each, default 4), so one batch's
rollout tail overlaps the next batches' work; every step is a whole batch.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--candidates 8192]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Multi-GPU: weak scaling, one process per GPU, each rank evaluates its own
8192-candidate block (seed = rank); no data-path collective -- only the
timing barrier and the max-over-ranks reduction.  Run directly with --gpus N
(no WORLD_SIZE in the environment), the script starts the N ranks itself as
child processes before any GPU call; under a launcher, WORLD_SIZE must equal N.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mj-grasp-sim_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

# one hardware queue per HIP stream: S pipeline streams + S escalation streams
# (the default of 4 queues would serialise an escalation re-run with the next
# step of the pipeline sharing its queue); set before the runtime starts
def _argv_streams(default=4):
    a = sys.argv
    for i, x in enumerate(a):
        if x == "--streams" and i + 1 < len(a):
            return int(a[i + 1])
        if x.startswith("--streams="):
            return int(x.split("=", 1)[1])
    return default


os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, max(8, 2 * _argv_streams())))

HBM_PEAK_GBS = 8000.0     # MI355X HBM3E peak (MI355X_MICROARCH.md)


def algorithmic_bytes(cm, steps, sum_ncon, sum_nefc, w=8):
    """SURVEY.md §8(d) B_cs summed over the executed candidate-steps of a launch:
    every per-candidate SoA array read once and written once per step (fp64)."""
    ngeom = len(cm.geom_bodyid)
    per_step = (2 * (cm.nq + 2 * cm.nv + cm.nu + 7 * cm.nmocap + 1) + 2 * 7 * cm.nbody
                + 2 * 12 * ngeom + 2 * cm.nv * cm.nv)
    return w * (per_step * steps + 2 * 18 * sum_ncon + 2 * (cm.nv + 6) * sum_nefc)


def executed_steps(labels, fail_step, active, horizon):
    """candidate-steps actually simulated (early exits stop a rollout)."""
    s = np.where(labels, horizon, fail_step + 1)
    return int(np.sum(np.where(active, s, 0)))


def pmc_record():
    """the committed PMC pass (profiles/pmc_rollout.json) and a label of where it
    came from -- its numbers are read from that file, not measured in this run"""
    p = os.path.join(ROOT, "profiles", "pmc_rollout.json")
    if not os.path.isfile(p):
        return None, None
    with open(p) as f:
        j = json.load(f)
    m = j.get("measured") or {}
    label = ("stored: profiles/pmc_rollout.json, rocprofv3 PMC pass %s (commit %s, %s) on a one-pipeline bench, "
             "per candidate-step scaled to this launch" % (m.get("tag", "?"), m.get("commit", "?"), m.get("date", "?")))
    return j, label


def load_traffic(launch_steps):
    """HBM bytes per rollout launch from the committed PMC pass (profiles/), scaled
    to this launch's candidate-steps; None if no PMC summary is present."""
    j, _ = pmc_record()
    if j is None:
        return None
    per_cs = j.get("hbm_bytes_per_candidate_step")
    return None if per_cs is None else float(per_cs) * launch_steps


def cpu_baseline(env, poses, joints, h, budget_s, threads):
    """The oracle (C restatement, OpenMP over candidates) on the host cores, on a
    bounded leading sample of the same candidate block; returns a dict."""
    from oracle import oracle as O
    om = O.OracleModel(env.model, ncon_max=40)         # the escalation ceiling: MuJoCo has no cap
    q, mp, mq, _ = env.initial_state(poses, joints)
    # pilot (two candidates per thread, at least 16) to size the sample to the time budget
    n_pilot = min(max(16, 2 * threads), len(poses))
    t0 = time.perf_counter()
    free = om.collision_free(q[:n_pilot], mp[:n_pilot], mq[:n_pilot], nthreads=threads)
    idx = np.nonzero(free)[0]
    if len(idx):
        plan = env.rollout_plan(poses[idx], joints[idx], nstep_lift=h["nstep_lift"], shake_steps=h["shake_steps"],
                                close_steps=h["close_steps"], lift_check_every=h["lift_check_every"])
        om.rollout(plan, nthreads=threads)
    dt_pilot = max(time.perf_counter() - t0, 1e-6)
    want = n_pilot * budget_s / dt_pilot
    n = int(min(len(poses), max(n_pilot, want)))
    reps = 0
    t0 = time.perf_counter()
    # whole passes until the budget is spent (at least one): a block shorter
    # than the budget is timed over repeated passes
    while reps == 0 or (n == len(poses) and time.perf_counter() - t0 < budget_s):
        reps += 1
        free = om.collision_free(q[:n], mp[:n], mq[:n], nthreads=threads)
        idx = np.nonzero(free)[0]
        labels = np.zeros(n, bool)
        if len(idx):
            plan = env.rollout_plan(poses[idx], joints[idx], nstep_lift=h["nstep_lift"],
                                    shake_steps=h["shake_steps"], close_steps=h["close_steps"],
                                    lift_check_every=h["lift_check_every"])
            labels[idx] = om.rollout(plan, nthreads=threads)["label"]
    dt = time.perf_counter() - t0
    return dict(value=n * reps / dt, n=n, reps=reps, seconds=dt, free=free, labels=labels)


def cpu_share():
    """CPUs this process can actually run on: the affinity mask, capped by the
    cgroup v2 CPU quota (rounded up)"""
    n = len(os.sched_getaffinity(0))
    q = host_info()["cgroup_cpu_quota"]
    return max(1, min(n, int(-(-q // 1)))) if q else n


def host_info():
    """the CPU the baseline ran on: model name and the cores visible to this process"""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    quota = None
    try:
        # cgroup v2 CPU bandwidth limit ("max 100000" = none): the share of the
        # visible CPUs this process can actually use
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()
            quota = None if q == "max" else float(q) / float(period)
    except (OSError, ValueError):
        pass
    return {"cpu_model": model, "cpus_visible": len(os.sched_getaffinity(0)), "cpu_count": os.cpu_count(),
            "cgroup_cpu_quota": quota}


# VALU issue peak of the chip (MI355X_MICROARCH.md: 256 CUs x 4 SIMDs; a wave64
# VALU instruction issues over 2 cycles on a SIMD-32 at f32, and f64 vector
# arithmetic runs at half that lane rate -- 78.6 TF f64 vector = 256 x 4 x 16
# lanes x 2 flops x 2.4 GHz -- so 4 cycles; the sustained clock under this load
# is 2.39-2.40 GHz, profiles/r03_clock_probe.txt)
CHIP_SIMDS = 256 * 4
CLOCK_HZ = 2.4e9
VALU_CYC_F64, VALU_CYC_OTHER = 4.0, 2.0


def valu_roofline(candidate_steps_per_s):
    """the rollout kernel against the chip's VALU issue peak: VALU wave-
    instructions per candidate-step (the committed PMC pass) x this run's
    candidate-steps/s / (CHIP_SIMDS x CLOCK_HZ / c), c the mix's mean issue
    cycles per wave-instruction (f64 arithmetic 4, the rest 2)"""
    j, label = pmc_record()
    if j is None:
        return None
    sq, cs = j.get("sq", {}), j.get("executed_candidate_steps")
    if not sq.get("SQ_INSTS_VALU") or not cs:
        return None
    valu = sq["SQ_INSTS_VALU"]
    f64 = sum(sq.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                        "SQ_INSTS_VALU_TRANS_F64"))
    share = f64 / valu
    cyc = share * VALU_CYC_F64 + (1.0 - share) * VALU_CYC_OTHER
    peak = CHIP_SIMDS * CLOCK_HZ / cyc
    per_cs = valu / cs
    achieved = per_cs * candidate_steps_per_s
    return {"bound": "valu_issue", "achieved": achieved, "peak": peak, "unit": "wave-instructions/s",
            "frac": achieved / peak, "valu_per_candidate_step": per_cs, "f64_share": share,
            "mean_issue_cycles": cyc, "candidate_steps_per_s": candidate_steps_per_s,
            "source": label,
            "what": "VALU wave-instructions per candidate-step (PMC pass) x this run's executed candidate-steps/s "
                    "(device level: all launches in flight) / the chip's VALU issue peak for this f64 / other mix"}


def issue_summary():
    """latency / issue view of the rollout kernel from the committed PMC pass
    (profiles/pmc_rollout.json): instructions and wave cycles per executed
    candidate-step; None if absent"""
    j, label = pmc_record()
    if j is None:
        return None
    sq, cs = j.get("sq", {}), j.get("executed_candidate_steps")
    if not sq or not cs:
        return None
    # SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles
    # (MI355X_MICROARCH.md, per-instruction constants table); instruction
    # counters count wave-instructions
    quad = ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU")
    out = {}
    for k, v in sq.items():
        name = k.replace("SQ_", "").lower()
        if k in quad:
            out[name + "_cycles_per_candidate_step"] = 4.0 * v / cs
        else:
            out[name + "_per_candidate_step"] = v / cs
    if "SQ_WAIT_ANY" in sq and "SQ_WAVE_CYCLES" in sq:
        # latency view: the share of a wave's lifetime spent issuing, parked at
        # s_waitcnt (LDS / memory) and stalled at issue; one wave per SIMD
        # (register-limited), so parked cycles are idle SIMD cycles
        w = sq["SQ_WAVE_CYCLES"]
        out["issue_frac"] = sq.get("SQ_ACTIVE_INST_ANY", 0.0) / w
        out["wait_any_frac"] = sq["SQ_WAIT_ANY"] / w
        out["wait_inst_any_frac"] = sq.get("SQ_WAIT_INST_ANY", 0.0) / w
    f64 = sum(sq.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                        "SQ_INSTS_VALU_TRANS_F64"))
    if f64 and sq.get("SQ_INSTS_VALU"):
        out["f64_arith_share_of_valu"] = f64 / sq["SQ_INSTS_VALU"]
    out["source"] = label + " (" + j.get("kernel", "") + ")"
    return out


def e2e_api(env, poses, J, h, steps):
    """the drop-in path as the reference's filter_to_stable calls it
    (mgs/cli/filter_to_stable.py:39-50): host arrays in, collision mask, then
    the rollout of the collision-free subset, labels back on the host; host
    pose processing, schedule building and PCIe copies included"""
    ts = []
    for _ in range(steps):
        t0 = time.perf_counter()
        mask = env.grasp_collision_mask(poses, J)
        idx = np.nonzero(mask)[0]
        labels = np.zeros(len(poses), bool)
        if len(idx):
            labels[idx] = env.grasp_stability_evaluation_from_joints(
                poses[idx], J[idx], nstep_lift=h["nstep_lift"], shake_steps=h["shake_steps"],
                close_steps=h["close_steps"], lift_check_every=h["lift_check_every"])
        ts.append(time.perf_counter() - t0)
    return mask, labels, float(np.median(ts))


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n):
    """`bench.py --gpus N` run directly (no WORLD_SIZE from a launcher): start N
    fresh child processes of this script, one rank per GPU (RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* set), before anything in this parent touches the GPU,
    and exit with the worst child status.  Rank 0 prints the JSON line."""
    import subprocess
    port = str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), *sys.argv[1:]], env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--candidates", type=int, default=8192)
    ap.add_argument("--horizon", default="h200")
    ap.add_argument("--solver", default=None, help="override the model's solver (Newton | PGS)")
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of CPU baseline work (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="CPU baseline threads (default: the CPUs this process may use, cgroup quota included)")
    ap.add_argument("--no-shard-check", dest="shard_check", action="store_false",
                    help="N > 1: skip rank 0's single-GPU re-evaluation of every rank's block")
    ap.add_argument("--e2e-large", type=int, default=8,
                    help="also time the drop-in API on the batch repeated this many times in one call (0 = skip)")
    ap.add_argument("--e2e-steps", type=int, default=5,
                    help="batches timed through the drop-in env API on host arrays (0 = skip)")
    ap.add_argument("--e2e-slices", type=int, default=None,
                    help="time slices by relaunch of the env API's rollout calls (default: the env's SLICES)")
    ap.add_argument("--e2e-yield", type=int, default=None,
                    help="in-launch rotation of the env API's rollout launches, steps per slice (default: the "
                         "env's YIELD_EVERY; 0 = off)")
    ap.add_argument("--yield-every", type=int, default=32,
                    help="in-launch rotation (mgs_schedule.yield_every, the env API's default too) of the timed "
                         "pipelines' launches, steps per slice (0 = off; needs the resume records of "
                         "--esc-resume 1); profiles/r04e_rotation_ab.txt")
    ap.add_argument("--streams", type=int, default=4,
                    help="batches in flight: pipelines (engine + HIP stream) the steps rotate over")
    ap.add_argument("--ncon-max", type=int, default=20, help="per-candidate contact capacity of the main kernel")
    ap.add_argument("--nefc-max", type=int, default=None,
                    help="per-candidate constraint-row capacity of the main kernel (default: auto_capacity)")
    ap.add_argument("--esc-grid", type=int, default=1, help="workgroups of the escalation list re-run")
    ap.add_argument("--esc-side", type=int, default=1, help="1: escalation re-runs on a side stream per pipeline")
    ap.add_argument("--fused", type=int, default=1,
                    help="1: collision mask and rollout in one launch per step (mgs_mask_rollout_device); "
                         "0: a mask launch, then the rollout launch over its collision-free candidates")
    ap.add_argument("--esc-resume", type=int, default=1,
                    help="1: overflowing candidates stop at the overflowing step and the escalation continues "
                         "them from there (0: re-run from the start)")
    ap.add_argument("--warmup-s", type=float, default=0.0,
                    help="untimed warm-up continues past --warmup steps until this much wall time has passed "
                         "(probe of the fresh-box first-process deficit, profiles/r03q_first_process.txt)")
    ap.add_argument("--queue", type=int, default=None,
                    help="rollout launch mode (mgs_rollout_queue): 0 one workgroup per candidate, 1 the work queue "
                         "on the resident grid (the library default)")
    ap.add_argument("--no-escalate", dest="escalate", action="store_false",
                    help="skip the contact-capacity re-run of overflowed candidates")
    ap.add_argument("--dry-run", action="store_true", help="print each rank's layout and exit (no GPU work)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if args.cpu_threads is None:
        # every CPU this process may use (all cores), whatever
        # OMP_NUM_THREADS the box exports: the affinity mask, capped by the
        # cgroup CPU bandwidth quota (a 16-CPU quota over 256 visible CPUs on the
        # GPU box: 256 threads there run 3.5x slower than 16, time-sliced)
        args.cpu_threads = cpu_share()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
        sys.exit(2)
    if args.dry_run:
        # launcher check (tests/test_bench_launch.py): the rank layout, no GPU work
        print(json.dumps({"rank": int(os.environ.get("RANK", "0")), "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
                          "world": world, "master": os.environ.get("MASTER_ADDR")}), flush=True)
        return
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    # one GPU per rank; a rehearsal with more ranks than GPUs (a 1-GPU box)
    # shares the devices round-robin over gloo, since RCCL needs distinct GPUs
    ngpu = torch.cuda.device_count()
    shared = world > 1 and world > ngpu
    local = local % max(1, ngpu) if shared else local
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if shared:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)

    # the headline engines run their model-specialised code objects, compiled
    # here (outside the timed region) if build() did not leave them cached
    os.environ.setdefault("MGS_SPECIALIZE", "1")
    from mgs.core import abi
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping, HORIZONS
    from mgs.gripper.robotiq2f85 import GripperRobotiq2f85
    from mgs.obj.selector import get_object
    from mgs.sampler.antipodal import robotiq_candidates
    from mgs.util.geo.transforms import SE3Pose

    grip = GripperRobotiq2f85(SE3Pose(np.zeros(3), np.array([1.0, 0, 0, 0]), "wxyz"))
    obj = get_object("003_cracker_box")
    env = GravitylessObjectGrasping(grip, obj, device=local, ncon_max=args.ncon_max, nefc_max=args.nefc_max)
    if args.solver:
        env.model.options["solver"] = args.solver
    h = HORIZONS[args.horizon]
    N = args.candidates
    H, J, _ = robotiq_candidates(obj, N, seed=rank)
    poses = SE3Pose.from_mat(H)
    qpos, mpos, mquat, _ = env.initial_state(poses, J)
    plan = env.rollout_plan(poses, J, nstep_lift=h["nstep_lift"], shake_steps=h["shake_steps"],
                            close_steps=h["close_steps"], lift_check_every=h["lift_check_every"])
    sched = abi.make_schedule(plan.nsteps, plan.check_every, plan.check_at_end, plan.ctrl, plan.obj_qposadr,
                                  check_offset=getattr(plan, "check_offset", None))
    sched.yield_every = int(args.yield_every)
    horizon = plan.horizon
    eng = env.engine
    if args.queue is not None:
        eng.lib.mgs_rollout_queue(args.queue)
    dev = torch.device("cuda", local)
    f64 = dict(dtype=torch.float64, device=dev)
    d_q = torch.as_tensor(qpos, **f64).contiguous()
    d_mp = torch.as_tensor(mpos, **f64).contiguous()
    d_mq = torch.as_tensor(mquat, **f64).contiguous()
    d_ps = torch.as_tensor(plan.phase_start, **f64).contiguous()
    d_pt = torch.as_tensor(plan.phase_target, **f64).contiguous()
    # S pipelines, each with its own engine (device work buffers, HIP events),
    # output buffers and HIP stream; step k runs on pipeline k % S, so one batch's
    # rollout tail overlaps the next batch's start (no host synchronisation
    # inside the timed loop).  Every step does the whole filter_to_stable pass.
    from mgs.core.engine import Engine
    NS = abi.MGS["MGS_NSTATS"]
    ESC_GRID = args.esc_grid
    RESUME = bool(args.escalate and args.esc_resume)
    FUSED = bool(args.fused)
    RW = env.engine.resume_width()
    LH = abi.MGS["MGS_LIST_HEADER"]

    class Pipe:
        def __init__(self, s):
            self.eng = env.engine if s == 0 else Engine(env.model, device=local, ncon_max=env.ncon_max,
                                                          nefc_max=env.nefc_max, g_rows_hbm="auto")
            self.stream = torch.cuda.current_stream(dev) if s == 0 else torch.cuda.Stream(dev)
            self.free = torch.zeros(N, dtype=torch.uint8, device=dev)
            self.label = torch.zeros(N, dtype=torch.uint8, device=dev)
            self.fail = torch.zeros(N, dtype=torch.int32, device=dev)
            self.objq = torch.zeros((N, 7), **f64)
            self.stats = torch.zeros((N, NS), dtype=torch.int32, device=dev)
            # contact-capacity escalation (GravitylessObjectGrasping.rollout: the
            # candidates whose contacts / rows exceeded the capacity are re-run
            # with twice the capacity): the step's rollout appends each
            # overflowing candidate to the step's device list itself (ABI 17:
            # a list header + n indices, zeroed once here and left zeroed by
            # each list re-run) and stops it at that step, leaving its state in
            # the step's resume records; the list re-run (mgs_rollout_list_device,
            # ESC_GRID workgroups looping over the list) continues them on this
            # pipeline's escalation stream into the step's own escalation
            # outputs.  Nothing runs between two rollouts of a pipeline's
            # stream, and the pipeline never waits for its side stream.
            self.wide = Engine(env.model, device=local, ncon_max=2 * env.ncon_max,
                               specialize="cached", role="escalation") if args.escalate else None
            self.esc_stream = torch.cuda.Stream(dev)
            self.esc = []          # per step: list (header + indices), label, fail, objq, stats, resume records
            self.events = []
            self.last = -1

        def esc_buffers(self, k):
            while len(self.esc) <= k:
                self.esc.append((torch.zeros(LH + N, dtype=torch.int32, device=dev),
                                 torch.zeros(N, dtype=torch.uint8, device=dev),
                                 torch.zeros(N, dtype=torch.int32, device=dev), torch.zeros((N, 7), **f64),
                                 torch.zeros((N, NS), dtype=torch.int32, device=dev),
                                 torch.zeros((N, RW) if RESUME else 1, **f64)))
            return self.esc[k]

        def step(self, k, timed):
            sp = self.stream.cuda_stream
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)] if timed else None
            ovf, el, ef, eo, es, rec = self.esc_buffers(k) if self.wide is not None else (None,) * 6
            d_ovf = ovf.data_ptr() if ovf is not None else None
            with torch.cuda.stream(self.stream):
                if ev:
                    ev[0].record(self.stream)
                if not FUSED:
                    self.eng.collision_free_device(N, d_q.data_ptr(), d_mp.data_ptr(), d_mq.data_ptr(),
                                                   self.free.data_ptr(), predicate="any", stream=sp)
                if ev:
                    ev[1].record(self.stream)
                if FUSED:
                    # mask + rollout in one launch (mgs_mask_rollout_device): each
                    # workgroup computes its candidate's mask and, if collision-free,
                    # its rollout; no rollout waits for a separate mask launch
                    self.eng.mask_rollout_device(sched, N, d_q.data_ptr(), d_mp.data_ptr(), d_mq.data_ptr(),
                                                 d_ps.data_ptr(), d_pt.data_ptr(), self.free.data_ptr(),
                                                 self.label.data_ptr(), self.fail.data_ptr(), self.objq.data_ptr(),
                                                 self.stats.data_ptr(),
                                                 d_resume_out=rec.data_ptr() if RESUME else None,
                                                 predicate="any", stream=sp, d_ovf=d_ovf)
                else:
                    self.eng.rollout_resumable_device(sched, N, d_q.data_ptr(), d_mq.data_ptr(), d_ps.data_ptr(),
                                                      d_pt.data_ptr(), self.label.data_ptr(), self.fail.data_ptr(),
                                                      self.objq.data_ptr(), self.stats.data_ptr(),
                                                      (rec if RESUME else self.res_scratch()).data_ptr(),
                                                      d_active=self.free.data_ptr(), stream=sp, d_ovf=d_ovf)
                if ev:
                    ev[2].record(self.stream)
                    self.events.append(ev)
                if self.wide is not None:
                    done = torch.cuda.Event()
                    done.record(self.stream)
                    es_ = self.esc_stream if args.esc_side else self.stream
                    es_.wait_event(done)
                    self.wide.rollout_list_device(sched, N, d_ovf, d_ovf + 4 * LH, ESC_GRID, d_q.data_ptr(),
                                                  d_mq.data_ptr(), d_ps.data_ptr(), d_pt.data_ptr(), el.data_ptr(),
                                                  ef.data_ptr(), eo.data_ptr(), es.data_ptr(),
                                                  stream=es_.cuda_stream,
                                                  d_resume_in=rec.data_ptr() if RESUME else None)
            self.last = k

        def res_scratch(self):
            # the non-resumed escalation (--esc-resume 0) re-runs from the start:
            # the capped launch still needs somewhere to put its records
            if not hasattr(self, "_rs"):
                self._rs = torch.zeros((N, RW), **f64)
            return self._rs

        def merge_last(self):
            """this pipeline's last step with its escalated candidates merged;
            returns (escalated count, still capped after escalation)"""
            if self.wide is None or self.last < 0:
                return 0, 0
            ovf, el, ef, eo, es, _ = self.esc[self.last]
            m = int(ovf[2].item())        # the count the list re-run ran
            if m == 0:
                return 0, 0
            idx = ovf[LH:LH + m].long()
            self.label[idx] = el[idx]
            self.fail[idx] = ef[idx]
            self.objq[idx] = eo[idx]
            self.stats[idx] = es[idx]
            return m, int(((es[idx, 2] & abi.MGS["MGS_FLAG_CAPACITY"]) != 0).sum().item())

    pipes = [Pipe(s) for s in range(max(1, args.streams))]
    # every step's escalation buffers allocated up front: first-touch device
    # allocations inside the timed loop cost several % on a fresh box
    per_pipe = -(-max(args.warmup, len(pipes), args.steps) // len(pipes))
    for p in pipes:
        if p.wide is not None:
            p.esc_buffers(per_pipe)
    torch.cuda.synchronize(dev)
    tw = time.perf_counter()
    nwarm = max(args.warmup, len(pipes))
    for k in range(nwarm):       # every pipeline (and its escalation) warmed up
        pipes[k % len(pipes)].step(k // len(pipes), False)
    torch.cuda.synchronize(dev)
    # optional warm-up floor in wall time: further untimed rounds over the
    # pipelines (outputs overwritten by the timed steps; nothing carries over)
    while time.perf_counter() - tw < args.warmup_s:
        for p in pipes:
            p.step(0, False)
        nwarm += len(pipes)
        torch.cuda.synchronize(dev)
    for p in pipes:            # the warm-up launches' device spans, dropped
        p.eng.queue_spans()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        pipes[k % len(pipes)].step(k // len(pipes), True)
    t_enq = time.perf_counter() - t0      # host time to enqueue the K steps (diagnostic)
    torch.cuda.synchronize(dev)
    merged = [p.merge_last() for p in pipes]
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    # in-launch rotation audit (outside the timed region): no ring spin expired
    # in any pipeline's launches and no candidate kept the MGS_FAIL_YIELDED
    # sentinel (a lost candidate) -- else the line is not printed
    from mgs.core.engine import check_no_lost_candidates
    qs = [p.eng.queue_stats() for p in pipes]
    for p in pipes:
        check_no_lost_candidates(p.fail.cpu().numpy(), sum(x[1] for x in qs))
    rotation = {"yields": int(sum(x[0] for x in qs)), "expired_spins": int(sum(x[1] for x in qs)),
                "lost_candidates": 0}
    # the timed main launches' execution spans on the device clock (first
    # candidate taken -> last workgroup out, mgs_queue_spans): what a kernel
    # trace reports as their durations, without a profiler attached
    spans, spans_lost = [], 0
    for p in pipes:
        spans += p.eng.queue_spans()
        spans_lost += p.eng.spans_overwritten
    if spans_lost:
        print(f"bench: {spans_lost} timed launch span(s) overwritten before they were read (more than 64 "
              "launches per pipeline); launch_ms averages the rest", file=sys.stderr)
    t = torch.tensor([dt], dtype=torch.float64, device="cpu" if shared else dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    # per-launch kernel durations from the HIP events on each pipeline's stream
    coll_ms = [e[0].elapsed_time(e[1]) for p in pipes for e in p.events]
    roll_ms = [e[1].elapsed_time(e[2]) for p in pipes for e in p.events]
    P0 = pipes[0]
    d_free, d_label, d_fail, d_stats = P0.free, P0.label, P0.fail, P0.stats
    same_pipes = all(torch.equal(p.label, P0.label) and torch.equal(p.free, P0.free) and
                     torch.equal(p.fail, P0.fail) for p in pipes[1:])
    wide = P0.wide

    free = d_free.cpu().numpy().astype(bool)
    labels = d_label.cpu().numpy().astype(bool)
    fail = d_fail.cpu().numpy()
    stats = d_stats.cpu().numpy()
    e2e = None
    if args.e2e_slices is not None:
        env.SLICES = args.e2e_slices
    if args.e2e_yield is not None:
        env.YIELD_EVERY = args.e2e_yield
    if args.e2e_steps > 0:
        # the env's engines are created once per env (as a CLI run creates them
        # once): one untimed call builds the small-call engine
        # (GravitylessObjectGrasping.engine_for_rollouts) before the timed ones
        e2e_api(env, poses, J, h, 1)
        m2, l2, t2 = e2e_api(env, poses, J, h, args.e2e_steps)
        large = None
        if args.e2e_large > 1:
            # one call over the batch repeated k times (the CLI evaluates a whole
            # candidate file per call): the rollout launch's last-round tail is
            # amortised over more rounds of waves
            k = args.e2e_large
            pk = SE3Pose.from_mat(np.tile(np.asarray(H), (k, 1, 1)))
            mk, lk, tk = e2e_api(env, pk, np.tile(J, (k, 1)), h, 1)
            large = {"candidates": N * k, "candidates_per_s": N * k / tk, "seconds": tk,
                     "labels_identical_to_device_run": bool(np.array_equal(mk, np.tile(free, k)) and
                                                            np.array_equal(lk, np.tile(labels, k)))}
        e2e = {"candidates_per_s": N / t2, "ms_per_batch": t2 * 1e3, "batches": args.e2e_steps,
               "rollout_slices": getattr(env, "SLICES", 1),
               "rollout_yield_every": getattr(env, "YIELD_EVERY", 0),
               "one_call_over_repeated_batch": large,
               "labels_identical_to_device_run": bool(np.array_equal(m2, free) and np.array_equal(l2, labels)),
               "what": "env.grasp_collision_mask + grasp_stability_evaluation_from_joints on host arrays "
                       "(filter_to_stable.py:39-50 call pattern): host SE3 processing, schedule, PCIe "
                       "copies and the host round trip between mask and rollout included; per rank, "
                       "median over batches after one untimed call",
               "rollout_engine": ("G rows in LDS" if env.engine_for_rollouts(int(free.sum())) is not env.engine
                                  else "G rows in HBM" if int(env.engine.desc.g_rows_hbm) else "G rows in LDS")}
    shard_check = None
    if world > 1 and args.shard_check:
        # the global candidate set is the concatenation of the
        # seed-b blocks (rank b evaluates block b); rank 0 re-evaluates every
        # block on its own GPU and compares the gathered labels bit for bit
        from mgs.env.sharding import gather_results
        t0c = time.perf_counter()
        g = gather_results({"H": np.asarray(H)[None], "J": np.asarray(J)[None], "free": free[None],
                            "labels": labels[None]})
        if rank == 0:
            same = True
            for b in range(world):
                pb = SE3Pose.from_mat(g["H"][b])
                mb, lb, _ = e2e_api(env, pb, g["J"][b], h, 1)
                same = same and bool(np.array_equal(mb, g["free"][b]) and np.array_equal(lb, g["labels"][b]))
            shard_check = {"blocks": world, "candidates": world * N, "labels_identical_to_single_rank": same,
                           "seconds": time.perf_counter() - t0c,
                           "what": "labels gathered from the N ranks == rank 0 evaluating every block alone"}
        dist.barrier()
    if rank != 0:
        if world > 1:
            dist.destroy_process_group()
        return
    steps_exec = executed_steps(labels, fail, free, horizon)
    alg = algorithmic_bytes(env.model, steps_exec, int(stats[:, 4].sum()), int(stats[:, 5].sum()))
    roll_avg = float(np.mean(roll_ms))
    span_avg = float(np.mean(spans)) if spans else None
    launch_ms = span_avg if span_avg else roll_avg
    achieved = alg / (launch_ms * 1e-3) / 1e9
    # the same bytes over the step time: the device-level rate with the
    # --streams launches in flight (a launch's span overlaps the others')
    achieved_device = alg / (dt / args.steps) / 1e9
    _, pmc_label = pmc_record()
    traffic = load_traffic(steps_exec)
    out = {
        "metric": "grasp candidates evaluated/sec at 200-step horizon, Robotiq2F85xYCB",
        "value": N * world * args.steps / dt,
        "unit": "candidates/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded antipodal candidates on a 003_cracker_box stand-in; rank r uses seed r)",
        "config": {"workload": f"Robotiq2F85 x YCB 003_cracker_box, {N} candidates/GPU, collision mask + "
                               f"{args.horizon} close-lift-shake rollout ({horizon} steps, dt 1 ms)",
                   "candidates_per_gpu": N, "horizon_steps": horizon, "solver": env.model.options.get("solver"),
                   "parallelism": f"batch split x{world}", "streams": len(pipes),
                   "yield_every": int(args.yield_every)},
        "detail": {"collision_free": int(free.sum()), "stable": int(labels.sum()),
                   "rollouts_per_s": float(free.sum()) * world * args.steps / dt,
                   "host_enqueue_s": t_enq,
                   "warmup_steps_executed": nwarm,
                   "pipelines_identical": bool(same_pipes),
                   "static_layout_kernel": env.engine.static_layout(),
                   "rollout_grid": env.engine.rollout_grid(N),
                   "shard_check": shard_check,
                   "end_to_end_api": e2e,
                   "issue": issue_summary(),
                   "rotation": rotation,
                   "rollout_kernel_ms": roll_avg, "collision_kernel_ms": float(np.mean(coll_ms)),
                   "executed_candidate_steps": steps_exec,
                   "mean_ncon": float(stats[:, 4].sum() / max(1, steps_exec)),
                   "mean_nefc": float(stats[:, 5].sum() / max(1, steps_exec)),
                   "solver_iters_per_step": float(stats[:, 3].sum() / max(1, steps_exec)),
                   "overflow_candidates": merged[0][0] if wide is not None
                   else int((stats[:, 2] & abi.MGS["MGS_FLAG_CAPACITY"] != 0).sum()),
                   "diverged_candidates": int((stats[:, 2] & abi.MGS["MGS_FLAG_DIVERGED"] != 0).sum()),
                   "escalation": "per step on the device: overflow list + list re-run (grid %d) on a side stream, %s"
                   % (ESC_GRID, "resumed from the overflowing step" if RESUME else "from the start")
                   if wide is not None else None,
                   "still_capped_after_escalation": merged[0][1] if wide is not None else None},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic,
                     "traffic_source": pmc_label,
                     "kernel": "mgs_special_rollout" if env.engine.static_layout() else "mgs_rollout_kernel",
                     "algorithmic_bytes_per_launch": alg,
                     "launch_ms": launch_ms,
                     "launch_ms_device_span": span_avg,
                     "launch_spans_measured": len(spans), "launch_spans_overwritten": spans_lost,
                     "launch_ms_hip_events": roll_avg,
                     "launches_in_flight": len(pipes),
                     "achieved_device": achieved_device,
                     "frac_device": achieved_device / HBM_PEAK_GBS,
                     "valu": valu_roofline(steps_exec * args.steps / dt),
                     "what": "achieved = SURVEY 8(d) bytes of one main rollout launch (its executed "
                             "candidate-steps) / launch_ms, the timed main launches' mean execution span on "
                             "the device clock (mgs_queue_spans: first candidate taken -> last workgroup out, "
                             "the duration a kernel trace reports; HIP events on the stream, which also count "
                             "the wait for CUs held by the other pipelines' launches, beside it); "
                             "achieved_device = the same bytes / ms_per_step (launches overlap); the escalation "
                             "re-runs are mgs_special_rollout_esc in a trace"},
        "cpu_baseline": None,
    }
    if world == 1 and args.cpu_budget > 0:
        cb = cpu_baseline(env, poses, J, h, args.cpu_budget, args.cpu_threads)
        n = cb["n"]
        agree = bool(np.array_equal(cb["free"], free[:n]) and np.array_equal(cb["labels"], labels[:n]))
        # one thread (the reference is single-threaded MuJoCo): a smaller bounded sample
        c1 = cpu_baseline(env, poses, J, h, max(2.0, args.cpu_budget / 3), 1)
        agree1 = bool(np.array_equal(c1["free"], free[:c1["n"]]) and np.array_equal(c1["labels"], labels[:c1["n"]]))
        out["cpu_baseline"] = {"value": cb["value"], "unit": "candidates/s", "cores": args.cpu_threads,
                               "kind": "port", "host": host_info(),
                               "sample": f"first {n} of the {N} candidates x {cb['reps']} passes (mask + h200 "
                                         f"rollouts of the collision-free ones), oracle/ C restatement, OpenMP "
                                         f"{args.cpu_threads} threads (every CPU of the affinity mask within "
                                         f"the cgroup CPU quota), "
                                         f"{cb['seconds']:.1f} s",
                               "labels_identical_to_gpu": agree,
                               "one_thread": {"value": c1["value"], "unit": "candidates/s", "cores": 1,
                                              "sample": f"first {c1['n']} candidates x {c1['reps']} passes, "
                                                        f"{c1['seconds']:.1f} s",
                                              "labels_identical_to_gpu": agree1}}
    print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
