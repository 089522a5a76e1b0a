"""Secondary BASELINE.json configurations on one MI355X (bench.py keeps the
headline C2 line).  One JSON line per configuration:

  c3  Franka Panda over the (synthetic) YCB set, 16384 candidates per object
  c4  Allegro on a GSO-format object stand-in (GSO is not shipped), 32768 candidates
      (the whole 8-GPU job on one GPU; per-GPU share = 4096)
  c5  Shadow Hand on a settled 5-object clutter pile (tests/golden/
      clutter_scene_shadow.npz): collision mask + 3000-step close + 3000-step
      lift per candidate (the reference's grasp_stable_mask schedule)

Timing: wall clock of the env API calls (collision mask + stability rollout,
host buffers, PCIe included), and the kernels' own HIP-event durations.
Horizons: c3/c4 use h200 (bench.py's), c5 the reference's clutter schedule
(scaled down with --c5-steps for a bounded run).

    python tools/bench_configs.py [c3 c4 c5] [--c5-steps 600]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mj-grasp-sim_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import numpy as np  # noqa: E402

YIELD = None    # --yield: the envs' in-launch rotation (steps per slice; None = the env default)


def gravityless(gripper_name, object_ids, n, horizon="h200", cpu_sample=0, threads=16):
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping, HORIZONS
    from mgs.gripper.selector import get_gripper
    from mgs.obj.selector import get_object
    from mgs.sampler import antipodal
    from mgs.util.geo.transforms import SE3Pose
    h = HORIZONS[horizon]
    tot_n = tot_t = tot_k = 0.0
    per = []
    for oid in object_ids:
        g = get_gripper({"name": gripper_name})
        env = GravitylessObjectGrasping(g, get_object(oid))
        if YIELD is not None:
            env.YIELD_EVERY = YIELD
        if gripper_name == "PandaGripper":
            H, J, _ = antipodal.panda_candidates(env.obj, n, seed=0, gripper=g)
        else:
            H, J, _ = antipodal.hand_candidates(env.obj, n, g, seed=0)
        P = SE3Pose.from_mat(H)
        env.grasp_collision_mask(P[:64], J[:64])          # warm up (model upload, code objects)
        t0 = time.perf_counter()
        mask = env.grasp_collision_mask(P, J)
        km = env.engine.last_collision_ms()
        idx = np.nonzero(mask)[0]
        res = env.grasp_stability_evaluation_from_joints(P[idx], J[idx], nstep_lift=h["nstep_lift"],
                                                         shake_steps=h["shake_steps"],
                                                         close_steps=h["close_steps"],
                                                         lift_check_every=h["lift_check_every"],
                                                         return_details=True) if len(idx) else None
        dt = time.perf_counter() - t0
        kr = res["kernel_ms"] if res is not None else 0.0
        per.append(dict(object=oid, candidates=n, collision_free=int(mask.sum()),
                        stable=int(res["label"].sum()) if res is not None else 0, seconds=dt,
                        kernel_ms=km + kr, static_layout_kernel=bool(env.engine.specialized())))
        if cpu_sample:
            per[-1]["cpu"] = gravityless_cpu(env, P, J, cpu_sample, h, threads)
        tot_n += n
        tot_t += dt
        tot_k += (km + kr) * 1e-3
    out = dict(value=tot_n / tot_t, kernel_only=tot_n / tot_k, objects=per)
    if cpu_sample:
        cs = sum(o["cpu"]["candidates"] for o in per)
        ct = sum(o["cpu"]["seconds"] for o in per)
        out["cpu_baseline"] = dict(value=cs / ct, unit="grasp candidates/s", cores=threads, kind="port",
                                   seconds=ct, sample=f"{cpu_sample} evenly spaced candidates per object "
                                   f"({len(per)} objects): mask + the collision-free rollouts at {horizon}, the "
                                   "C oracle (checker build) on the host cores, same run")
        for o in per:
            o.pop("cpu")
    return out


def gravityless_cpu(env, P, J, sample, h, threads):
    """the C oracle over a bounded evenly spaced sample of the same candidates:
    the collision mask, then the h-horizon rollouts of the collision-free ones
    at the env's main capacity (the oracle flags what the GPU escalates)"""
    from oracle import oracle as O
    sel = np.linspace(0, len(P) - 1, sample).astype(int)
    Ps, Js = P[sel], J[sel]
    om = O.OracleModel(env.model, ncon_max=64, nefc_max=256)
    t0 = time.perf_counter()
    q, mp, mq, _ = env.initial_state(Ps, Js)
    free = om.collision_free(q, mp, mq, nthreads=threads)
    idx = np.nonzero(free)[0]
    if len(idx):
        om.rollout(env.rollout_plan(Ps[idx], Js[idx], nstep_lift=h["nstep_lift"], shake_steps=h["shake_steps"],
                                    close_steps=h["close_steps"], lift_check_every=h["lift_check_every"]),
                   nthreads=threads)
    return dict(candidates=int(sample), seconds=time.perf_counter() - t0)


def clutter(n_per_obj, steps, cpu_sample=0, threads=16):
    from make_clutter_scene import make_env
    from mgs.sampler.antipodal import hand_candidates
    from mgs.util.geo.transforms import SE3Pose
    z = np.load(os.path.join(ROOT, "tests", "golden", "clutter_scene_shadow.npz"))
    env = make_env("ShadowHand")
    if YIELD is not None:
        env.YIELD_EVERY = YIELD
    env.set_state(z["state"])
    H, J = [], []
    for k, o in enumerate(env.objects):
        h, j, _ = hand_candidates(o, n_per_obj, env.gripper, seed=k)
        H.append((env.get_obj_pose(o.name) @ SE3Pose.from_mat(h)).to_mat())
        J.append(j)
    P = SE3Pose.from_mat(np.concatenate(H).astype(np.float32))
    J = np.concatenate(J)
    st = env.get_state()
    env.grasp_collision_mask(P[:8], J[:8])
    t0 = time.perf_counter()
    mask = env.grasp_collision_mask(P, J)
    idx = np.nonzero(mask)[0]
    res = env.grasp_stable_mask(P[idx], J[idx], st, nstep_lift=steps, close_steps=steps, return_details=True)
    dt = time.perf_counter() - t0
    eng = env.engine_for_state(st)
    out = dict(value=len(P) / dt, candidates=len(P), collision_free=int(mask.sum()),
               stable=int(res["label"].sum()), seconds=dt, rollout_kernel_ms=res["kernel_ms"],
               overflow_rerun=int((res["stats"][:, 2] != 0).sum()), steps_per_phase=steps,
               nv=int(env.model.nv), nefc_max=int(eng.desc.nefc_max), library=os.path.basename(eng.lib._name),
               static_layout_kernel=bool(eng.specialized()),
               mean_ncon=float(res["stats"][:, 4].sum() / max(1, (2 * steps) * len(idx))))
    if cpu_sample:
        out["cpu_baseline"] = clutter_cpu(env, st, P, J, cpu_sample, steps, threads)
    return out


def clutter_cpu(env, st, P, J, sample, steps, threads):
    """the C oracle on the host cores over a bounded sample of the same job: the
    collision mask of `sample` evenly spaced candidates, then the close + lift
    rollouts of the collision-free ones; candidates/s = sample / time"""
    from oracle import oracle as O
    sel = np.linspace(0, len(P) - 1, sample).astype(int)
    Ps, Js = P[sel], J[sel]
    eng = env.engine_for_state(st)
    om = O.OracleModel(env.model_for(st), ncon_max=env.ncon_max, nefc_max=eng.desc.nefc_max)
    t0 = time.perf_counter()
    free = np.zeros(sample, bool)
    inb = np.nonzero(env.in_bounds(Ps))[0]
    q, mp, mq = env._initial_qpos(Ps[inb], Js[inb], st)
    free[inb] = om.collision_free(q, mp, mq, predicate="partition_incl", nthreads=threads)
    idx = np.nonzero(free)[0]
    if len(idx):
        om.rollout(env.stable_plan(Ps[idx], Js[idx], st, nstep_lift=steps, close_steps=steps), nthreads=threads)
    dc = time.perf_counter() - t0
    return dict(value=sample / dc, unit="grasp candidates/s", cores=threads, kind="port", seconds=dc,
                sample=f"{sample} of the candidates (evenly spaced): mask + {len(idx)} collision-free "
                       f"rollouts of {steps}+{steps} steps")


def scenes(n=256, steps_each=900, steps_final=9000, cpu_states=16, cpu_steps=200, ncon=None):
    """gen_clutter (clutter_table.py:197-222) + is_stable (:160-195) for n Robotiq
    piles of 5 fast-subset objects at once (mgs_simulate, one wave per pile), at
    the reference's 5 x 900 + 9000 steps.  CPU: the oracle on 16 host threads,
    cpu_states of the settled piles advanced cpu_steps free steps."""
    from mgs.env.clutter_table import ClutterTableEnv
    from mgs.gripper.selector import get_gripper
    from mgs.obj.selector import get_objects
    from mgs.util.geo.transforms import SE3Pose
    from oracle import oracle as O
    grip = get_gripper({"name": "Robotiq2f85Gripper"},
                       default_pose=SE3Pose(np.array([5.0, 5.0, 1.0]), np.array([1.0, 0, 0, 0]), "wxyz"))
    objs = get_objects({"name": "Fast_Data_Subset", "num_objects": 5}, 0)
    env = ClutterTableEnv(grip, objs, scene_randomization=False)
    env.gen_clutter_states(4, np.random.default_rng(1), steps_each=10, steps_final=10)     # warm-up
    t0 = time.perf_counter()
    st = env.gen_clutter_states(n, np.random.default_rng(0), steps_each, steps_final, ncon_max=ncon)
    t1 = time.perf_counter()
    ok, mx, _ = env.is_stable_states(st)
    t2 = time.perf_counter()
    steps = len(objs) * steps_each + steps_final
    plan, vs = env.free_plan(st[:cpu_states], cpu_steps)
    eng = env.engine_for_state(st[0])
    om = O.OracleModel(env.model_for(st[0]), ncon_max=env.ncon_max, nefc_max=eng.desc.nefc_max)
    t3 = time.perf_counter()
    om.simulate_batch(plan, vstate=vs, nthreads=16)
    dc = time.perf_counter() - t3
    return dict(value=n / (t2 - t0), unit="settled + checked piles/s", piles=n, stable=int(ok.sum()),
                gen_clutter_s=t1 - t0, is_stable_s=t2 - t1, pile_steps_per_s=n * (steps + 1000) / (t2 - t0),
                nv=int(env.model.nv), overflow_after_escalation=int(env.last_overflow),
                start_capacity=ncon or env.ncon_max,
                cpu_baseline=dict(value=cpu_states * cpu_steps / dc, unit="pile-steps/s", cores=16, kind="port",
                                  sample=f"{cpu_states} settled piles x {cpu_steps} free steps"))


def sampler(n=8192, subdiv=5):
    """Antipodal candidate ray casting on a 20480-face icosphere (a YCB-scale
    mesh): device kernel vs the C restatement on 16 host threads."""
    import tempfile
    from make_synthetic_ycb_mesh import icosphere_obj
    from mgs.core.engine import antipodal_contacts
    from mgs.sampler.antipodal import AntipodalGraspGenerator
    from oracle import oracle as O
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "sphere.obj")
        with open(path, "w") as f:
            f.write(icosphere_obj(0.04, subdiv))
        g = AntipodalGraspGenerator(path, rng=np.random.default_rng(0))
        g.normalize_load()
        r = g.draw(n)
    antipodal_contacts(r["tri"], r["points"][:256], r["dirs"][:256], r["u"][:256], 1e-5)   # warm-up
    t0 = time.perf_counter()
    sg, cg, ms = antipodal_contacts(r["tri"], r["points"], r["dirs"], r["u"], 1e-5)
    dt = time.perf_counter() - t0
    t1 = time.perf_counter()
    so, co = O.antipodal_contacts(r["tri"], r["points"], r["dirs"], r["u"], 1e-5, nthreads=16)
    dc = time.perf_counter() - t1
    tests = 2 * 2 * n * len(r["tri"])          # two rays, two sweeps
    return dict(value=n / (ms * 1e-3), unit="candidate points/s (kernel)", points=n, triangles=len(r["tri"]),
                kernel_ms=ms, wall_ms=dt * 1e3, ray_triangle_tests_per_s=tests / (ms * 1e-3),
                cpu_baseline=dict(value=n / dc, cores=16, kind="port", seconds=dc),
                bit_exact=bool(np.array_equal(sg, so) and np.array_equal(cg, co)))


def contact(n=10000, cpu_n=256):
    """the contact-based Shadow Hand sampler (mgs.sampler.contact): n grasps on
    one object; GPU stages timed by HIP events, the wall clock of
    generate_grasps, and the C oracle's fit on a cpu_n sample (16 threads)"""
    import copy
    from mgs.obj.selector import get_object
    from mgs.sampler import contact as C
    from mgs.sampler.kin.model import ShadowKinematicsModel
    from oracle import oracle as O
    kin = ShadowKinematicsModel()
    obj = get_object("005_tomato_soup_can")
    C.ContactBasedDiff(obj, rng=np.random.default_rng(9)).generate_grasps(64, kin)     # warm-up
    s = C.ContactBasedDiff(obj, rng=np.random.default_rng(0))
    t0 = time.perf_counter()
    H, aux = s.generate_grasps(n, kin)
    dt = time.perf_counter() - t0
    inp, desc = C.ContactBasedDiff(obj, rng=np.random.default_rng(0)).prepare(n, kin)
    t1 = time.perf_counter()
    O.contact_optimize(desc, inp["rot_init"][:cpu_n], inp["pos_init"][:cpu_n], inp["targets"][:cpu_n],
                       inp["normals"][:cpu_n], nthreads=16)
    cpu = (time.perf_counter() - t1) / cpu_n
    km = s.last["kernel_ms"]
    return dict(value=n / dt, unit="grasps/s", grasps=n, seconds=dt, kernel_ms=km,
                fit_grasps_per_s_gpu=n / (km["optimize"] * 1e-3),
                fit_grasps_per_s_cpu_oracle_16t=1.0 / cpu, median_final_loss=float(np.median(s.last["loss"])),
                iterations=desc.iters)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["c3", "c4", "c5", "sampler"])
    ap.add_argument("--c5-steps", type=int, default=600)
    ap.add_argument("--c5-per-object", type=int, default=256)
    ap.add_argument("--c5-cpu-sample", type=int, default=0, help="candidates for the C5 CPU baseline (0: none)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--cpu-sample", type=int, default=1024,
                    help="candidates per object for the C3 / C4 CPU baselines (0: none)")
    ap.add_argument("--yield", dest="yield_every", type=int, default=None,
                    help="in-launch rotation of the envs' rollout launches, steps per slice (0 = off)")
    ap.add_argument("--scene-piles", type=int, default=256)
    ap.add_argument("--scene-ncon", type=int, default=None)
    a = ap.parse_args()
    global YIELD
    YIELD = a.yield_every
    os.environ.setdefault("MGS_SPECIALIZE", "1")
    import torch
    torch.cuda.init()
    from mgs.obj.ycb import ObjectYCB
    ycb = ObjectYCB.all_object_ids()
    for c in a.configs:
        if c == "c3":
            r = gravityless("PandaGripper", ycb, 16384, cpu_sample=a.cpu_sample, threads=a.cpu_threads)
            out = dict(config="c3", workload=f"Franka Panda x {len(ycb)} synthetic YCB stand-ins (the YCB set is not "
                                             "shipped: 5 stand-in objects, not the full set), 16384 candidates/object,"
                                             " mask + h200 rollout, 1 GPU", unit="candidates/s", **r)
        elif c == "c4":
            r = gravityless("AllegroGripper", ["Synthetic_Mug_Body"], 32768, cpu_sample=a.cpu_sample,
                            threads=a.cpu_threads)
            out = dict(config="c4", workload="Allegro x GSO-format stand-in (Synthetic_Mug_Body), 32768 candidates, "
                                             "measured on 1 GPU (BASELINE names 8 GPUs: the whole 8-GPU job on one; "
                                             "per-GPU share 4096), mask + h200 rollout", unit="candidates/s", **r)
        elif c == "c5":
            r = clutter(a.c5_per_object, a.c5_steps, a.c5_cpu_sample, a.cpu_threads)
            out = dict(config="c5", workload=f"Shadow Hand x settled 5-object pile, {r['candidates']} candidates, "
                                             f"mask + close {a.c5_steps} + lift {a.c5_steps} (reference: 3000 + 3000)",
                       unit="candidates/s", **r)
        elif c == "scenes":
            out = dict(config="scenes", workload=f"gen_clutter + is_stable, {a.scene_piles} Robotiq piles of 5 "
                                                 "fast-subset objects, 5 x 900 + 9000 + 1000 steps",
                       **scenes(a.scene_piles, ncon=a.scene_ncon))
        elif c == "contact":
            out = dict(config="contact", workload="contact-based Shadow Hand sampler (FPS seeds, local targets, "
                                                  "150 AdamW steps), 10000 grasps on 005_tomato_soup_can", **contact())
        elif c == "sampler":
            out = dict(config="sampler", workload="antipodal ray casting, 8192 points x 20480-face icosphere",
                       **sampler())
        else:
            raise SystemExit(f"unknown config {c}")
        out["yield_every"] = "env default" if YIELD is None else YIELD
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
