"""Diagnostic: per-stage s_memtime breakdown of the rollout kernel (MGS_PROFILE build)."""
import sys, os, ctypes
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'mj-grasp-sim_amd'))
import mgs.core.engine as E

NAMES = ['loop/ctrl/checks', 'kinematics', 'com_pos', 'coll: certificate checks', 'coll: MPR', 'coll: feature+clip',
         'crb', 'ldl(M)', 'act+passive+rne+smooth', 'con: J rows', 'con: G transform', 'con: params+blocks',
         'newton: setup', 'newton: hessian', 'newton: ldl+solve+jv', 'newton: linesearch', 'newton: eval+grad',
         'noslip', 'finalize', 'int: crb', 'int: qDeriv+M', 'int: ldl+solve+qpos', 'coll: small-hull support calls',
         'newton: H accumulate', 'newton: H to rows', 'newton: H factor',
         'con: equality rows', 'con: limit/friction rows', 'actuation', 'passive', 'rne',
         'coll: big-hull support calls', 'coll: feature passes', 'coll: select4+add / multiccd',
         'noslip/pgs block: residual', 'noslip/pgs block: qcqp', 'noslip/pgs block: update',
         'coll: sort+dedup', 'coll: hull chains', 'coll: clip+depth filter', 'coll: broadphase AABB',
         'coll: broadphase OBB']


def report(buf, r, ncand, horizon):
    v = np.concatenate([np.array(buf[:26], dtype=np.float64), np.array(buf[31:36], dtype=np.float64),
                        np.array(buf[39:45], dtype=np.float64),
                        np.array(buf[47:50], dtype=np.float64), np.array(buf[59:61], dtype=np.float64)])
    cnt = np.array(buf[26:31], dtype=np.float64)
    tot = v.sum()
    print('N=%d candidates, kernel %.1f ms, labels %d, overflow %d' % (
        ncand, r['kernel_ms'], r['label'].sum(), (r['stats'][:, 2] != 0).sum()))
    for n_, x in zip(NAMES, v):
        print('%-28s %6.1f%%  %.3g ticks' % (n_, 100 * x / tot, x))
    steps = ncand * horizon
    print('ticks per candidate-step: %.0f' % (tot / steps))
    print('per candidate-step: narrowphase pairs %.2f, hits %.2f, support calls %.2f, big-hull scans %.2f, '
          'big-hull pairs %.2f' % tuple(cnt / steps))
    c2 = np.array(buf[36:39], dtype=np.float64) / steps
    c3 = np.array(buf[45:47], dtype=np.float64) / steps
    print('per candidate-step: ls_eval calls %.2f, newton_eval calls %.2f, noslip sweeps %.2f, '
          'qcqp iterations %.2f, block updates %.2f' % (*c2, *c3))
    c4 = np.array(buf[51:59], dtype=np.float64)
    print('per candidate-step: pairs skipped by a separation certificate %.2f' % (c4[7] / steps))
    if buf[62]:
        print('clock held in the kernel: %.2f GHz (shader-clock / 100 MHz real-time spans, summed over '
              'workgroups)' % (0.1 * buf[61] / buf[62]))
    if c4[3] + c4[4] > 0:
        print('narrowphase MPR (incl. supports): missed pairs %.1f%% of ticks (%.2f support calls per step), '
              'hit pairs %.1f%% (%.2f support calls per step)' % (100 * c4[3] / tot, c4[5] / steps,
                                                                  100 * c4[4] / tot, c4[6] / steps))


def main():
    """stage timers of the headline engine's specialised kernels: the profile
    build of its code object (-DMGS_PROFILE, compiled if not cached) attached
    in place of the product one"""
    from mgs.core import special
    from mgs.gripper.robotiq2f85 import GripperRobotiq2f85
    from mgs.obj.selector import get_object
    from mgs.util.geo.transforms import SE3Pose
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping, HORIZONS
    from mgs.sampler.antipodal import robotiq_candidates
    grip = GripperRobotiq2f85(SE3Pose(np.zeros(3), np.array([1, 0, 0, 0]), 'wxyz'))
    obj = get_object('003_cracker_box')
    env = GravitylessObjectGrasping(grip, obj)
    if "--compile-only" in sys.argv:
        # the profile object of the headline engine, built here (no device needed)
        from mgs.core import abi
        from mgs.core.engine import library_for
        fields, _, _ = env.model.pack(ncon_max=env.ncon_max, nefc_max=env.nefc_max)
        lib = library_for(env.model.nv, int(fields["nefc_max"]))
        if "--lds-rows" not in sys.argv and lib.mgs_rows_per_lane() != 4:
            fields["g_rows_hbm"] = 1      # as env.engine (Engine(g_rows_hbm="auto")) runs it
        print(special.code_object(lib, abi.make_desc(fields), profile=True))
        return
    N = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 64
    heavy = "--heavy" in sys.argv
    # --heavy: the N candidates with the most constraint rows over their rollout
    # among the collision-free ones of the headline's 8192-candidate batch (the
    # critical path of a single launch, tools/probes/critical_path_probe.py)
    H, J, W = robotiq_candidates(obj, 8192 if heavy else 4 * N, seed=0 if heavy else 2)
    poses = SE3Pose.from_mat(H)
    q, mp, mq, _ = env.initial_state(poses, J)
    eng = env.engine
    free = eng.collision_free(q, mp, mq)
    idx = np.nonzero(free)[0]
    h = HORIZONS['h200']

    def plan_of(sel):
        return env.rollout_plan(poses[sel], J[sel], nstep_lift=h['nstep_lift'], shake_steps=h['shake_steps'],
                                close_steps=h['close_steps'], lift_check_every=h['lift_check_every'])
    if heavy:
        st = eng.rollout(plan_of(idx))["stats"]
        idx = idx[np.argsort(-st[:, 5], kind="stable")[:N]]
    else:
        idx = idx[:N]
    plan = plan_of(idx)
    path = special.code_object(eng.lib, eng.desc, profile=True)
    eng._ck(eng.lib.mgs_model_attach_special(eng._model, path.encode()), 'mgs_model_attach_special')
    L = eng.lib
    L.mgs_model_prof_read.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_ulonglong)]
    buf = (ctypes.c_ulonglong * 64)()
    L.mgs_model_prof_read(eng._model, buf)
    r = eng.rollout(plan)
    eng._ck(L.mgs_model_prof_read(eng._model, buf), 'mgs_model_prof_read')
    report(buf, r, len(idx), 200)


if __name__ == "__main__":
    main()
