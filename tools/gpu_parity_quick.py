"""Quick GPU-vs-oracle parity probe (dev tool; the pytest suite is tests/)."""
import sys, time, os, json
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..', 'mj-grasp-sim_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), '..'))
from oracle import oracle as O
from mgs.core import engine as E
from mgs.gripper.robotiq2f85 import GripperRobotiq2f85
from mgs.obj.selector import get_object
from mgs.util.geo.transforms import SE3Pose
from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping, HORIZONS
from mgs.sampler.antipodal import robotiq_candidates

rng = np.random.default_rng(1)
x = np.concatenate([rng.uniform(-20, 20, 20000), rng.uniform(-1e-3, 1e-3, 1000)])
y = rng.uniform(0.1, 10, len(x))
g = E.arith_probe(x, y)
s, c = O.sincos(x)
print('arith: sqrt exact', np.array_equal(g[:, 0], np.sqrt(np.abs(x))), 'div exact', np.array_equal(g[:, 1], x / y),
      'sin exact', np.array_equal(g[:, 2], s), 'cos exact', np.array_equal(g[:, 3], c), flush=True)

tree_ok = True
for n in [1, 2, 3, 5, 8, 9, 16, 17, 20, 31, 32, 33, 50, 64]:
    a = rng.standard_normal((16, 64)); cc = rng.standard_normal((16, 64))
    dev = E.tree_probe(a, cc, n)
    ref = np.array([O.tree_dot(a[i], cc[i], n) for i in range(16)])
    tree_ok &= bool(np.array_equal(dev, ref))
print('tree probe exact', tree_ok, flush=True)
grip = GripperRobotiq2f85(SE3Pose(np.zeros(3), np.array([1, 0, 0, 0]), 'wxyz'))
obj = get_object('003_cracker_box')
env = GravitylessObjectGrasping(grip, obj)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 64
H, J, W = robotiq_candidates(obj, N, seed=0)
poses = SE3Pose.from_mat(H)
q, mp, mq, _ = env.initial_state(poses, J)
om = O.OracleModel(env.model)
t = time.time(); free_o = om.collision_free(q, mp, mq, nthreads=8); to = time.time() - t
t = time.time(); free_g = env.engine.collision_free(q, mp, mq); tg = time.time() - t
print('mask equal', np.array_equal(free_o, free_g), free_g.sum(), '/', N, 'oracle %.3fs gpu %.3fs' % (to, tg), flush=True)
h = HORIZONS['h200']
idx = np.nonzero(free_o)[0]
plan = env.rollout_plan(poses[idx], J[idx], nstep_lift=h['nstep_lift'], shake_steps=h['shake_steps'],
                        close_steps=h['close_steps'], lift_check_every=h['lift_check_every'])
import copy
for solver in ['Newton', 'PGS']:
    cm2 = copy.copy(env.model); cm2.options = dict(env.model.options); cm2.options['solver'] = solver
    om2 = O.OracleModel(cm2); eng = E.Engine(cm2)
    t = time.time(); ro = om2.rollout(plan, nthreads=16); to = time.time() - t
    t = time.time(); rg = eng.rollout(plan); tg = time.time() - t
    print(solver, 'rollout labels equal', np.array_equal(ro['label'], rg['label']), 'fail equal', np.array_equal(ro['fail_step'], rg['fail_step']),
          'objq bit-equal', np.array_equal(ro['obj_qpos'], rg['obj_qpos']), 'max|dq|', np.abs(ro['obj_qpos'] - rg['obj_qpos']).max(),
          'stats equal', np.array_equal(ro['stats'], rg['stats']))
    print('  labels', rg['label'].sum(), '/', len(idx), 'oracle %.3fs gpu %.3fs kernel %.2f ms' % (to, tg, rg['kernel_ms']))
    bad = np.nonzero((ro['stats'] != rg['stats']).any(1) | (ro['obj_qpos'] != rg['obj_qpos']).any(1))[0]
    print('  mismatching candidates', bad[:10].tolist(), 'of', len(bad), flush=True)
    if len(bad):
        print('  stats gpu', rg['stats'][bad[:4]].tolist(), 'oracle', ro['stats'][bad[:4]].tolist())

if len(sys.argv) > 2:
    import copy
    NB = int(sys.argv[2])
    H, J, W = robotiq_candidates(obj, NB, seed=1)
    poses = SE3Pose.from_mat(H)
    plan = env.rollout_plan(poses, J, nstep_lift=h['nstep_lift'], shake_steps=h['shake_steps'],
                            close_steps=h['close_steps'], lift_check_every=h['lift_check_every'])
    print('lds bytes', env.engine.lds_bytes())
    for rep in range(2):
        rg = env.engine.rollout(plan)
        print('N=%d kernel %.1f ms  -> %.0f cand/s ; labels %d; mean iters/step %.1f maxcon %d maxefc %d overflow %d' % (
            NB, rg['kernel_ms'], NB / rg['kernel_ms'] * 1e3, rg['label'].sum(), rg['stats'][:, 3].sum() / 200.0 / NB,
            rg['stats'][:, 0].max(), rg['stats'][:, 1].max(), (rg['stats'][:, 2] != 0).sum()), flush=True)
    cm2 = copy.copy(env.model); cm2.options = dict(env.model.options); cm2.options['solver'] = 'PGS'
    e2 = E.Engine(cm2)
    rg = e2.rollout(plan)
    print('PGS: kernel %.1f ms -> %.0f cand/s' % (rg['kernel_ms'], NB / rg['kernel_ms'] * 1e3), flush=True)
