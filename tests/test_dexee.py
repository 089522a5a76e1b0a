"""DEXEE hand x YCB (reference mgs/gripper/dexee.py:32-476).

The DEXEE is the reference's one gripper with condim-6 contacts (torsional and
rolling friction on the fingertip pads, dexee.py:41-43), mujoco.pid plugin
actuators with actuator state (dexee.py:84-121,383-407) and gravcomp
(dexee.py:125-179), closed by 500 steps at the yaml's qpos_close
(dexee.py:450-456).  MuJoCo's pid plugin and its general QCQP are not in the
reference or this image: their restatement (oracle pid_force / qcqpn,
DESIGN.md §2) is parity unpinned -- these tests pin the restated semantics by
hand and the GPU to the oracle bit for bit.

CPU: model structure; the pid semantics on a one-joint model against a
by-hand step loop; the free-space close settles on qpos_close; oracle
rollouts grasp.  GPU: mask, rollout (h200 and the reference's 500-step
close) and the free simulation's act state bit-exact against the oracle
through the C-ABI (the model's code object is built with -DMGS_MAXDIM=6)."""
import numpy as np
import pytest

CLOSE = np.array([0, -0.0325, 0, 0.00143, 0.0655, -0.0369, 0, 0, -0.0654, -0.0337, 0, 0])


@pytest.fixture(scope="module")
def denv():
    from mgs.core.shipped import DEXEE_OBJECT
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
    from mgs.gripper.selector import get_gripper
    from mgs.obj.selector import get_object
    return GravitylessObjectGrasping(get_gripper({"name": "DexeeGripper"}), get_object(DEXEE_OBJECT))


@pytest.fixture(scope="module")
def dcand(denv):
    from mgs.sampler.antipodal import hand_candidates
    from mgs.util.geo.transforms import SE3Pose
    H, J, _ = hand_candidates(denv.obj, 256, denv.gripper, seed=0)
    return SE3Pose.from_mat(H), J


@pytest.fixture(scope="module")
def dom(denv):
    from oracle import oracle as O
    return O.OracleModel(denv.model, ncon_max=denv.ncon_max, nefc_max=denv.nefc_max)


def test_dexee_model(denv):
    cm = denv.model
    assert (cm.nv, cm.nu, cm.nact) == (24, 12, 24)          # gripper free joint + 12 finger joints + object
    # the hand base's two collision geoms have MuJoCo's defaults (condim 3)
    assert set(np.unique(cm.pair_condim)) == {3, 4, 6}
    assert list(cm.actuator_actadr) == list(range(0, 24, 2))
    fields, _, _ = cm.pack(ncon_max=denv.ncon_max)
    assert fields["maxcondim"] == 6 and fields["nact"] == 24
    # J0's gains (dexee.py:86-92), imax / slewmax set
    assert np.allclose(cm.actuator_pidprm[0], [2.8, 4.0, 0.03, 0.1, 3.14159])
    assert denv.gripper.close_steps == 500
    assert np.array_equal(denv.gripper.close_ctrl(None), CLOSE)


def test_dexee_collision_geom_classes(denv):
    """every DEXEE collision geom's condim / friction / solref / priority as the
    template's default classes give them (dexee.py:39-47): finger/collision_hard
    on the finger links (dexee.py:154-186), finger/collision_soft on the
    fingertip pads (:187), and no class -- MuJoCo's geom defaults -- on the hand
    base's two geoms (:132,135-136)"""
    cm = denv.model
    hard = (4, [1.0, 0.001, 2e-05], [-7000.0, -167.0])
    soft = (6, [1.0, 0.005, 0.0001], [-2500.0, -100.0])
    default = (3, [1.0, 0.005, 0.0001], [0.02, 1.0])
    want = {"hand_base_geom_col": default, "hand_base_puck_geom_col": default}
    for f in ("F0", "F1", "F2"):
        for link in ("base", "knuckle", "proximal", "middle", "distal"):
            want[f"{f}/{link}_geom_col"] = hard
        want[f"{f}/distal_geom_tip_col"] = soft
    names = list(cm.geom_names)
    for name, (condim, fr, sr) in want.items():
        g = names.index(name)
        assert cm.geom_condim[g] == condim, name
        assert np.array_equal(cm.geom_friction[g], fr), name
        assert np.array_equal(cm.geom_solref[g], sr), name
        assert cm.geom_priority[g] == 0, name
    # the gripper's collision geoms are exactly these (the object and the ground follow)
    assert sum(n in want for n in names) == len(want) == 20


PID_XML = """
<mujoco><option gravity="0 0 0" cone="elliptic" integrator="implicitfast" timestep="0.002"/>
<extension><plugin plugin="mujoco.pid"><instance name="p">
  <config key="kp" value="2.8"/><config key="ki" value="4.0"/><config key="kd" value="0.03"/>
  <config key="imax" value="0.1"/><config key="slewmax" value="3.14159"/>
</instance></plugin></extension>
<worldbody><body name="b"><joint name="j" axis="0 0 1"/>
  <geom type="box" size="0.1 0.02 0.02" mass="1" contype="0" conaffinity="0"/></body></worldbody>
<actuator><plugin plugin="mujoco.pid" instance="p" joint="j" ctrlrange="-1 1" forcerange="-0.9 0.53" actdim="2"/>
</actuator></mujoco>"""


def _pid_by_hand(ctrl, nsteps, dt=0.002, inertia=(0.1 ** 2 + 0.02 ** 2) / 3.0):
    """mujoco.pid on one free hinge (box about its z axis), step by step:
    setpoint slew-limited from the previous one, force kp e + kd (setpoint rate
    - v) + ki integral clamped to forcerange, integral clamped to imax / ki"""
    kp, ki, kd, imax, slew = 2.8, 4.0, 0.03, 0.1, 3.14159
    q = v = prev = integ = 0.0
    out = []
    for _ in range(nsteps):
        c = min(max(ctrl, -1.0), 1.0)
        c = min(max(c, prev - slew * dt), prev + slew * dt)
        cdot = (c - prev) / dt
        err = c - q
        f = kp * err + kd * (cdot - v) + ki * integ
        f = min(max(f, -0.9), 0.53)
        v = v + dt * (f / inertia)
        q = q + dt * v
        prev = prev + dt * cdot
        integ = min(max(integ + dt * err, -imax / ki), imax / ki)
        out.append((q, v, prev, integ))
    return np.array(out)


@pytest.mark.parametrize("ctrl,nsteps", [(0.8, 40), (0.8, 400), (-2.0, 300)])
def test_pid_semantics_by_hand(ctrl, nsteps):
    """the restated plugin (oracle pid_force + the act advance) against the
    by-hand step loop: slew-limited setpoint (act 0), integral with its imax
    clamp (act 1), force clamp; 1e-9 (the model's inertia and the implicit
    solve round differently from the closed form)"""
    from types import SimpleNamespace
    from mgs.core.mjcf import compile_xml
    from oracle import oracle as O
    cm = compile_xml(PID_XML)
    assert (cm.nu, cm.nact) == (1, 2)
    om = O.OracleModel(cm)
    z = np.zeros((1, 1, 3))
    plan = SimpleNamespace(nsteps=[nsteps], check_every=[0], check_at_end=[0], ctrl=[np.array([ctrl])],
                           obj_qposadr=-1, check_offset=None, qpos_init=cm.qpos0.reshape(1, -1),
                           mocap_quat=np.array([[1.0, 0, 0, 0]]), phase_start=z, phase_target=z)
    r = om.simulate_batch(plan)
    want = _pid_by_hand(ctrl, nsteps)[-1]
    got = np.array([r["qpos"][0, 0], r["qvel"][0, 0], r["act"][0, 0], r["act"][0, 1]])
    assert np.allclose(got, want, rtol=1e-9, atol=1e-12), (got, want)


@pytest.mark.parametrize("gc", [1.0, 0.5])
def test_gravcomp_semantics(gc):
    """gravcomp (dexee.py:125-179 puts gravcomp="1" on every body; MuJoCo
    mj_gravcomp): gravcomp 1 cancels gravity -- a jointed free body under
    gravity stays at rest; gravcomp 0.5 on every body -- the whole system
    falls at g / 2 without the hinge turning (semi-implicit Euler: z_n = z_0 -
    a dt^2 n (n + 1) / 2)"""
    from types import SimpleNamespace
    from mgs.core.mjcf import compile_xml
    from mgs.core.shipped import GRAVCOMP_XML
    from oracle import oracle as O
    cm = compile_xml(GRAVCOMP_XML.format(gc=gc))
    om = O.OracleModel(cm)
    n, dt = 200, 0.002
    z = np.zeros((1, 1, 3))
    plan = SimpleNamespace(nsteps=[n], check_every=[0], check_at_end=[0], ctrl=[np.zeros(0)], obj_qposadr=-1,
                           check_offset=None, qpos_init=cm.qpos0.reshape(1, -1),
                           mocap_quat=np.array([[1.0, 0, 0, 0]]), phase_start=z, phase_target=z)
    r = om.simulate_batch(plan)
    a = (1.0 - gc) * 9.81
    assert abs(r["qpos"][0, 2] - (1.0 - a * dt * dt * n * (n + 1) / 2)) < 1e-9
    assert np.abs(r["qvel"][0, [0, 1, 3, 4, 5, 6]]).max() < 1e-9
    assert abs(r["qvel"][0, 2] + a * dt * n) < 1e-9


def test_dexee_free_close_settles(denv, dom):
    """free-space close (object out of reach): 500 steps at qpos_close; the
    slew-limited setpoints reach it after 0.44 s and the PID holds the fingers
    near it: the three fingertips meet (qpos_close closes them onto each
    other), so the contacts at rest are gripper-gripper only and J1 rests
    about 0.02 rad short"""
    from mgs.util.geo.transforms import SE3Pose
    pose = SE3Pose(np.array([[0.0, 0.0, 0.0]]), np.array([[1.0, 0, 0, 0]]), "wxyz")
    q, mp, mq, _ = denv.initial_state(pose, denv.gripper.open_joints()[None])
    oq = denv.model.nq - 7
    q[0, oq] = 2.0                      # object x: far from the hand
    tr, nc, qv = dom.trace(q[0], mp[0], mq[0], CLOSE, 500)
    idx = denv.get_joint_idxs(denv.gripper.get_actuator_joint_names())
    qf = tr[-1, idx]
    assert np.abs(qf - CLOSE).max() < 2.5e-2
    n, _, _, _, g = dom.contacts(tr[-1], mp[0], mq[0])
    assert n == nc[-1] > 0
    assert np.all(denv.model.geom_side[g[:n]] < 0)     # fingertip against fingertip, not the object


def test_dexee_oracle_grasps(denv, dcand, dom):
    from conftest import plan_for
    poses, J = dcand
    q, mp, mq, _ = denv.initial_state(poses, J)
    free = dom.collision_free(q, mp, mq, nthreads=8)
    idx = np.nonzero(free)[0][:24]
    assert len(idx) >= 16
    r = dom.rollout(plan_for(denv, poses[idx], J[idx]), nthreads=8)
    assert r["label"].sum() >= 4


@pytest.mark.gpu
def test_dexee_gpu_parity(denv, dcand, dom):
    """mask and h200 rollouts bit-exact (the env's engine: its specialised
    MGS_MAXDIM=6 code object), then the reference's 500-step close.  A
    grasp past the engine's contact capacity (20) runs on capped and flagged
    (capped_continue), which is the oracle's one semantics at a capacity --
    the envs' escalation continues such candidates wider"""
    from conftest import plan_for
    poses, J = dcand
    q, mp, mq, _ = denv.initial_state(poses, J)
    fg = denv.engine.collision_free(q, mp, mq)
    assert np.array_equal(fg, dom.collision_free(q, mp, mq, nthreads=8))
    idx = np.nonzero(fg)[0][:96]
    plan = plan_for(denv, poses[idx], J[idx])
    rg = denv.engine.rollout(plan, resumable=True, capped_continue=True)
    ro = dom.rollout(plan, nthreads=8)
    for k in ("label", "fail_step", "obj_qpos", "stats"):
        assert np.array_equal(rg[k], ro[k]), k
    assert denv.engine.specialized()
    assert ro["label"].sum() >= 8
    idx = idx[:24]
    plan = denv.rollout_plan(poses[idx], J[idx], nstep_lift=100, shake_steps=20, close_steps=500,
                             lift_check_every=50)
    rg = denv.engine.rollout(plan, resumable=True, capped_continue=True)
    ro = dom.rollout(plan, nthreads=8)
    for k in ("label", "fail_step", "obj_qpos", "stats"):
        assert np.array_equal(rg[k], ro[k]), k


@pytest.mark.gpu
def test_dexee_gpu_act_state(denv, dcand, dom):
    """free simulation from mid-close states: final qpos, qvel, warmstart and
    the 24 act entries (setpoints, integrals) bit-exact, also when continued
    from a given act state (vstate's act columns)"""
    from types import SimpleNamespace
    poses, J = dcand
    q, mp, mq, _ = denv.initial_state(poses[:16], J[:16])
    oq = denv.model.nq - 7
    q[:, oq] = 2.0
    mp3 = mp.reshape(16, 1, 3)
    plan = SimpleNamespace(nsteps=[120], check_every=[0], check_at_end=[0], ctrl=[CLOSE], obj_qposadr=-1,
                           check_offset=None, qpos_init=q, mocap_quat=mq, phase_start=mp3, phase_target=mp3)
    g = denv.engine.simulate(plan)
    o = dom.simulate_batch(plan)
    for k in ("qpos", "qvel", "qacc_warmstart", "act"):
        assert np.array_equal(g[k], o[k]), k
    assert np.abs(g["act"]).max() > 0
    vs = np.concatenate([g["qvel"], g["qacc_warmstart"], g["act"]], axis=1)
    plan.qpos_init = g["qpos"]
    g2, o2 = denv.engine.simulate(plan, vstate=vs), dom.simulate_batch(plan, vstate=vs)
    for k in ("qpos", "qvel", "qacc_warmstart", "act"):
        assert np.array_equal(g2[k], o2[k]), k


@pytest.mark.gpu
def test_gravcomp_gpu_parity():
    """gravity compensation on the device (passive(): the cinert moment arm,
    bodies in order) bit-exact against the oracle: the half-compensated
    jointed body of test_gravcomp_semantics, from a tilted, spinning start"""
    from types import SimpleNamespace
    from mgs.core.engine import Engine
    from mgs.core.mjcf import compile_xml
    from mgs.core.shipped import GRAVCOMP_XML
    from oracle import oracle as O
    cm = compile_xml(GRAVCOMP_XML.format(gc=0.5))
    eng, om = Engine(cm, ncon_max=4), O.OracleModel(cm, ncon_max=4)
    n = 8
    rng = np.random.default_rng(3)
    q = np.tile(cm.qpos0, (n, 1))
    q[:, 3:7] = rng.normal(size=(n, 4))
    q[:, 3:7] /= np.linalg.norm(q[:, 3:7], axis=1, keepdims=True)
    q[:, 7] = rng.uniform(-1, 1, n)
    vs = np.concatenate([rng.normal(size=(n, cm.nv)), np.zeros((n, cm.nv))], axis=1)
    z = np.zeros((n, 1, 3))
    plan = SimpleNamespace(nsteps=[300], check_every=[0], check_at_end=[0], ctrl=[np.zeros(0)], obj_qposadr=-1,
                           check_offset=None, qpos_init=q, mocap_quat=np.tile([1.0, 0, 0, 0], (n, 1)),
                           phase_start=z, phase_target=z)
    g, o = eng.simulate(plan, vstate=vs), om.simulate_batch(plan, vstate=vs)
    for k in ("qpos", "qvel", "qacc_warmstart"):
        assert np.array_equal(g[k], o[k]), k


PID_KPKD_XML = PID_XML.replace('<config key="ki" value="4.0"/>', '<config key="ki" value="0"/>') \
    .replace('<config key="imax" value="0.1"/><config key="slewmax" value="3.14159"/>', '') \
    .replace(' actdim="2"', ' actdim="0"')


def _pid_plan(cm, ctrl, nsteps, n=1, q=None, vs=None):
    from types import SimpleNamespace
    z = np.zeros((n, 1, 3))
    return SimpleNamespace(nsteps=[nsteps], check_every=[0], check_at_end=[0], ctrl=[np.array([ctrl])],
                           obj_qposadr=-1, check_offset=None,
                           qpos_init=np.tile(cm.qpos0, (n, 1)) if q is None else q,
                           mocap_quat=np.tile([1.0, 0, 0, 0], (n, 1)), phase_start=z, phase_target=z)


def test_pid_kp_kd_only_has_no_act_state():
    """a mujoco.pid actuator with ki = 0 and no slewmax has no act entries
    (nact 0) and is still a pid: force kp (ctrl - q) + kd (0 - v), clamped"""
    from mgs.core.mjcf import compile_xml
    from oracle import oracle as O
    cm = compile_xml(PID_KPKD_XML)
    assert (cm.nu, cm.nact) == (1, 0)
    fields, _, _ = cm.pack()
    assert fields["npid"] == 1 and fields["nact"] == 0
    r = O.OracleModel(cm).simulate_batch(_pid_plan(cm, 0.8, 200))
    # by hand: the same loop without slew / integral
    kp, kd, dt, inertia = 2.8, 0.03, 0.002, (0.1 ** 2 + 0.02 ** 2) / 3.0
    q = v = 0.0
    for _ in range(200):
        f = min(max(kp * (0.8 - q) + kd * (0.0 - v), -0.9), 0.53)
        v = v + dt * (f / inertia)
        q = q + dt * v
    assert np.allclose([r["qpos"][0, 0], r["qvel"][0, 0]], [q, v], rtol=1e-9, atol=1e-12)


def test_pid_negative_ki_clamps_by_magnitude():
    """|ki integral| <= imax also for ki < 0 (the clamp bound is imax / |ki|)"""
    from mgs.core.mjcf import compile_xml
    from oracle import oracle as O
    cm = compile_xml(PID_XML.replace('value="4.0"', 'value="-4.0"'))
    r = O.OracleModel(cm).simulate_batch(_pid_plan(cm, 0.8, 400))
    assert abs(r["act"][0, 1]) <= 0.1 / 4.0 + 1e-15
    assert r["act"][0, 1] > 0.0          # the error stays positive: the integral sits at +imax / |ki|


@pytest.mark.gpu
def test_pid_kp_kd_only_gpu_parity():
    """the kernel took the pid branch only for models with act
    state; a kp / kd-only pid (nact 0) now runs it on the device too (npid)"""
    from mgs.core.engine import Engine
    from mgs.core.mjcf import compile_xml
    from oracle import oracle as O
    cm = compile_xml(PID_KPKD_XML)
    eng, om = Engine(cm, ncon_max=4), O.OracleModel(cm, ncon_max=4)
    rng = np.random.default_rng(5)
    n = 8
    q = np.tile(cm.qpos0, (n, 1)) + rng.uniform(-0.5, 0.5, (n, cm.nq))
    plan = _pid_plan(cm, 0.8, 300, n=n, q=q)
    g, o = eng.simulate(plan), om.simulate_batch(plan)
    for k in ("qpos", "qvel"):
        assert np.array_equal(g[k], o[k]), k
    assert np.abs(g["qpos"][:, 0] - 0.8).max() < 0.5
