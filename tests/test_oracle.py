"""The CPU oracle (oracle/mgs_oracle.c): the checker the GPU path is compared
with.  Pinned here by (1) the reference's own known answer for the physics,
Robotiq's recorded closed state `state_close` (mgs/cli/config/gripper/
robotiq_2f_85.yaml:11, values copied as data below), run in the model it was
recorded in, (2) its arithmetic primitives, (3) determinism and solver
consistency."""
import copy

import numpy as np
import pytest

# state_close (robotiq_2f_85.yaml:11): right driver, coupler, spring link,
# follower, then the left chain, after a long ctrl=255 close in free space
# (time 223.376 s, |qvel| <= 2e-14).
KAT_JOINTS = np.array([7.93116751e-01, 3.48441304e-04, 7.89591521e-01, -7.76735418e-01,
                       7.93117030e-01, 3.47173334e-04, 7.89598436e-01, -7.76696653e-01])
# rest state of the oracle minus KAT_JOINTS (rad) in the scan-env model, MuJoCo
# 3.2.2's legacy mesh inertia (test_state_close_offset_is_the_base_mount_mass),
# the box-box edge rule and the equality impedance at the constraint's
# violation norm (round 5, test_state_close_contact_set_study): drivers
# -7.7e-6 / -8.3e-6, couplers -1.1e-6 / +1.5e-6, spring links -1.1e-6 /
# -2.1e-5, followers +4.7e-5 / -5.1e-5 -- every joint within SURVEY §8c's
# 1e-4 bar.  (Round 4: drivers +1.1e-4, spring links -2.9e-4 / -3.2e-4.)
# Per-joint bounds are ~1.3x those offsets (at least 5e-6).
KAT_TOL = np.array([1.2e-5, 5.0e-6, 5.0e-6, 6.2e-5, 1.2e-5, 5.0e-6, 2.8e-5, 6.7e-5])

# GripperScanEnv's model (reference mgs/env/gripper_scan.py:26-49), the model
# state_close was recorded in (its 22 qpos = 15 gripper + 7 of the free
# camera body): the option sequence, the gripper, a world-fixed 1e-6 m sphere
# at the origin and a free camera body 0.4 m above it (lights and the camera
# element do not enter the physics and are left out)
SCAN_XML = r"""
<mujoco>
  <compiler angle="radian" autolimits="true" />
  <option integrator="implicitfast" timestep="0.001"/>
  <compiler discardvisual="false"/>
  <option noslip_iterations="1"> </option>
  <option><flag multiccd="enable"/> </option>
  <option cone="elliptic" gravity="0 0 -9.81" impratio="3" timestep="0.001" noslip_iterations="2"
          noslip_tolerance="1e-8" tolerance="1e-8"/>
  <option gravity="0 0 0" />
  {gripper}
  <option gravity="0 0 0" />
  <worldbody>
    <body name="center" pos="0.0 0.0 0.0" quat="1.0 0.0 0 0">
      <geom name="geom:center" size="0.000001" rgba="0 0 0 1.0"/>
    </body>
    <body name="body:camera" pos="0.0 0.0 .4" quat="1.0 0.0 0 0">
      <freejoint name="camera:joint"/>
      <geom name="geom:camera" size="0.01" />
    </body>
  </worldbody>
</mujoco>
"""


@pytest.fixture(scope="module")
def scan_model():
    from mgs.core.mjcf import compile_xml
    from mgs.gripper.robotiq2f85 import GripperRobotiq2f85
    from mgs.util.geo.transforms import SE3Pose
    g = GripperRobotiq2f85(SE3Pose(np.zeros(3), np.array([1.0, 0, 0, 0]), "wxyz"))
    gx, ga = g.to_xml()
    cm = compile_xml(SCAN_XML.format(gripper=gx), ga)
    # GripperScanEnv.__init__ (gripper_scan.py:86-91): identity pose @ b2c
    pose = SE3Pose(np.zeros(3), np.array([1.0, 0, 0, 0]), "wxyz") @ g.base_to_contact_transform()
    q = np.array(cm.qpos0, np.float64).copy()
    q[0:3], q[3:7] = pose.pos, pose.quat
    return cm, q, np.array(pose.pos, np.float64), np.array(pose.quat, np.float64)


def scan_close(scan_model, solver="Newton", noslip=2, nsteps=6000, cm=None):
    from oracle import oracle as O
    cm0, q, mp, mq = scan_model
    cm = copy.copy(cm0 if cm is None else cm)
    cm.options = dict(cm.options)
    cm.options["solver"] = solver
    om = O.OracleModel(cm)
    om.desc.noslip_iterations = noslip
    tr, nc, qv = om.trace(q, mp, mq, np.array([255.0]), nsteps)
    return tr, nc, qv, om


def test_scan_model_is_the_recorded_one(scan_model):
    """state_close's layout: 22 qpos (15 gripper + 7 camera), 20 dofs; the
    scan env's options after the gripper's own <option> (impratio 10)"""
    cm = scan_model[0]
    assert (cm.nq, cm.nv) == (22, 20)
    o = cm.options
    assert (o["impratio"], o["noslip_iterations"], o["tolerance"], o["cone"]) == (10.0, 2, 1e-8, "elliptic")
    assert np.all(o["gravity"] == 0.0)


@pytest.mark.parametrize("solver", ["Newton", "PGS"])
def test_state_close_known_answer(scan_model, solver):
    """Free-space close in GripperScanEnv's model (noslip off: MuJoCo reached
    rest): every joint within ~1.3x its known offset (KAT_TOL) of the recorded
    state.  The world-fixed 1e-6 m sphere stays 16 mm below the pads' contact
    line and the camera sphere 0.55 m away: the pads touch only each other."""
    cm = scan_model[0]
    tr, nc, qv, om = scan_close(scan_model, solver, noslip=0, nsteps=6000)
    assert np.all(np.abs(tr[-1, 7:15] - KAT_JOINTS) < KAT_TOL)
    assert np.abs(qv).max() < (1e-12 if solver == "Newton" else 1e-10)
    _, _, _, _, g = om.contacts(tr[-1], scan_model[2], scan_model[3])
    names = {cm.geom_names[i] for i in g.ravel()}
    assert names == {"right_pad1", "left_pad1"}
    assert np.array_equal(tr[-1, 15:22], scan_model[1][15:22])       # the camera body never moves


def test_state_close_with_noslip(scan_model):
    """With the scan env's noslip_iterations=2 the close comes to rest at the
    same joints and at MuJoCo's recorded rest (|qvel| <= 2e-14 there, < 1e-13
    here).  Round 4 kept a 40 Hz limit cycle of ~6e-7 rad/s: its two pad-pad
    contacts on one edge had identical tangent rows, which the unregularised
    noslip sweep cannot split; the edge rule's single contact has none
    (test_state_close_contact_set_study)."""
    tr, nc, qv, _ = scan_close(scan_model, noslip=2, nsteps=6000)
    assert np.all(np.abs(tr[-1, 7:15] - KAT_JOINTS) < KAT_TOL)
    assert np.abs(qv).max() < 1e-13
    amp = np.abs(tr[-2000:, 7:15] - tr[-2000:, 7:15].mean(0)).max()
    assert amp < 1e-12


def test_pgs_cost_change_revert_noslip_free_close(scan_model):
    """PGS main solver + noslip, same rest criterion (PGS at 100 iterations is
    not converged, so the bound is the solver's, not the revert rule's)."""
    tr, nc, qv, _ = scan_close(scan_model, "PGS", noslip=2, nsteps=6000)
    assert np.all(np.abs(tr[-1, 7:15] - KAT_JOINTS) < KAT_TOL)
    assert np.abs(qv).max() < 1e-5


def test_state_close_offset_is_the_base_mount_mass(scan_model):
    """Which modelled term the state_close offset came from.  The rest state is
    a static balance of soft constraints whose stiffness is
    K imp^2 / ((1 - imp) diagApprox), and diagApprox is built from the qpos0
    inverse weights, which every gripper body inherits from the free base.
    base_mount has no <inertial>, so its mass comes from its two mesh geoms at
    density 1000, and MuJoCo 3.2.2's default <mesh inertia="legacy"> sums
    |volume| per face pyramid: 74.98 cm^3 for this non-convex mesh against its
    34.77 cm^3 exact volume.  With the exact volume (the round-3 model) the
    drivers rest 4.0e-4 rad and the followers 6.6e-4 / 7.8e-4 rad off the
    recorded state; with the legacy mass 8e-6 and 4.7e-5 / 5.1e-5 (round-5
    contract; round 4's contract gave 4.7e-4 / 5.8e-4 / 6.9e-4 exact and 1.1e-4 /
    3.1e-5 / 6.5e-5 legacy, the spring links' -3e-4 being the term the round-5
    study explains, test_state_close_contact_set_study)."""
    from mgs.core.mjcf import _invweight0, mesh_mass_properties
    from mgs.gripper.robotiq2f85 import _ASSET
    cm = scan_model[0]
    b = cm.body_names.index("base_mount")
    d = np.load(_ASSET)
    vol = float(d["vol_base_mount"])
    assert abs(cm.body_mass[b] - 2 * 1000.0 * vol) < 1e-12
    # the exact-volume variant of the same body (the mesh's own vertices are
    # not shipped: scale the legacy properties to the exact volume 34.769 cm^3
    # and centroid, which is what the round-3 model carried)
    ex = copy.copy(cm)
    ex.body_mass = cm.body_mass.copy()
    ex.body_mass[b] = 2 * 1000.0 * 3.4769031848943e-05
    ex.body_inertia = cm.body_inertia.copy()
    ex.body_inertia[b] = cm.body_inertia[b] * (3.4769031848943e-05 / vol)
    ex.body_ipos = cm.body_ipos.copy()
    ex.body_ipos[b] = [-1.41673786e-03, -3.79796273e-05, -8.98408191e-04]
    ex.body_invweight0, ex.dof_invweight0, ex.meaninertia = _invweight0(ex)
    tr_l, *_ = scan_close(scan_model, noslip=0)
    tr_e, *_ = scan_close(scan_model, noslip=0, cm=ex)
    off_l = np.abs(tr_l[-1, 7:15] - KAT_JOINTS)
    off_e = np.abs(tr_e[-1, 7:15] - KAT_JOINTS)
    drv, fol = [0, 4], [3, 7]
    assert off_e[drv].min() > 3.5e-4 and off_e[fol].min() > 5e-4
    assert off_l[drv].max() < 1.5e-5 and off_l[fol].max() < 7e-5
    assert (off_l[drv] < off_e[drv] / 20).all() and (off_l[fol] < off_e[fol] / 8).all()
    # the legacy rule itself (mgs.core.mjcf.mesh_mass_properties): a convex
    # mesh is unchanged, a non-convex one is over-counted
    cube = np.array([[x, y, z] for x in (0, 1) for y in (0, 1) for z in (0, 1)], float)
    assert abs(mesh_mass_properties(cube, None)[0] - 1.0) < 1e-12
    # a U-shaped prism (volume 7): its area-weighted face centroid lies in the
    # notch, outside the solid, so some face pyramids are negative and legacy
    # counts them positive
    P = np.array([[0, 0], [1, 0], [2, 0], [3, 0], [3, 3], [2, 3], [2, 1], [1, 1], [1, 3], [0, 3]], float)
    verts = np.vstack([np.c_[P, np.zeros(10)], np.c_[P, np.ones(10)]])
    up = [[0, 1, 8], [0, 8, 9], [1, 2, 6], [1, 6, 7], [2, 3, 4], [2, 4, 5]]   # CCW seen from +z
    faces = [[a, c, b] for a, b, c in up] + [[10 + a, 10 + b, 10 + c] for a, b, c in up]
    for i in range(10):
        j = (i + 1) % 10
        faces += [[i, j, 10 + j], [i, 10 + j, 10 + i]]
    faces = np.array(faces)
    assert abs(mesh_mass_properties(verts, faces, "exact")[0] - 7.0) < 1e-12
    assert mesh_mass_properties(verts, faces, "legacy")[0] > 7.0 + 1e-3


def test_state_close_contact_set_study(scan_model):
    """Round-5 study (verdict r4 item 1): which pad-pad contact set and which
    row term explain the round-4 residuals against state_close -- the spring
    links 3e-4 rad off and, with noslip, a limit cycle where MuJoCo rested at
    |qvel| 2e-14.  The model variants are oracle knobs (mgs_oracle.c
    oracle_set_bbmode / oracle_set_eqimp); (0, 0) is the contract the kernels
    follow.  At rest the pads touch along one edge (two penetrating clipped
    vertices of the incident face):

      box-box set \\ equality impedance   own row's violation   violation norm
      both edge vertices (round 4)       max 3.2e-4, cycle     max 2.9e-4, cycle
      the deeper vertex (round 5)        max 2.9e-4            max 5.1e-5, rest

    The single contact alone removes the noslip cycle and moves the spring
    links by 2.6e-4 (to -3e-5 / -5e-5) but the drivers 1.8e-4 the other way;
    the impedance at the connect constraints' violation norm alone moves the
    drivers back; together every joint is within 5.1e-5 and the close comes to
    rest as MuJoCo's did.  The connect rows carry ~20 N at rest with R ~0.6 (a
    0.3 mm soft violation), so the linkage angles are this sensitive to their
    impedance.  Two other sets change nothing: the face-overlap corners
    (non-penetrating corners are inactive rows) and one contact at the edge's
    midpoint instead of its deeper vertex (the hinge axes are along the
    edge)."""
    from oracle import oracle as O
    res = {}
    try:
        for bb, eq in ((1, 1), (0, 1), (1, 0), (0, 0), (2, 1), (4, 0)):
            O.set_study_variant(bb, eq)
            tr, nc, qv, om = scan_close(scan_model, noslip=2, nsteps=6000)
            amp = np.abs(tr[-2000:, 7:15] - tr[-2000:, 7:15].mean(0)).max()
            n = om.contacts(tr[-1], scan_model[2], scan_model[3])[0]
            res[bb, eq] = (tr[-1, 7:15] - KAT_JOINTS, np.abs(qv).max(), amp, n)
    finally:
        O.set_study_variant(0, 0)
    off4, qv4, amp4, n4 = res[1, 1]          # the round-4 contract
    assert n4 == 2 and np.abs(off4[[2, 6]]).min() > 2.5e-4 and qv4 > 1e-7 and amp4 > 1e-9
    off, qv, amp, n = res[0, 0]               # the round-5 contract
    assert n == 1 and np.abs(off).max() < 6e-5 and qv < 1e-13 and amp < 1e-12
    # each change alone: the spring links or the drivers stay > 1.5e-4 off
    assert np.abs(res[0, 1][0]).max() > 2.5e-4 and res[0, 1][1] < 1e-13      # no cycle, drivers off
    assert np.abs(res[1, 0][0][[2, 6]]).min() > 2.5e-4 and res[1, 0][1] > 1e-7
    # the corners and the midpoint variants equal their base sets
    assert np.allclose(res[2, 1][0], off4, atol=1e-9, rtol=0) and res[2, 1][3] == 4
    assert np.allclose(res[4, 0][0], off, atol=1e-9, rtol=0)


def test_equality_row_impedance_by_hand(scan_model):
    """One connect row and one weld row at the state_close rest state against
    MuJoCo's documented soft-constraint formulas (Computation chapter):
    diagApprox = the two bodies' qpos0 inverse weights (translational for a
    connect and a weld's first 3 rows, rotational for the weld's last 3),
    imp = solimp's sigmoid at x = |violation| / width (power 2, midpoint 0.5)
    with the violation the constraint's norm, R = (1 - imp) / imp * diagApprox,
    K = 1 / (dmax^2 timeconst^2 dampratio^2), B = 2 / (dmax timeconst),
    aref = -B v - K imp pos"""
    tr, nc, qv, om = scan_close(scan_model, noslip=0, nsteps=6000)
    cm = scan_model[0]
    r = om.forward_debug(tr[-1], scan_model[2], scan_model[3], np.array([255.0]))
    eq = np.nonzero(r["type"] == 0)[0]
    assert len(eq) == 13                        # 2 connect (3 each), joint (1), weld (6)

    def imp_of(si, x):
        x = min(abs(x) / si[2], 1.0)
        y = x ** 2 / 0.5 if x <= 0.5 else 1.0 - (1.0 - x) ** 2 / 0.5
        assert si[3] == 0.5 and si[4] == 2.0
        return si[0] + y * (si[1] - si[0])

    iw = cm.body_invweight0.reshape(-1, 2)
    for e, rows in ((0, eq[0:3]), (3, eq[7:13])):
        e = int(np.nonzero(cm.eq_type == (0 if e == 0 else 1))[0][0])
        b1, b2 = int(cm.eq_obj1id[e]), int(cm.eq_obj2id[e])
        sr, si = cm.eq_solref[e], cm.eq_solimp[e]
        nrm = np.sqrt(np.sum(r["pos"][rows] ** 2))
        imp = imp_of(si, nrm)
        tc = max(sr[0], 2 * cm.options["timestep"])
        K = 1.0 / (si[1] ** 2 * tc ** 2 * sr[1] ** 2)
        B = 2.0 / (si[1] * tc)
        for k, q in enumerate(rows):
            dA = iw[b1, int(k > 2)] + iw[b2, int(k > 2)]
            assert abs(r["diag"][q] - dA) <= 1e-12 * dA
            assert abs(r["R"][q] - (1 - imp) / imp * dA) <= 1e-12 * r["R"][q]
            aref = -B * r["vel"][q] - K * imp * r["pos"][q]
            assert abs(r["aref"][q] - aref) <= 1e-9 * (abs(aref) + 1e-9)
    # the connect constraint at rest: ~20 N through a ~0.3 mm soft violation
    c = eq[0:3]
    assert np.abs(r["force"][c]).max() > 10 and 1e-4 < np.sqrt(np.sum(r["pos"][c] ** 2)) < 1e-3


def test_sincos_and_tree_primitives():
    from oracle import oracle as O
    x = np.concatenate([np.linspace(-30, 30, 4001), np.array([0.0, 1e-300, -1e-8, np.pi / 2, np.pi])])
    s, c = O.sincos(x)
    assert np.abs(s - np.sin(x)).max() < 4e-16 * 30
    assert np.abs(c - np.cos(x)).max() < 4e-16 * 30
    rng = np.random.default_rng(0)
    for n in [1, 2, 3, 7, 16, 20, 33, 64]:
        a, b = rng.standard_normal(64), rng.standard_normal(64)
        leaf = np.zeros(64)
        P = 1
        while P < n:
            P *= 2
        leaf[:n] = a[:n] * b[:n]
        s_ = 1
        v = leaf[:P].copy()
        while s_ < P:
            v = v + v[np.arange(P) ^ s_]
            s_ *= 2
        assert O.tree_dot(a, b, n) == v[0]


def test_rollout_deterministic_across_threads(env, candidates, oracle_model):
    from conftest import plan_for
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    free = oracle_model.collision_free(q, mp, mq, nthreads=4)
    idx = np.nonzero(free)[0][:12]
    plan = plan_for(env, poses[idx], J[idx])
    r1 = oracle_model.rollout(plan, nthreads=1)
    r4 = oracle_model.rollout(plan, nthreads=4)
    for k in r1:
        assert np.array_equal(r1[k], r4[k]), k


def test_collision_free_fraction(env, candidates, oracle_model):
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    free = oracle_model.collision_free(q, mp, mq, nthreads=4)
    assert 0.05 < free.mean() < 0.5
    part = oracle_model.collision_free(q, mp, mq, predicate="partition", nthreads=4)
    assert np.all(part >= free)        # gripper-object contact implies any contact


def test_newton_and_pgs_agree_on_labels(env, candidates):
    """Same convex problem, two solvers: labels agree on most candidates."""
    from conftest import plan_for
    from oracle import oracle as O
    poses, J = candidates
    res = {}
    for solver in ["Newton", "PGS"]:
        cm = copy.copy(env.model)
        cm.options = dict(env.model.options)
        cm.options["solver"] = solver
        om = O.OracleModel(cm)
        q, mp, mq, _ = env.initial_state(poses, J)
        idx = np.nonzero(om.collision_free(q, mp, mq, nthreads=4))[0]
        res[solver] = om.rollout(plan_for(env, poses[idx], J[idx]), nthreads=4)["label"]
    assert (res["Newton"] == res["PGS"]).mean() >= 0.85


def test_empty_batch(env, oracle_model):
    from conftest import plan_for
    from mgs.util.geo.transforms import SE3Pose
    poses = SE3Pose(np.zeros((0, 3), np.float32), np.zeros((0, 4), np.float32), "wxyz")
    q, mp, mq, _ = env.initial_state(poses, np.zeros((0, 8)))
    assert oracle_model.collision_free(q, mp, mq).shape == (0,)


def _guard_plan(env, candidates, oracle_model, n=4):
    """n collision-free candidates (the rollouts the pipeline runs), two of them
    given a bad initial state"""
    from conftest import plan_for
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    idx = np.nonzero(oracle_model.collision_free(q, mp, mq))[0][:n]
    plan = plan_for(env, poses[idx], J[idx])
    plan.qpos_init = plan.qpos_init.copy()
    plan.qpos_init[1, 17] = np.nan        # object x: a NaN state
    plan.qpos_init[2, 0] = 2e10           # gripper x beyond mjMAXVAL
    return plan


def test_divergence_guard_oracle(env, candidates, oracle_model):
    """MuJoCo's mj_checkPos / mj_checkVel / mj_checkAcc (NaN or |x| > 1e10) stop a
    candidate: label 0, fail step = the step that produced the bad state, flag
    MGS_FLAG_DIVERGED in stats[:, 2]; healthy candidates are untouched."""
    from mgs.core.abi import MGS
    plan = _guard_plan(env, candidates, oracle_model)
    r = oracle_model.rollout(plan)
    div = MGS["MGS_FLAG_DIVERGED"]
    assert list(r["stats"][:, 2] & div) == [0, div, div, 0]
    assert not r["label"][1] and not r["label"][2]
    assert r["fail_step"][1] == 0 and r["fail_step"][2] == 0
    clean = oracle_model.rollout(plan.subset([0, 3]))
    for k in ("label", "fail_step", "obj_qpos", "stats"):
        assert np.array_equal(clean[k], r[k][[0, 3]])


@pytest.mark.parametrize("horizon,n", [("h200", 160), ("ref8000", 3)])
def test_separation_certificates_are_exact(env, candidates, oracle_model, horizon, n):
    """Pairs skipped by a separation certificate (kernel / oracle cert_check)
    are pairs MPR would miss: rollouts with the skipping turned off give the
    same labels, fail steps, object poses and contact / row statistics, bit
    for bit, and the skipping removes narrowphase support calls"""
    import ctypes
    from conftest import plan_for
    from oracle import oracle as O
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    idx = np.nonzero(oracle_model.collision_free(q, mp, mq, nthreads=8))[0][:n]
    plan = plan_for(env, poses[idx], J[idx], horizon)
    L = O.lib()
    L.oracle_set_cull.argtypes = [ctypes.c_int]
    try:
        L.oracle_set_cull(0)
        off = oracle_model.rollout(plan, nthreads=8)
    finally:
        L.oracle_set_cull(1)
    on = oracle_model.rollout(plan, nthreads=8)
    for k in ("label", "fail_step", "obj_qpos", "stats"):
        assert np.array_equal(on[k], off[k]), k
