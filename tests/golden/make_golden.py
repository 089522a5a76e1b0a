"""Generate tests/golden/harness_golden.npz from the REFERENCE harness.

TEST INFRASTRUCTURE ONLY -- run here (never on the GPU box; the reference does
not travel).  It imports the reference's own Python modules read-only from
/root/reference with:

  * a `typing.Self` shim (reference needs Python >= 3.11, transforms.py:18),
  * the Protocol-__init__ workaround for Python 3.10 (gripper/base.py:33-39),
  * a recording `mujoco` stand-in: MuJoCo itself is not installed, so physics is
    NOT exercised.  `mj_step` logs the control inputs the harness wrote
    (mocap_pos, mocap_quat, ctrl, and qpos at the first step), and
    `data.contact.geom` / `data.ncon` follow a scripted contact oracle
    ("gripper-object contact is lost after global step k").

What this pins: the float32 pose processing, the joint
index quirk, the per-step mocap trajectory of close/lift/back/right/left, the
check points, early exits and labels under the scripted oracle -- i.e. the
whole host-side schedule the GPU rollout consumes.  Physics parity against
MuJoCo stays unpinned (MuJoCo absent).

Two subprocesses, because both the reference and this build are the `mgs`
package: phase "build" dumps this build's model name tables + the candidate
inputs, phase "reference" runs the reference harness against them.

    python tests/golden/make_golden.py          # writes tests/golden/harness_golden.npz
"""
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"

# horizon used for the goldens: the reference's close (3000, fixed in
# close_gripper_at) with a short lift/shake (the reference's own parameters)
NSTEP_LIFT = 300
SHAKE_STEPS = 50
NCAND = 8


def phase_build(tmp):
    sys.path.insert(0, os.path.join(REPO, "mj-grasp-sim_amd"))
    import numpy as np
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
    from mgs.gripper.robotiq2f85 import GripperRobotiq2f85
    from mgs.obj.selector import get_object
    from mgs.sampler.antipodal import robotiq_candidates
    from mgs.util.geo.transforms import SE3Pose

    grip = GripperRobotiq2f85(SE3Pose(np.zeros(3), np.array([1, 0, 0, 0]), "wxyz"))
    obj = get_object("003_cracker_box")
    env = GravitylessObjectGrasping(grip, obj)
    cm = env.model
    H, J, _ = robotiq_candidates(obj, NCAND, seed=0)
    J = np.asarray(J, np.float64)
    # exercise the index quirk: joints[:, 2] / joints[:, 6] land in the object's x
    J[1, 2] = 0.25
    J[2, 6] = -0.125
    J[3, :] = np.linspace(0.01, 0.08, 8)
    tables = dict(jnt_names=list(cm.jnt_names), jnt_qposadr=[int(x) for x in cm.jnt_qposadr],
                  geom_names=list(cm.geom_names), nq=int(cm.nq), nu=int(cm.nu),
                  qpos0=[float(x) for x in cm.qpos0], obj_name=obj.name)
    with open(os.path.join(tmp, "tables.json"), "w") as f:
        json.dump(tables, f)
    np.savez(os.path.join(tmp, "inputs.npz"), poses=np.asarray(H, np.float32), joints=J)


def phase_reference(tmp):
    sys.dont_write_bytecode = True          # never write into /root/reference
    import types
    import typing

    import numpy as np
    import typing_extensions
    typing.Self = typing_extensions.Self

    with open(os.path.join(tmp, "tables.json")) as f:
        T = json.load(f)
    inp = np.load(os.path.join(tmp, "inputs.npz"))

    # ---------------- recording mujoco stand-in ----------------
    LOG = dict(steps=[], checks=[], ncon_calls=[])
    SCRIPT = dict(lose_after=None, step=0, collide=False)
    mj = types.ModuleType("mujoco")
    mj.viewer = types.ModuleType("mujoco.viewer")
    ground = T["geom_names"].index("geom:ground")
    g_grip, g_obj = 0, len(T["geom_names"]) - 1

    class _Obj:
        def __init__(self, **kw):
            self.__dict__.update(kw)

    class MjModel:
        def __init__(self):
            self.nq, self.nu = T["nq"], T["nu"]
            self.jnt_qposadr = np.array(T["jnt_qposadr"], dtype=np.int32)
            self.qpos0 = np.array(T["qpos0"])

        @staticmethod
        def from_xml_string(xml, assets=None):
            return MjModel()

        def jnt(self, name):
            return _Obj(qposadr=np.array([self.jnt_qposadr[T["jnt_names"].index(name)]]))

        def geom(self, name):
            return _Obj(id=T["geom_names"].index(name))

    class _Contact:
        @property
        def geom(self):
            LOG["checks"].append(SCRIPT["step"])
            lost = SCRIPT["lose_after"] is not None and SCRIPT["step"] > SCRIPT["lose_after"]
            return np.zeros((0, 2), np.int32) if lost else np.array([[g_grip, g_obj]], np.int32)

    class MjData:
        def __init__(self, model):
            self.model = model
            self.qpos = model.qpos0.copy()
            self._mocap_pos = np.zeros((1, 3))
            self._mocap_quat = np.array([[1.0, 0, 0, 0]])
            self.ctrl = np.zeros(model.nu)
            self.contact = _Contact()

        mocap_pos = property(lambda s: s._mocap_pos, lambda s, v: s._mocap_pos.__setitem__(Ellipsis, v))
        mocap_quat = property(lambda s: s._mocap_quat, lambda s, v: s._mocap_quat.__setitem__(Ellipsis, v))

        @property
        def ncon(self):
            LOG["ncon_calls"].append(SCRIPT["step"])
            return 1 if SCRIPT["collide"] else 0

    def mj_step(m, d, nstep=1):
        for _ in range(nstep):
            if SCRIPT["step"] == 0:
                LOG["qpos0"] = d.qpos.copy()
            LOG["steps"].append(np.concatenate([d.mocap_pos[0], d.mocap_quat[0], d.ctrl]))
            SCRIPT["step"] += 1

    def mj_resetData(m, d):
        d.qpos[:] = m.qpos0
        d._mocap_pos[:] = 0.0
        d._mocap_quat[:] = [1.0, 0, 0, 0]
        d.ctrl[:] = 0.0

    def mj_name2id(m, objtype, name):
        return T["jnt_names"].index(name) if name in T["jnt_names"] else -1

    mj.MjModel, mj.MjData = MjModel, MjData
    mj.mj_step, mj.mj_forward, mj.mj_resetData, mj.mj_name2id = mj_step, (lambda m, d: None), mj_resetData, mj_name2id
    mj.mjtObj = _Obj(mjOBJ_JOINT=3)
    mj.mjtState = _Obj(mjSTATE_INTEGRATION=0)
    mj.mj_stateSize = lambda m, spec: m.nq
    mj.mj_getState = lambda m, d, out, spec: out.__setitem__(Ellipsis, d.qpos)
    mj.mj_setState = lambda m, d, st, spec: d.qpos.__setitem__(Ellipsis, st)
    mj.MjvOption = lambda: _Obj(flags=np.zeros(64, bool), geomgroup=np.zeros(6, bool))
    mj.mjtVisFlag = _Obj()
    sys.modules["mujoco"] = mj
    sys.modules["mujoco.viewer"] = mj.viewer

    sys.path.insert(0, REF)
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
    from mgs.gripper.robotiq2f85 import GripperRobotiq2f85
    from mgs.util.geo.transforms import SE3Pose

    grip = GripperRobotiq2f85.__new__(GripperRobotiq2f85)
    pv = SE3Pose(np.zeros(3), np.array([1.0, 0, 0, 0]), "wxyz").to_vec(layout="pq", type="wxyz")
    grip.pos, grip.quat, grip.base = pv[:3], pv[3:], "base_mount"

    class FakeObj:
        name = T["obj_name"]

        def to_xml(self):
            return "", {}

    env = GravitylessObjectGrasping(grip, FakeObj())
    poses = SE3Pose.from_mat(inp["poses"])
    joints = inp["joints"]
    n = len(joints)

    # collision mask: scripted ncon (odd candidates collide)
    mask_script = np.array([i % 2 == 1 for i in range(n)])
    mask = []
    for i in range(n):
        SCRIPT["collide"] = bool(mask_script[i])
        mask.append(bool(env.grasp_collision_mask(poses[i:i + 1], joints[i:i + 1])[0]))

    # stability: scripted contact loss per candidate (global step after which
    # gripper-object contact disappears; -1 = never)
    close = 3000
    L = NSTEP_LIFT
    lose = [-1, 1500, close + 150, close + 250, close + L + 10, close + L + SHAKE_STEPS + 5,
            close + L + 2 * SHAKE_STEPS + 60, -1][:n]
    traj, checks, labels, nsteps, qpos0 = [], [], [], [], []
    for i in range(n):
        LOG["steps"], LOG["checks"] = [], []
        SCRIPT["step"] = 0
        SCRIPT["lose_after"] = None if lose[i] < 0 else lose[i]
        lab = env.grasp_stability_evaluation_from_joints(poses[i:i + 1], joints[i:i + 1],
                                                         nstep_lift=NSTEP_LIFT, shake_steps=SHAKE_STEPS)
        labels.append(bool(lab[0]))
        nsteps.append(len(LOG["steps"]))
        tr = np.zeros((close + L + 4 * SHAKE_STEPS, 8))
        tr[:len(LOG["steps"])] = np.array(LOG["steps"])
        traj.append(tr)
        ck = np.full(64, -1, np.int32)
        ck[:len(LOG["checks"])] = LOG["checks"]
        checks.append(ck)
        qpos0.append(LOG["qpos0"])

    np.savez_compressed(
        os.path.join(tmp, "golden.npz"),
        poses=inp["poses"], joints=joints, mask_script=mask_script, mask=np.array(mask),
        lose_after=np.array(lose, np.int32), labels=np.array(labels), nsteps=np.array(nsteps, np.int32),
        traj=np.array(traj), checks=np.array(checks), qpos0=np.array(qpos0),
        nstep_lift=NSTEP_LIFT, shake_steps=SHAKE_STEPS, close_steps=close)


def main():
    if len(sys.argv) > 2:
        {"build": phase_build, "reference": phase_reference}[sys.argv[1]](sys.argv[2])
        return
    with tempfile.TemporaryDirectory() as tmp:
        env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
        for ph in ("build", "reference"):
            subprocess.run([sys.executable, os.path.abspath(__file__), ph, tmp], check=True, env=env)
        out = os.path.join(HERE, "harness_golden.npz")
        os.replace(os.path.join(tmp, "golden.npz"), out)
        print("wrote", out)


if __name__ == "__main__":
    main()
