"""DEXEE hand (Shadow Robot / DeepMind), 3 fingers x 4 joints (reference:
mgs/gripper/dexee.py:413-476).

The MJCF is re-authored from the model's parameters (Menagerie-derived,
Apache-2.0; the reference template is dexee.py:32-410) rather than copied:

  * the kinematic tree (three fingers at the template's mount poses, each
    base -> knuckle -> proximal -> middle -> distal), joint axes / ranges,
    armature 8e-5, damping 0.009, frictionloss 0.009;
  * the contact classes: "hard" links (condim 4, friction 1 0.001 2e-5, direct
    solref -7000 -167) and the "soft" fingertip sensor pads (condim 6 --
    torsional and rolling friction -- friction 1 0.005 1e-4, solref -2500
    -100);
  * the twelve mujoco.pid plugin actuators (the four per-joint gain sets of the
    template's <extension>: kp, ki, kd, imax, slewmax), their ctrl and force
    ranges, actdim 2 (integral and previous setpoint);
  * the collision meshes emitted inline as the convex hulls MuJoCo collides
    (tools/derive_dexee_assets.py, each after its mesh's refquat); the mass of
    every link -- carried in the template by one visual mesh with an explicit
    mass -- as an <inertial> from that mesh's volume, centroid and inertia
    (MuJoCo's default legacy mesh inertia); visual geoms and the group-5
    helper capsules / cylinders (contype = conaffinity = 0, massless) have no
    physical effect and are dropped;
  * gravcomp="1" on every body (the template's gravity compensation; the
    engine supports it where gravity is zero, the gravityless env, where it is
    exactly no force);
  * the contact excludes and the mocap weld (torquescale 1).

close_gripper_at (dexee.py:450-456): set_pose, ctrl = qpos_close
(dexee.yaml:7), 500 steps.
"""
from __future__ import annotations

import os
from typing import Any, Dict, List, Tuple

import numpy as np

from mgs.gripper.base import MjShakableOpenCloseGripper, fmt32, mesh_inertial_xml
from mgs.util.const import PACKAGE_PATH
from mgs.util.geo.transforms import SE3Pose

_ASSET = os.path.join(PACKAGE_PATH, "assets", "dexee.npz")

# dexee.yaml:6-7
OPEN_QPOS = np.array([0, -1.3963, 0, 0, 0, -1.3963, 0, 0, 0, -1.3963, 0, 0], np.float64)
CLOSE_QPOS = np.array([0, -0.0325, 0, 0.00143, 0.0655, -0.0369, 0, 0, -0.0654, -0.0337, 0, 0], np.float64)

# per joint: axis, range, pid (kp, ki, kd, imax, slewmax), forcerange  (dexee.py:85-120, 150-178, 384-406)
_JOINTS = [
    ("J0", "0 0 -1", "-0.8727 0.8727", (2.8, 4.0, 0.03, 0.1, 3.14159), "-0.9 0.53"),
    ("J1", "1 0 0", "-1.3963 0.7854", (2.5, 3.0, 0.02, 0.2, 3.14159), "-0.35 1.2"),
    ("J2", "1 0 0", "0 1.3963", (1.1, 3.0, 0.01, 0.2, 3.14159), "-0.52 0.7"),
    ("J3", "-1 0 0", "-0.5236 1.4835", (0.6, 3.0, 0.008, 0.1, 3.14159), "-0.3 0.3"),
]
# finger mounts in the gripper frame: pos, quat (dexee.py:140, 216, 292)
_FINGERS = [("F0", "0 0.05 0.017", "1 0 0 0"),
            ("F1", "0.039 -0.029 0.017", "-0.16212752892551119 0 0 0.98676981326168844"),
            ("F2", "-0.039 -0.029 0.017", "0.16212752892551119 0 0 0.98676981326168844")]
# link masses (the visual mesh that carries each, dexee.py:128-178)
_MASS = {"base": 0.51, "finger_base": 0.89937782, "knuckle": 0.13077995, "proximal": 0.09614332,
         "middle": 0.05585897, "distal": 0.02766365}
_HARD = 'condim="4" friction="1 0.001 2e-05" solref="-7000 -167"'
_SOFT = 'condim="6" friction="1 0.005 0.0001" solref="-2500 -100"'
# knuckle body orientation: euler="-1.0472 0 0" (radians)
_KNUCKLE_QUAT = f"{float(np.cos(-1.0472 / 2))!r} {float(np.sin(-1.0472 / 2))!r} 0 0"


class GripperDexee(MjShakableOpenCloseGripper):
    close_steps = 500

    def __init__(self, pose: SE3Pose):
        super().__init__(pose, "dexee_gripper")

    def base_to_contact_transform(self) -> SE3Pose:
        # dexee.py:434-437
        return SE3Pose(np.array([0.0, 0, -0.31]), np.array([0.707106781, 0.0, 0.0, 0.707106781]), type="wxyz")

    def close_ctrl(self, sim) -> np.ndarray:
        # dexee.py:450-456 (close_gripper_at re-applies set_pose, a no-op at
        # the candidate's own pose, then holds this target for 500 steps)
        return CLOSE_QPOS.copy()

    def open_ctrl(self, sim) -> np.ndarray:
        # dexee.py:439-444 (open_gripper)
        return OPEN_QPOS.copy()

    def open_joints(self) -> np.ndarray:
        return OPEN_QPOS.copy()

    def get_actuator_joint_names(self) -> List[str]:
        # dexee.py:458-472
        return [f"F{i}/J{k}" for i in range(3) for k in range(4)]

    @staticmethod
    def _inertial(data, name):
        vol = float(data["vol_" + name])
        return mesh_inertial_xml(vol, data["com_" + name], data["inertia_" + name], _MASS[name] / vol)

    def _finger(self, data, f, pos, quat):
        def col(mesh, cls, extra="", name=None):
            return f'<geom name="{f}/{name or mesh.replace("_col", "_geom_col")}" type="mesh" mesh="{mesh}" {cls}{extra}/>'

        def joint(k):
            j, axis, rng, _, _ = _JOINTS[k]
            return (f'<joint name="{f}/{j}" axis="{axis}" range="{rng}" armature="8e-05" damping="0.009" '
                    'frictionloss="0.009"/>')
        return [f'<body name="{f}/" pos="{pos}" quat="{quat}">',
                f'<body name="{f}/finger_base" gravcomp="1">', self._inertial(data, "finger_base"),
                col("finger_base_col", _HARD, ' quat="1 -1 0 0"', name="base_geom_col"),
                f'<body name="{f}/finger_knuckle" pos="0 0.015 0.17902" quat="{_KNUCKLE_QUAT}" gravcomp="1">',
                joint(0), self._inertial(data, "knuckle"), col("knuckle_col", _HARD),
                f'<body name="{f}/finger_proximal" pos="0 -0.03 0" gravcomp="1">',
                joint(1), self._inertial(data, "proximal"), col("proximal_col", _HARD),
                f'<body name="{f}/finger_middle" pos="0 -0.05 0" gravcomp="1">',
                joint(2), self._inertial(data, "middle"), col("middle_col", _HARD),
                f'<body name="{f}/finger_distal" pos="0 -0.035 0" quat="0 0 -1 1" gravcomp="1">',
                joint(3), self._inertial(data, "distal"), col("distal_col", _HARD),
                col("tip_col", _SOFT, name="distal_geom_tip_col"),
                "</body></body></body></body></body></body>"]

    def to_xml(self) -> Tuple[str, Dict[str, Any]]:
        data = np.load(_ASSET)
        pos = f"{self.pos[0]} {self.pos[1]} {self.pos[2]}"
        quat = f"{self.quat[0]} {self.quat[1]} {self.quat[2]} {self.quat[3]}"
        out = ["<extension>"]
        for j, _, _, (kp, ki, kd, imax, slew), _ in _JOINTS:
            out.append(f'<plugin plugin="mujoco.pid"><instance name="actuator_{j}">'
                       f'<config key="kp" value="{kp}"/><config key="ki" value="{ki}"/>'
                       f'<config key="kd" value="{kd}"/><config key="imax" value="{imax}"/>'
                       f'<config key="slewmax" value="{slew}"/></instance></plugin>')
        out += ["</extension>", "<asset>"]
        for m in ("base", "puck", "finger_base", "knuckle", "proximal", "middle", "distal", "tip"):
            out.append(f'<mesh name="{m}_col" vertex="{fmt32(data["hull_" + m])}"/>')
        out += ["</asset>", "<worldbody>", f'<body name="mocap" mocap="true" pos="{pos}" quat="{quat}"/>',
                f'<body name="dexee_gripper" pos="{pos}" quat="{quat}" gravcomp="1">',
                '<freejoint name="freejoint"/>',
                '<body name="hand_base" gravcomp="1">', self._inertial(data, "base"),
                # the hand base's collision geoms carry no class (dexee.py:132,135-136):
                # MuJoCo's geom defaults, condim 3, friction 1 0.005 0.0001, solref 0.02 1
                '<geom name="hand_base_geom_col" type="mesh" mesh="base_col"/>',
                '<geom name="hand_base_puck_geom_col" type="mesh" mesh="puck_col"/>',
                "</body>"]
        for f, p, q in _FINGERS:
            out += self._finger(data, f, p, q)
        out += ["</body>", "</worldbody>", "<contact>"]
        for f, _, _ in _FINGERS:
            out.append(f'<exclude body1="hand_base" body2="{f}/finger_knuckle"/>')
        for f, _, _ in _FINGERS:
            out.append(f'<exclude body1="{f}/finger_base" body2="{f}/finger_knuckle"/>')
        out += ["</contact>", '<equality><weld body1="mocap" body2="dexee_gripper" torquescale="1.0"/></equality>',
                "<actuator>"]
        for f, _, _ in _FINGERS:
            for j, _, rng, _, frc in _JOINTS:
                out.append(f'<plugin name="{f}/{j}_actuator" plugin="mujoco.pid" instance="actuator_{j}" '
                           f'ctrlrange="{rng}" forcerange="{frc}" dyntype="none" joint="{f}/{j}" actdim="2"/>')
        out.append("</actuator>")
        return "\n".join(out), {}
