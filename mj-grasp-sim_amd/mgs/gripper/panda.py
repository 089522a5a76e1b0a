"""Franka Panda parallel gripper (reference: mgs/gripper/panda.py:142-273).

The MJCF is re-authored from the model's parameters (Menagerie-derived,
Apache-2.0; the reference template is panda.py:32-139) rather than copied:

  * every body, inertial, joint, equality, tendon and actuator parameter of the
    reference template is kept (hand 0.73 kg on a free joint welded to a mocap
    body, two slide fingers with damping 100, armature 1, frictionloss 1 and
    limits, position actuators kp 1000 clamped to +-15 N, the `split` tendon,
    the hand/finger contact excludes);
  * the two collision meshes are emitted inline (`<mesh vertex=...>`) as the
    convex hulls of the Menagerie meshes, which is what MuJoCo collides
    (tools/derive_panda_assets.py);
  * visual geoms (contype=conaffinity=0) are dropped: every body carries an
    explicit <inertial>, so they have no physical effect.
"""
from __future__ import annotations

import os
from typing import Any, Dict, List, Tuple

import numpy as np

from mgs.gripper.base import MjShakableOpenCloseGripper
from mgs.util.const import PACKAGE_PATH
from mgs.util.geo.transforms import SE3Pose

_ASSET = os.path.join(PACKAGE_PATH, "assets", "panda.npz")

# fingertip pad boxes shared by both fingers: (size, pos) -- panda.py:41-55,
# all with friction "2.4 0.3 0.1"
_PADS = [("0.0085 0.004 0.0085", "0 0.0055 0.0445"),
         ("0.003 0.002 0.003", "0.0055 0.002 0.05"),
         ("0.003 0.002 0.003", "-0.0055 0.002 0.05"),
         ("0.003 0.002 0.0035", "0.0055 0.002 0.0395"),
         ("0.003 0.002 0.0035", "-0.0055 0.002 0.0395")]
# (body, pos, quat, joint, range, first collision-geom index)
_FINGERS = [("left_finger", "0 0 0.0584", None, "finger_joint1", "0.0 0.04", 1),
            ("right_finger", "0 -0.04 0.0584", "0 0 0 1", "finger_joint2", "-0.04 0.0", 7)]


def _fmt(v):
    return " ".join(repr(float(np.float32(x))) if abs(x) > 0 else "0" for x in np.ravel(v))


class GripperPanda(MjShakableOpenCloseGripper):
    MIN_WIDTH_TARGET = 0.0
    MAX_WIDTH = 0.08
    MIN_WIDTH_CLAMP = 0.003
    Q1_RANGE = [0.0, 0.04]
    Q2_RANGE = [-0.04, 0.0]
    close_steps = 3000

    def __init__(self, pose: SE3Pose):
        super().__init__(pose, "hand")

    def base_to_contact_transform(self) -> SE3Pose:
        # reference panda.py:190-193
        return SE3Pose(np.array([0, 0, -0.102]), np.array([0.707106781, 0.0, 0.0, 0.707106781]), type="wxyz")

    def close_ctrl(self, sim) -> np.ndarray:
        # reference panda.py:225-241: ctrl = (0.0, -0.04), then 3000 steps
        return np.array([0.0, -0.04])

    def open_ctrl(self, sim) -> np.ndarray:
        # reference panda.py:195-207
        return np.array([self.Q1_RANGE[1], self.Q2_RANGE[1]])

    def width_to_joints(self, width):
        # reference panda.py:217-223
        w = np.clip(width, self.MIN_WIDTH_CLAMP, self.MAX_WIDTH)
        q1 = np.clip(w / 2.0, self.Q1_RANGE[0], self.Q1_RANGE[1])
        q2 = np.clip(-0.04 + w / 2.0, self.Q2_RANGE[0], self.Q2_RANGE[1])
        return q1, q2

    def _clamp_width(self, width):
        # reference panda.py:264-266
        return np.clip(width + 0.025, self.MIN_WIDTH_CLAMP, self.MAX_WIDTH)

    def get_actuator_joint_names(self) -> List[str]:
        return ["finger_joint1", "finger_joint2"]

    # ------------------------------------------------------------------
    def to_xml(self) -> Tuple[str, Dict[str, Any]]:
        data = np.load(_ASSET)
        pos = f"{self.pos[0]} {self.pos[1]} {self.pos[2]}"
        quat = f"{self.quat[0]} {self.quat[1]} {self.quat[2]} {self.quat[3]}"
        out = ["<asset>"]
        for m in ("hand_c", "finger_0"):
            out.append(f'<mesh name="{m}" vertex="{_fmt(data["hull_" + m])}"/>')
        out.append("</asset>")
        out.append("<worldbody>")
        out.append(f'<body name="mocap" mocap="true" pos="{pos}" quat="{quat}"/>')
        out.append(f'<body name="hand" quat="{quat}" pos="{pos}">')
        out.append('<freejoint name="freejoint"/>')
        out.append('<inertial mass="0.73" pos="-0.01 0 0.03" diaginertia="0.001 0.0025 0.0017"/>')
        out.append('<geom type="mesh" mesh="hand_c"/>')
        for body, bpos, bquat, jname, jrange, g0 in _FINGERS:
            q = f' quat="{bquat}"' if bquat else ""
            out.append(f'<body name="{body}" pos="{bpos}"{q}>')
            out.append('<inertial mass="0.015" pos="0 0 0" diaginertia="2.375e-6 2.375e-6 7.5e-7"/>')
            out.append(f'<joint name="{jname}" type="slide" axis="0 1 0" limited="true" range="{jrange}" '
                       'damping="100" armature="1.0" frictionloss="1.0"/>')
            out.append(f'<geom name="panda_col_{g0}" type="mesh" mesh="finger_0"/>')
            for k, (size, ppos) in enumerate(_PADS):
                out.append(f'<geom name="panda_col_{g0 + 1 + k}" type="box" size="{size}" pos="{ppos}" '
                           'friction="2.4 0.3 0.1"/>')
            out.append("</body>")
        out.append("</body></worldbody>")
        out.append('<contact><exclude body1="hand" body2="left_finger"/>'
                   '<exclude body1="hand" body2="right_finger"/></contact>')
        out.append('<tendon><fixed name="split"><joint joint="finger_joint1" coef="0.5"/>'
                   '<joint joint="finger_joint2" coef="0.5"/></fixed></tendon>')
        out.append('<equality><weld body1="mocap" body2="hand"/></equality>')
        out.append("<actuator>")
        for k, (_, _, _, jname, jrange, _) in enumerate(_FINGERS):
            out.append(f'<position name="gripper_finger_joint{k + 1}" joint="{jname}" kp="1000" '
                       f'ctrllimited="true" ctrlrange="{jrange}" forcelimited="true" forcerange="-15 15"/>')
        out.append("</actuator>")
        return "\n".join(out), {}
