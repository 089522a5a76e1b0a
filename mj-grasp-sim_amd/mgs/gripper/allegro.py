"""Wonik Allegro hand, right (reference: mgs/gripper/allegro.py:254-361).

The MJCF is re-authored from the model's parameters (Menagerie-derived,
BSD-2; the reference template is allegro.py:32-251) rather than copied:

  * kinematic tree, joint axes/ranges (per finger-segment class), damping 0.1,
    the 16 position servos (kp 1, ctrlrange = joint range), the massless
    collision boxes and fingertip capsules, the palm excludes and the
    mocap weld are kept;
  * the template has no <inertial> (allegro.py:158 is commented out), so
    MuJoCo derives every body's mass from its density-800 visual mesh; the
    visual geoms (contype=conaffinity=0) are dropped and replaced by the
    equivalent explicit <inertial> (tools/derive_allegro_assets.py).
"""
from __future__ import annotations

import os
from typing import Any, Dict, List, Tuple

import numpy as np

from mgs.gripper.base import MjShakableOpenCloseGripper, mesh_inertial_xml
from mgs.util.const import PACKAGE_PATH
from mgs.util.geo.transforms import SE3Pose

_ASSET = os.path.join(PACKAGE_PATH, "assets", "allegro.npz")
_DENSITY = 800.0

# segment classes: joint axis, range; collision box (half sizes, pos)   (allegro.py:65-133)
_SEG = {
    "base": ("0 0 1", "-0.47 0.47", "0.0098 0.01375 0.0082", "0 0 0.0082"),
    "proximal": ("0 1 0", "-0.196 1.61", "0.0098 0.01375 0.027", "0 0 0.027"),
    "medial": ("0 1 0", "-0.174 1.709", "0.0098 0.01375 0.0192", "0 0 0.0192"),
    "distal": ("0 1 0", "-0.227 1.618", "0.0098 0.01375 0.008", "0 0 0.008"),
    "thumb_base": ("-1 0 0", "0.263 1.396", "0.0179 0.017 0.02275", "-0.0179 0.009 0.0145"),
    "thumb_proximal": ("0 0 1", "-0.105 1.163", "0.0098 0.01375 0.00885", "0 0 0.00885"),
    "thumb_medial": ("0 1 0", "-0.189 1.644", "0.0098 0.01375 0.0257", "0 0 0.0257"),
    "thumb_distal": ("0 1 0", "-0.162 1.719", "0.0098 0.01375 0.0157", "0 0 0.0157"),
}
# fingers: prefix, base pos, base quat, segment classes, visual meshes, segment offsets, tip
_FINGERS = [
    ("ff", "0 0.0435 -0.001542", "0.999048 -0.0436194 0 0"),
    ("mf", "0 0 0.0007", None),
    ("rf", "0 -0.0435 -0.001542", "0.999048 0.0436194 0 0"),
]
_FINGER_SEGS = [("base", "link_0.0", None), ("proximal", "link_1.0", "0 0 0.0164"),
                ("medial", "link_2.0", "0 0 0.054"), ("distal", "link_3.0", "0 0 0.0384")]
_THUMB_SEGS = [("thumb_base", "link_12.0_right", None), ("thumb_proximal", "link_13.0", "-0.027 0.005 0.0399"),
               ("thumb_medial", "link_14.0", "0 0 0.0177"), ("thumb_distal", "link_15.0", "0 0 0.0514")]
_THUMB_POS, _THUMB_QUAT = "-0.0182 0.019333 -0.045987", "0.477714 -0.521334 -0.521334 -0.477714"
# tips: visual mesh offset, capsule (radius half-length), capsule pos
_TIP = ("link_3.0_tip", 0.0267, "0.012 0.01", "0 0 0.019")
_THUMB_TIP = ("link_15.0_tip", 0.0423, "0.012 0.008", "0 0 0.035")

OPEN_POSE = np.array([-0.08, 0.715, 0.710, 0.95, 0, 0.8, 0.71, 0.67, 0.08, 0.715, 0.710, 0.95,
                      1.4, 0.55, -0.19, 1.45])
CLOSE_POSE = np.array([-0.08, 0.95, 1, 0.95, 0, 0.95, 1.2, 0.85, 0.08, 0.95, 1.2, 0.9,
                       1.4, 0.55, 0.29, 1.45])


class GripperAllegro(MjShakableOpenCloseGripper):
    close_steps = 3000

    def __init__(self, pose: SE3Pose):
        super().__init__(pose, "palm")
        self.open_pose = OPEN_POSE.copy()      # allegro.py:255-274
        self.close_pose = CLOSE_POSE.copy()    # allegro.py:275-294

    def base_to_contact_transform(self) -> SE3Pose:
        # allegro.py:296-302: rotate -90 deg about y, offset (-0.08, 0, 0.01) in that frame
        theta = -np.pi / 2.0
        q = np.array([np.cos(theta / 2.0), 0.0, np.sin(theta / 2.0), 0.0])
        rot = SE3Pose(np.array([0, 0, 0]), q, type="wxyz")
        off = rot @ SE3Pose(np.array([-0.08, 0.0, 0.01]), np.array([1.0, 0, 0, 0]), type="wxyz")
        return SE3Pose(off.pos, q, type="wxyz")

    def close_ctrl(self, sim) -> np.ndarray:
        # allegro.py:354-357: set_pose (no state change after the env's own
        # set_pose + forward), ctrl = close_pose, 3000 steps
        return self.close_pose.copy()

    def open_ctrl(self, sim) -> np.ndarray:
        return self.open_pose.copy()

    def get_actuator_joint_names(self) -> List[str]:
        return [f"{f}j{k}" for f in ("ff", "mf", "rf", "th") for k in range(4)]

    # ------------------------------------------------------------------
    def to_xml(self) -> Tuple[str, Dict[str, Any]]:
        data = np.load(_ASSET)

        def inertial(mesh, z=0.0):
            return mesh_inertial_xml(float(data["vol_" + mesh]), data["com_" + mesh], data["inertia_" + mesh],
                                     _DENSITY, (0.0, 0.0, z))

        def chain(prefix, segs, tip, first_pos, first_quat):
            out, depth = [], 0
            for k, (cls, mesh, pos) in enumerate(segs):
                axis, rng, bsize, bpos = _SEG[cls]
                bp = first_pos if k == 0 else pos
                q = f' quat="{first_quat}"' if (k == 0 and first_quat) else ""
                seg = {"base": "base", "proximal": "proximal", "medial": "medial", "distal": "distal"}.get(
                    cls, cls.replace("thumb_", ""))
                out.append(f'<body name="{prefix}_{seg}" pos="{bp}"{q}>')
                out.append(inertial(mesh))
                out.append(f'<joint name="{prefix}j{k}" axis="{axis}" range="{rng}" damping="0.1"/>')
                out.append(f'<geom type="box" size="{bsize}" pos="{bpos}" mass="0"/>')
                depth += 1
            tmesh, tz, csize, cpos = tip
            out.append(f'<body name="{prefix}_tip">')
            out.append(inertial(tmesh, tz))
            out.append(f'<geom type="capsule" size="{csize}" pos="{cpos}" mass="0"/>')
            out.append("</body>" * (depth + 1))
            return out

        pos = f"{self.pos[0]} {self.pos[1]} {self.pos[2]}"
        quat = f"{self.quat[0]} {self.quat[1]} {self.quat[2]} {self.quat[3]}"
        out = ["<worldbody>", f'<body name="mocap" mocap="true" pos="{pos}" quat="{quat}"/>',
               f'<body name="palm" pos="{pos}" quat="{quat}">', '<freejoint name="freejoint"/>',
               inertial("base_link"),
               '<geom type="box" size="0.0204 0.0565 0.0475" pos="-0.0093 0 -0.0475" mass="0"/>']
        for prefix, bpos, bquat in _FINGERS:
            out += chain(prefix, _FINGER_SEGS, _TIP, bpos, bquat)
        out += chain("th", _THUMB_SEGS, _THUMB_TIP, _THUMB_POS, _THUMB_QUAT)
        out.append("</body></worldbody>")
        out.append('<equality><weld body1="mocap" body2="palm"/></equality>')
        out.append("<contact>" + "".join(f'<exclude body1="palm" body2="{b}"/>' for b in
                                         ("ff_base", "mf_base", "rf_base", "th_base", "th_proximal")) + "</contact>")
        out.append("<actuator>")
        classes = [c for c, _, _ in _FINGER_SEGS] * 3 + [c for c, _, _ in _THUMB_SEGS]
        for name, cls in zip(self.get_actuator_joint_names(), classes):
            out.append(f'<position name="{name.replace("j", "a")}" joint="{name}" kp="1" ctrlrange="{_SEG[cls][1]}"/>')
        out.append("</actuator>")
        return "\n".join(out), {}
