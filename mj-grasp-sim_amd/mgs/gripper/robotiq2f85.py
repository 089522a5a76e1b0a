"""Robotiq 2F-85 gripper (reference: mgs/gripper/robotiq2f85.py:228-284).

The MJCF is re-authored from the model's parameters (Menagerie-derived, BSD-2;
the reference template is robotiq2f85.py:32-225) rather than copied:

  * every body, inertial, joint, equality, tendon and actuator parameter of the
    reference template is kept (including its edits to Menagerie: elliptic cone,
    impratio 10, armature 0.001 on coupler/spring_link/follower, pad friction 0.8,
    the mocap body + free joint + weld, forcerange +-100);
  * collision meshes are emitted inline (`<mesh vertex=...>`) as the convex
    hulls of the Menagerie meshes -- MuJoCo collides meshes through their hull,
    so the contact geometry is unchanged (tools/derive_robotiq_assets.py);
  * visual geoms (contype=0) are dropped; the only physical effect they had is
    mass on bodies without <inertial> (base_mount: visual + collision mesh at
    density 1000; the silicone pads: visual mesh), which is folded into
    explicit <inertial> elements computed from the same meshes.
"""
from __future__ import annotations

import os
from typing import Any, Dict, List, Tuple

import numpy as np

from mgs.gripper.base import MjShakableOpenCloseGripper
from mgs.util.const import PACKAGE_PATH
from mgs.util.geo.transforms import SE3Pose

_ASSET = os.path.join(PACKAGE_PATH, "assets", "robotiq2f85.npz")

# limit/equality softness shared by driver, coupler, follower and the 4-bar equalities
_SOFT = dict(solimp="0.95 0.99 0.001", solref="0.005 1")

# (name, parent, pos, quat, inertial(mass,pos,quat,diag) | None, joint | None, collision mesh | None)
_LINKS = [
    ("base", "base_mount", "0 0 0.0038", "1 0 0 -1",
     ("0.777441", "0 -2.70394e-05 0.0354675", "1 -0.00152849 0 0", "0.000260285 0.000225381 0.000152708"),
     None, "base"),
]
_SIDE = {
    "right": dict(driver_pos="0 0.0306011 0.054904", spring_pos="0 0.0132 0.0609", quat=None,
                  driver_ipos="2.96931e-12 0.0177547 0.00107314", pad_iquat="0.707107 0 0 0.707107"),
    "left": dict(driver_pos="0 -0.0306011 0.054904", spring_pos="0 -0.0132 0.0609", quat="0 0 0 1",
                 driver_ipos="0 0.0177547 0.00107314", pad_iquat="1 0 0 1"),
}
_PAD_BOX = dict(size="0.011 0.004 0.009375", friction="0.8", solimp="0.95 0.99 0.001",
                solref="0.004 1", priority="1", mass="0")


def _fmt(v):
    return " ".join(repr(float(np.float32(x))) if abs(x) > 0 else "0" for x in np.ravel(v))


def _inertial_from_mesh(vol, com, inertia, density, copies):
    mass = density * vol * copies
    w, V = np.linalg.eigh(inertia * density * copies)
    if np.linalg.det(V) < 0:
        V[:, 2] = -V[:, 2]
    from mgs.core.mjcf import mat2quat
    return mass, com, mat2quat(V), w


class GripperRobotiq2f85(MjShakableOpenCloseGripper):
    close_steps = 3000

    def __init__(self, pose: SE3Pose):
        super().__init__(pose, "base_mount")

    def base_to_contact_transform(self) -> SE3Pose:
        # reference robotiq2f85.py:232-235
        return SE3Pose(np.array([0.0, 0.0, -0.15]), np.array([1, 0, 0, 0]), type="wxyz")

    def close_ctrl(self, sim) -> np.ndarray:
        # reference robotiq2f85.py:243: sim.data.ctrl[:] = 255.0
        return np.full(sim.model.nu, 255.0)

    def get_actuator_joint_names(self) -> List[str]:
        # kept verbatim, including the reference's "*_spring_link" names that do
        # not exist in the model (robotiq2f85.py:271-281): the
        # lookup then falls back to the last joint's qpos address.
        return ["right_driver_joint", "right_coupler_joint", "right_spring_link",
                "right_follower_joint", "left_driver_joint", "left_coupler_joint",
                "left_spring_link", "left_follower_joint"]

    # ------------------------------------------------------------------
    def to_xml(self) -> Tuple[str, Dict[str, Any]]:
        data = np.load(_ASSET)
        pos = f"{self.pos[0]} {self.pos[1]} {self.pos[2]}"
        quat = f"{self.quat[0]} {self.quat[1]} {self.quat[2]} {self.quat[3]}"
        out = ['<compiler angle="radian" autolimits="true"/>',
               '<option cone="elliptic" impratio="10"/>', "<asset>"]
        for m in ["base_mount", "base", "driver", "coupler", "follower", "spring_link"]:
            out.append(f'<mesh name="{m}" vertex="{_fmt(data["hull_" + m])}"/>')
        out.append("</asset>")
        bm = _inertial_from_mesh(float(data["vol_base_mount"]), data["com_base_mount"],
                                 data["inertia_base_mount"], 1000.0, 2)
        sp = _inertial_from_mesh(float(data["vol_silicone_pad"]), data["com_silicone_pad"],
                                 data["inertia_silicone_pad"], 1000.0, 1)
        out.append("<worldbody>")
        out.append(f'<body name="mocap" mocap="true" pos="{pos}" quat="{quat}"/>')
        out.append(f'<body name="base_mount" pos="{pos}" quat="{quat}">')
        out.append('<freejoint name="freejoint"/>')
        out.append(f'<inertial mass="{bm[0]!r}" pos="{_fmt(bm[1])}" quat="{_fmt(bm[2])}" '
                   f'diaginertia="{_fmt(bm[3])}"/>')
        out.append('<geom type="mesh" mesh="base_mount"/>')
        name, parent, bpos, bquat, ine, _, mesh = _LINKS[0]
        out.append(f'<body name="{name}" pos="{bpos}" quat="{bquat}">')
        out.append(f'<inertial mass="{ine[0]}" pos="{ine[1]}" quat="{ine[2]}" diaginertia="{ine[3]}"/>')
        out.append(f'<geom type="mesh" mesh="{mesh}"/>')
        for side in ("right", "left"):
            s = _SIDE[side]
            q = f' quat="{s["quat"]}"' if s["quat"] else ""
            # driver -> coupler
            out.append(f'<body name="{side}_driver" pos="{s["driver_pos"]}"{q}>')
            out.append(f'<inertial mass="0.00899563" pos="{s["driver_ipos"]}" quat="0.681301 0.732003 0 0" '
                       'diaginertia="1.72352e-06 1.60906e-06 3.22006e-07"/>')
            out.append(f'<joint name="{side}_driver_joint" axis="1 0 0" range="0 0.8" armature="0.005" '
                       f'damping="0.1" solimplimit="{_SOFT["solimp"]}" solreflimit="{_SOFT["solref"]}"/>')
            out.append('<geom type="mesh" mesh="driver"/>')
            out.append(f'<body name="{side}_coupler" pos="0 0.0315 -0.0041">')
            out.append('<inertial mass="0.0140974" pos="0 0.00301209 0.0232175" '
                       'quat="0.705636 -0.0455904 0.0455904 0.705636" '
                       'diaginertia="4.16206e-06 3.52216e-06 8.88131e-07"/>')
            out.append(f'<joint name="{side}_coupler_joint" axis="1 0 0" range="-1.57 0" armature="0.001" '
                       f'solimplimit="{_SOFT["solimp"]}" solreflimit="{_SOFT["solref"]}"/>')
            out.append('<geom type="mesh" mesh="coupler"/>')
            out.append("</body></body>")
            # spring link -> follower -> pad -> silicone pad
            out.append(f'<body name="{side}_spring_link" pos="{s["spring_pos"]}"{q}>')
            out.append('<inertial mass="0.0221642" pos="-8.65005e-09 0.0181624 0.0212658" '
                       'quat="0.663403 -0.244737 0.244737 0.663403" '
                       'diaginertia="8.96853e-06 6.71733e-06 2.63931e-06"/>')
            out.append(f'<joint name="{side}_spring_link_joint" axis="1 0 0" range="-0.29670597283 0.8" '
                       'armature="0.001" stiffness="0.05" springref="2.62" damping="0.00125"/>')
            out.append('<geom type="mesh" mesh="spring_link"/>')
            out.append(f'<body name="{side}_follower" pos="0 0.055 0.0375">')
            out.append('<inertial mass="0.0125222" pos="0 -0.011046 0.0124786" quat="1 0.1664 0 0" '
                       'diaginertia="2.67415e-06 2.4559e-06 6.02031e-07"/>')
            out.append(f'<joint name="{side}_follower_joint" axis="1 0 0" range="-0.872664 0.872664" '
                       f'armature="0.001" pos="0 -0.018 0.0065" solimplimit="{_SOFT["solimp"]}" '
                       f'solreflimit="{_SOFT["solref"]}"/>')
            out.append('<geom type="mesh" mesh="follower"/>')
            out.append(f'<body name="{side}_pad" pos="0 -0.0189 0.01352">')
            pb = " ".join(f'{k}="{v}"' for k, v in _PAD_BOX.items())
            out.append(f'<geom name="{side}_pad1" type="box" pos="0 -0.0026 0.028125" {pb}/>')
            out.append(f'<geom name="{side}_pad2" type="box" pos="0 -0.0026 0.009375" {pb}/>')
            out.append(f'<inertial mass="0.0035" pos="0 -0.0025 0.0185" quat="{s["pad_iquat"]}" '
                       'diaginertia="4.73958e-07 3.64583e-07 1.23958e-07"/>')
            out.append(f'<body name="{side}_silicone_pad">')
            out.append(f'<inertial mass="{sp[0]!r}" pos="{_fmt(sp[1])}" quat="{_fmt(sp[2])}" '
                       f'diaginertia="{_fmt(sp[3])}"/>')
            out.append("</body></body></body></body>")
        out.append("</body></body></worldbody>")
        out.append("<contact>")
        for b1, b2 in [("base", "left_driver"), ("base", "right_driver"), ("base", "left_spring_link"),
                       ("base", "right_spring_link"), ("right_coupler", "right_follower"),
                       ("left_coupler", "left_follower")]:
            out.append(f'<exclude body1="{b1}" body2="{b2}"/>')
        out.append("</contact>")
        out.append('<tendon><fixed name="split"><joint joint="right_driver_joint" coef="0.5"/>'
                   '<joint joint="left_driver_joint" coef="0.5"/></fixed></tendon>')
        out.append("<equality>")
        for side in ("right", "left"):
            out.append(f'<connect anchor="0 0 0" body1="{side}_follower" body2="{side}_coupler" '
                       f'solimp="{_SOFT["solimp"]}" solref="{_SOFT["solref"]}"/>')
        out.append('<joint joint1="right_driver_joint" joint2="left_driver_joint" polycoef="0 1 0 0 0" '
                   f'solimp="{_SOFT["solimp"]}" solref="{_SOFT["solref"]}"/>')
        out.append('<weld body1="mocap" body2="base_mount"/>')
        out.append("</equality>")
        out.append('<actuator><general name="fingers_actuator" tendon="split" forcerange="-100 100" '
                   'ctrlrange="0 255" gainprm="0.3137255 0 0" biasprm="0 -100 -10" biastype="affine"/>'
                   "</actuator>")
        return "\n".join(out), {}
