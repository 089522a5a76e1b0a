"""Shadow Dexterous Hand, right (reference: mgs/gripper/shadow.py:348-455).

The MJCF is re-authored from the model's parameters (Menagerie-derived,
Apache-2.0; the reference template is shadow.py:32-345) rather than copied:

  * kinematic tree, explicit inertials, the per-class joint axes / ranges,
    damping 0.05, armature 2e-4, frictionloss 0.01, the "plastic" contact
    softness (solimp 0.5 0.99 1e-4, solref 0.005 1) with friction 3.5 on every
    collision geom, the four coupled middle/distal tendons, the 18 position
    servos (per-class kp, ctrl and force ranges), the thumb exclude and the
    mocap weld are kept;
  * the two fingertip collision meshes are emitted inline as the convex hulls
    MuJoCo collides (tools/derive_shadow_assets.py); visual geoms
    (contype=conaffinity=0) are dropped -- every body has an <inertial>.
"""
from __future__ import annotations

import os
from typing import Any, Dict, List, Tuple

import numpy as np

from mgs.gripper.base import MjShakableOpenCloseGripper, fmt32
from mgs.util.const import PACKAGE_PATH
from mgs.util.geo.transforms import SE3Pose

_ASSET = os.path.join(PACKAGE_PATH, "assets", "shadow.npz")

# joint classes: axis, range; servo kp, ctrlrange, forcerange  (shadow.py:37-92)
_CLS = {
    "thbase": ("0 0 -1", "-1.0472 1.0472", 0.4, "-1.0472 1.0472", "-30 30"),
    "thproximal": ("1 0 0", "0 1.22173", 1.0, "0 1.22173", "-20 20"),
    "thhub": ("1 0 0", "-0.20944 0.20944", 0.5, "-0.20944 0.20944", "-10 10"),
    "thmiddle": ("0 -1 0", "-0.698132 0.698132", 1.5, "-0.698132 0.698132", "-10 10"),
    "thdistal": ("1 0 0", "-0.261799 1.5708", 1.0, "-0.261799 1.5708", "-10 10"),
    "metacarpal": ("0.573576 0 0.819152", "0 0.785398", 1.0, "0 0.785398", "-10 10"),
    "knuckle": ("0 -1 0", "-0.349066 0.349066", 1.0, "-0.349066 0.349066", "-10 10"),
    "proximal": ("1 0 0", "-0.261799 1.5708", 1.0, "-0.261799 1.5708", "-10 10"),
    "middle_distal": ("1 0 0", "0 1.5708", 0.5, "0 3.1415", "-10 10"),
}
_PLASTIC = 'solimp="0.5 0.99 0.0001" solref="0.005 1" friction="3.5"'
_KNUCKLE_INERTIAL = '<inertial mass="0.008" pos="0 0 0" quat="0.5 0.5 -0.5 0.5" diaginertia="3.2e-07 2.6e-07 2.6e-07"/>'
_PROX_INERTIAL = '<inertial mass="0.03" pos="0 0 0.0225" quat="1 0 0 1" diaginertia="1e-05 9.8e-06 1.8e-06"/>'
_MID_INERTIAL = '<inertial mass="0.017" pos="0 0 0.0125" quat="1 0 0 1" diaginertia="2.7e-06 2.6e-06 8.7e-07"/>'
_DIST_INERTIAL = ('<inertial mass="0.013" pos="0 0 0.0130769" quat="1 0 0 1" '
                  'diaginertia="1.28092e-06 1.12092e-06 5.3e-07"/>')
# wrist collision geoms (shadow.py:133-139): type, size, pos, quat
_WRIST_GEOMS = [("cylinder", "0.0135 0.015", "0 0 0", "0.499998 0.5 0.5 -0.500002"),
                ("cylinder", "0.011 0.005", "-0.026 0 0.034", "1 0 1 0"),
                ("cylinder", "0.011 0.005", "0.031 0 0.034", "1 0 1 0"),
                ("box", "0.0135 0.009 0.005", "-0.021 0 0.011", "0.923879 0 0.382684 0"),
                ("box", "0.0135 0.009 0.005", "0.026 0 0.01", "0.923879 0 -0.382684 0")]
# palm collision boxes (shadow.py:144-153): size, pos, quat
_PALM_BOXES = [("0.031 0.0035 0.049", "0.011 0.0085 0.038", None),
               ("0.018 0.0085 0.049", "-0.002 -0.0035 0.038", None),
               ("0.013 0.0085 0.005", "0.029 -0.0035 0.082", None),
               ("0.013 0.007 0.009", "0.0265 -0.001 0.07", "0.987241 0.0990545 0.0124467 0.124052"),
               ("0.0105 0.0135 0.012", "0.0315 -0.0085 0.001", None),
               ("0.011 0.0025 0.015", "0.0125 -0.015 0.004", "0.971338 0 0 -0.237703"),
               ("0.009 0.012 0.002", "0.011 0 0.089", None),
               ("0.01 0.012 0.02", "-0.03 0 0.009", None)]
# fingers: prefix, knuckle body pos, knuckle axis override
_FINGERS = [("ff", "0.033 0 0.095", None), ("mf", "0.011 0 0.099", None), ("rf", "-0.011 0 0.095", "0 1 0")]

CLOSE_QPOS = np.array([-0.3464, 1.253, 0.7836, -0.001106, 0.01103, 1.475, 0.6181, 0.0155, -0.2083, 1.45, 0.75,
                       0.0, 0.13, -0.4, 1.5, 0.95, 0.35, 0.07708, 1.21, 0.2023, 0.6614, 0.0102])


def _joint(name, cls, axis=None):
    a, rng = _CLS[cls][0], _CLS[cls][1]
    return (f'<joint name="{name}" axis="{axis or a}" range="{rng}" damping="0.05" armature="0.0002" '
            'frictionloss="0.01"/>')


def _geom(t, size, pos=None, quat=None, extra=""):
    p = f' pos="{pos}"' if pos else ""
    q = f' quat="{quat}"' if quat else ""
    return f'<geom type="{t}" size="{size}"{p}{q} {_PLASTIC}{extra}/>'


class GripperShadowRight(MjShakableOpenCloseGripper):
    close_steps = 3000
    # in front of the palm (the template's grasp_site, shadow.py:142, moved off
    # the palm surface): where synthetic test candidates put the object centre
    grasp_site = np.array([0.0, -0.07, 0.125])

    def __init__(self, pose: SE3Pose, grasp_type=None):
        super().__init__(pose, "rh_wrist")

    def base_to_contact_transform(self) -> SE3Pose:
        # shadow.py:368-371: identity
        return SE3Pose(np.array([0, 0, 0.0]), np.array([1.0, 0.0, 0.0, 0.0]), type="wxyz")

    @staticmethod
    def _qpos_to_qacc(qpos):
        """22 joint targets -> 18 servo ctrls (shadow.py:444-455): thumb first,
        the coupled middle+distal joints summed onto their tendon servo."""
        acc = np.zeros((18,))
        acc[:5] = qpos[-5:]
        acc[5:7] = qpos[0:2]
        acc[7] = qpos[2] + qpos[3]
        acc[8:10] = qpos[4:6]
        acc[10] = qpos[6] + qpos[7]
        acc[11:13] = qpos[8:10]
        acc[13] = qpos[10] + qpos[11]
        acc[14:17] = qpos[12:15]
        acc[17] = qpos[15] + qpos[16]
        return acc

    def close_ctrl(self, sim) -> np.ndarray:
        # shadow.py:379-410
        return self._qpos_to_qacc(CLOSE_QPOS.copy())

    def open_ctrl(self, sim) -> np.ndarray:
        # shadow.py:373-377: open pose = zeros(22)
        return self._qpos_to_qacc(np.zeros(22))

    def open_joints(self) -> np.ndarray:
        return np.zeros(22)

    def get_actuator_joint_names(self) -> List[str]:
        return [f"rh_{f}J{k}" for f in ("FF", "MF", "RF") for k in (4, 3, 2, 1)] + \
               [f"rh_LFJ{k}" for k in (5, 4, 3, 2, 1)] + [f"rh_THJ{k}" for k in (5, 4, 3, 2, 1)]

    # ------------------------------------------------------------------
    @staticmethod
    def _finger(prefix, axis4):
        P = prefix.upper()
        return [_KNUCKLE_INERTIAL, _joint(f"rh_{P}J4", "knuckle", axis4),
                _geom("cylinder", "0.009 0.009", quat="1 0 1 0"),
                f'<body name="rh_{prefix}proximal">', _PROX_INERTIAL, _joint(f"rh_{P}J3", "proximal"),
                _geom("capsule", "0.009 0.02", pos="0 0 0.025"),
                f'<body name="rh_{prefix}middle" pos="0 0 0.045">', _MID_INERTIAL,
                _joint(f"rh_{P}J2", "middle_distal"), _geom("capsule", "0.009 0.0125", pos="0 0 0.0125"),
                f'<body name="rh_{prefix}distal" pos="0 0 0.025">', _DIST_INERTIAL,
                _joint(f"rh_{P}J1", "middle_distal"), f'<geom type="mesh" mesh="f_distal_pst" {_PLASTIC}/>',
                "</body></body></body>"]

    def to_xml(self) -> Tuple[str, Dict[str, Any]]:
        data = np.load(_ASSET)
        pos = f"{self.pos[0]} {self.pos[1]} {self.pos[2]}"
        quat = f"{self.quat[0]} {self.quat[1]} {self.quat[2]} {self.quat[3]}"
        out = ['<option cone="elliptic" impratio="10"/>', "<asset>"]
        for m in ("f_distal_pst", "th_distal_pst"):
            out.append(f'<mesh name="{m}" vertex="{fmt32(data["hull_" + m])}"/>')
        out += ["</asset>", "<worldbody>", f'<body name="mocap" mocap="true" pos="{pos}" quat="{quat}"/>',
                f'<body name="rh_wrist" pos="{pos}" quat="{quat}">', '<freejoint name="freejoint"/>',
                '<inertial mass="0.1" pos="0 0 0.029" quat="0.5 0.5 0.5 0.5" diaginertia="6.4e-05 4.38e-05 3.5e-05"/>']
        out += [_geom(t, s, p, q) for t, s, p, q in _WRIST_GEOMS]
        out += ['<body name="rh_palm" pos="0 0 0.034">',
                '<inertial mass="0.3" pos="0 0 0.035" quat="1 0 0 1" diaginertia="0.0005287 0.0003581 0.000191"/>']
        out += [_geom("box", s, p, q) for s, p, q in _PALM_BOXES]
        for prefix, kpos, axis4 in _FINGERS:
            out.append(f'<body name="rh_{prefix}knuckle" pos="{kpos}">')
            out += self._finger(prefix, axis4)
            out.append("</body>")
        out += ['<body name="rh_lfmetacarpal" pos="-0.033 0 0.02071">',
                '<inertial mass="0.03" pos="0 0 0.04" quat="1 0 0 1" diaginertia="1.638e-05 1.45e-05 4.272e-06"/>',
                _joint("rh_LFJ5", "metacarpal"), _geom("box", "0.011 0.012 0.025", pos="0.002 0 0.033"),
                '<body name="rh_lfknuckle" pos="0 0 0.06579">']
        out += self._finger("lf", "0 1 0")
        out += ["</body></body>"]
        # thumb (shadow.py:282-300)
        out += ['<body name="rh_thbase" pos="0.034 -0.00858 0.029" quat="0.92388 0 0.382683 0">',
                '<inertial mass="0.01" pos="0 0 0" diaginertia="1.6e-07 1.6e-07 1.6e-07"/>',
                _joint("rh_THJ5", "thbase"), _geom("sphere", "0.013"),
                '<body name="rh_thproximal">',
                '<inertial mass="0.04" pos="0 0 0.019" diaginertia="1.36e-05 1.36e-05 3.13e-06"/>',
                _joint("rh_THJ4", "thproximal"), _geom("capsule", "0.0105 0.009", pos="0 0 0.02"),
                '<body name="rh_thhub" pos="0 0 0.038">',
                '<inertial mass="0.005" pos="0 0 0" diaginertia="1e-06 1e-06 3e-07"/>',
                _joint("rh_THJ3", "thhub"), _geom("sphere", "0.011"),
                '<body name="rh_thmiddle">',
                '<inertial mass="0.02" pos="0 0 0.016" diaginertia="5.1e-06 5.1e-06 1.21e-06"/>',
                _joint("rh_THJ2", "thmiddle"), _geom("capsule", "0.009 0.009", pos="0 0 0.012"),
                _geom("sphere", "0.01", pos="0 0 0.03"),
                '<body name="rh_thdistal" pos="0 0 0.032" quat="1 0 0 -1">',
                '<inertial mass="0.017" pos="0 0 0.0145588" quat="1 0 0 1" '
                'diaginertia="2.37794e-06 2.27794e-06 1e-06"/>',
                _joint("rh_THJ1", "thdistal"), f'<geom type="mesh" mesh="th_distal_pst" {_PLASTIC}/>',
                "</body></body></body></body></body>"]
        out += ["</body></body></worldbody>",
                '<contact><exclude body1="rh_thproximal" body2="rh_thmiddle"/></contact>', "<tendon>"]
        for f in ("FF", "MF", "RF", "LF"):
            out.append(f'<fixed name="rh_{f}J0"><joint joint="rh_{f}J2" coef="1"/>'
                       f'<joint joint="rh_{f}J1" coef="1"/></fixed>')
        out.append("</tendon><actuator>")
        acts = [("THJ5", "thbase"), ("THJ4", "thproximal"), ("THJ3", "thhub"), ("THJ2", "thmiddle"),
                ("THJ1", "thdistal")]
        for f in ("FF", "MF", "RF"):
            acts += [(f"{f}J4", "knuckle"), (f"{f}J3", "proximal"), (f"{f}J0", "middle_distal")]
        acts += [("LFJ5", "metacarpal"), ("LFJ4", "knuckle"), ("LFJ3", "proximal"), ("LFJ0", "middle_distal")]
        for j, cls in acts:
            _, _, kp, crange, frange = _CLS[cls]
            trn = f'tendon="rh_{j}"' if j.endswith("J0") else f'joint="rh_{j}"'
            out.append(f'<position name="rh_A_{j}" {trn} kp="{kp}" ctrlrange="{crange}" forcerange="{frange}"/>')
        out.append('</actuator><equality><weld body1="mocap" body2="rh_wrist"/></equality>')
        return "\n".join(out), {}
