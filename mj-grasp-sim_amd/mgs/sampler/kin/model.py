"""Kinematic hand models for the contact-based sampler.

A model is data: per-dof static transforms (parent link -> joint frame, as
quaternion wxyz + translation), per-dof joint axes (prismatic direction and
revolute axis), joint ranges, the finger chains, the fingertip links with their
candidate contact points and contact normals, the pre-grasp joint vector and
the approach alignment.  The reference keeps the same tables on flax modules
(mgs/sampler/kin/base.py:15-31 the field list, mgs/sampler/kin/shadow.py:17-223
the Shadow Hand values); the forward kinematics that consumes them is
forward_kinematic_point_transform (base.py:80-113), restated in
csrc/mgs_contact.hip (device) and oracle/mgs_contact_oracle.c (checker).

Only the Shadow Hand is provided: it is the dexterous hand whose simulation
(mgs.gripper.shadow) this build evaluates; the LEAP hand has no gripper model
here, so its kinematic table is not carried.
"""
from dataclasses import dataclass, field

import numpy as np


@dataclass
class KinematicsModel:
    name: str
    chains: list                     # dof indices per finger, root first
    kin_tf: np.ndarray               # (ndof, 7): parent -> joint frame, wxyz + xyz
    joint_tf: np.ndarray             # (ndof, 6): prismatic direction, revolute axis
    joint_ranges: np.ndarray         # (ndof, 2)
    fingertip_idx: np.ndarray        # (ntip,) link (dof) index of each fingertip
    tip_contacts: np.ndarray         # (ntip, ncand, 3) candidate contact points, tip frame
    tip_normals: np.ndarray          # (ntip, 3) contact normal, tip frame
    pregrasp: np.ndarray             # (ndof,) initial joints
    align_rot: np.ndarray            # (3, 3) approach alignment (right-multiplied)
    align_pos: np.ndarray            # (3,)
    extra: dict = field(default_factory=dict)

    @property
    def num_dofs(self):
        return len(self.kin_tf)

    def parents(self):
        """parent dof of each dof (-1: the palm), in the reference's parent_map
        construction (base.py:91-95)"""
        par = np.full(self.num_dofs, -1, np.int32)
        for ch in self.chains:
            for a, b in zip(ch[:-1], ch[1:]):
                par[b] = a
        return par


def _shadow():
    s2 = 1.0 / np.sqrt(2.0)
    palm = 0.034          # wrist -> palm frame offset folded into the finger roots
    # per finger: (root offset xyz, root quaternion, link lengths along z)
    ff = [0.033, 0.0, 0.095 + palm]
    mf = [0.011, 0.0, 0.099 + palm]
    rf = [-0.011, 0.0, 0.095 + palm]
    lf = [-0.033, 0.0, 0.02071 + palm]
    th = [0.034, -0.00858, 0.029 + palm]
    I = [1.0, 0.0, 0.0, 0.0]
    rows = []
    for root in (ff, mf, rf):
        rows += [I + root, I + [0, 0, 0.0], I + [0, 0, 0.045], I + [0, 0, 0.025]]
    rows += [I + lf, I + [0, 0, 0.06579], I + [0, 0, 0.0], I + [0, 0, 0.045], I + [0, 0, 0.025]]
    rows += [[0.92388, 0.0, 0.382683, 0.0] + th, I + [0, 0, 0.0], I + [0, 0, 0.038], I + [0, 0, 0.0],
             [s2, 0.0, 0.0, -s2, 0.0, 0.0, 0.032]]
    X, Y, Z = [1.0, 0, 0], [0, 1.0, 0], [0, 0, 1.0]
    neg = lambda v: [-c for c in v]  # noqa: E731
    axes = [neg(Y), X, X, X] + [neg(Y), X, X, X] + [Y, X, X, X] + \
        [[0.573576, 0.0, 0.819152], Y, X, X, X] + [neg(Z), X, X, neg(Y), X]
    jt = np.array([[0.0, 0.0, 0.0] + a for a in axes])
    knuckle, prox, mid = [-0.349066, 0.349066], [-0.261799, 1.5708], [0.0, 1.5708]
    ranges = [knuckle, prox, mid, mid] * 3 + [[0.0, 0.785398], knuckle, prox, mid, mid] + \
        [[-1.0472, 1.0472], [0.0, 1.22173], [-0.20944, 0.20944], [-0.698132, 0.698132], [-0.261799, 1.5708]]
    tips = np.array([3, 7, 11, 16, 21], np.int32)
    one = [[0.0, -0.01, 0.0], [0.0, -0.01, 0.01], [0.0, -0.01, -0.01]]
    pre = [-0.350, 0.425, 0.015, 0.005, -0.095, 0.415, 0.010, 0.0, -0.075, 0.435, 0.015, 0.005,
           0.0, -0.220, 0.255, 0.0, 0.0, -0.480, 1.05, -0.19, -0.080, 0.45]
    return KinematicsModel(
        name="ShadowHand",
        chains=[[0, 1, 2, 3], [4, 5, 6, 7], [8, 9, 10, 11], [12, 13, 14, 15, 16], [17, 18, 19, 20, 21]],
        kin_tf=np.array(rows, np.float64),
        joint_tf=jt,
        joint_ranges=np.array(ranges, np.float64),
        fingertip_idx=tips,
        tip_contacts=np.array([one] * 5, np.float64),
        tip_normals=np.tile([0.0, 1.0, 0.0], (5, 1)),
        pregrasp=np.array(pre, np.float64),
        align_rot=np.array([[0.0, 0, 1.0], [1.0, 0.0, 0], [0.0, 1.0, 0.0]]),
        align_pos=np.array([-0.1, 0.0, 0.0]),
    )


def ShadowKinematicsModel():
    """the Shadow Hand table (reference mgs/sampler/kin/shadow.py:17-223)"""
    return _shadow()


def get_kinematics(name):
    if name == "ShadowHand":
        return ShadowKinematicsModel()
    raise ValueError(f"no kinematic model for gripper {name!r} (ShadowHand only; SURVEY.md §8a-4)")
