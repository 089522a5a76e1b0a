"""Gripper protocol (reference: mgs/gripper/base.py:30-147).

The reference's grippers drive a MuJoCo MjData directly (`set_pose` writes the
free joint and the mocap, `close_gripper_at` sets ctrl and calls mj_step).  In
this engine a whole batch of candidates is stepped on the GPU, so a gripper
describes its close phase as data instead:

  * `to_xml()`                  -> (MJCF fragment, assets)        same as reference
  * `base_to_contact_transform()`                                  same as reference
  * `get_actuator_joint_names()`                                   same as reference
  * `close_ctrl(sim)`           -> ctrl vector applied during the close phase
  * `close_steps`               -> steps of the close phase (reference: 3000)

`set_pose` semantics (free-joint qpos[0:7] and mocap[0] both set to the
processed pose, gripper/base.py:48-59) are applied by the environment when it
builds the per-candidate initial state.
"""
from __future__ import annotations

from abc import ABC, abstractmethod
from typing import Any, Dict, List, Tuple

import numpy as np

from mgs.util.geo.transforms import SE3Pose


class MjGripper(ABC):
    pos: np.ndarray
    quat: np.ndarray
    base: str

    def __init__(self, pose: SE3Pose, base_body: str):
        v = pose.to_vec(layout="pq", type="wxyz")
        self.pos, self.quat = v[:3], v[3:]
        self.base = base_body

    def set_load_pose(self, pose: SE3Pose):
        v = pose.to_vec(layout="pq", type="wxyz")
        self.pos, self.quat = v[:3], v[3:]

    @abstractmethod
    def to_xml(self) -> Tuple[str, Dict[str, Any]]:
        ...

    @abstractmethod
    def get_actuator_joint_names(self) -> List[str]:
        ...

    @abstractmethod
    def base_to_contact_transform(self) -> SE3Pose:
        ...

    def get_freejoint_idxs(self, sim) -> List[int]:
        start = sim.get_joint_idxs(["freejoint"])[0]
        return list(range(start, start + 7))


class MjShakableOpenCloseGripper(MjGripper):
    """Open/close + shake protocol; the close phase is described by data."""

    close_steps: int = 3000

    @abstractmethod
    def close_ctrl(self, sim) -> np.ndarray:
        """ctrl vector set by close_gripper_at (e.g. Robotiq: [255])."""

    def open_ctrl(self, sim) -> np.ndarray:
        return np.zeros(sim.model.nu)

    def open_joints(self) -> np.ndarray:
        """actuated-joint values of the open hand (order of get_actuator_joint_names)."""
        return np.asarray(self.open_ctrl(None), dtype=np.float64)


def fmt32(v) -> str:
    """space-separated float32-rounded values (MJCF attribute text)."""
    return " ".join(repr(float(np.float32(x))) if abs(x) > 0 else "0" for x in np.ravel(v))


def mesh_inertial_xml(vol, com, inertia, density, offset=(0.0, 0.0, 0.0)) -> str:
    """<inertial> equal to MuJoCo's mass from one mesh geom at `density`, placed
    at `offset` in the body frame (geom pos, identity geom orientation)."""
    from mgs.core.mjcf import mat2quat
    w, V = np.linalg.eigh(np.asarray(inertia) * density)
    if np.linalg.det(V) < 0:
        V[:, 2] = -V[:, 2]
    pos = np.asarray(com) + np.asarray(offset)
    return (f'<inertial mass="{float(density * vol)!r}" pos="{fmt32(pos)}" quat="{fmt32(mat2quat(V))}" '
            f'diaginertia="{fmt32(w)}"/>')
