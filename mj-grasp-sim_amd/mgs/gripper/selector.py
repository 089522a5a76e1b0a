"""Gripper factory (reference: mgs/gripper/selector.py:33-66)."""
import numpy as np

from mgs.gripper.base import MjShakableOpenCloseGripper
from mgs.gripper.allegro import GripperAllegro
from mgs.gripper.dexee import GripperDexee
from mgs.gripper.panda import GripperPanda
from mgs.gripper.robotiq2f85 import GripperRobotiq2f85
from mgs.gripper.shadow import GripperShadowRight
from mgs.util.geo.transforms import SE3Pose

_GRIPPERS = {"Robotiq2f85Gripper": GripperRobotiq2f85, "PandaGripper": GripperPanda,
             "AllegroGripper": GripperAllegro,
             "ShadowHand": GripperShadowRight, "DexeeGripper": GripperDexee}


def get_gripper(cfg, default_pose=None) -> MjShakableOpenCloseGripper:
    pose = SE3Pose(np.array([0, 0, 0]), np.array([1, 0, 0, 0]), type="wxyz") if default_pose is None else default_pose
    name = cfg["name"] if isinstance(cfg, dict) else cfg.name
    if name not in _GRIPPERS:
        raise ValueError(f"Unknown gripper: {name}")
    return _GRIPPERS[name](pose)


def gripper_class(class_name: str):
    """gripper class by its Python class name (scene files store it)."""
    for cls in _GRIPPERS.values():
        if cls.__name__ == class_name:
            return cls
    raise ValueError(f"Unknown gripper class: {class_name}")
