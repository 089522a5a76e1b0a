"""Object factory (reference: mgs/obj/selector.py:33-51)."""
import secrets

import numpy as np

from mgs.obj.base import CollisionMeshObject
from mgs.obj.gso import ObjectGSO
from mgs.obj.ycb import ObjectYCB
from mgs.util.geo.transforms import SE3Pose


def generate_unique_hash(length=16):
    return secrets.token_hex(length)


def get_object(id, name=None) -> CollisionMeshObject:
    ycb = [o for o in ObjectYCB.all_object_ids() if o == id]
    gso = [o for o in ObjectGSO.all_object_ids() if o == id]
    if len(ycb) + len(gso) != 1:
        raise AssertionError(f"object {id!r} not found exactly once")
    pose = SE3Pose(np.array([0, 0, 0]), np.array([1, 0, 0, 0]), type="wxyz")
    cls = ObjectGSO if gso else ObjectYCB
    return cls(pose, object_id=id, name=name or generate_unique_hash())
