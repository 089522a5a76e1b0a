"""Object factory (reference: mgs/obj/selector.py:33-246)."""
import os
import random
import secrets

import numpy as np

from mgs.obj.base import CollisionMeshObject
from mgs.obj.gso import ObjectGSO
from mgs.obj.ycb import ObjectYCB
from mgs.util.const import ASSET_PATH
from mgs.util.geo.transforms import SE3Pose


def generate_unique_hash(length=16):
    return secrets.token_hex(length)


def _make(cls, oid, pos=(0.0, 0.0, 0.0), name=None):
    pose = SE3Pose(np.array([float(p) for p in pos]), np.array([1, 0, 0, 0]), type="wxyz")
    return cls(pose, object_id=oid, name=name or generate_unique_hash())


def get_object(id, name=None) -> CollisionMeshObject:
    ycb = [o for o in ObjectYCB.all_object_ids() if o == id]
    gso = [o for o in ObjectGSO.all_object_ids() if o == id]
    if len(ycb) + len(gso) != 1:
        raise AssertionError(f"object {id!r} not found exactly once")
    return _make(ObjectGSO if gso else ObjectYCB, id, name=name)


def parked_objects(chosen):
    """selector.py:149-182: (class, id) pairs placed off the drop zone, ten per
    row: x = -8.5 + 0.5 per started row, y = -8 + 0.5 within the row."""
    out, x, y = [], -8.5, -8.0
    for i, (cls, oid) in enumerate(chosen):
        if i % 10 == 0:
            x += 0.5
            y = -8.0
        else:
            y += 0.5
        out.append(_make(cls, oid, (x, y, 0.0)))
    return out


def _pool(ids):
    """(class, id) of the YCB then GSO objects whose id is in `ids`."""
    keep = set(ids)
    return [(ObjectYCB, i) for i in ObjectYCB.all_object_ids() if i in keep] + \
           [(ObjectGSO, i) for i in ObjectGSO.all_object_ids() if i in keep]


def get_objects(cfg, rng=None):
    """selector.py:54-246.  Random subsets draw from `rng` (a random.Random or a
    seed) instead of the global `random` module.  Full_Data_Subset: the
    reference restricts the draw to mgs/cli/stats/graspable_object_set.pickle, a
    pickle this build never loads, so every YCB / GSO object is eligible."""
    r = rng if isinstance(rng, random.Random) else random.Random(rng)
    name = cfg["name"]
    if name == "SingleObject":
        return [get_object(cfg["id"])]
    if name == "YCB":
        return [_make(ObjectYCB, i) for i in sorted(ObjectYCB.all_object_ids())]
    if name == "GSO":
        return [_make(ObjectGSO, i) for i in ObjectGSO.all_object_ids()]
    if name == "Full_Dataset":
        return [_make(ObjectGSO, i) for i in sorted(ObjectGSO.all_object_ids())] + \
               [_make(ObjectYCB, i) for i in sorted(ObjectYCB.all_object_ids())]
    if name == "Fast_Data_Subset":
        with open(os.path.join(ASSET_PATH, "mj-objects", "fast_eta_objects.txt")) as f:
            pool = _pool(f.read().splitlines())
        return parked_objects(r.choices(pool, k=int(cfg["num_objects"])))
    if name == "Full_Data_Subset":
        k = r.randint(int(cfg["num_objects_min"]), int(cfg["num_objects_max"]))
        pool = _pool(ObjectYCB.all_object_ids() + ObjectGSO.all_object_ids())
        return parked_objects(r.choices(pool, k=k))
    raise ValueError(f"Unknown object set {name!r}")
