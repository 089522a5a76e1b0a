"""Derive the Franka Panda hand's collision hulls.

Run once, in the build container only (it reads the Menagerie meshes that ship
with the reference under /root/reference/asset/panda, Apache-2.0):

    python tools/derive_panda_assets.py

Output: mj-grasp-sim_amd/mgs/assets/panda.npz -- DERIVED DATA only: the convex
hull vertices (float32-rounded, as MuJoCo stores mesh vertices) of the two
meshes the reference template uses as collision geoms (`hand_c` = hand.stl,
`finger_0` = finger_0.obj; mgs/gripper/panda.py:65-67,96,104,114).  Every Panda
body has an explicit <inertial>, so no mesh mass properties are needed, and the
visual meshes (contype=conaffinity=0) have no physical effect.
No mesh file and no reference source is copied into the repository.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mj-grasp-sim_amd"))
from mgs.core.mjcf import convex_hull_vertices, load_mesh_bytes  # noqa: E402

SRC = "/root/reference/asset/panda"
DST = os.path.join(os.path.dirname(__file__), "..", "mj-grasp-sim_amd", "mgs", "assets", "panda.npz")
HULLS = {"hand_c": "hand.stl", "finger_0": "finger_0.obj"}


def main():
    if not os.path.isdir(SRC):
        print("reference meshes not found at", SRC)
        return 1
    out = {}
    for name, fname in HULLS.items():
        v, _ = load_mesh_bytes(open(os.path.join(SRC, fname), "rb").read(), fname)
        v = v.astype(np.float32).astype(np.float64)
        out["hull_" + name] = np.unique(convex_hull_vertices(v), axis=0)
    np.savez_compressed(DST, **out)
    for k, v in out.items():
        print(k, v.shape)
    return 0


if __name__ == "__main__":
    sys.exit(main())
