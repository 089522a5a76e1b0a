"""Derive the Shadow Hand's collision hulls.

Run once, in the build container only (it reads the Menagerie meshes that ship
with the reference under /root/reference/asset/shadow, Apache-2.0):

    python tools/derive_shadow_assets.py

Output: mj-grasp-sim_amd/mgs/assets/shadow.npz -- DERIVED DATA only: the convex
hull vertices (mesh scale 0.001 of class right_hand, float32-rounded as MuJoCo
stores mesh vertices) of the two meshes the reference template uses as
collision geoms, f_distal_pst and th_distal_pst (mgs/gripper/shadow.py:39,174,
296).  Every Shadow body has an explicit <inertial>, so no mesh mass
properties are needed, and the visual meshes (contype=conaffinity=0) have no
physical effect.  No mesh file and no reference source is copied.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mj-grasp-sim_amd"))
from mgs.core.mjcf import convex_hull_vertices, load_mesh_bytes  # noqa: E402

SRC = "/root/reference/asset/shadow"
DST = os.path.join(os.path.dirname(__file__), "..", "mj-grasp-sim_amd", "mgs", "assets", "shadow.npz")
HULLS = ["f_distal_pst", "th_distal_pst"]
SCALE = 0.001


def main():
    if not os.path.isdir(SRC):
        print("reference meshes not found at", SRC)
        return 1
    out = {}
    for name in HULLS:
        fname = name + ".obj"
        v, _ = load_mesh_bytes(open(os.path.join(SRC, fname), "rb").read(), fname)
        v = (v * SCALE).astype(np.float32).astype(np.float64)
        out["hull_" + name] = np.unique(convex_hull_vertices(v), axis=0)
    np.savez_compressed(DST, **out)
    for k, v in out.items():
        print(k, v.shape, v.min(0), v.max(0))
    return 0


if __name__ == "__main__":
    sys.exit(main())
