"""Derive the Robotiq 2F-85 collision hulls and mesh mass properties.

Run once, in the build container only (it reads the Menagerie meshes that ship
with the reference under /root/reference/asset/robotiq2f85, BSD-2 licensed):

    python tools/derive_robotiq_assets.py

Output: mj-grasp-sim_amd/mgs/assets/robotiq2f85.npz — DERIVED DATA only:
  * for every mesh used as a collision geom, the vertices of its convex hull
    (MuJoCo collides meshes through their convex hull; vertices are scaled by
    the template's mesh scale 0.001 and rounded to float32 as MuJoCo stores
    mesh vertices),
  * for every mesh whose body has no <inertial> (base_mount, silicone_pad),
    its volume, centroid and inertia tensor about the centroid (density 1),
    as MuJoCo 3.2.2's mesh compiler computes them with its default
    <mesh inertia="legacy"> (mgs.core.mjcf.mesh_mass_properties: |volume| per
    face pyramid, so the non-convex base_mount counts 2.16x its volume).

No STL file and no reference source is copied into the repository.
Reference: mgs/gripper/robotiq2f85.py:32-225 (template), asset/robotiq2f85/*.stl.
"""
import os
import struct
import sys

import numpy as np
from scipy.spatial import ConvexHull

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mj-grasp-sim_amd"))
from mgs.core.mjcf import mesh_mass_properties  # noqa: E402

SRC = "/root/reference/asset/robotiq2f85"
DST = os.path.join(os.path.dirname(__file__), "..", "mj-grasp-sim_amd", "mgs",
                   "assets", "robotiq2f85.npz")
SCALE = 0.001
HULL_MESHES = ["base_mount", "base", "driver", "coupler", "follower", "spring_link"]
MASS_MESHES = ["base_mount", "silicone_pad"]


def load_stl(path):
    data = open(path, "rb").read()
    n = struct.unpack("<I", data[80:84])[0]
    rec = np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")])
    arr = np.frombuffer(data[84:84 + n * 50], dtype=rec)
    return arr["v"].astype(np.float64)


def main():
    if not os.path.isdir(SRC):
        print("reference meshes not found at", SRC)
        return 1
    out = {}
    for name in HULL_MESHES:
        pts = load_stl(os.path.join(SRC, name + ".stl")).reshape(-1, 3) * SCALE
        pts = pts.astype(np.float32).astype(np.float64)
        hull = ConvexHull(pts)
        verts = np.unique(pts[hull.vertices], axis=0)
        out["hull_" + name] = verts
    for name in MASS_MESHES:
        tri = (load_stl(os.path.join(SRC, name + ".stl")) * SCALE).astype(np.float32).astype(np.float64)
        v = tri.reshape(-1, 3)
        vol, com, inertia = mesh_mass_properties(v, np.arange(len(v)).reshape(-1, 3))
        out["vol_" + name] = np.array(vol)
        out["com_" + name] = com
        out["inertia_" + name] = inertia
    os.makedirs(os.path.dirname(DST), exist_ok=True)
    np.savez_compressed(DST, **out)
    for k, v in out.items():
        print(k, np.shape(v))
    return 0


if __name__ == "__main__":
    sys.exit(main())
