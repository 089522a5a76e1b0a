"""Derive the DEXEE hand's collision hulls and link mass properties.

Run once, in the build container only (it reads the meshes that ship with the
reference under /root/reference/asset/dexee; the template is derived from
MuJoCo Menagerie, Apache-2.0):

    python tools/derive_dexee_assets.py

Output: mj-grasp-sim_amd/mgs/assets/dexee.npz -- DERIVED DATA only:
  * hull_<name>: the convex hull vertices (float32-rounded, as MuJoCo stores
    mesh vertices) of the eight meshes the reference template collides
    (mgs/gripper/dexee.py:52-76, the "*_col" meshes), each after its mesh's
    refquat: MuJoCo expresses the vertices in the frame rotated by refquat, i.e.
    stores R(refquat)^T v (checked on the links: every finger link mesh then
    extends from its joint toward its child body along -y);
  * vol_/com_/inertia_<name>: volume, centroid and inertia about the centroid
    at density 1 of the six visual meshes that carry a link's mass (geoms with
    an explicit mass, dexee.py:128-178; MuJoCo 3.2.2's default legacy mesh
    inertia), after the same refquat.
No mesh file and no reference source is copied into the repository.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mj-grasp-sim_amd"))
from mgs.core.mjcf import convex_hull_vertices, load_mesh_bytes, mesh_mass_properties, quat2mat  # noqa: E402

SRC = "/root/reference/asset/dexee"
DST = os.path.join(os.path.dirname(__file__), "..", "mj-grasp-sim_amd", "mgs", "assets", "dexee.npz")
Q_LINK = (1.0, -1.0, 0.0, 0.0)       # knuckle / proximal / middle meshes
Q_DISTAL = (0.0, 0.0, 0.0, 1.0)
Q_TIP = (0.0, -1.0, 0.0, 0.0)
# name: (file, refquat)
HULLS = {
    "base": ("Asm-MRH-HB1-Visual,00-Plastic.stl", None),
    "puck": ("Asm-MRH-HB1-Visual,00-Puck.stl", None),
    "finger_base": ("r3_finger_base_col.stl", None),
    "knuckle": ("MRH-F-J0Link-Visual,00.stl", Q_LINK),
    "proximal": ("Asm-MRH-F-Prox-Visual,00+Magtac,00.stl", Q_LINK),
    "middle": ("Asm-MRH-F-Mid-Visual,00+MagTac,00.stl", Q_LINK),
    "distal": ("MRH-F-Distal-Visual,00.stl", Q_DISTAL),
    "tip": ("MRH-F-Distal-Sensor-Visual,00.stl", Q_TIP),
}
MASS_MESHES = {
    "base": ("Asm-MRH-HB1-Visual,00-Plastic.stl", None),
    "finger_base": ("MRH-FB-MainALU-Visual,00.stl", None),
    "knuckle": ("MRH-F-J0Link-Visual,00.stl", Q_LINK),
    "proximal": ("MRH-F-Prox-Visual,00-Main.stl", Q_LINK),
    "middle": ("MRH-F-Mid-Visual,00.stl", Q_LINK),
    "distal": ("MRH-F-Distal-Visual,00.stl", Q_DISTAL),
}


def load(fname, refquat):
    v, f = load_mesh_bytes(open(os.path.join(SRC, fname), "rb").read(), fname)
    if refquat is not None:
        q = np.asarray(refquat, np.float64)
        v = v @ quat2mat(q / np.linalg.norm(q))      # rows: R^T v
    return v.astype(np.float32).astype(np.float64), f


def main():
    if not os.path.isdir(SRC):
        print("reference meshes not found at", SRC)
        return 1
    out = {}
    for name, (fname, rq) in HULLS.items():
        v, _ = load(fname, rq)
        out["hull_" + name] = np.unique(convex_hull_vertices(v), axis=0)
    for name, (fname, rq) in MASS_MESHES.items():
        v, f = load(fname, rq)
        vol, com, inertia = mesh_mass_properties(v, f)
        out["vol_" + name] = np.array(vol)
        out["com_" + name] = com
        out["inertia_" + name] = inertia
    np.savez_compressed(DST, **out)
    for k, v in out.items():
        if k.startswith("hull_"):
            print(k, v.shape, np.round(v.min(0), 4), np.round(v.max(0), 4))
        elif k.startswith("com_"):
            print(k, np.round(v, 4))
    return 0


if __name__ == "__main__":
    sys.exit(main())
