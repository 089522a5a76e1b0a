"""Derive the Allegro hand's link mass properties.

Run once, in the build container only (it reads the Menagerie meshes that ship
with the reference under /root/reference/asset/allegro, BSD-2):

    python tools/derive_allegro_assets.py

Output: mj-grasp-sim_amd/mgs/assets/allegro.npz -- DERIVED DATA only.  The
reference template gives no body an <inertial> (allegro.py:158 is commented
out), so MuJoCo takes every body's mass from its geoms: the collision boxes and
capsules are massless (class "collision", mass="0", allegro.py:66) and the
visual meshes carry density 800 (class "allegro_right", allegro.py:37).  For
each visual mesh this stores its volume, centroid and inertia about the
centroid at density 1 (exact signed-volume integration over the closed,
float32-rounded triangle mesh, as tools/derive_robotiq_assets.py).
No mesh file and no reference source is copied into the repository.
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mj-grasp-sim_amd"))
from mgs.core.mjcf import load_mesh_bytes, mesh_mass_properties  # noqa: E402

SRC = "/root/reference/asset/allegro"
DST = os.path.join(os.path.dirname(__file__), "..", "mj-grasp-sim_amd", "mgs", "assets", "allegro.npz")
MESHES = ["base_link", "link_0.0", "link_1.0", "link_2.0", "link_3.0", "link_3.0_tip", "link_12.0_right",
          "link_13.0", "link_14.0", "link_15.0", "link_15.0_tip"]


def main():
    if not os.path.isdir(SRC):
        print("reference meshes not found at", SRC)
        return 1
    out = {}
    for name in MESHES:
        fname = name + ".stl"
        v, f = load_mesh_bytes(open(os.path.join(SRC, fname), "rb").read(), fname)
        v = v.astype(np.float32).astype(np.float64)
        vol, com, inertia = mesh_mass_properties(v, f)
        out["vol_" + name] = np.array(vol)
        out["com_" + name] = com
        out["inertia_" + name] = inertia
    np.savez_compressed(DST, **out)
    print(len(out), "arrays ->", DST)
    return 0


if __name__ == "__main__":
    sys.exit(main())
