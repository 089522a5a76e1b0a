"""Write synthetic YCB-format stand-in objects (SURVEY.md §8d "Synthetic inputs").

The YCB / GSO object sets are not shipped with the reference (git-ignored
asset/mj-objects, reference README.md:49-50) and there is no network here, so
the benchmark object is a stand-in written in the exact YCB directory format
read by mgs/obj/ycb.py (info.yml with original_file, submesh_files,
submesh_props, weight, material_map; reference mgs/obj/ycb.py:70-83):

  003_cracker_box   box 0.060 x 0.158 x 0.210 m, weight 0.411 kg, one convex submesh.

Real YCB directories are drop-in replacements (set MGS_ASSET_PATH).
"""
import os
import sys

import yaml

ROOT = os.path.join(os.path.dirname(__file__), "..", "mj-grasp-sim_amd", "mgs", "assets", "mj-objects", "YCB")

OBJECTS = {
    "003_cracker_box": dict(half=(0.030, 0.079, 0.105), weight=0.411),
}


def box_obj(hx, hy, hz):
    v = [(sx * hx, sy * hy, sz * hz) for sz in (-1, 1) for sy in (-1, 1) for sx in (-1, 1)]
    # outward-facing quads (1-based)
    f = [(1, 3, 4, 2), (5, 6, 8, 7), (1, 2, 6, 5), (3, 7, 8, 4), (1, 5, 7, 3), (2, 4, 8, 6)]
    lines = ["# synthetic YCB stand-in (box)"]
    lines += ["v %.6f %.6f %.6f" % p for p in v]
    for q in f:
        lines.append("f %d %d %d" % (q[0], q[1], q[2]))
        lines.append("f %d %d %d" % (q[0], q[2], q[3]))
    return "\n".join(lines) + "\n"


def main():
    for oid, spec in OBJECTS.items():
        d = os.path.join(ROOT, oid)
        os.makedirs(d, exist_ok=True)
        body = box_obj(*spec["half"])
        open(os.path.join(d, "textured.obj"), "w").write(body)
        open(os.path.join(d, "collision_0.obj"), "w").write(body)
        info = dict(original_file="textured.obj", submesh_files=["collision_0.obj"],
                    submesh_props=[1.0], weight=spec["weight"], material_map="texture_map.png",
                    synthetic=True)
        with open(os.path.join(d, "info.yml"), "w") as fh:
            yaml.safe_dump(info, fh, sort_keys=False)
    with open(os.path.join(ROOT, "..", "fast_eta_objects.txt"), "w") as fh:
        fh.write("\n".join(OBJECTS) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
