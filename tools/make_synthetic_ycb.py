"""Write synthetic YCB-format stand-in objects (SURVEY.md §8d "Synthetic inputs").

The YCB / GSO object sets are not shipped with the reference (git-ignored
asset/mj-objects, reference README.md:49-50) and there is no network here, so
the benchmark object is a stand-in written in the exact YCB directory format
read by mgs/obj/ycb.py (info.yml with original_file, submesh_files,
submesh_props, weight, material_map; reference mgs/obj/ycb.py:70-83):

  003_cracker_box       box 0.060 x 0.158 x 0.210 m, 0.411 kg (the benchmark object)
  005_tomato_soup_can   32-gon cylinder r 0.0335, h 0.101 m, 0.349 kg
  010_potted_meat_can   box 0.100 x 0.058 x 0.084 m, 0.370 kg
  017_orange            icosphere (2 subdivisions) r 0.0365 m, 0.047 kg
  061_foam_brick        box 0.050 x 0.075 x 0.050 m, 0.028 kg
each with one convex submesh (nominal YCB sizes and weights).

Real YCB directories are drop-in replacements (set MGS_ASSET_PATH).
"""
import os
import sys

import yaml

ROOT = os.path.join(os.path.dirname(__file__), "..", "mj-grasp-sim_amd", "mgs", "assets", "mj-objects", "YCB")

OBJECTS = {
    "003_cracker_box": dict(half=(0.030, 0.079, 0.105), weight=0.411),
    "005_tomato_soup_can": dict(cyl=(0.0335, 0.0505, 32), weight=0.349),
    "010_potted_meat_can": dict(half=(0.050, 0.029, 0.042), weight=0.370),
    "017_orange": dict(sphere=(0.0365, 2), weight=0.047),
    "061_foam_brick": dict(half=(0.025, 0.0375, 0.025), weight=0.028),
}


# GSO stand-in: a 24-gon mug-sized cylinder r 0.04, h 0.09 m, 0.3 kg
GSO_OBJECTS = {"Synthetic_Mug_Body": dict(cyl=(0.04, 0.045, 24), weight=0.3)}


def convex_obj(verts, title):
    """OBJ text of the convex hull of `verts` with outward-oriented triangles."""
    import numpy as np
    from scipy.spatial import ConvexHull
    v = np.asarray(verts, dtype=np.float64)
    h = ConvexHull(v)
    c = v.mean(0)
    lines = [f"# synthetic YCB stand-in ({title})"] + ["v %.6f %.6f %.6f" % tuple(p) for p in v]
    for f in h.simplices:
        a, b, cc = v[f[0]], v[f[1]], v[f[2]]
        if np.dot(np.cross(b - a, cc - a), a - c) < 0:
            f = f[[0, 2, 1]]
        lines.append("f %d %d %d" % tuple(f + 1))
    return "\n".join(lines) + "\n"


def cylinder_verts(r, hz, n):
    import numpy as np
    a = 2 * np.pi * np.arange(n) / n
    rim = np.stack([r * np.cos(a), r * np.sin(a)], 1)
    return np.concatenate([np.c_[rim, np.full(n, -hz)], np.c_[rim, np.full(n, hz)]])


def icosphere_verts(r, subdiv):
    import numpy as np
    t = (1 + 5 ** 0.5) / 2
    v = [(-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0), (0, -1, t), (0, 1, t), (0, -1, -t), (0, 1, -t),
         (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1)]
    f = [(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4), (11, 10, 2),
         (10, 7, 6), (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8), (3, 8, 9), (4, 9, 5), (2, 4, 11),
         (6, 2, 10), (8, 6, 7), (9, 8, 1)]
    v = [np.array(p, float) / np.linalg.norm(p) for p in v]
    for _ in range(subdiv):
        mid, nf = {}, []
        for a, b, c in f:
            ids = []
            for i, j in ((a, b), (b, c), (c, a)):
                k = (min(i, j), max(i, j))
                if k not in mid:
                    m = v[i] + v[j]
                    v.append(m / np.linalg.norm(m))
                    mid[k] = len(v) - 1
                ids.append(mid[k])
            nf += [(a, ids[0], ids[2]), (b, ids[1], ids[0]), (c, ids[2], ids[1]), tuple(ids)]
        f = nf
    return np.array(v) * r


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
        if "half" in spec:
            body = box_obj(*spec["half"])
        elif "cyl" in spec:
            body = convex_obj(cylinder_verts(*spec["cyl"]), "cylinder")
        else:
            body = convex_obj(icosphere_verts(*spec["sphere"]), "icosphere")
        open(os.path.join(d, "textured.obj"), "w").write(body)
        open(os.path.join(d, "collision_0.obj"), "w").write(body)
        info = dict(original_file="textured.obj", submesh_files=["collision_0.obj"],
                    submesh_props=[1.0], weight=spec["weight"], material_map="texture_map.png",
                    synthetic=True)
        with open(os.path.join(d, "info.yml"), "w") as fh:
            yaml.safe_dump(info, fh, sort_keys=False)
    with open(os.path.join(ROOT, "..", "fast_eta_objects.txt"), "w") as fh:
        fh.write("\n".join(OBJECTS) + "\n")
    # one Google-Scanned-Objects-format stand-in (model.obj; reference gso.py:50-52)
    for oid, spec in GSO_OBJECTS.items():
        d = os.path.join(ROOT, "..", "GoogleScannedObjects", oid)
        os.makedirs(d, exist_ok=True)
        body = convex_obj(cylinder_verts(*spec["cyl"]), "cylinder")
        open(os.path.join(d, "model.obj"), "w").write(body)
        open(os.path.join(d, "collision_0.obj"), "w").write(body)
        info = dict(original_file="model.obj", submesh_files=["collision_0.obj"], submesh_props=[1.0],
                    weight=spec["weight"], material_map="texture.png", synthetic=True)
        with open(os.path.join(d, "info.yml"), "w") as fh:
            yaml.safe_dump(info, fh, sort_keys=False)
    return 0


if __name__ == "__main__":
    sys.exit(main())
