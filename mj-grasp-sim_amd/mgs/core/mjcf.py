"""MJCF-subset compiler: XML string + asset dict -> flat model for libmgs_gpu.

This replaces `mujoco.MjModel.from_xml_string(xml, assets)` as called at
mgs/env/gravityless_object_grasping.py:67-69 for the subset of MJCF the
reference's gripper/object/env templates use:

  * <compiler angle meshdir autolimits discardvisual>, repeated <option>
    elements merged attribute-wise in document order (the reference relies on
    this: gravityless_object_grasping.py:36-42 then robotiq2f85.py:35 sets
    impratio=10 after the env's impratio=3);
  * <default> classes with nesting, `class` and `childclass`;
  * <asset><mesh file=.. | vertex=..  scale=..>, STL and OBJ files;
  * bodies (pos/quat/axisangle/euler/zaxis, mocap), <inertial>, <joint>
    (free/hinge/slide), <freejoint>, <geom> (box/mesh collide; sphere/capsule/
    cylinder/ellipsoid contribute mass only), <include file=..> from the assets;
  * <contact><exclude>, <tendon><fixed>, <equality> connect/weld/joint,
    <actuator> general/position/motor.

Semantics follow MuJoCo 3.2.2's documented compiler (the engine the reference
pins, requirements.txt:1): mass from geoms when a body has no <inertial>
(visual geoms included: discardvisual=false), meshes collide through their
convex hull, weld/connect anchors are resolved at qpos0, contact pairs are
filtered by weld-body, contype/conaffinity, parent/child and <exclude>, and
pair parameters are mixed by priority (higher wins) else max/solmix.
"""
from __future__ import annotations

import io
import os
import re
import struct
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

_MINVAL = 1e-15

# ----------------------------------------------------------------------------
# defaults
_GEOM_DEFAULTS = dict(type="sphere", size="0 0 0", contype="1", conaffinity="1",
                      condim="3", friction="1 0.005 0.0001", solref="0.02 1",
                      solimp="0.9 0.95 0.001 0.5 2", margin="0", gap="0",
                      priority="0", solmix="1", density="1000", group="0",
                      pos="0 0 0")
_JOINT_DEFAULTS = dict(type="hinge", axis="0 0 1", pos="0 0 0", range="0 0",
                       limited="auto", stiffness="0", springref="0", damping="0",
                       armature="0", frictionloss="0", solreflimit="0.02 1",
                       solimplimit="0.9 0.95 0.001 0.5 2", solreffriction="0.02 1",
                       solimpfriction="0.9 0.95 0.001 0.5 2", margin="0", ref="0")
_EQ_DEFAULTS = dict(solref="0.02 1", solimp="0.9 0.95 0.001 0.5 2", active="true")

PAIR_CONVEX, PAIR_BOXBOX = 0, 1   # pair_kind: narrowphase used for the pair (mgs_gpu.h MGS_PAIR_*)
# ABI 23: MuJoCo 3.2.2's collision table restated (ccd_mode 1 / 2): MPR pairs
# with a sphere (no multiccd), and the analytic primitive colliders
PAIR_CONVEX_SMOOTH, PAIR_SPHERE_SPHERE, PAIR_SPHERE_CAPSULE, PAIR_CAPSULE_CAPSULE = 2, 3, 4, 5
PAIR_SPHERE_BOX, PAIR_CAPSULE_BOX, PAIR_SPHERE_CYLINDER = 6, 7, 8
# MuJoCo mjtGeom numbering (the collision table is indexed type1 <= type2)
GEOM_TYPES = {"plane": 0, "hfield": 1, "sphere": 2, "capsule": 3, "ellipsoid": 4, "cylinder": 5, "box": 6,
              "mesh": 7}
_PRIM_KIND = {(2, 2): PAIR_SPHERE_SPHERE, (2, 3): PAIR_SPHERE_CAPSULE, (3, 3): PAIR_CAPSULE_CAPSULE,
              (2, 6): PAIR_SPHERE_BOX, (3, 6): PAIR_CAPSULE_BOX, (2, 5): PAIR_SPHERE_CYLINDER,
              (6, 6): PAIR_BOXBOX}
CCD_MODES = {"r5": 0, "multiccd": 1, "single": 2}   # mgs_model_desc.ccd_mode
GAIN_PID = 16                      # actuator_gaintype of a mujoco.pid plugin actuator (mgs_gpu.h MGS_GAIN_PID)
CYL_SIDES = 16   # cylinder collision geoms: 32-vertex prisms (a cap fits one contact feature, K_MAXF)
_JNT_TYPES = {"free": 0, "ball": 1, "slide": 2, "hinge": 3}


def _f(s, n=None):
    v = np.array([float(x) for x in str(s).split()], dtype=np.float64)
    if n is not None and v.size < n:
        v = np.concatenate([v, np.zeros(n - v.size)])
    return v


_VEC_DEFAULTS = {"friction": "1 0.005 0.0001", "solref": "0.02 1", "solimp": "0.9 0.95 0.001 0.5 2",
                 "solreflimit": "0.02 1", "solimplimit": "0.9 0.95 0.001 0.5 2",
                 "solreffriction": "0.02 1", "solimpfriction": "0.9 0.95 0.001 0.5 2",
                 "gainprm": "1 0 0", "biasprm": "0 0 0"}


def _fv(attrs, key):
    """Vector attribute; trailing entries not given keep MuJoCo's defaults."""
    d = _f(_VEC_DEFAULTS[key])
    v = _f(attrs.get(key, _VEC_DEFAULTS[key]))
    out = d.copy()
    out[:min(len(v), len(d))] = v[:len(d)]
    return out


# ----------------------------------------------------------------------------
# small rotation helpers (wxyz)
def quat_mul(a, b):
    return np.array([
        a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
        a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
        a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
        a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]])


def quat_conj(q):
    return np.array([q[0], -q[1], -q[2], -q[3]])


def quat2mat(q):
    w, x, y, z = q
    return np.array([
        [w * w + x * x - y * y - z * z, 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), w * w - x * x + y * y - z * z, 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), w * w - x * x - y * y + z * z]])


def mat2quat(R):
    t = np.trace(R)
    if t > 0:
        s = np.sqrt(t + 1.0) * 2
        q = [0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s]
    elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = np.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
        q = [(R[2, 1] - R[1, 2]) / s, 0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s]
    elif R[1, 1] > R[2, 2]:
        s = np.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
        q = [(R[0, 2] - R[2, 0]) / s, (R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s]
    else:
        s = np.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
        q = [(R[1, 0] - R[0, 1]) / s, (R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s]
    q = np.array(q)
    if q[0] < 0:
        q = -q
    return q / np.linalg.norm(q)


def _normq(q):
    n = np.linalg.norm(q)
    return np.array([1.0, 0, 0, 0]) if n < _MINVAL else q / n


def eig3(mat):
    """MuJoCo's mju_eig3 (engine_util_solve.c): eigen-decomposition of a
    symmetric 3x3 matrix by Jacobi rotations accumulated in a quaternion
    (at most 500 sweeps of the largest off-diagonal element, eps 1e-12), then
    the eigenvalues sorted in decreasing order by quarter-turn rotations of the
    quaternion.  Returns (eigenvalues, quaternion wxyz); the columns of
    quat2mat(quaternion) are the eigenvectors.  MuJoCo's mesh compiler takes
    the mesh frame (mesh_quat) from it, so principal axes of degenerate
    inertias (axisymmetric meshes) are chosen as MuJoCo chooses them rather
    than as a LAPACK solver would."""
    eps = 1e-12
    A = np.asarray(mat, np.float64).reshape(3, 3)
    quat = np.array([1.0, 0.0, 0.0, 0.0])
    ev = np.zeros(3)
    for _ in range(500):
        V = quat2mat(quat)
        D = V.T @ A @ V
        ev = np.array([D[0, 0], D[1, 1], D[2, 2]])
        d1, d2, d5 = D.flat[1], D.flat[2], D.flat[5]
        if abs(d1) > abs(d2) and abs(d1) > abs(d5):
            rk, ck, rotk = 0, 1, 2
        elif abs(d2) > abs(d5):
            rk, ck, rotk = 0, 2, 1
        else:
            rk, ck, rotk = 1, 2, 0
        off = D.flat[3 * rk + ck]
        if abs(off) < eps:
            break
        tau = (D.flat[4 * ck] - D.flat[4 * rk]) / (2 * off)
        t = 1.0 / (tau + np.sqrt(1 + tau * tau)) if tau >= 0 else -1.0 / (-tau + np.sqrt(1 + tau * tau))
        c = 1.0 / np.sqrt(1 + t * t)
        if c > 1.0 - eps:
            break
        r = np.zeros(4)
        r[rotk + 1] = -np.sqrt(0.5 - 0.5 * c) if tau >= 0 else np.sqrt(0.5 - 0.5 * c)
        if rotk == 1:
            r[rotk + 1] = -r[rotk + 1]
        r[0] = np.sqrt(1.0 - r[rotk + 1] * r[rotk + 1])
        r = _normq(r)
        quat = _normq(quat_mul(quat, r))
    for j in range(3):
        j1 = j % 2
        if ev[j1] < ev[j1 + 1]:
            ev[j1], ev[j1 + 1] = ev[j1 + 1], ev[j1]
            r = np.zeros(4)
            r[0] = 0.707106781186548
            r[(j1 + 2) % 3 + 1] = r[0]
            quat = _normq(quat_mul(quat, r))
    return ev, quat


# ----------------------------------------------------------------------------
# meshes
def load_mesh_bytes(data: bytes, fname: str):
    """Return (vertices (n,3), faces (m,3) or None)."""
    low = fname.lower()
    if low.endswith(".stl"):
        if data[:5] == b"solid" and b"facet" in data[:400]:
            pts = [list(map(float, l.split()[1:4])) for l in data.decode().splitlines()
                   if l.strip().startswith("vertex")]
            tri = np.array(pts).reshape(-1, 3, 3)
        else:
            n = struct.unpack("<I", data[80:84])[0]
            rec = np.dtype([("n", "<f4", 3), ("v", "<f4", (3, 3)), ("a", "<u2")])
            tri = np.frombuffer(data[84:84 + 50 * n], dtype=rec)["v"].astype(np.float64)
        verts = tri.reshape(-1, 3)
        faces = np.arange(len(verts)).reshape(-1, 3)
        return verts, faces
    if low.endswith(".obj"):
        verts, faces = [], []
        for line in io.StringIO(data.decode(errors="ignore")):
            p = line.split()
            if not p:
                continue
            if p[0] == "v":
                verts.append([float(p[1]), float(p[2]), float(p[3])])
            elif p[0] == "f":
                idx = [int(t.split("/")[0]) for t in p[1:]]
                idx = [i - 1 if i > 0 else len(verts) + i for i in idx]
                for k in range(1, len(idx) - 1):
                    faces.append([idx[0], idx[k], idx[k + 1]])
        return np.array(verts, dtype=np.float64), np.array(faces, dtype=np.int64)
    raise ValueError(f"unsupported mesh file {fname}")


def _hull_faces(verts):
    """outward-oriented triangles of the convex hull"""
    from scipy.spatial import ConvexHull
    h = ConvexHull(verts)
    faces = h.simplices.copy()
    c = verts[h.vertices].mean(0)
    a, b, cc = verts[faces[:, 0]], verts[faces[:, 1]], verts[faces[:, 2]]
    flip = np.einsum("ij,ij->i", np.cross(b - a, cc - a), a - c) < 0
    faces[flip] = faces[flip][:, [0, 2, 1]]
    return faces


# products of inertia accumulated per tetrahedron: xx, yy, zz, xy, xz, yz
_PI = ((0, 0), (1, 1), (2, 2), (0, 1), (0, 2), (1, 2))


def mesh_mass_properties(verts, faces, inertia="legacy"):
    """volume, centroid, inertia about centroid (density 1) of a mesh, as
    MuJoCo 3.2's mesh compiler computes them (user_mesh.cc) for
    <mesh inertia=...> (default "legacy", the value MuJoCo 3.2.2 uses when the
    attribute is absent):

      * a pyramid per face with its apex at the area-weighted centroid of the
        face centres: signed volume dot(cen - facecen, n) * area / 3; "legacy"
        takes its absolute value (a non-convex mesh is over-counted: the
        Robotiq base_mount mesh by 2.16x), "exact" keeps the sign;
      * centre of mass: pyramid volumes times pyramid centroids
        (3/4 face centre + 1/4 apex);
      * inertia: a tetrahedron per face with its apex at the centre of mass
        (again |volume| for "legacy"), the standard second-moment formula;
      * "convex": the same over the convex hull's faces (a mesh given by
        vertices only is its hull, so every inertia mode agrees on it).
    """
    verts = np.asarray(verts, np.float64)
    if faces is None or len(faces) == 0 or inertia == "convex":
        faces = _hull_faces(verts)
    faces = np.asarray(faces)
    a, b, c = verts[faces[:, 0]], verts[faces[:, 1]], verts[faces[:, 2]]
    cr = np.cross(b - a, c - a)
    nn = np.linalg.norm(cr, axis=1)
    keep = nn > 0
    a, b, c, cr, nn = a[keep], b[keep], c[keep], cr[keep], nn[keep]
    area = 0.5 * nn
    nrm = cr / nn[:, None]
    cen = (a + b + c) / 3.0
    facecen = (area[:, None] * cen).sum(0) / area.sum()
    vol = np.einsum("ij,ij->i", cen - facecen, nrm) * area / 3.0
    if inertia == "legacy":
        vol = np.abs(vol)
    V = vol.sum()
    if V < 0:
        V, vol = -V, -vol
    if V < 1e-20:
        return 0.0, verts.mean(0), np.zeros((3, 3))
    com = (vol[:, None] * (0.75 * cen + 0.25 * facecen)).sum(0) / V
    D, E, F = a - com, b - com, c - com
    v2 = np.einsum("ij,ij->i", (D + E + F) / 3.0, nrm) * area / 3.0
    if inertia == "legacy":
        v2 = np.abs(v2)
    elif v2.sum() < 0:
        v2 = -v2
    P = np.zeros(6)
    for j, (k0, k1) in enumerate(_PI):
        P[j] = (v2 / 20.0 * (2.0 * (D[:, k0] * D[:, k1] + E[:, k0] * E[:, k1] + F[:, k0] * F[:, k1])
                             + D[:, k0] * E[:, k1] + D[:, k1] * E[:, k0] + D[:, k0] * F[:, k1]
                             + D[:, k1] * F[:, k0] + E[:, k0] * F[:, k1] + E[:, k1] * F[:, k0])).sum()
    I = np.array([[P[1] + P[2], -P[3], -P[4]],
                  [-P[3], P[0] + P[2], -P[5]],
                  [-P[4], -P[5], P[0] + P[1]]])
    return V, com, I


def convex_hull_vertices(verts):
    from scipy.spatial import ConvexHull
    v = np.asarray(verts, dtype=np.float64)
    if len(v) <= 4:
        return v.copy()
    h = ConvexHull(v)
    return np.unique(v[h.vertices], axis=0)


# ----------------------------------------------------------------------------
@dataclass
class _Body:
    name: str
    parent: int
    pos: np.ndarray
    quat: np.ndarray
    mocap: bool = False
    inertial: Optional[dict] = None
    joints: List[dict] = field(default_factory=list)
    geoms: List[dict] = field(default_factory=list)
    childclass: Optional[str] = None
    gravcomp: float = 0.0


class MJCFError(ValueError):
    pass


class Compiler:
    def __init__(self, xml: str, assets: Optional[Dict[str, bytes]] = None):
        self.assets = dict(assets or {})
        self.options = dict(timestep=0.002, impratio=1.0, tolerance=1e-8, iterations=100,
                            noslip_iterations=0, noslip_tolerance=1e-6, gravity=np.array([0, 0, -9.81]),
                            cone="pyramidal", integrator="Euler", mpr_tolerance=1e-6, solver="Newton",
                            ls_iterations=50, ls_tolerance=0.01, ccd_iterations=50, multiccd=False,
                            contact_model="mujoco")
        self.compiler = dict(angle="degree", meshdir="", autolimits=True, discardvisual=False)
        self.defaults: Dict[str, dict] = {"main": {"parent": None}}
        self.meshes: Dict[str, dict] = {}
        self.bodies: List[_Body] = [_Body("world", -1, np.zeros(3), np.array([1.0, 0, 0, 0]))]
        self.excludes: List[tuple] = []
        self.tendons: List[dict] = []
        self.equalities: List[dict] = []
        self.actuators: List[dict] = []
        self.plugin_instances: Dict[str, dict] = {}   # <extension> instances: plugin, config
        root = ET.fromstring(xml)
        root = self._expand_includes(root)
        self._parse(root)

    # -- includes ------------------------------------------------------------
    def _expand_includes(self, elem):
        new_children = []
        for ch in list(elem):
            if ch.tag == "include":
                fname = ch.get("file")
                if fname not in self.assets:
                    raise MJCFError(f"include file {fname} not in assets")
                data = self.assets[fname]
                sub = ET.fromstring(data if isinstance(data, (bytes, str)) else bytes(data))
                sub = self._expand_includes(sub)
                if sub.tag == "mujoco":
                    new_children.extend(list(sub))
                else:
                    new_children.append(sub)
            else:
                new_children.append(self._expand_includes(ch))
        for ch in list(elem):
            elem.remove(ch)
        for ch in new_children:
            elem.append(ch)
        return elem

    # -- parsing -------------------------------------------------------------
    def _parse(self, root):
        # pass 1: compiler/option/default/asset (order independent in MJCF)
        for el in root:
            if el.tag == "compiler":
                for k, v in el.attrib.items():
                    if k == "autolimits":
                        self.compiler[k] = v == "true"
                    elif k == "discardvisual":
                        self.compiler[k] = v == "true"
                    else:
                        self.compiler[k] = v
            elif el.tag == "option":
                self._parse_option(el)
            elif el.tag == "default":
                self._parse_default(el, "main", top=True)
            elif el.tag == "extension":
                # <plugin plugin="..."><instance name="..."><config key= value=/>
                for pl in el:
                    if pl.tag != "plugin":
                        continue
                    for inst in pl:
                        if inst.tag == "instance":
                            cfg = {c.get("key"): c.get("value") for c in inst if c.tag == "config"}
                            self.plugin_instances[inst.get("name")] = dict(plugin=pl.get("plugin"), config=cfg)
        for el in root:
            if el.tag == "asset":
                for a in el:
                    if a.tag == "mesh":
                        self._parse_mesh(a)
        for el in root:
            if el.tag == "worldbody":
                self._parse_body_children(el, 0, None)
        for el in root:
            if el.tag == "contact":
                for c in el:
                    if c.tag == "exclude":
                        self.excludes.append((c.get("body1"), c.get("body2")))
                    elif c.tag == "pair":
                        raise MJCFError("explicit <pair> is not supported")
            elif el.tag == "tendon":
                for t in el:
                    if t.tag == "fixed":
                        wr = [(j.get("joint"), float(j.get("coef", "1"))) for j in t if j.tag == "joint"]
                        self.tendons.append(dict(name=t.get("name"), wraps=wr))
                    else:
                        raise MJCFError(f"tendon type {t.tag} not supported")
            elif el.tag == "equality":
                for e in el:
                    self.equalities.append(self._resolve(e, "equality", None))
            elif el.tag == "actuator":
                for a in el:
                    self.actuators.append((a.tag, self._resolve(a, a.tag, None)))

    def _parse_option(self, el):
        o = self.options
        for k, v in el.attrib.items():
            if k in ("timestep", "impratio", "tolerance", "noslip_tolerance", "mpr_tolerance", "ls_tolerance"):
                o[k] = float(v)
            elif k == "ccd_tolerance":          # MuJoCo 3.x name of mpr_tolerance
                o["mpr_tolerance"] = float(v)
            elif k in ("iterations", "noslip_iterations", "ls_iterations"):
                o[k] = int(v)
            elif k in ("ccd_iterations", "mpr_iterations"):
                o["ccd_iterations"] = int(v)
            elif k == "gravity":
                o[k] = _f(v, 3)
            elif k in ("cone", "integrator", "solver", "jacobian"):
                o[k] = v
        # <flag multiccd="enable"/>: MuJoCo's multi-contact convex collisions
        # (perturbed MPR, ccd_mode 1); other flags are accepted and ignored
        for fl in el:
            if fl.tag == "flag" and "multiccd" in fl.attrib:
                o["multiccd"] = fl.get("multiccd") == "enable"

    def _parse_default(self, el, name, top=False):
        if top:
            cls = "main"
        else:
            cls = el.get("class")
            self.defaults[cls] = {"parent": name}
        for ch in el:
            if ch.tag == "default":
                self._parse_default(ch, cls)
            else:
                self.defaults[cls][ch.tag] = dict(ch.attrib)

    def _class_attrs(self, cls, tag):
        chain = []
        c = cls
        while c is not None:
            if c not in self.defaults:
                raise MJCFError(f"unknown default class {c}")
            chain.append(c)
            c = self.defaults[c]["parent"]
        out = {}
        for c in reversed(chain):
            out.update(self.defaults[c].get(tag, {}))
        return out

    def _resolve(self, el, tag, childclass):
        cls = el.get("class", childclass or "main")
        base = {"joint": _JOINT_DEFAULTS, "geom": _GEOM_DEFAULTS, "equality": _EQ_DEFAULTS}.get(tag, {})
        dtag = {"connect": "equality", "weld": "equality", "joint": "joint"}.get(tag, tag)
        if tag in ("connect", "weld") or (tag == "joint" and el.tag == "joint" and "joint1" in el.attrib):
            dtag, base = "equality", _EQ_DEFAULTS
        out = dict(base)
        out.update(self._class_attrs(cls, dtag))
        out.update(el.attrib)
        out["_tag"] = el.tag
        return out

    def _angle(self, v):
        return v if self.compiler["angle"] == "radian" else v * np.pi / 180.0

    def _orientation(self, attrs):
        if "quat" in attrs:
            return _normq(_f(attrs["quat"]))
        if "axisangle" in attrs:
            a = _f(attrs["axisangle"])
            ax = a[:3] / np.linalg.norm(a[:3])
            ang = self._angle(a[3])
            return np.concatenate([[np.cos(ang / 2)], ax * np.sin(ang / 2)])
        if "euler" in attrs:
            e = self._angle(_f(attrs["euler"]))
            q = np.array([1.0, 0, 0, 0])
            for i, ang in enumerate(e):  # default eulerseq xyz (intrinsic)
                ax = np.zeros(3)
                ax[i] = 1
                q = quat_mul(q, np.concatenate([[np.cos(ang / 2)], ax * np.sin(ang / 2)]))
            return q
        if "zaxis" in attrs:
            z = _f(attrs["zaxis"])
            z = z / np.linalg.norm(z)
            a = np.cross([0, 0, 1.0], z)
            s = np.linalg.norm(a)
            if s < 1e-12:
                return np.array([1.0, 0, 0, 0]) if z[2] > 0 else np.array([0, 1.0, 0, 0])
            ang = np.arctan2(s, z[2])
            return np.concatenate([[np.cos(ang / 2)], a / s * np.sin(ang / 2)])
        if "xyaxes" in attrs:
            v = _f(attrs["xyaxes"])
            x = v[:3] / np.linalg.norm(v[:3])
            y = v[3:] - x * np.dot(x, v[3:])
            y /= np.linalg.norm(y)
            return mat2quat(np.stack([x, y, np.cross(x, y)], axis=1))
        return np.array([1.0, 0, 0, 0])

    def _parse_mesh(self, a):
        cls = a.get("class", "main")
        attrs = dict(self._class_attrs(cls, "mesh"))
        attrs.update(a.attrib)
        scale = _f(attrs.get("scale", "1 1 1"), 3)
        if "vertex" in attrs:
            verts = _f(attrs["vertex"]).reshape(-1, 3)
            faces = None
            fname = attrs.get("name")
        else:
            fname = attrs["file"]
            key = fname if fname in self.assets else os.path.join(self.compiler.get("meshdir", ""), fname)
            if key in self.assets:
                data = self.assets[key]
            elif os.path.isfile(fname):
                data = open(fname, "rb").read()
            elif os.path.isfile(key):
                data = open(key, "rb").read()
            else:
                base = os.path.basename(fname)
                if base not in self.assets:
                    raise MJCFError(f"mesh file {fname} not found")
                data = self.assets[base]
            verts, faces = load_mesh_bytes(data, fname)
        verts = (verts * scale).astype(np.float32).astype(np.float64)
        name = attrs.get("name") or os.path.splitext(os.path.basename(fname))[0]
        self.meshes[name] = dict(verts=verts, faces=faces, hull=None, mass=None,
                                 inertia=attrs.get("inertia", "legacy"))

    def _mesh_hull(self, name):
        m = self.meshes[name]
        if m["hull"] is None:
            m["hull"] = convex_hull_vertices(m["verts"])
        return m["hull"]

    def _mesh_frame(self, name):
        """MuJoCo's mesh compilation (user_mesh.cc): the mesh is moved to its
        inertial frame -- centre of mass at the origin, principal axes along x,
        y, z (mesh_pos, mesh_quat) -- and its vertices are stored as float32
        (mesh_vert).  Returns (mesh_pos, mesh_quat, float32-rounded hull
        vertices in that frame as float64).  The principal axes come from
        MuJoCo's own eigensolver restated (eig3: decreasing moments, MuJoCo's
        choice of axes for equal moments)."""
        m = self.meshes[name]
        if m.get("frame") is None:
            vol, com, I = self._mesh_massprops(name)
            if vol > 0 and np.any(I):
                _, q = eig3(I)
            else:
                q = np.array([1.0, 0.0, 0.0, 0.0])
            V = quat2mat(q)
            hull = self._mesh_hull(name)
            local = ((hull - com) @ V).astype(np.float32).astype(np.float64)
            m["frame"] = (np.asarray(com, np.float64), q, local)
        return m["frame"]

    def _mesh_massprops(self, name):
        m = self.meshes[name]
        if m["mass"] is None:
            m["mass"] = mesh_mass_properties(m["verts"], m["faces"], m.get("inertia", "legacy"))
        return m["mass"]

    def _parse_body_children(self, el, parent, childclass):
        for ch in el:
            if ch.tag == "body":
                cc = ch.get("childclass", childclass)
                b = _Body(ch.get("name", f"body{len(self.bodies)}"), parent,
                          _f(ch.get("pos", "0 0 0"), 3), self._orientation(ch.attrib),
                          mocap=ch.get("mocap", "false") == "true", childclass=cc,
                          gravcomp=float(ch.get("gravcomp", "0")))
                bid = len(self.bodies)
                self.bodies.append(b)
                for sub in ch:
                    if sub.tag == "inertial":
                        b.inertial = dict(sub.attrib)
                    elif sub.tag == "joint":
                        b.joints.append(self._resolve(sub, "joint", cc))
                    elif sub.tag == "freejoint":
                        b.joints.append(dict(_JOINT_DEFAULTS, type="free", name=sub.get("name", ""),
                                             _tag="freejoint"))
                    elif sub.tag == "geom":
                        b.geoms.append(self._resolve(sub, "geom", cc))
                self._parse_body_children(ch, bid, cc)
            elif ch.tag == "geom" and parent == 0:
                self.bodies[0].geoms.append(self._resolve(ch, "geom", childclass))

    # -- compile ---------------------------------------------------------------
    def _geom_massprops(self, g):
        """mass, local com, inertia about com in geom frame."""
        t = g.get("type", "sphere")
        size = _f(g.get("size", "0 0 0"), 3)
        if t == "box":
            vol = 8 * size[0] * size[1] * size[2]
            com = np.zeros(3)
            I = np.diag([size[1] ** 2 + size[2] ** 2, size[0] ** 2 + size[2] ** 2, size[0] ** 2 + size[1] ** 2]) * vol / 3
        elif t == "sphere":
            r = size[0]
            vol = 4 / 3 * np.pi * r ** 3
            com = np.zeros(3)
            I = np.eye(3) * 0.4 * vol * r * r
        elif t == "capsule":
            r, h = size[0], size[1]
            vc = np.pi * r * r * 2 * h
            vs = 4 / 3 * np.pi * r ** 3
            vol = vc + vs
            ixx_c = vc * (3 * r * r + 4 * h * h) / 12
            izz_c = vc * r * r / 2
            ixx_s = vs * (0.4 * r * r + h * h + 0.75 * h * r)
            izz_s = vs * 0.4 * r * r
            com = np.zeros(3)
            I = np.diag([ixx_c + ixx_s, ixx_c + ixx_s, izz_c + izz_s])
        elif t == "cylinder":
            r, h = size[0], size[1]
            vol = np.pi * r * r * 2 * h
            com = np.zeros(3)
            I = np.diag([vol * (3 * r * r + 4 * h * h) / 12] * 2 + [vol * r * r / 2])
        elif t == "ellipsoid":
            vol = 4 / 3 * np.pi * size[0] * size[1] * size[2]
            com = np.zeros(3)
            I = np.diag([size[1] ** 2 + size[2] ** 2, size[0] ** 2 + size[2] ** 2, size[0] ** 2 + size[1] ** 2]) * vol / 5
        elif t == "mesh":
            vol, com, I = self._mesh_massprops(g["mesh"])
        else:
            return 0.0, np.zeros(3), np.zeros((3, 3))
        if "mass" in g:
            mass = float(g["mass"])
            scale = mass / vol if vol > 0 else 0.0
        else:
            scale = float(g.get("density", "1000"))
            mass = vol * scale
        return mass, com, I * scale

    def compile(self) -> "CompiledModel":
        opt = self.options
        if opt.get("integrator", "Euler") != "implicitfast":
            raise MJCFError("only integrator=implicitfast is supported (the reference's setting)")
        if opt.get("cone") != "elliptic":
            raise MJCFError("only cone=elliptic is supported (the reference's setting)")
        autolimits = self.compiler.get("autolimits", True)
        nb = len(self.bodies)
        names = [b.name for b in self.bodies]
        body_id = {n: i for i, n in enumerate(names)}

        # --- joints / dofs / qpos
        jnt, dof = [], []
        qpos0, qspring = [], []
        body_jntadr = np.full(nb, -1, np.int32)
        body_jntnum = np.zeros(nb, np.int32)
        body_dofadr = np.full(nb, -1, np.int32)
        body_dofnum = np.zeros(nb, np.int32)
        body_mocapid = np.full(nb, -1, np.int32)
        nmocap = 0
        for bi, b in enumerate(self.bodies):
            if b.mocap:
                if b.joints or b.parent != 0:
                    raise MJCFError("mocap bodies must be top-level and jointless")
                body_mocapid[bi] = nmocap
                nmocap += 1
            if b.joints:
                body_jntadr[bi] = len(jnt)
                body_jntnum[bi] = len(b.joints)
                body_dofadr[bi] = len(dof)
            for j in b.joints:
                jt = _JNT_TYPES[j.get("type", "hinge")]
                rng = _f(j.get("range", "0 0"), 2)
                lim = j.get("limited", "auto")
                limited = (rng[0] < rng[1]) if (lim == "auto" and autolimits) else (lim == "true")
                if jt in (2, 3) and self.compiler["angle"] != "radian" and jt == 3:
                    rng = rng * np.pi / 180.0
                ax = _f(j.get("axis", "0 0 1"), 3)
                ax = ax / max(np.linalg.norm(ax), _MINVAL)
                rec = dict(name=j.get("name", ""), type=jt, bodyid=bi, qposadr=len(qpos0),
                           dofadr=len(dof), limited=int(limited and jt in (2, 3)),
                           pos=_f(j.get("pos", "0 0 0"), 3), axis=ax, range=rng,
                           solref=_fv(j, "solreflimit"), solimp=_fv(j, "solimplimit"),
                           margin=float(j.get("margin", "0")), stiffness=float(j.get("stiffness", "0")))
                if jt == 0:
                    qpos0 += list(b.pos) + list(b.quat)
                    qspring += list(b.pos) + list(b.quat)
                    nd = 6
                elif jt == 1:
                    qpos0 += [1.0, 0, 0, 0]
                    qspring += [1.0, 0, 0, 0]
                    nd = 3
                else:
                    ref = float(j.get("ref", "0"))
                    sref = float(j.get("springref", "0"))
                    if jt == 3 and self.compiler["angle"] != "radian":
                        ref, sref = np.deg2rad(ref), np.deg2rad(sref)
                    qpos0.append(ref)
                    qspring.append(sref)
                    nd = 1
                jid = len(jnt)
                jnt.append(rec)
                for k in range(nd):
                    dof.append(dict(bodyid=bi, jntid=jid, armature=float(j.get("armature", "0")),
                                    damping=float(j.get("damping", "0")),
                                    frictionloss=float(j.get("frictionloss", "0")),
                                    solref=_fv(j, "solreffriction"), solimp=_fv(j, "solimpfriction")))
            body_dofnum[bi] = len(dof) - (body_dofadr[bi] if body_dofadr[bi] >= 0 else len(dof))
        nq, nv = len(qpos0), len(dof)
        parent = np.array([b.parent for b in self.bodies], np.int32)
        # dof parent: previous dof of the same body, else last dof of the ancestor chain
        body_lastdof = np.full(nb, -1, np.int32)
        dof_parent = np.full(nv, -1, np.int32)
        for bi in range(1, nb):
            last = body_lastdof[parent[bi]] if parent[bi] >= 0 else -1
            if body_dofnum[bi] > 0:
                for k in range(body_dofnum[bi]):
                    d = body_dofadr[bi] + k
                    dof_parent[d] = last
                    last = d
            body_lastdof[bi] = last
        rootid = np.zeros(nb, np.int32)
        weldid = np.zeros(nb, np.int32)
        for bi in range(1, nb):
            rootid[bi] = bi if parent[bi] == 0 else rootid[parent[bi]]
            weldid[bi] = bi if (body_jntnum[bi] > 0 or body_mocapid[bi] >= 0) else weldid[parent[bi]]

        # --- body global frames at qpos0 (joints at qpos0 are identity)
        xpos = np.zeros((nb, 3))
        xquat = np.zeros((nb, 4))
        xquat[0] = [1, 0, 0, 0]
        for bi in range(1, nb):
            b = self.bodies[bi]
            p = parent[bi]
            xpos[bi] = xpos[p] + quat2mat(xquat[p]) @ b.pos
            xquat[bi] = _normq(quat_mul(xquat[p], b.quat))

        # --- inertia
        body_mass = np.zeros(nb)
        body_ipos = np.zeros((nb, 3))
        body_iquat = np.tile([1.0, 0, 0, 0], (nb, 1))
        body_inertia = np.zeros((nb, 3))
        for bi in range(1, nb):
            b = self.bodies[bi]
            if b.inertial is not None:
                ia = b.inertial
                body_mass[bi] = float(ia["mass"])
                body_ipos[bi] = _f(ia.get("pos", "0 0 0"), 3)
                if "fullinertia" in ia:
                    fi = _f(ia["fullinertia"], 6)
                    I = np.array([[fi[0], fi[3], fi[4]], [fi[3], fi[1], fi[5]], [fi[4], fi[5], fi[2]]])
                    w, V = np.linalg.eigh(I)
                    if np.linalg.det(V) < 0:
                        V[:, 2] = -V[:, 2]
                    body_inertia[bi] = w
                    body_iquat[bi] = quat_mul(self._orientation(ia), mat2quat(V))
                else:
                    body_inertia[bi] = _f(ia.get("diaginertia", "0 0 0"), 3)
                    body_iquat[bi] = self._orientation(ia)
            else:
                mtot, c, Itot = 0.0, np.zeros(3), np.zeros((3, 3))
                parts = []
                for g in b.geoms:
                    m, gc, gI = self._geom_massprops(g)
                    if m <= 0:
                        continue
                    R = quat2mat(self._orientation(g))
                    gp = _f(g.get("pos", "0 0 0"), 3) + R @ gc
                    parts.append((m, gp, R @ gI @ R.T))
                    mtot += m
                    c += m * gp
                if mtot > 0:
                    c /= mtot
                    for m, gp, gI in parts:
                        d = gp - c
                        Itot += gI + m * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
                    w, V = np.linalg.eigh(Itot)
                    if np.linalg.det(V) < 0:
                        V[:, 2] = -V[:, 2]
                    body_mass[bi] = mtot
                    body_ipos[bi] = c
                    body_inertia[bi] = w
                    body_iquat[bi] = mat2quat(V)

        # --- geoms (all, to know MuJoCo geom ids), then collision subset
        allgeoms = []
        for bi, b in enumerate(self.bodies):
            for g in b.geoms:
                allgeoms.append((bi, g))
        partition = None
        for gid, (bi, g) in enumerate(allgeoms):
            if g.get("name") in ("geom:ground", "geom:table", "table"):
                partition = gid
        cgeoms = []
        hulls = []
        hull_of_mesh = {}
        for gid, (bi, g) in enumerate(allgeoms):
            ct, ca = int(g.get("contype", "1")), int(g.get("conaffinity", "1"))
            if ct == 0 and ca == 0:
                continue
            t = g.get("type", "sphere")
            gpos = _f(g.get("pos", "0 0 0"), 3)
            gquat = self._orientation(g)
            if t == "box":
                s = _f(g["size"], 3)
                verts = np.array([[sx * s[0], sy * s[1], sz * s[2]]
                                  for sz in (-1, 1) for sy in (-1, 1) for sx in (-1, 1)])
                hid = len(hulls)
                hulls.append(verts)
            elif t == "mesh":
                mname = g["mesh"]
                mpos, mquat, mverts = self._mesh_frame(mname)
                if mname not in hull_of_mesh:
                    hull_of_mesh[mname] = len(hulls)
                    hulls.append(mverts)
                hid = hull_of_mesh[mname]
                # MuJoCo offsets a mesh geom's frame by the mesh frame (mesh_pos /
                # mesh_quat), so the geom origin is the mesh's centre of mass
                gpos = gpos + quat2mat(gquat) @ mpos
                gquat = _normq(quat_mul(gquat, mquat))
            elif t in ("sphere", "capsule"):
                # rounded geoms: a point / a z-segment swept by a ball of radius size[0]
                s = _f(g["size"], 3)
                hid = len(hulls)
                hulls.append(np.zeros((1, 3)) if t == "sphere" else np.array([[0, 0, -s[1]], [0, 0, s[1]]]))
            elif t == "cylinder":
                # a CYL_SIDES-sided prism inscribed in the cylinder (vertices on the
                # true rim): the broadphase box and the cap polygon; supports and
                # contact features use the exact cylinder (geom_cyl)
                s = _f(g["size"], 3)
                a = 2 * np.pi * np.arange(CYL_SIDES) / CYL_SIDES
                rim = np.stack([s[0] * np.cos(a), s[0] * np.sin(a)], 1)
                hid = len(hulls)
                hulls.append(np.concatenate([np.c_[rim, np.full(CYL_SIDES, -s[1])],
                                             np.c_[rim, np.full(CYL_SIDES, s[1])]]))
            else:
                raise MJCFError(f"collision geom type {t} not supported yet")
            radius = float(_f(g["size"], 3)[0]) if t in ("sphere", "capsule") else 0.0
            cyl = _f(g["size"], 3)[:2].copy() if t == "cylinder" else np.zeros(2)
            side = 0 if partition is None else int(np.sign(gid - partition))
            fr = _fv(g, "friction")
            size3 = np.zeros(3)
            sz = _f(g["size"])
            size3[:min(3, len(sz))] = sz[:3]
            cgeoms.append(dict(gid=gid, body=bi, hull=hid, pos=gpos, quat=gquat, contype=ct, size=size3,
                               conaffinity=ca, condim=int(g.get("condim", "3")), friction=fr,
                               solref=_fv(g, "solref"), solimp=_fv(g, "solimp"),
                               margin=float(g.get("margin", "0")), gap=float(g.get("gap", "0")),
                               priority=int(g.get("priority", "0")), solmix=float(g.get("solmix", "1")),
                               side=side, name=g.get("name", ""), radius=radius, type=t, cyl=cyl))
        # --- admissible pairs
        excl = set()
        for b1, b2 in self.excludes:
            i1, i2 = body_id[b1], body_id[b2]
            excl.add((min(i1, i2), max(i1, i2)))
        pairs = []
        for a in range(len(cgeoms)):
            for b in range(a + 1, len(cgeoms)):
                g1, g2 = cgeoms[a], cgeoms[b]
                w1, w2 = weldid[g1["body"]], weldid[g2["body"]]
                if w1 == w2:
                    continue
                if not ((g1["contype"] & g2["conaffinity"]) or (g2["contype"] & g1["conaffinity"])):
                    continue
                if w1 != 0 and w2 != 0 and (w1 == weldid[parent[w2]] or w2 == weldid[parent[w1]]):
                    continue
                key = (min(g1["body"], g2["body"]), max(g1["body"], g2["body"]))
                if key in excl:
                    continue
                if g1["priority"] > g2["priority"]:
                    src = [g1]
                elif g2["priority"] > g1["priority"]:
                    src = [g2]
                else:
                    src = None
                if src is not None:
                    s = src[0]
                    condim, fr, sr, si = s["condim"], s["friction"], s["solref"], s["solimp"]
                else:
                    condim = max(g1["condim"], g2["condim"])
                    fr = np.maximum(g1["friction"], g2["friction"])
                    tot = g1["solmix"] + g2["solmix"]
                    mix = 0.5 if tot < _MINVAL else g1["solmix"] / tot
                    if g1["solref"][0] > 0 and g2["solref"][0] > 0:
                        sr = mix * g1["solref"] + (1 - mix) * g2["solref"]
                    else:
                        sr = np.minimum(g1["solref"], g2["solref"])
                    si = mix * g1["solimp"] + (1 - mix) * g2["solimp"]
                if condim not in (1, 3, 4, 6):
                    raise MJCFError(f"condim {condim} not supported")
                # collider: MuJoCo dispatches box-box pairs to its dedicated box
                # collider (mjc_BoxBox), everything else here to the convex path
                kind = PAIR_BOXBOX if (g1["type"] == "box" and g2["type"] == "box") else PAIR_CONVEX
                pairs.append(dict(g1=a, g2=b, condim=condim, kind=kind,
                                  friction=np.array([fr[0], fr[0], fr[1], fr[2], fr[2]]),
                                  solref=np.array(sr), solimp=np.array(si),
                                  margin=max(g1["margin"], g2["margin"]) - max(g1["gap"], g2["gap"])))

        # --- equality
        jnt_id = {j["name"]: i for i, j in enumerate(jnt)}
        eqs = []
        for e in self.equalities:
            tag = e["_tag"]
            if e.get("active", "true") != "true":
                continue
            data = np.zeros(11)
            if tag == "connect":
                b1, b2 = body_id[e["body1"]], body_id[e["body2"]]
                anchor = _f(e.get("anchor", "0 0 0"), 3)
                pw = xpos[b1] + quat2mat(xquat[b1]) @ anchor
                a2 = quat2mat(xquat[b2]).T @ (pw - xpos[b2])
                data[0:3], data[3:6] = anchor, a2
                eqs.append(dict(type=0, o1=b1, o2=b2, data=data, e=e))
            elif tag == "weld":
                b1 = body_id[e["body1"]]
                b2 = body_id[e.get("body2", "world")] if e.get("body2") else 0
                if np.any(_f(e.get("anchor", "0 0 0"), 3) != 0):
                    raise MJCFError("weld anchor != 0 not supported")
                if "relpose" in e and np.any(_f(e["relpose"], 7)[3:] != 0):
                    rp = _f(e["relpose"], 7)
                    relpos, relq = rp[:3], _normq(rp[3:])
                else:
                    R1 = quat2mat(xquat[b1])
                    relpos = R1.T @ (xpos[b2] - xpos[b1])
                    relq = _normq(quat_mul(quat_conj(xquat[b1]), xquat[b2]))
                data[0:3], data[3:7] = relpos, relq
                data[7] = float(e.get("torquescale", "1"))
                eqs.append(dict(type=1, o1=b1, o2=b2, data=data, e=e))
            elif tag == "joint":
                j1 = jnt_id[e["joint1"]]
                j2 = jnt_id[e["joint2"]] if e.get("joint2") else -1
                pc = _f(e.get("polycoef", "0 1 0 0 0"), 5)
                data[0:5] = pc
                data[5] = qpos0[jnt[j1]["qposadr"]]
                data[6] = qpos0[jnt[j2]["qposadr"]] if j2 >= 0 else 0.0
                eqs.append(dict(type=2, o1=j1, o2=j2, data=data, e=e))
            else:
                raise MJCFError(f"equality {tag} not supported")

        # --- tendons
        wraps, tadr, tnum = [], [], []
        ten_id = {}
        for t in self.tendons:
            ten_id[t["name"]] = len(tadr)
            tadr.append(len(wraps))
            tnum.append(len(t["wraps"]))
            for jn, coef in t["wraps"]:
                j = jnt[jnt_id[jn]]
                if j["type"] not in (2, 3):
                    raise MJCFError("fixed tendon on non-scalar joint")
                wraps.append((j["dofadr"], j["qposadr"], coef))

        # --- actuators
        acts = []
        for tag, a in self.actuators:
            if "joint" in a:
                trn, tid = 0, jnt_id[a["joint"]]
            elif "tendon" in a:
                trn, tid = 3, ten_id[a["tendon"]]
            else:
                raise MJCFError("actuator transmission not supported")
            gainprm = np.zeros(3)
            biasprm = np.zeros(3)
            if tag == "general":
                gainprm[:] = _fv(a, "gainprm")
                biasprm[:] = _fv(a, "biasprm")
                gt = {"fixed": 0, "affine": 1}[a.get("gaintype", "fixed")]
                bt = {"none": 0, "affine": 1}[a.get("biastype", "none")]
            elif tag == "position":
                kp = float(a.get("kp", "1"))
                kv = float(a.get("kv", "0"))
                gainprm[0] = kp
                biasprm[:] = [0, -kp, -kv]
                gt, bt = 0, 1
            elif tag == "motor":
                gainprm[0] = 1.0
                gt, bt = 0, 0
            elif tag == "plugin":
                # MuJoCo's mujoco.pid actuator plugin: gains and limits from its
                # <extension> instance, its state (integral, previous setpoint)
                # in the actuator's act slots
                inst = self.plugin_instances.get(a.get("instance", ""))
                plug = a.get("plugin") or (inst or {}).get("plugin")
                if inst is None or plug != "mujoco.pid":
                    raise MJCFError(f"actuator plugin {plug!r} not supported (mujoco.pid instances only)")
                cfg = inst["config"]
                pid = np.array([float(cfg.get("kp", "0")), float(cfg.get("ki", "0")), float(cfg.get("kd", "0")),
                                float(cfg.get("imax", "-1")), float(cfg.get("slewmax", "-1"))])
                if a.get("dyntype", "none") != "none":
                    raise MJCFError("mujoco.pid with a dyntype is not supported")
                nst = int(pid[1] != 0.0) + int(pid[4] >= 0.0)
                if int(a.get("actdim", str(nst))) != nst:
                    raise MJCFError(f"mujoco.pid actdim {a.get('actdim')} does not match its state ({nst})")
                gt, bt = GAIN_PID, 0
            else:
                raise MJCFError(f"actuator {tag} not supported")
            cr = _f(a.get("ctrlrange", "0 0"), 2)
            fr = _f(a.get("forcerange", "0 0"), 2)
            cl = a.get("ctrllimited", "auto")
            fl = a.get("forcelimited", "auto")
            if gt != GAIN_PID:
                pid = np.zeros(5)
                nst = 0
            acts.append(dict(trn=trn, tid=tid, gt=gt, bt=bt, gainprm=gainprm, biasprm=biasprm, pid=pid, actnum=nst,
                             ctrlrange=cr, forcerange=fr,
                             ctrllimited=int(("ctrlrange" in a) if cl == "auto" else cl == "true"),
                             forcelimited=int(("forcerange" in a) if fl == "auto" else fl == "true"),
                             gear=_f(a.get("gear", "1"), 1)[0], name=a.get("name", "")))

        cm = CompiledModel()
        cm.options = dict(opt)
        cm.nq, cm.nv, cm.nbody, cm.nmocap = nq, nv, nb, nmocap
        cm.body_names = names
        cm.jnt_names = [j["name"] for j in jnt]
        cm.geom_names = [g["name"] for g in cgeoms]
        cm.actuator_names = [a["name"] for a in acts]
        cm.partition_geom = partition
        cm.body_parentid = parent
        cm.body_rootid = rootid
        cm.body_weldid = weldid
        cm.body_mocapid = body_mocapid
        cm.body_jntnum, cm.body_jntadr = body_jntnum, body_jntadr
        cm.body_dofnum, cm.body_dofadr = body_dofnum, body_dofadr
        cm.body_lastdof = body_lastdof
        cm.body_pos = np.array([b.pos for b in self.bodies])
        cm.body_quat = np.array([b.quat for b in self.bodies])
        cm.body_ipos, cm.body_iquat = body_ipos, body_iquat
        cm.body_mass, cm.body_inertia = body_mass, body_inertia
        cm.jnt_type = np.array([j["type"] for j in jnt], np.int32)
        cm.jnt_qposadr = np.array([j["qposadr"] for j in jnt], np.int32)
        cm.jnt_dofadr = np.array([j["dofadr"] for j in jnt], np.int32)
        cm.jnt_bodyid = np.array([j["bodyid"] for j in jnt], np.int32)
        cm.jnt_limited = np.array([j["limited"] for j in jnt], np.int32)
        cm.jnt_pos = np.array([j["pos"] for j in jnt]).reshape(-1, 3)
        cm.jnt_axis = np.array([j["axis"] for j in jnt]).reshape(-1, 3)
        cm.jnt_range = np.array([j["range"] for j in jnt]).reshape(-1, 2)
        cm.jnt_solref = np.array([j["solref"] for j in jnt]).reshape(-1, 2)
        cm.jnt_solimp = np.array([j["solimp"] for j in jnt]).reshape(-1, 5)
        cm.jnt_margin = np.array([j["margin"] for j in jnt])
        cm.jnt_stiffness = np.array([j["stiffness"] for j in jnt])
        cm.dof_bodyid = np.array([d["bodyid"] for d in dof], np.int32)
        cm.dof_jntid = np.array([d["jntid"] for d in dof], np.int32)
        cm.dof_parentid = dof_parent
        cm.dof_armature = np.array([d["armature"] for d in dof])
        cm.dof_damping = np.array([d["damping"] for d in dof])
        cm.dof_frictionloss = np.array([d["frictionloss"] for d in dof])
        cm.dof_solref = np.array([d["solref"] for d in dof]).reshape(-1, 2)
        cm.dof_solimp = np.array([d["solimp"] for d in dof]).reshape(-1, 5)
        cm.qpos0 = np.array(qpos0, dtype=np.float64)
        cm.qpos_spring = np.array(qspring, dtype=np.float64)
        cm.geom_bodyid = np.array([g["body"] for g in cgeoms], np.int32)
        cm.geom_hullid = np.array([g["hull"] for g in cgeoms], np.int32)
        cm.geom_side = np.array([g["side"] for g in cgeoms], np.int32)
        cm.geom_origid = np.array([g["gid"] for g in cgeoms], np.int32)
        cm.geom_pos = np.array([g["pos"] for g in cgeoms]).reshape(-1, 3)
        cm.geom_quat = np.array([g["quat"] for g in cgeoms]).reshape(-1, 4)
        aabb = []
        for g in cgeoms:
            v = hulls[g["hull"]]
            lo, hi = v.min(0) - g["radius"], v.max(0) + g["radius"]
            aabb.append(np.concatenate([(lo + hi) / 2, (hi - lo) / 2]))
        cm.geom_aabb = np.array(aabb).reshape(-1, 6)
        cm.geom_radius = np.array([g["radius"] for g in cgeoms], np.float64)
        cm.geom_cyl = np.array([g["cyl"] for g in cgeoms], np.float64).reshape(-1, 2)
        cm.geom_rbound = np.array([float(np.max(np.linalg.norm(hulls[g["hull"]], axis=1)))
                                   for g in cgeoms], np.float64)
        cm.geom_type = np.array([GEOM_TYPES[g["type"]] for g in cgeoms], np.int32)
        # per-geom contact parameters after the default-class cascade (the pairs
        # mix them; kept for tests of a template's classes)
        cm.geom_condim = np.array([g["condim"] for g in cgeoms], np.int32)
        cm.geom_friction = np.array([g["friction"] for g in cgeoms], np.float64).reshape(-1, 3)
        cm.geom_solref = np.array([g["solref"] for g in cgeoms], np.float64).reshape(-1, 2)
        cm.geom_priority = np.array([g["priority"] for g in cgeoms], np.int32)
        cm.geom_size = np.array([g["size"] for g in cgeoms], np.float64).reshape(-1, 3)
        cm.hull_vertnum = np.array([len(h) for h in hulls], np.int32)
        cm.hull_vertadr = np.concatenate([[0], np.cumsum(cm.hull_vertnum)[:-1]]).astype(np.int32) if hulls else np.zeros(0, np.int32)
        cm.hull_vert = np.concatenate(hulls).reshape(-1, 3) if hulls else np.zeros((0, 3))
        # interior point of each hull for MPR: the geom frame origin, as MuJoCo's
        # ccd centre (geom_xpos); for meshes that is the mesh's centre of mass
        cm.hull_center = np.zeros((len(hulls), 3))
        cm.pair_geom1 = np.array([p["g1"] for p in pairs], np.int32)
        cm.pair_geom2 = np.array([p["g2"] for p in pairs], np.int32)
        cm.pair_condim = np.array([p["condim"] for p in pairs], np.int32)
        cm.pair_kind = np.array([p["kind"] for p in pairs], np.int32)
        cm.pair_friction = np.array([p["friction"] for p in pairs]).reshape(-1, 5)
        cm.pair_solref = np.array([p["solref"] for p in pairs]).reshape(-1, 2)
        cm.pair_solimp = np.array([p["solimp"] for p in pairs]).reshape(-1, 5)
        cm.pair_margin = np.array([p["margin"] for p in pairs])
        cm.eq_type = np.array([e["type"] for e in eqs], np.int32)
        cm.eq_obj1id = np.array([e["o1"] for e in eqs], np.int32)
        cm.eq_obj2id = np.array([e["o2"] for e in eqs], np.int32)
        cm.eq_data = np.array([e["data"] for e in eqs]).reshape(-1, 11)
        cm.eq_solref = np.array([_fv(e["e"], "solref") for e in eqs]).reshape(-1, 2)
        cm.eq_solimp = np.array([_fv(e["e"], "solimp") for e in eqs]).reshape(-1, 5)
        cm.tendon_adr = np.array(tadr, np.int32)
        cm.tendon_num = np.array(tnum, np.int32)
        cm.wrap_dofid = np.array([w[0] for w in wraps], np.int32)
        cm.wrap_qposadr = np.array([w[1] for w in wraps], np.int32)
        cm.wrap_coef = np.array([w[2] for w in wraps], np.float64)
        cm.actuator_trntype = np.array([a["trn"] for a in acts], np.int32)
        cm.actuator_trnid = np.array([a["tid"] for a in acts], np.int32)
        cm.actuator_gaintype = np.array([a["gt"] for a in acts], np.int32)
        cm.actuator_biastype = np.array([a["bt"] for a in acts], np.int32)
        cm.actuator_ctrllimited = np.array([a["ctrllimited"] for a in acts], np.int32)
        cm.actuator_forcelimited = np.array([a["forcelimited"] for a in acts], np.int32)
        cm.actuator_gainprm = np.array([a["gainprm"] for a in acts]).reshape(-1, 3)
        cm.actuator_biasprm = np.array([a["biasprm"] for a in acts]).reshape(-1, 3)
        cm.actuator_ctrlrange = np.array([a["ctrlrange"] for a in acts]).reshape(-1, 2)
        cm.actuator_forcerange = np.array([a["forcerange"] for a in acts]).reshape(-1, 2)
        cm.actuator_gear = np.array([a["gear"] for a in acts], np.float64)
        # actuator state (mujoco.pid: integral, previous setpoint), mjData.act
        cm.actuator_actnum = np.array([a["actnum"] for a in acts], np.int32)
        cm.actuator_actadr = np.where(cm.actuator_actnum > 0,
                                      np.concatenate([[0], np.cumsum(cm.actuator_actnum)[:-1]]) if acts else 0,
                                      -1).astype(np.int32)
        cm.nact = int(cm.actuator_actnum.sum()) if acts else 0
        cm.actuator_pidprm = np.array([a["pid"] for a in acts], np.float64).reshape(-1, 5)
        # gravity compensation (body gravcomp, MuJoCo mj_gravcomp): a passive
        # force -gravity * mass * gravcomp at the body's centre of mass
        cm.body_gravcomp = np.array([b.gravcomp for b in self.bodies], np.float64)
        cm.body_xpos0 = xpos
        cm.body_xquat0 = xquat
        cm.body_invweight0, cm.dof_invweight0, cm.meaninertia = _invweight0(cm)
        return cm


def _invweight0(cm):
    """MuJoCo's mj_setConst inverse weights at qpos0 (engine_setconst.c):

      body_invweight0[b] = (mean diag of Jt M^-1 Jt', mean diag of Jr M^-1 Jr')
                           with J the body-COM Jacobian (0 for world-welded bodies),
      dof_invweight0[d]  = diag(M^-1) (free joints: mean over the 3 translational
                           and over the 3 rotational dofs).

    They define efc_diagApprox, from which the constraint regulariser R is built
    (R = (1 - imp) / imp * diagApprox; engine_core_constraint.c mj_diagApprox /
    mj_makeImpedance).  Joint values at qpos0 are the reference configuration,
    so body frames are the compiled body_xpos0 / body_xquat0."""
    nb, nv = cm.nbody, cm.nv
    xpos, xquat = cm.body_xpos0, cm.body_xquat0
    xmat = np.array([quat2mat(q) for q in xquat])
    xipos = np.array([xpos[b] + xmat[b] @ cm.body_ipos[b] for b in range(nb)])
    ximat = np.array([xmat[b] @ quat2mat(cm.body_iquat[b]) for b in range(nb)])
    # world-frame dof axes (angular part) and anchors
    dof_w = np.zeros((nv, 3))      # angular direction (0 for translations)
    dof_v = np.zeros((nv, 3))      # translational direction (slide / free xyz)
    dof_anchor = np.zeros((nv, 3))
    for j in range(len(cm.jnt_type)):
        b, da, t = cm.jnt_bodyid[j], cm.jnt_dofadr[j], cm.jnt_type[j]
        anchor = xpos[b] + xmat[b] @ cm.jnt_pos[j]
        axis = xmat[b] @ cm.jnt_axis[j]
        if t == 0:
            for k in range(3):
                dof_v[da + k, k] = 1.0
                dof_w[da + 3 + k] = xmat[b][:, k]
                dof_anchor[da + 3 + k] = anchor
        elif t == 1:
            for k in range(3):
                dof_w[da + k] = xmat[b][:, k]
                dof_anchor[da + k] = anchor
        elif t == 2:
            dof_v[da] = axis
        else:
            dof_w[da] = axis
            dof_anchor[da] = anchor
    # body COM Jacobians (dofs on the path to the root)
    def jac(b):
        Jt, Jr = np.zeros((3, nv)), np.zeros((3, nv))
        d = cm.body_lastdof[b]
        while d >= 0:
            Jr[:, d] = dof_w[d]
            Jt[:, d] = dof_v[d] + np.cross(dof_w[d], xipos[b] - dof_anchor[d])
            d = cm.dof_parentid[d]
        return Jt, Jr
    M = np.diag(np.asarray(cm.dof_armature, np.float64)).copy() if nv else np.zeros((0, 0))
    Js = [None] * nb
    for b in range(1, nb):
        Jt, Jr = jac(b)
        Js[b] = (Jt, Jr)
        I = ximat[b] @ np.diag(cm.body_inertia[b]) @ ximat[b].T
        M += cm.body_mass[b] * Jt.T @ Jt + Jr.T @ I @ Jr
    Minv = np.linalg.inv(M) if nv else M
    biw = np.zeros((nb, 2))
    for b in range(1, nb):
        if cm.body_weldid[b] == 0 or cm.body_lastdof[b] < 0:
            continue
        Jt, Jr = Js[b]
        biw[b, 0] = max(_MINVAL, np.trace(Jt @ Minv @ Jt.T) / 3.0)
        biw[b, 1] = max(_MINVAL, np.trace(Jr @ Minv @ Jr.T) / 3.0)
    diw = np.diag(Minv).copy() if nv else np.zeros(0)
    for j in range(len(cm.jnt_type)):
        da, t = cm.jnt_dofadr[j], cm.jnt_type[j]
        if t == 0:
            diw[da:da + 3] = diw[da:da + 3].mean()
            diw[da + 3:da + 6] = diw[da + 3:da + 6].mean()
        elif t == 1:
            diw[da:da + 3] = diw[da:da + 3].mean()
    # stat.meaninertia: mean diagonal of M (armature included) at qpos0
    meaninertia = float(np.trace(M) / nv) if nv else 1.0
    return biw, diw, meaninertia


class CompiledModel:
    """Flat model arrays (numpy) + packing into the mgs_model_desc buffers."""

    nq: int
    nv: int

    def jnt_qposadr_by_name(self, name):
        """mujoco.mj_name2id + jnt_qposadr, including the reference's -1 quirk:
        an unknown joint name gives id -1 and numpy's jnt_qposadr[-1] is the
        LAST joint's address (mgs/core/simualtion.py:37-43)."""
        try:
            jid = self.jnt_names.index(name)
        except ValueError:
            jid = -1
        return int(self.jnt_qposadr[jid])

    def actuator_moment(self):
        """(nu, nv) actuator moment rows, constant for joint and fixed-tendon
        transmissions: the kernels' / oracle's actuation() sums (joint: gear at
        the joint's dof; tendon: 0 + wrap coef x gear over the wraps in order)"""
        mom = np.zeros((self.nu, self.nv))
        for u in range(self.nu):
            g = float(self.actuator_gear[u])
            t = int(self.actuator_trnid[u])
            if int(self.actuator_trntype[u]) == 0:
                mom[u, int(self.jnt_dofadr[t])] = g
            else:
                for w in range(int(self.tendon_adr[t]), int(self.tendon_adr[t]) + int(self.tendon_num[t])):
                    k = int(self.wrap_dofid[w])
                    mom[u, k] = float(mom[u, k]) + float(self.wrap_coef[w]) * g
        return mom

    def body_dofmask(self):
        """(nbody, W) int32 bit masks of the dofs on each body's chain to the root:
        W = 2 words (dofs 0-63), 4 for models of more than 64 dofs (mgs_gpu.h)"""
        m = np.zeros((self.nbody, 4 if self.nv > 64 else 2), np.uint32)
        for b in range(self.nbody):
            d = int(self.body_lastdof[b])
            while d >= 0:
                m[b, d // 32] |= np.uint32(1) << np.uint32(d % 32)
                d = int(self.dof_parentid[d])
        return m.view(np.int32)

    @property
    def nu(self):
        return len(self.actuator_trntype)

    def geom_id(self, name):
        return self.geom_names.index(name)

    def ccd_mode(self):
        """mgs_model_desc.ccd_mode of this model: options["contact_model"] "r5"
        (round 5's face-clipping manifold, kept for the contact-set study) -> 0;
        else MuJoCo 3.2.2's collision table restated, with the multiccd flag
        (<flag multiccd="enable"/>) -> 1, without -> 2"""
        o = self.options
        if o.get("contact_model", "mujoco") == "r5":
            return 0
        return 1 if o.get("multiccd", False) else 2

    def pair_table(self, ccd_mode):
        """(geom1, geom2, kind) of every admissible pair for a ccd mode.  Mode 0:
        the compiled order (geom index) with the convex / box-box kinds.  Modes
        1-2: MuJoCo's collision table (engine_collision_driver.c mjCOLLISIONFUNC,
        indexed by type1 <= type2: mj_collideGeoms swaps a pair whose first geom
        has the larger type): the analytic colliders for sphere / capsule / box /
        cylinder pairs (engine_collision_primitive.c), mjc_BoxBox for box pairs,
        and mjc_Convex (MPR) for the rest -- a pair with a sphere never takes
        multiccd (mjc_Convex skips spheres and ellipsoids)."""
        g1 = np.asarray(self.pair_geom1, np.int32).copy()
        g2 = np.asarray(self.pair_geom2, np.int32).copy()
        kind = np.asarray(self.pair_kind, np.int32).copy()
        if ccd_mode == 0 or len(g1) == 0:
            return g1, g2, kind
        t = np.asarray(self.geom_type)
        for p in range(len(g1)):
            a, b = int(g1[p]), int(g2[p])
            if t[a] > t[b]:
                a, b = b, a
            g1[p], g2[p] = a, b
            ta, tb = int(t[a]), int(t[b])
            k = _PRIM_KIND.get((ta, tb))
            if k is None:
                k = PAIR_CONVEX_SMOOTH if GEOM_TYPES["sphere"] in (ta, tb) else PAIR_CONVEX
            kind[p] = k
        return g1, g2, kind

    def pack(self, ncon_max=16, nefc_max=None):
        """Build (desc_fields dict, ibuf int32 array, dbuf float64 array)."""
        ibuf, dbuf = [], []
        fields = {}

        def put_i(name, arr):
            a = np.ascontiguousarray(np.asarray(arr, np.int32).ravel())
            fields["i_" + name] = sum(len(x) for x in ibuf)
            ibuf.append(a)

        def put_d(name, arr):
            a = np.ascontiguousarray(np.asarray(arr, np.float64).ravel())
            fields["d_" + name] = sum(len(x) for x in dbuf)
            dbuf.append(a)

        for n in ["body_parentid", "body_rootid", "body_mocapid", "body_jntnum", "body_jntadr",
                  "body_dofnum", "body_dofadr", "body_lastdof"]:
            put_i(n, getattr(self, n))
        put_i("body_dofmask", self.body_dofmask())
        depth = np.zeros(self.nbody + 1, np.int32)
        for b in range(1, self.nbody):
            depth[b] = depth[self.body_parentid[b]] + 1
        depth[self.nbody] = depth[:self.nbody].max()
        put_i("body_depth", depth)
        kids = [[c for c in range(self.nbody - 1, 0, -1) if self.body_parentid[c] == b] for b in range(self.nbody)]
        adr = np.cumsum([0] + [len(k) for k in kids])[:-1]
        put_i("body_childadr", adr)
        put_i("body_childnum", [len(k) for k in kids])
        put_i("body_child", [c for k in kids for c in k] or [0])
        for n in ["body_pos", "body_quat", "body_ipos", "body_iquat", "body_mass", "body_inertia",
                  "body_gravcomp", "body_invweight0", "dof_invweight0"]:
            put_d(n, getattr(self, n))
        for n in ["jnt_type", "jnt_qposadr", "jnt_dofadr", "jnt_bodyid", "jnt_limited"]:
            put_i(n, getattr(self, n))
        for n in ["jnt_pos", "jnt_axis", "jnt_range", "jnt_solref", "jnt_solimp", "jnt_margin",
                  "jnt_stiffness"]:
            put_d(n, getattr(self, n))
        for n in ["dof_bodyid", "dof_jntid", "dof_parentid"]:
            put_i(n, getattr(self, n))
        for n in ["dof_armature", "dof_damping", "dof_frictionloss", "dof_solref", "dof_solimp",
                  "qpos0", "qpos_spring"]:
            put_d(n, getattr(self, n))
        # initial velocity state shared by every candidate (mj_resetData: zeros;
        # ClutterTableEnv: the scene's env_state, clutter_table.py:290-291)
        put_d("qvel0", getattr(self, "qvel0", None) if getattr(self, "qvel0", None) is not None
              else np.zeros(self.nv))
        put_d("qacc_ws0", getattr(self, "qacc_ws0", None) if getattr(self, "qacc_ws0", None) is not None
              else np.zeros(self.nv))
        for n in ["geom_bodyid", "geom_hullid", "geom_side"]:
            put_i(n, getattr(self, n))
        for n in ["geom_pos", "geom_quat", "geom_aabb", "geom_radius", "geom_rbound", "geom_cyl"]:
            put_d(n, getattr(self, n))
        put_d("geom_size", self.geom_size)
        put_i("hull_vertadr", self.hull_vertadr)
        put_i("hull_vertnum", self.hull_vertnum)
        # per hull x[n], y[n], z[n] (SoA): the kernels' support scans then read
        # 64 consecutive doubles per load instead of a 24-byte stride
        put_d("hull_vert", np.concatenate([self.hull_vert[a:a + n].T.ravel()
                                           for a, n in zip(self.hull_vertadr, self.hull_vertnum)])
              if len(self.hull_vertnum) else self.hull_vert)
        put_d("hull_center", self.hull_center)
        ccd_mode = self.ccd_mode()
        g1, g2, kind = self.pair_table(ccd_mode)
        put_i("pair_geom1", g1)
        put_i("pair_geom2", g2)
        put_i("pair_condim", self.pair_condim)
        put_i("pair_kind", kind)
        for n in ["pair_friction", "pair_solref", "pair_solimp", "pair_margin"]:
            put_d(n, getattr(self, n))
        for n in ["eq_type", "eq_obj1id", "eq_obj2id"]:
            put_i(n, getattr(self, n))
        for n in ["eq_data", "eq_solref", "eq_solimp"]:
            put_d(n, getattr(self, n))
        for n in ["tendon_adr", "tendon_num", "wrap_dofid", "wrap_qposadr"]:
            put_i(n, getattr(self, n))
        put_d("wrap_coef", self.wrap_coef)
        for n in ["actuator_trntype", "actuator_trnid", "actuator_gaintype", "actuator_biastype",
                  "actuator_ctrllimited", "actuator_forcelimited"]:
            put_i(n, getattr(self, n))
        for n in ["actuator_gainprm", "actuator_biasprm", "actuator_ctrlrange", "actuator_forcerange",
                  "actuator_gear"]:
            put_d(n, getattr(self, n))
        put_d("actuator_moment", self.actuator_moment())
        put_i("actuator_actadr", self.actuator_actadr)
        put_d("actuator_pidprm", self.actuator_pidprm)
        # initial actuator state shared by every candidate (mj_resetData: zeros;
        # ClutterTableEnv: the scene's env_state)
        put_d("act0", getattr(self, "act0", None) if getattr(self, "act0", None) is not None
              else np.zeros(int(self.nact)))
        ib = np.concatenate(ibuf) if ibuf else np.zeros(0, np.int32)
        db = np.concatenate(dbuf) if dbuf else np.zeros(0, np.float64)
        neqrow = sum({0: 3, 1: 6, 2: 1}[int(t)] for t in self.eq_type)
        nfric = int(np.sum(self.dof_frictionloss > 0))
        nlim = int(np.sum(self.jnt_limited))
        maxdim = int(self.pair_condim.max()) if len(self.pair_condim) else 1
        if nefc_max is None:
            # worst case (every contact at the largest condim); the kernels hold
            # 2 (main build) or 4 (wide build) rows per lane: at most 256
            nefc_max = min(256, neqrow + nfric + nlim + ncon_max * maxdim)
        o = self.options
        fields.update(
            nq=self.nq, nv=self.nv, nbody=self.nbody, njnt=len(self.jnt_type),
            ngeom=len(self.geom_bodyid), nhull=len(self.hull_vertnum),
            nhullvert=len(self.hull_vert), npair=len(self.pair_geom1), neq=len(self.eq_type),
            ntendon=len(self.tendon_adr), nwrap=len(self.wrap_dofid), nu=self.nu, nmocap=self.nmocap,
            nact=int(self.nact), npid=int(np.sum(np.asarray(self.actuator_gaintype) == GAIN_PID)),
            maxcondim=maxdim, ncon_max=ncon_max, nefc_max=nefc_max,
            maxhullvert=int(self.hull_vertnum.max()) if len(self.hull_vertnum) else 0,
            iterations=int(o["iterations"]), noslip_iterations=int(o["noslip_iterations"]),
            cone=1, integrator=2, solver={"PGS": 0, "CG": 2, "Newton": 2}[o.get("solver", "Newton")],
            ls_iterations=int(o.get("ls_iterations", 50)), ls_tolerance=float(o.get("ls_tolerance", 0.01)),
            timestep=float(o["timestep"]), impratio=float(o["impratio"]),
            tolerance=float(o["tolerance"]), noslip_tolerance=float(o["noslip_tolerance"]),
            mpr_tolerance=float(o.get("mpr_tolerance", 1e-6)), meaninertia=float(self.meaninertia),
            ccd_mode=ccd_mode, ccd_iterations=int(o.get("ccd_iterations", 50)),
            gravity=[float(x) for x in o["gravity"]], isize=len(ib), dsize=len(db))
        return fields, ib, db


def compile_xml(xml: str, assets: Optional[Dict[str, bytes]] = None) -> CompiledModel:
    return Compiler(xml, assets).compile()
