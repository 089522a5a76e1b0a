"""Antipodal grasp candidates (reference: mgs/sampler/antipodal.py:96-298).

numpy restatement of AntipodalGraspGenerator without trimesh/rtree (absent
here): area-weighted surface sampling of 5N points, one von-Mises-Fisher ray
direction (kappa=10) around the inward normal per point, +-ray casting against
the object mesh (vectorised Moller-Trumbore), the reference's +-5 cm random
fallback partner, and define_gripper_pose (x = contact1 -> contact2,
z = x cross random, y = z cross x, centre = midpoint).  The reference's
normalise/denormalise round trip (normalize_load + denormalize_points, :41-93)
is kept, including its `(p - offset) * scale` formula.

Unlike the reference (no seeds anywhere, :107,142,147,217), every draw comes
from one numpy Generator so candidate sets are reproducible.
"""
from __future__ import annotations

import numpy as np
from scipy.stats import vonmises_fisher

from mgs.core.mjcf import load_mesh_bytes


def load_obj_mesh(path):
    v, f = load_mesh_bytes(open(path, "rb").read(), path)
    return v, f


def _ray_mesh(origins, dirs, tri, eps=1e-12):
    """all hits: returns list of arrays of hit points per ray."""
    v0, v1, v2 = tri[:, 0], tri[:, 1], tri[:, 2]
    e1, e2 = v1 - v0, v2 - v0
    hits = []
    for o, d in zip(origins, dirs):
        p = np.cross(d, e2)
        det = np.einsum("ij,ij->i", e1, p)
        ok = np.abs(det) > eps
        inv = np.where(ok, 1.0 / np.where(ok, det, 1.0), 0.0)
        tv = o - v0
        u = np.einsum("ij,ij->i", tv, p) * inv
        q = np.cross(tv, e1)
        w = (q @ d) * inv
        t = np.einsum("ij,ij->i", e2, q) * inv
        m = ok & (u >= 0) & (w >= 0) & (u + w <= 1) & (t > 0)
        hits.append(o + t[m, None] * d)
    return hits


class AntipodalGraspGenerator:
    def __init__(self, mesh_file_path: str, rng=None):
        self.mesh_file_path = mesh_file_path
        self.rng = np.random.default_rng(0) if rng is None else rng
        self.scale = 1.0
        self.offset = np.zeros(3)

    def denormalize_points(self, points):
        return (points - self.offset) * self.scale

    def normalize_load(self):
        v, f = load_obj_mesh(self.mesh_file_path)
        tri = v[f]
        area = 0.5 * np.linalg.norm(np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0]), axis=1)
        centroid = (tri.mean(1) * area[:, None]).sum(0) / area.sum()
        ext = v.max(0) - v.min(0)
        self.scale = float(np.linalg.norm(ext))          # trimesh.Trimesh.scale
        vn = v / self.scale
        c_n = centroid / self.scale
        self.offset = -c_n
        self.verts = vn - c_n
        self.faces = f

    def generate_grasps(self, num: int, kappa: float = 10.0, eps: float = 1e-5):
        self.normalize_load()
        rng = self.rng
        tri = self.verts[self.faces]
        cr = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
        area = 0.5 * np.linalg.norm(cr, axis=1)
        normals = cr / np.maximum(np.linalg.norm(cr, axis=1, keepdims=True), 1e-30)
        fidx = rng.choice(len(tri), size=5 * num, p=area / area.sum())
        r1, r2 = rng.random((2, 5 * num, 1))
        s1 = np.sqrt(r1)
        pts = (1 - s1) * tri[fidx, 0] + s1 * (1 - r2) * tri[fidx, 1] + s1 * r2 * tri[fidx, 2]
        nrm = normals[fidx]
        dirs = np.empty_like(pts)
        for i in range(len(pts)):
            d = vonmises_fisher.rvs(mu=-nrm[i], kappa=kappa, size=1, random_state=rng)[0]
            dirs[i] = d / np.linalg.norm(d)
        one, two = [], []
        for i in range(len(pts)):
            if len(one) >= num:
                break
            o = pts[i]
            hits = _ray_mesh([o, o], [dirs[i], -dirs[i]], tri)
            cand = [h for hh in hits for h in hh if np.linalg.norm(h - o) >= eps]
            if cand:
                loc = cand[rng.integers(len(cand))]
            else:
                loc = o + rng.uniform(-0.05, 0.05, size=3)
            one.append(o)
            two.append(loc)
        while len(one) < num:
            o = pts[rng.integers(len(pts))]
            one.append(o)
            two.append(o + rng.uniform(-0.05, 0.05, size=3))
        one, two = np.array(one), np.array(two)
        H = self.define_gripper_pose(one, two, rng)
        H[..., :3, 3] = self.denormalize_points(H[..., :3, 3])
        widths = np.maximum(np.linalg.norm(two - one, axis=1), 0) * self.scale
        return H, {"width": widths}

    def draw(self, num: int, kappa: float = 10.0):
        """All random inputs of one batch, drawn vectorised up front (the device
        path): surface points (area-weighted face, uniform barycentric), von
        Mises-Fisher directions around the inward normal (Wood's exact 3-D
        sampler), the hit-choice uniforms and the fallback offsets."""
        rng = self.rng
        tri = self.verts[self.faces]
        cr = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
        area = 0.5 * np.linalg.norm(cr, axis=1)
        normals = cr / np.maximum(np.linalg.norm(cr, axis=1, keepdims=True), 1e-30)
        fidx = rng.choice(len(tri), size=num, p=area / area.sum())
        r1, r2 = rng.random((2, num, 1))
        s1 = np.sqrt(r1)
        pts = (1 - s1) * tri[fidx, 0] + s1 * (1 - r2) * tri[fidx, 1] + s1 * r2 * tri[fidx, 2]
        mu = -normals[fidx]
        xi = rng.random(num)
        w = 1.0 + np.log(xi + (1.0 - xi) * np.exp(-2.0 * kappa)) / kappa
        v = rng.standard_normal((num, 3))
        v -= np.sum(v * mu, axis=1, keepdims=True) * mu
        v /= np.maximum(np.linalg.norm(v, axis=1, keepdims=True), 1e-30)
        dirs = w[:, None] * mu + np.sqrt(np.maximum(1.0 - w * w, 0.0))[:, None] * v
        dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
        return dict(tri=tri, points=pts, dirs=dirs, u=rng.random(num),
                    offset=rng.uniform(-0.05, 0.05, size=(num, 3)))

    def finish(self, one, two, rng):
        H = self.define_gripper_pose(one, two, rng)
        H[..., :3, 3] = self.denormalize_points(H[..., :3, 3])
        widths = np.maximum(np.linalg.norm(two - one, axis=1), 0) * self.scale
        return H, {"width": widths}

    def generate_grasps_device(self, num: int, kappa: float = 10.0, eps: float = 1e-5, device: int = 0):
        """generate_grasps with the ray casting of every point on the MI355X
        (mgs_antipodal_contacts): one batch, no per-point host loop."""
        from mgs.core.engine import antipodal_contacts
        self.normalize_load()
        r = self.draw(num, kappa)
        sec, cnt, ms = antipodal_contacts(r["tri"], r["points"], r["dirs"], r["u"], eps, device=device)
        two = np.where((cnt > 0)[:, None], sec, r["points"] + r["offset"])
        H, aux = self.finish(r["points"], two, self.rng)
        aux.update(kernel_ms=ms, hits=cnt)
        return H, aux

    @staticmethod
    def define_gripper_pose(c1, c2, rng):
        n = len(c1)
        center = (c1 + c2) / 2.0
        x = c2 - c1
        nx = np.linalg.norm(x, axis=1, keepdims=True)
        bad = np.isclose(nx, 0.0).ravel()
        x[~bad] /= nx[~bad]
        x[bad] = [1.0, 0.0, 0.0]
        z = np.cross(x, rng.standard_normal((n, 3)))
        nz = np.linalg.norm(z, axis=1, keepdims=True)
        badz = np.isclose(nz, 0.0).ravel()
        z[~badz] /= nz[~badz]
        z[badz] = [0.0, 0.0, 1.0]
        y = np.cross(z, x)
        H = np.zeros((n, 4, 4))
        H[:, :3, 0], H[:, :3, 1], H[:, :3, 2], H[:, :3, 3] = x, y, z, center
        H[:, 3, 3] = 1.0
        return H


def robotiq_candidates(obj, num, seed=0):
    """(pose (num,4,4) float32 contact frames, joints (num,8) zeros = open),
    the candidates.npz layout of gen_grasp_candidates.py:79-82."""
    gen = AntipodalGraspGenerator(obj.obj_file_path, rng=np.random.default_rng(seed))
    H, aux = gen.generate_grasps(num)
    return H.astype(np.float32), np.zeros((num, 8)), aux["width"]


def panda_candidates(obj, num, seed=0, gripper=None):
    """(pose, joints (num,2), width) as gen_grasp_candidates.py:66-71 builds them for
    the Panda: joints = width_to_joints(_clamp_width(width))."""
    from mgs.gripper.panda import GripperPanda
    from mgs.util.geo.transforms import SE3Pose
    g = gripper if gripper is not None else GripperPanda(SE3Pose(np.zeros(3), np.array([1.0, 0, 0, 0]), "wxyz"))
    gen = AntipodalGraspGenerator(obj.obj_file_path, rng=np.random.default_rng(seed))
    H, aux = gen.generate_grasps(num)
    j1, j2 = g.width_to_joints(g._clamp_width(aux["width"]))
    return H.astype(np.float32), np.stack([j1, j2], axis=-1), aux["width"]


def hand_candidates(obj, num, gripper, seed=0):
    """Antipodal contact frames with the hand's open joint configuration, for
    dexterous hands whose own sampler (the reference's JAX contact sampler,
    mgs/sampler/contact.py) is out of scope here: (pose, joints (num, nj), width)."""
    gen = AntipodalGraspGenerator(obj.obj_file_path, rng=np.random.default_rng(seed))
    H, aux = gen.generate_grasps(num)
    site = getattr(gripper, "grasp_site", None)
    if site is not None:
        # hands whose base frame is the wrist (identity base-to-contact): put the
        # hand's grasp site, not the wrist, on the antipodal centre
        H[:, :3, 3] -= H[:, :3, :3] @ np.asarray(site)
    J = np.tile(gripper.open_joints(), (num, 1))
    return H.astype(np.float32), J, aux["width"]
