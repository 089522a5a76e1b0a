"""Contact-based grasp sampler for dexterous hands (reference:
mgs/sampler/contact.py, ContactBasedDiff).

generate_grasps(num, kin) keeps the reference's steps and constants:

1. max(30000, 3 num) surface points, area-weighted with trimesh's uniform
   triangle sampling, and their face normals (contact.py:180-189);
2. num farthest-point seeds (contact.py:191-194)            -> GPU mgs_contact_fps
3. per seed the nearest other seed and ntip random seeds within 10 cm
   (contact.py:196-214, 226-228)                             -> GPU mgs_contact_seeds
4. targets = picked seeds + 2 cm along their normals; the initial frame
   z = seed normal, x toward the nearest seed, y = z x x, aligned by the
   model's approach transform, placed 5 cm out along the normal
   (contact.py:215-236);
5. 150 AdamW(0.005) steps on (6-D rotation, position, joints) per candidate
   with the fingertip-target assignment redone every step, joints clipped to
   their ranges (contact.py:98-158, 238-280)                -> GPU mgs_contact_optimize
6. poses [R | t] (float32, rows of the Gram-Schmidt matrix) and joints
   (contact.py:282-297).

Differences from the reference, all documented in DESIGN.md: float64
arithmetic (the reference runs JAX float32); random draws from a numpy
Generator and splitmix64 keys instead of jax.random (PRNGKey(0)); a fresh
optimiser state per call (the reference's Trainer reuses its optax state across
calls of one sampler object).  No CPU fallback: every numeric stage above the
host-side frame construction runs on the MI355X.
"""
from itertools import permutations

import numpy as np

from mgs.core import abi, engine
from mgs.sampler.antipodal import load_obj_mesh
from mgs.sampler.kin.model import KinematicsModel

NUM_SURFACE_SAMPLES = 30000
LOCAL_REGION_RADIUS = 0.10
TARGET_OFFSET_DISTANCE = 0.02
POSE_OFFSET_DISTANCE = 0.05
ITERATIONS = 150
LEARNING_RATE = 0.005
COS_WEIGHT = 0.001


def normalize_vector(v, eps=1e-6):
    """jax_util.normalize_vector: v / (|v| + eps)"""
    return v / (np.linalg.norm(v, axis=-1, keepdims=True) + eps)


def sample_surface(verts, faces, count, rng):
    """trimesh.sample.sample_surface: faces drawn by area, points by the
    reflected unit-square parametrisation; returns (points, face index)"""
    tri = verts[faces]
    cr = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
    area = 0.5 * np.linalg.norm(cr, axis=1)
    cum = np.cumsum(area)
    fidx = np.searchsorted(cum, rng.random(count) * cum[-1])
    fidx = np.minimum(fidx, len(faces) - 1)
    origin = tri[fidx, 0]
    vec = tri[fidx, 1:] - origin[:, None, :]
    lengths = rng.random((count, 2, 1))
    flip = lengths.sum(axis=1).reshape(-1) > 1.0
    lengths[flip] -= 1.0
    lengths = np.abs(lengths)
    return origin + (vec * lengths).sum(axis=1), fidx


def face_normals(verts, faces):
    tri = verts[faces]
    cr = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
    return cr / np.maximum(np.linalg.norm(cr, axis=1, keepdims=True), 1e-30)


def kin_desc(kin: KinematicsModel, contact_choice, iters=ITERATIONS, lr=LEARNING_RATE):
    """the C-ABI view of a kinematic model (include/mgs_gpu.h mgs_kin_desc);
    contact_choice[a] picks tip a's contact point (contact.py:248-253)"""
    M = abi.MGS
    d = abi.KinDesc()
    nd, nt = kin.num_dofs, len(kin.fingertip_idx)
    if nd > M["MGS_KIN_MAXDOF"] or nt > M["MGS_KIN_MAXTIP"]:
        raise ValueError("kinematic model too large for the contact kernels")
    perms = list(permutations(range(nt)))
    d.ndof, d.ntip, d.nperm, d.iters = nd, nt, len(perms), int(iters)
    par = kin.parents()
    for a, tip in enumerate(kin.fingertip_idx):
        ch = [int(tip)]
        while par[ch[-1]] >= 0:
            ch.append(int(par[ch[-1]]))
        ch.reverse()
        if len(ch) > M["MGS_KIN_MAXCHAIN"]:
            raise ValueError("finger chain too long for the contact kernels")
        d.chain_len[a] = len(ch)
        for s, i in enumerate(ch):
            d.chain[a][s] = i
        for j in range(3):
            d.tip_point[a][j] = float(kin.tip_contacts[a, contact_choice[a], j])
            d.tip_normal[a][j] = float(kin.tip_normals[a, j])
    for q, p in enumerate(perms):
        for a in range(nt):
            d.perm[q][a] = p[a]
    for i in range(nd):
        for j in range(7):
            d.kin_tf[i][j] = float(kin.kin_tf[i, j])
        for j in range(6):
            d.joint_tf[i][j] = float(kin.joint_tf[i, j])
        d.range[i][0], d.range[i][1] = float(kin.joint_ranges[i, 0]), float(kin.joint_ranges[i, 1])
        d.pregrasp[i] = float(kin.pregrasp[i])
    # optax.adamw(learning_rate) defaults
    d.lr, d.b1, d.b2, d.eps, d.eps_root, d.weight_decay = float(lr), 0.9, 0.999, 1e-8, 0.0, 1e-4
    d.w_cos = COS_WEIGHT
    return d


def initial_frames(seeds, seed_normals, nn, kin: KinematicsModel):
    """contact.py:226-236: the (non-orthonormal) initial rotation and position"""
    z = seed_normals
    x = normalize_vector(seeds[nn] - seeds)
    y = np.cross(z, x)
    R0 = np.stack([x, y, z], axis=-1)
    align_pos = np.einsum("...ij,j->...i", R0, kin.align_pos)
    R = np.einsum("...ij,jk->...ik", R0, kin.align_rot)
    p = seeds + POSE_OFFSET_DISTANCE * seed_normals + align_pos
    return R, p


class ContactBasedDiff:
    """drop-in for the reference's ContactBasedDiff(obj).generate_grasps(num, kin)"""

    def __init__(self, obj, rng=None, device=0):
        self.mesh_file_path = obj.obj_file_path
        self.verts, self.faces = load_obj_mesh(self.mesh_file_path)
        self.rng = rng if rng is not None else np.random.default_rng(0)
        self.device = device
        self.last = {}

    def update_object(self, obj):
        self.mesh_file_path = obj.obj_file_path
        self.verts, self.faces = load_obj_mesh(self.mesh_file_path)
        return self

    def prepare(self, num, kin: KinematicsModel):
        """steps 1-4 (seeds and targets on the GPU, frames on the host); returns
        the optimiser inputs and the kin descriptor"""
        rng = self.rng
        pts, fidx = sample_surface(self.verts, self.faces, max(NUM_SURFACE_SAMPLES, num * 3), rng)
        normals = normalize_vector(face_normals(self.verts, self.faces)[fidx])
        nt = len(kin.fingertip_idx)
        fps, ms_fps = engine.contact_fps(pts, num, device=self.device)
        seeds, seed_normals = pts[fps], normals[fps]
        key = int(rng.integers(0, 2**63))
        nn, sel, ms_sel = engine.contact_seeds(seeds, LOCAL_REGION_RADIUS, key, nt, device=self.device)
        targets = seeds[sel] + TARGET_OFFSET_DISTANCE * seed_normals[sel]
        tnormals = seed_normals[sel]
        R, p = initial_frames(seeds, seed_normals, nn, kin)
        choice = rng.integers(0, kin.tip_contacts.shape[1], size=nt)
        self.last = dict(points=pts, normals=normals, fps=fps, nn=nn, sel=sel, choice=choice,
                         kernel_ms={"fps": ms_fps, "seeds": ms_sel})
        return dict(rot_init=R, pos_init=p, targets=targets, normals=tnormals), kin_desc(kin, choice)

    def generate_grasps(self, num: int, gripper: KinematicsModel):
        inp, desc = self.prepare(num, gripper)
        r = engine.contact_optimize(desc, inp["rot_init"], inp["pos_init"], inp["targets"], inp["normals"],
                                    device=self.device)
        self.last["kernel_ms"]["optimize"] = r["kernel_ms"]
        self.last["loss"] = r["loss"]
        H = np.zeros((num, 4, 4), np.float32)
        H[:, :3, :3] = r["rot"]
        H[:, :3, 3] = r["pos"]
        H[:, 3, 3] = 1.0
        return H, {"joints": r["joints"].astype(np.float32)}
