"""SE(3) pose container with the reference's float32 semantics.

Mirrors mgs/util/geo/transforms.py:28-128 of the reference: positions and
quaternions are cast to float32 on construction (:34-45), composition goes
through 4x4 matrices built with scipy's Rotation (:93-97, :109-121) and
`from_mat` uses `as_quat(canonical=False)` (:79-88).  These casts define the
input quantisation of the hot path, so they are kept
bit-for-bit; tests/golden/se3_golden.npz (tests/golden/make_se3_golden.py, generated
from the reference's own SE3Pose) pins them (tests/test_model_and_host.py).
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import numpy as np
from scipy.spatial.transform import Rotation

from mgs.util.geo.operations import quaternion_apply, quaternion_invert


# large pose batches: scipy's from_matrix (an SVD per float32 matrix) over
# row blocks on 4 threads; 8 measured slower on the GPU box (GIL contention:
# 12.3 -> 18.4 ms for 8192 poses, profiles/r04o_api_breakdown.txt)
_PAR_MIN, _PAR_CHUNKS = 2048, 4
_POOL = None


def _pool():
    global _POOL
    if _POOL is None:
        from concurrent.futures import ThreadPoolExecutor
        _POOL = ThreadPoolExecutor(_PAR_CHUNKS)
    return _POOL


def _drop_pool():
    global _POOL
    _POOL = None


# a forked child inherits the executor object but not its threads
os.register_at_fork(after_in_child=_drop_pool)


# from_mat's fast path (round 6): scipy 1.15's Rotation.from_matrix takes the
# nearest rotation of every non-orthogonal matrix with an SVD (U @ Vt) and
# then Markley's method; a float32 pose product is never orthogonal to its
# 1e-12 test, so the SVD ran on every pose (most of the drop-in API's host
# time, profiles/r06p_api_breakdown.txt).  The same polar factor comes from
# three Newton steps X <- (X + X^-T) / 2 (quadratic from the float32 matrix's
# 1e-7 defect), followed by the same Markley formulas in the same operation
# order; measured against scipy the float64 quaternions differ by <= 3e-15
# (tests/test_model_and_host.py).  What SE3Pose keeps is their float32
# rounding, so a row takes scipy's own path whenever that rounding or the
# branch could depend on a difference that small: a component within
# _FAST_TOL of a float32 rounding midpoint or below _FAST_SMALL in magnitude,
# Markley's two largest decision values within _FAST_GAP, a matrix that scipy
# would take as already orthogonal (no SVD), or any non-finite / det <= 0
# input (scipy raises).  The result is scipy's, row for row.
_FAST_MIN = 64
_FAST_TOL = 1e-13
_FAST_SMALL = 1e-5
_FAST_GAP = 1e-9


def _scipy_quat(R):
    if R.ndim == 3 and len(R) >= _PAR_MIN:
        # scipy orthogonalises every float32 matrix with an SVD; chunks are
        # independent, so a thread pool over row blocks returns the identical
        # quaternions
        return np.concatenate(list(_pool().map(lambda c: Rotation.from_matrix(c).as_quat(canonical=False),
                                               np.array_split(R, _PAR_CHUNKS))))
    return Rotation.from_matrix(R).as_quat(canonical=False)


def _fast_quat(R):
    """(n, 3, 3) -> (n, 4) xyzw quaternions equal to scipy's from_matrix(R)
    .as_quat(canonical=False) (see _FAST_* above)"""
    m = np.ascontiguousarray(R.reshape(-1, 9).astype(np.float64).T)  # (9, n)
    if not np.isfinite(m).all():
        return _scipy_quat(R)
    a, b, c, d, e, f, g, h, i = m
    det0 = a * (e * i - f * h) + b * (f * g - d * i) + c * (d * h - e * g)
    if not (det0 > 0).all():
        return _scipy_quat(R)      # scipy's ValueError (or its own handling)
    # scipy's orthogonality test skips the SVD when every Gram entry is within
    # 1e-12 of the identity's: such rows (and near ones) go to scipy
    gram_off = np.maximum.reduce([np.abs(a * d + b * e + c * f), np.abs(a * g + b * h + c * i),
                                  np.abs(d * g + e * h + f * i)])
    for _ in range(3):
        c00, c01, c02 = e * i - f * h, f * g - d * i, d * h - e * g
        c10, c11, c12 = c * h - b * i, a * i - c * g, b * g - a * h
        c20, c21, c22 = b * f - c * e, c * d - a * f, a * e - b * d
        s = 0.5 / (a * c00 + b * c01 + c * c02)
        a, b, c = 0.5 * a + s * c00, 0.5 * b + s * c01, 0.5 * c + s * c02
        d, e, f = 0.5 * d + s * c10, 0.5 * e + s * c11, 0.5 * f + s * c12
        g, h, i = 0.5 * g + s * c20, 0.5 * h + s * c21, 0.5 * i + s * c22
    M = (a, b, c, d, e, f, g, h, i)
    dec = np.stack([a, e, i, a + e + i])
    ch = np.argmax(dec, axis=0)
    srt = np.sort(dec, axis=0)
    q = np.empty((4, m.shape[1]))
    q[0], q[1], q[2], q[3] = h - f, c - g, d - b, 1 + dec[3]
    for k0 in range(3):
        sel = ch == k0
        if not sel.any():
            continue
        k1 = (k0 + 1) % 3
        k2 = (k1 + 1) % 3

        def mm(r, col):
            return M[3 * r + col][sel]
        q[k0, sel] = 1 - dec[3, sel] + 2 * mm(k0, k0)
        q[k1, sel] = mm(k1, k0) + mm(k0, k1)
        q[k2, sel] = mm(k2, k0) + mm(k0, k2)
        q[3, sel] = mm(k2, k1) - mm(k1, k2)
    q = q / np.sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3])
    risky = _near_f32_midpoint(q).any(axis=0)
    risky |= (srt[3] - srt[2]) < _FAST_GAP
    risky |= gram_off < 1e-10
    q = np.ascontiguousarray(q.T)
    if risky.any():
        q[risky] = _scipy_quat(R[risky])
    return q


def _near_f32_midpoint(x):
    """x (float64) within _FAST_TOL of a float32 rounding midpoint, or small"""
    # |x - float32(x)| (exact) against the half spacings on either side of
    # float32(x): u / 2 above, u / 2 or u / 4 (at a power of two) below --
    # both are tested, which only ever flags more rows
    x32 = x.astype(np.float32)
    err = np.abs(x - x32)
    half = np.spacing(np.abs(x32)).astype(np.float64) * 0.5
    return (np.abs(err - half) < _FAST_TOL) | (np.abs(err - 0.5 * half) < _FAST_TOL) | (np.abs(x) < _FAST_SMALL)


def _fast_mat(q_xyzw):
    """(n, 4) xyzw -> (n, 3, 3) float32 equal to scipy's Rotation.from_quat(q)
    .as_matrix() cast to float32: scipy's normalisation and products in its
    order (float64-identical on 300k random rotations), rows whose entries sit
    near a float32 rounding midpoint (or are small) from scipy itself"""
    q = np.ascontiguousarray(np.asarray(q_xyzw).reshape(-1, 4).astype(np.float64).T)
    nrm = np.sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3])
    if not (np.isfinite(nrm).all() and (nrm > 0).all()):
        return Rotation.from_quat(np.copy(q_xyzw)).as_matrix().astype(np.float32)
    x, y, z, w = q / nrm
    x2, y2, z2, w2 = x * x, y * y, z * z, w * w
    xy, zw, xz, yw, yz, xw = x * y, z * w, x * z, y * w, y * z, x * w
    m = np.stack([x2 - y2 - z2 + w2, 2 * (xy - zw), 2 * (xz + yw),
                  2 * (xy + zw), -x2 + y2 - z2 + w2, 2 * (yz - xw),
                  2 * (xz - yw), 2 * (yz + xw), -x2 - y2 + z2 + w2])
    risky = _near_f32_midpoint(m).any(axis=0)
    out = np.ascontiguousarray(m.T).reshape(-1, 3, 3).astype(np.float32)
    if risky.any():
        out[risky] = Rotation.from_quat(np.copy(q_xyzw[risky])).as_matrix().astype(np.float32)
    return out


def _wxyz_to_xyzw(q):
    return np.concatenate([q[..., 1:], q[..., :1]], axis=-1)


def _xyzw_to_wxyz(q):
    return np.concatenate([q[..., 3:], q[..., :3]], axis=-1)


@dataclass
class SE3Pose:
    pos: np.ndarray
    quat: np.ndarray
    type: str  # "wxyz" or "xyzw"

    def __post_init__(self):
        if self.pos.shape[-1] != 3 or self.quat.shape[-1] != 4:
            raise AssertionError("SE3Pose expects (...,3) positions and (...,4) quaternions")
        if self.type not in ("wxyz", "xyzw"):
            raise AssertionError("SE3Pose type must be 'wxyz' or 'xyzw'")
        self.pos = np.asarray(self.pos).astype(np.float32)
        self.quat = np.asarray(self.quat).astype(np.float32)
        sq = np.sum(self.quat ** 2, axis=-1, keepdims=True)
        if not np.all(np.isclose(sq, np.ones_like(sq), rtol=1e-4)):
            raise AssertionError("SE3Pose quaternions must be unit length")

    def to_vec(self, layout="pq", type=None) -> np.ndarray:
        q = np.copy(self.quat)
        if type is not None and type != self.type:
            q = _xyzw_to_wxyz(q) if type == "wxyz" else _wxyz_to_xyzw(q)
        if layout == "pq":
            return np.concatenate([self.pos, q], axis=-1)
        if layout == "qp":
            return np.concatenate([q, self.pos], axis=-1)
        return np.array([])

    @classmethod
    def from_vec(cls, vec: np.ndarray, type: str = "wxyz", layout: str = "pq") -> "SE3Pose":
        if layout == "pq":
            return cls(vec[..., -7:-4], vec[..., -4:], type)
        if layout == "qp":
            return cls(vec[..., 4:7], vec[..., 0:4], type)
        raise ValueError(layout)

    @classmethod
    def from_mat(cls, mat: np.ndarray, type: str = "wxyz") -> "SE3Pose":
        if mat.shape[-2:] != (4, 4):
            raise AssertionError("from_mat expects (...,4,4)")
        if type != "wxyz":
            raise ValueError(type)
        R = mat[..., :3, :3]
        if R.ndim == 3 and len(R) >= _FAST_MIN:
            q = _fast_quat(R)
        else:
            q = _scipy_quat(R)
        return cls(mat[..., :3, 3], _xyzw_to_wxyz(q), type)

    def __getitem__(self, idx) -> "SE3Pose":
        return self.__class__(self.pos[idx], self.quat[idx], self.type)

    def __matmul__(self, other: "SE3Pose") -> "SE3Pose":
        m = np.einsum("...ij,...jk->...ik", self.to_mat(), other.to_mat())
        return self.__class__.from_mat(m, type=self.type)

    def __len__(self) -> int:
        return len(self.pos)

    def to_mat(self) -> np.ndarray:
        q = _wxyz_to_xyzw(self.quat) if self.type == "wxyz" else self.quat
        out = np.zeros((*self.quat.shape[:-1], 4, 4), dtype=np.float32)
        if q.ndim == 2 and len(q) >= _FAST_MIN:
            out[..., :3, :3] = _fast_mat(q)
        else:
            out[..., :3, :3] = Rotation.from_quat(np.copy(q)).as_matrix()
        out[..., :3, 3] = self.pos
        out[..., 3, 3] = 1.0
        return out

    def inverse(self) -> "SE3Pose":
        """reference transforms.py:102-107: conjugate quaternion and
        -quaternion_apply(conj, pos) in the reference's numpy arithmetic
        (operations.py); the receiver is mutated with the un-cast (float64)
        values and a new, float32 SE3Pose is returned."""
        inv_quat = quaternion_invert(self.quat, type=self.type)
        inv_pos = -quaternion_apply(inv_quat, self.pos, type=self.type)
        self.pos = inv_pos
        self.quat = inv_quat
        return SE3Pose(inv_pos, inv_quat, self.type)

    @classmethod
    def randn_se3(cls, num, rng=None) -> "SE3Pose":
        rng = np.random.default_rng() if rng is None else rng
        q = Rotation.random(num, random_state=rng).as_quat(canonical=False)
        return cls(rng.standard_normal((num, 3)), _xyzw_to_wxyz(q), "wxyz")
