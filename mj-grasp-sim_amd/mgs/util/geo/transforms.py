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
        if R.ndim == 3 and len(R) >= _PAR_MIN:
            # scipy orthogonalises every float32 matrix with an SVD (most of the
            # host time of a large batch); chunks are independent, so a thread
            # pool over row blocks returns the identical quaternions
            q = np.concatenate(list(_pool().map(lambda c: Rotation.from_matrix(c).as_quat(canonical=False),
                                                 np.array_split(R, _PAR_CHUNKS))))
        else:
            q = Rotation.from_matrix(R).as_quat(canonical=False)
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
