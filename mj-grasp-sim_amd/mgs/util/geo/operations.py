"""Quaternion helpers with the reference's arithmetic (mgs/util/geo/operations.py
of the reference): elementwise numpy products in the order the reference writes
them, so results match bit for bit.  Used by SE3Pose.inverse.

Quirks kept on purpose (they define outputs): `quaternion_invert` multiplies by
an int64 sign vector, so a float32 quaternion comes back float64; the "xyzw"
branch of `quaternion_raw_multiply` reads the components as (w, x, y, z) =
(a[3], a[1], a[2], a[0]) and drops the trailing axis, as the reference does.
"""
from __future__ import annotations

import numpy as np

_SIGN = {"wxyz": np.array([1, -1, -1, -1]), "xyzw": np.array([-1, -1, -1, 1])}


def quaternion_invert(quaternion: np.ndarray, type: str = "wxyz") -> np.ndarray:
    """conjugate of a unit quaternion (reference operations.py:20-37)"""
    return quaternion * _SIGN.get(type, np.array([]))


def quaternion_raw_multiply(a: np.ndarray, b: np.ndarray, type: str = "wxyz") -> np.ndarray:
    """Hamilton product (reference operations.py:80-112)"""
    if type == "wxyz":
        aw, ax, ay, az = a[..., [0]], a[..., [1]], a[..., [2]], a[..., [3]]
        bw, bx, by, bz = b[..., [0]], b[..., [1]], b[..., [2]], b[..., [3]]
    elif type == "xyzw":
        aw, ax, ay, az = a[..., 3], a[..., 1], a[..., 2], a[..., 0]
        bw, bx, by, bz = b[..., 3], b[..., 1], b[..., 2], b[..., 0]
    else:
        raise ValueError
    ow = aw * bw - ax * bx - ay * by - az * bz
    ox = aw * bx + ax * bw + ay * bz - az * by
    oy = aw * by - ax * bz + ay * bw + az * bx
    oz = aw * bz + ax * by - ay * bx + az * bw
    if type == "wxyz":
        return np.concatenate([ow, ox, oy, oz], axis=-1)
    return np.concatenate([ox, oy, oz, ow], axis=-1)


def quaternion_apply(quaternion: np.ndarray, point: np.ndarray, type: str = "wxyz") -> np.ndarray:
    """rotate 3-D points: q (0, p) q* (reference operations.py:40-77)"""
    if point.shape[-1] != 3:
        raise ValueError(f"Points are not in 3D, {point.shape}.")
    real = np.zeros(point.shape[:-1] + (1,))
    if type == "wxyz":
        pq = np.concatenate((real, point), -1)
    elif type == "xyzw":
        pq = np.concatenate((point, real), -1)
    else:
        pq = np.array([])
    qp = quaternion_raw_multiply(quaternion, pq, type=type)
    out = quaternion_raw_multiply(qp, quaternion_invert(quaternion, type=type), type=type)
    return out[..., 1:]
