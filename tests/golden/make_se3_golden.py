"""Generate tests/golden/se3_golden.npz from the REFERENCE's SE3Pose.

TEST INFRASTRUCTURE ONLY -- run here (never on the GPU box; the reference does
not travel).  Imports /root/reference's mgs.util.geo.transforms read-only with a
`typing.Self` shim (the reference needs Python >= 3.11, transforms.py:18) and
records, for seeded random poses (float32, the reference's casts), the outputs
of from_mat, __matmul__, to_mat and inverse (its return value and the
mutated receiver, transforms.py:102-107 via operations.py quaternion_invert /
quaternion_apply).  Only data is stored.

    python tests/golden/make_se3_golden.py      # writes tests/golden/se3_golden.npz
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def main():
    sys.dont_write_bytecode = True          # never write into /root/reference
    import typing

    import numpy as np
    import typing_extensions
    typing.Self = typing_extensions.Self
    sys.path.insert(0, REF)
    from mgs.util.geo.transforms import SE3Pose
    from scipy.spatial.transform import Rotation

    rng = np.random.default_rng(7)
    n = 256
    H = np.tile(np.eye(4), (n, 1, 1))
    H[:, :3, :3] = Rotation.random(n, random_state=rng).as_matrix()
    H[:, :3, 3] = rng.uniform(-0.5, 0.5, (n, 3))
    a = SE3Pose.from_mat(H)
    b = SE3Pose(rng.uniform(-0.2, 0.2, (n, 3)), Rotation.random(n, random_state=rng).as_quat()[:, [3, 0, 1, 2]],
                "wxyz")
    ab = a @ b
    c = SE3Pose(np.copy(a.pos), np.copy(a.quat), "wxyz")
    inv = c.inverse()
    out = dict(H=H, a_pos=a.pos, a_quat=a.quat, b_pos=b.pos, b_quat=b.quat, ab_pos=ab.pos, ab_quat=ab.quat,
               a_mat=a.to_mat(), inv_pos=inv.pos, inv_quat=inv.quat, self_pos=np.asarray(c.pos),
               self_quat=np.asarray(c.quat))
    np.savez_compressed(os.path.join(HERE, "se3_golden.npz"), **out)
    print("wrote", os.path.join(HERE, "se3_golden.npz"), {k: (v.dtype, v.shape) for k, v in out.items()})


if __name__ == "__main__":
    main()
