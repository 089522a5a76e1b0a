"""Regression fixture of the contact-based Shadow Hand sampler:
the final per-candidate loss of ContactBasedDiff.generate_grasps on the
005_tomato_soup_can stand-in (64 candidates, numpy seed 0), computed by the
product's host logic with the device stages served by the C oracle (the GPU
is bit-equal to it, tests/test_contact_sampler.py), plus the loss of the same
candidates before optimisation.  The reference (JAX / optax, float32) cannot
run here, so this pins the restatement against itself and records the
acceptance statistics it meets; it is not a reference output.

    python tests/golden/make_contact_sampler_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mj-grasp-sim_amd")]
OUT = os.path.join(HERE, "contact_sampler_golden.npz")
N = 64


def run():
    from mgs.core import engine
    from mgs.obj.selector import get_object
    from mgs.sampler import contact as C
    from mgs.sampler.kin.model import ShadowKinematicsModel
    from oracle import oracle as O
    saved = engine.contact_fps, engine.contact_seeds, engine.contact_optimize
    engine.contact_fps = lambda pts, k, device=0: (O.contact_fps(pts, k), 0.0)
    engine.contact_seeds = lambda s, r, key, nt, device=0: (*O.contact_seeds(s, r, key, nt), 0.0)
    engine.contact_optimize = lambda d, R, p, T, Nm, device=0: dict(O.contact_optimize(d, R, p, T, Nm), kernel_ms=0.0)
    try:
        kin = ShadowKinematicsModel()
        obj = get_object("005_tomato_soup_can")
        s = C.ContactBasedDiff(obj, rng=np.random.default_rng(0))
        inp, desc = s.prepare(N, kin)
        before = np.array([O.contact_loss_grad(desc, np.concatenate([inp["rot_init"][c][:2].ravel(),
                                                                     inp["pos_init"][c], kin.pregrasp]),
                                               inp["targets"][c], inp["normals"][c])[0] for c in range(N)])
        s2 = C.ContactBasedDiff(obj, rng=np.random.default_rng(0))
        H, aux = s2.generate_grasps(N, kin)
        return dict(loss=np.asarray(s2.last["loss"], np.float64), loss_before=before,
                    joints=np.asarray(aux["joints"], np.float64), H=np.asarray(H, np.float32))
    finally:
        engine.contact_fps, engine.contact_seeds, engine.contact_optimize = saved


if __name__ == "__main__":
    r = run()
    np.savez_compressed(OUT, **r)
    q = np.quantile(r["loss"], [0.1, 0.5, 0.9])
    print(OUT, "loss quantiles", q, "before", np.quantile(r["loss_before"], [0.1, 0.5, 0.9]))
