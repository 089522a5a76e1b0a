"""Contact-based dexterous-hand sampler (reference
mgs/sampler/contact.py, mgs/sampler/kin/{base,jax_util,shadow}.py).

Parity status: UNPINNED against the reference -- it is a JAX/flax/optax
program (float32, jax.random keys) and none of those packages is installed,
so no reference output can be produced here and the reference holds no
fixtures for it.  What is pinned instead:
  * the forward kinematics against an independent numpy transcription of the
    reference's formulas (forward_kinematic_point_transform, base.py:80-113;
    quaternion algebra jax_util.py:22-130);
  * the optimiser's gradient against central finite differences of its loss;
  * optax.adamw's update rule (scale_by_adam -> add_decayed_weights ->
    scale(-lr)) against a numpy transcription on a one-parameter problem;
  * farthest-point sampling, the seed neighbourhoods and the initial
    permutation assignment against direct numpy restatements;
  * GPU == oracle bit for bit (-m gpu).
"""
from itertools import permutations

import numpy as np
import pytest


@pytest.fixture(scope="module")
def kin():
    from mgs.sampler.kin.model import ShadowKinematicsModel
    return ShadowKinematicsModel()


@pytest.fixture(scope="module")
def desc(kin):
    from mgs.sampler import contact as C
    return C.kin_desc(kin, [0, 1, 2, 0, 1])


# --- an independent numpy transcription of the reference's JAX formulas ------
def q_mul(a, b):
    aw, ax, ay, az = a
    bw, bx, by, bz = b
    return np.array([aw * bw - ax * bx - ay * by - az * bz, aw * bx + ax * bw + ay * bz - az * by,
                     aw * by - ax * bz + ay * bw + az * bx, aw * bz + ax * by - ay * bx + az * bw])


def q_apply(q, p):
    return q_mul(q_mul(q, np.r_[0.0, p]), q * np.array([1, -1, -1, -1]))[1:]


def se3_mul(A, B):
    return np.r_[q_mul(A[:4], B[:4]), q_apply(A[:4], B[4:]) + A[4:]]


def ref_fk_point(kin, theta, point, joint_idx):
    """forward_kinematic_point_transform (base.py:80-113)"""
    par = kin.parents()
    links = [np.array([1.0, 0, 0, 0, 0, 0, 0])]
    for i in range(kin.num_dofs):
        axis = kin.joint_tf[i, 3:] / np.linalg.norm(kin.joint_tf[i, 3:])
        rq = np.r_[np.cos(theta[i] / 2), axis * np.sin(theta[i] / 2)]
        dyn = np.r_[rq, kin.joint_tf[i, :3] * theta[i]]
        links.append(se3_mul(se3_mul(links[par[i] + 1], kin.kin_tf[i]), dyn))
    T = links[joint_idx + 1]
    return q_apply(T[:4], point) + T[4:]


def test_shadow_model_tables(kin):
    assert kin.num_dofs == 22
    assert list(kin.fingertip_idx) == [3, 7, 11, 16, 21]
    assert kin.tip_contacts.shape == (5, 3, 3)
    # the reference's pre-grasp first-finger knuckle (-0.350) sits just below
    # its range (-0.349066); the first optimiser step clips it
    out = (kin.pregrasp < kin.joint_ranges[:, 0]) | (kin.pregrasp > kin.joint_ranges[:, 1])
    assert list(np.nonzero(out)[0]) == [0]
    par = kin.parents()
    assert par[0] == -1 and par[3] == 2 and par[12] == -1 and par[16] == 15 and par[17] == -1


def test_fk_matches_reference_formulas(kin, desc):
    from oracle import oracle as O
    rng = np.random.default_rng(1)
    for _ in range(5):
        th = rng.uniform(kin.joint_ranges[:, 0], kin.joint_ranges[:, 1])
        X, _ = O.contact_fk(desc, th)
        for a, tip in enumerate(kin.fingertip_idx):
            pts = [np.array([desc.tip_point[a][j] for j in range(3)]), np.zeros(3), kin.tip_normals[a]]
            for p in range(3):
                ref = ref_fk_point(kin, th, pts[p], int(tip))
                assert np.abs(X[a, p] - ref).max() < 1e-14


def test_fk_derivatives_finite_difference(kin, desc):
    from oracle import oracle as O
    th = kin.pregrasp.copy()
    X, dX = O.contact_fk(desc, th)
    for a in range(desc.ntip):
        for s in range(desc.chain_len[a]):
            i = desc.chain[a][s]
            tp, tm = th.copy(), th.copy()
            tp[i] += 1e-6
            tm[i] -= 1e-6
            fd = (O.contact_fk(desc, tp)[0][a] - O.contact_fk(desc, tm)[0][a]) / 2e-6
            assert np.abs(fd - dX[a, s]).max() < 1e-8


def test_loss_gradient_finite_difference(kin, desc):
    from oracle import oracle as O
    rng = np.random.default_rng(2)
    for trial in range(3):
        prm = np.concatenate([rng.normal(size=6), rng.normal(size=3) * 0.05, kin.pregrasp])
        T = rng.normal(size=(5, 3)) * 0.05 + np.array([0.0, 0.0, 0.3])
        N = rng.normal(size=(5, 3))
        N /= np.linalg.norm(N, axis=1, keepdims=True)
        loss, g = O.contact_loss_grad(desc, prm, T, N)
        fd = np.zeros_like(g)
        for j in range(len(prm)):
            p1, p2 = prm.copy(), prm.copy()
            p1[j] += 1e-6
            p2[j] -= 1e-6
            fd[j] = (O.contact_loss_grad(desc, p1, T, N)[0] - O.contact_loss_grad(desc, p2, T, N)[0]) / 2e-6
        assert np.abs(fd - g).max() < 1e-8 * max(1.0, np.abs(g).max())


def test_adamw_rule_matches_optax_transcription(desc):
    """the optimiser's first step against a numpy transcription of optax.adamw
    (scale_by_adam -> add_decayed_weights(1e-4) -> scale(-lr)) applied to the
    oracle's gradient at the initial parameters, joints clipped after it"""
    from oracle import oracle as O
    from mgs.sampler import contact as C
    import copy
    d1 = copy.copy(desc)
    d1.iters = 1
    rng = np.random.default_rng(3)
    R0 = np.eye(3)[None]
    p0 = np.array([[0.0, 0.0, 0.0]])
    T = rng.normal(size=(1, 5, 3)) * 0.05
    N = np.tile([0.0, 0.0, 1.0], (1, 5, 1))
    out = O.contact_optimize(d1, R0, p0, T, N, nthreads=1)
    # numpy transcription: initial assignment with R0 (identity), then one step
    from mgs.sampler.kin.model import ShadowKinematicsModel
    kin = ShadowKinematicsModel()
    X, _ = O.contact_fk(d1, kin.pregrasp)
    D = np.linalg.norm(X[:, 0][:, None, :] - T[0][None], axis=-1)
    perms = np.array(list(permutations(range(5))))
    best = perms[np.argmin(D[np.arange(5), perms].sum(1))]
    prm = np.concatenate([R0[0, :2].ravel(), p0[0], kin.pregrasp])
    _, g = O.contact_loss_grad(d1, prm, T[0][best], N[0])
    m = 0.1 * g
    v = 0.001 * g * g
    u = (m / 0.1) / (np.sqrt(v / 0.001) + 1e-8) + 1e-4 * prm
    new = prm - C.LEARNING_RATE * u
    new[9:] = np.clip(new[9:], kin.joint_ranges[:, 0], kin.joint_ranges[:, 1])
    assert np.allclose(out["pos"][0], new[6:9], atol=1e-15, rtol=0)
    assert np.allclose(out["joints"][0], new[9:], atol=1e-15, rtol=0)


def test_fps_matches_numpy():
    from oracle import oracle as O
    rng = np.random.default_rng(4)
    x = rng.normal(size=(3000, 3))
    idx = O.contact_fps(x, 64)
    dist = np.full(len(x), np.inf)
    ref = [0]
    for i in range(1, 64):
        d = np.sum((x - x[ref[-1]]) ** 2, axis=-1)
        dist = np.minimum(dist, d)
        ref.append(int(np.argmax(dist)))
    assert list(idx) == ref


def test_seeds_match_numpy_argsort():
    from oracle import oracle as O
    rng = np.random.default_rng(5)
    s = rng.uniform(-0.1, 0.1, size=(300, 3))
    s[:40] *= 10.0                       # a sparse region: fewer than ntip admissible
    nn, sel = O.contact_seeds(s, 0.1, 12345, 5, nthreads=2)
    d = np.linalg.norm(s[:, None] - s[None], axis=-1)
    assert np.array_equal(nn, np.argsort(d, axis=1, kind="stable")[:, 1])
    for i in [0, 3, 50, 299]:
        adm = d[i] < 0.1
        picked = sel[i]
        assert adm[picked[-min(5, adm.sum()):]].all()
        assert (adm.sum() >= 5) == adm[picked].all()


def test_single_seed_nearest_is_itself():
    """one seed has no second-nearest: the reference's sorted_indices[:, 1]
    (sampler/contact.py:213-214) clamps to column 0, the seed itself"""
    from oracle import oracle as O
    nn, sel = O.contact_seeds(np.array([[0.01, 0.02, 0.03]]), 0.1, 7, 3)
    assert list(nn) == [0]
    assert sel.tolist() == [[0, 0, 0]]          # fewer seeds than tips: the seed itself


def _oracle_pipeline(monkeypatch):
    """the product's host logic with the device stages served by the oracle"""
    from mgs.core import engine
    from oracle import oracle as O
    monkeypatch.setattr(engine, "contact_fps", lambda pts, k, device=0: (O.contact_fps(pts, k), 0.0))
    monkeypatch.setattr(engine, "contact_seeds",
                        lambda s, r, key, nt, device=0: (*O.contact_seeds(s, r, key, nt), 0.0))
    monkeypatch.setattr(engine, "contact_optimize",
                        lambda d, R, p, T, N, device=0: dict(O.contact_optimize(d, R, p, T, N), kernel_ms=0.0))


def test_generate_grasps_host_logic(monkeypatch, kin):
    """the whole sampler on a small object, device stages replaced by the
    oracle: valid poses, joints in range, fingertips pulled to the targets"""
    from mgs.obj.selector import get_object
    from mgs.sampler import contact as C
    _oracle_pipeline(monkeypatch)
    obj = get_object("005_tomato_soup_can")
    s = C.ContactBasedDiff(obj, rng=np.random.default_rng(0))
    inp, desc = s.prepare(48, kin)
    from oracle import oracle as O
    d0 = __import__("copy").copy(desc)
    d0.iters = 0
    before = O.contact_optimize(d0, inp["rot_init"], inp["pos_init"], inp["targets"], inp["normals"])
    s2 = C.ContactBasedDiff(obj, rng=np.random.default_rng(0))
    H, aux = s2.generate_grasps(48, kin)
    assert H.shape == (48, 4, 4) and H.dtype == np.float32
    R = H[:, :3, :3].astype(np.float64)
    assert np.abs(R @ R.transpose(0, 2, 1) - np.eye(3)).max() < 1e-5
    J = aux["joints"]
    assert J.shape == (48, 22)
    assert np.all(J >= kin.joint_ranges[:, 0] - 1e-6) and np.all(J <= kin.joint_ranges[:, 1] + 1e-6)
    loss = s2.last["loss"]
    assert np.isfinite(loss).all()
    # 150 steps lower the loss against the untrained (0-step) pose
    lb = []
    for c in range(48):
        lb.append(O.contact_loss_grad(desc, np.concatenate([inp["rot_init"][c][:2].ravel(), inp["pos_init"][c],
                                                            kin.pregrasp]), inp["targets"][c], inp["normals"][c])[0])
    assert np.median(loss) < 0.5 * np.median(lb)
    assert before["pos"].shape == (48, 3)


def test_sampler_regression_fixture():
    """the whole sampler (oracle-served device stages) reproduces the committed
    regression fixture bit for bit (tests/golden/make_contact_sampler_golden.py:
    64 candidates on 005_tomato_soup_can, seed 0), and the optimisation meets
    the fixture's acceptance statistics: every candidate's loss drops, the
    median by more than 5x, the 90th percentile by more than 5x.  Pins the
    restatement against itself (parity with the JAX reference is unpinned)."""
    import os
    import sys
    here = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
    if here not in sys.path:
        sys.path.insert(0, here)
    import make_contact_sampler_golden as G
    g = np.load(os.path.join(here, "contact_sampler_golden.npz"))
    r = G.run()
    for k in ("loss", "loss_before", "joints", "H"):
        assert np.array_equal(r[k], g[k]), k
    assert np.all(g["loss"] < g["loss_before"])
    assert np.median(g["loss"]) * 5 < np.median(g["loss_before"])
    assert np.quantile(g["loss"], 0.9) * 5 < np.quantile(g["loss_before"], 0.9)


def test_cli_contact_sampler_selected_for_shadow():
    from mgs.cli.gen_grasp_candidates import sampler_kind
    assert sampler_kind("ShadowHand") == "contact"
    assert sampler_kind("PandaGripper") == "antipodal"


# ------------------------------------------------------------------ GPU parity
@pytest.mark.gpu
def test_contact_kernels_gpu_parity(kin):
    import torch
    if torch.cuda.is_available():
        torch.cuda.init()
    from mgs.core import engine
    from mgs.sampler import contact as C
    from oracle import oracle as O
    rng = np.random.default_rng(7)
    pts = rng.normal(size=(5000, 3)) * 0.05
    idx, _ = engine.contact_fps(pts, 300)
    assert np.array_equal(idx, O.contact_fps(pts, 300))
    seeds = pts[idx]
    nn, sel, _ = engine.contact_seeds(seeds, 0.1, 99, 5)
    nn_o, sel_o = O.contact_seeds(seeds, 0.1, 99, 5)
    assert np.array_equal(nn, nn_o) and np.array_equal(sel, sel_o)
    one = seeds[:1]
    nn1, sel1, _ = engine.contact_seeds(one, 0.1, 99, 5)
    assert list(nn1) == [0] and np.array_equal(sel1, O.contact_seeds(one, 0.1, 99, 5)[1])
    desc = C.kin_desc(kin, [2, 1, 0, 1, 2])
    n = 200
    R = np.einsum("nij,jk->nik", np.linalg.qr(rng.normal(size=(n, 3, 3)))[0], kin.align_rot)
    p = rng.normal(size=(n, 3)) * 0.05
    T = rng.normal(size=(n, 5, 3)) * 0.04
    N = rng.normal(size=(n, 5, 3))
    N /= np.linalg.norm(N, axis=-1, keepdims=True)
    g = engine.contact_optimize(desc, R, p, T, N)
    o = O.contact_optimize(desc, R, p, T, N)
    for k in ("rot", "pos", "joints", "loss"):
        assert np.array_equal(g[k], o[k]), k


@pytest.mark.gpu
def test_generate_grasps_gpu_equals_oracle_pipeline(monkeypatch, kin):
    import torch
    if torch.cuda.is_available():
        torch.cuda.init()
    from mgs.obj.selector import get_object
    from mgs.sampler import contact as C
    obj = get_object("005_tomato_soup_can")
    Hg, ag = C.ContactBasedDiff(obj, rng=np.random.default_rng(1)).generate_grasps(256, kin)
    _oracle_pipeline(monkeypatch)
    Ho, ao = C.ContactBasedDiff(obj, rng=np.random.default_rng(1)).generate_grasps(256, kin)
    assert np.array_equal(Hg, Ho)
    assert np.array_equal(ag["joints"], ao["joints"])
