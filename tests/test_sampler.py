"""Antipodal candidate sampler (reference mgs/sampler/
antipodal.py:96-298): the device ray-casting path (mgs_antipodal_contacts) and
its CPU restatement (oracle_antipodal_contacts).

CPU: analytic ray-box hits, the choice rule over several hits, Wood's von
Mises-Fisher sampler's mean resultant (coth k - 1/k), the reference's
denormalisation.  GPU: bit-exact against the oracle on real meshes, and the
whole generate_grasps_device batch against a host restatement."""
import numpy as np
import pytest


def box_tris(h):
    v = np.array([[sx * h[0], sy * h[1], sz * h[2]] for sz in (-1, 1) for sy in (-1, 1) for sx in (-1, 1)])
    quads = [(0, 2, 3, 1), (4, 5, 7, 6), (0, 1, 5, 4), (2, 6, 7, 3), (0, 4, 6, 2), (1, 3, 7, 5)]
    f = [(a, b, c) for a, b, c, d in quads] + [(a, c, d) for a, b, c, d in quads]
    return v[np.array(f)].reshape(-1, 9)


def test_ray_box_known_hits():
    from oracle import oracle as O
    tri = box_tris([0.03, 0.079, 0.105])
    o = np.array([[0.03, 0.01, 0.02], [0.001, 0.02, 0.0], [0.03, 0.01, -0.03]])
    d = np.array([[-1.0, 0, 0], [0, 0, 1.0], [1.0, 0, 0]])
    sec, cnt = O.antipodal_contacts(tri, o, d, np.array([0.3, 0.99, 0.5]), 1e-5)
    assert cnt[0] == 1 and np.allclose(sec[0], [-0.03, 0.01, 0.02], atol=1e-15)
    # from inside (off the faces' diagonals): +z hits the top, -z the bottom;
    # u = 0.99 picks the second, i.e. the -d hit
    assert cnt[1] == 2 and np.allclose(sec[1], [0.001, 0.02, -0.105], atol=1e-15)
    # ray leaving the face: only the far face through -d
    assert cnt[2] == 1 and np.allclose(sec[2], [-0.03, 0.01, -0.03], atol=1e-15)


def test_vmf_mean_resultant_and_denormalisation():
    from mgs.obj.selector import get_object
    from mgs.sampler.antipodal import AntipodalGraspGenerator
    g = AntipodalGraspGenerator(get_object("017_orange").obj_file_path, rng=np.random.default_rng(0))
    g.normalize_load()
    r = g.draw(20000, kappa=10.0)
    tri = r["tri"]
    assert np.all(np.abs(np.linalg.norm(r["dirs"], axis=1) - 1) < 1e-12)
    # points lie on the (normalised) surface: inside the mesh's bounding box
    assert np.all(r["points"].min(0) >= tri.reshape(-1, 3).min(0) - 1e-12)
    # directions cluster around the inward normals with E[cos] = coth(k) - 1/k
    cr = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
    assert abs(np.mean(np.sum(r["dirs"] * -(r["points"] / np.linalg.norm(r["points"], axis=1, keepdims=True)), 1))
               - (1 / np.tanh(10) - 0.1)) < 0.02
    p = np.array([[0.1, -0.2, 0.3]])
    assert np.allclose(g.denormalize_points(p), (p - g.offset) * g.scale)


@pytest.mark.gpu
def test_device_rays_bit_exact():
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:
        pass
    from mgs.core.engine import antipodal_contacts
    from mgs.obj.selector import get_object
    from mgs.sampler.antipodal import AntipodalGraspGenerator
    from oracle import oracle as O
    for oid in ("017_orange", "005_tomato_soup_can", "003_cracker_box"):
        g = AntipodalGraspGenerator(get_object(oid).obj_file_path, rng=np.random.default_rng(1))
        g.normalize_load()
        r = g.draw(8192)
        sg, cg, ms = antipodal_contacts(r["tri"], r["points"], r["dirs"], r["u"], 1e-5)
        so, co = O.antipodal_contacts(r["tri"], r["points"], r["dirs"], r["u"], 1e-5)
        assert np.array_equal(cg, co) and np.array_equal(sg, so), oid
        assert (cg > 0).mean() > 0.9


@pytest.mark.gpu
def test_generate_grasps_device_batch():
    from mgs.obj.selector import get_object
    from mgs.sampler.antipodal import AntipodalGraspGenerator
    from oracle import oracle as O
    path = get_object("005_tomato_soup_can").obj_file_path
    g = AntipodalGraspGenerator(path, rng=np.random.default_rng(5))
    H, aux = g.generate_grasps_device(4096)
    h = AntipodalGraspGenerator(path, rng=np.random.default_rng(5))
    h.normalize_load()
    r = h.draw(4096)
    so, co = O.antipodal_contacts(r["tri"], r["points"], r["dirs"], r["u"], 1e-5)
    two = np.where((co > 0)[:, None], so, r["points"] + r["offset"])
    H2, aux2 = h.finish(r["points"], two, h.rng)
    assert np.array_equal(H, H2) and np.array_equal(aux["width"], aux2["width"])
    assert np.allclose(np.einsum("nij,nik->njk", H[:, :3, :3], H[:, :3, :3]), np.eye(3), atol=1e-9)
