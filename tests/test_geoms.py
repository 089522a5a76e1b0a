"""Rounded and prism collision geoms (sphere / capsule = hull (+) ball; cylinder
= 16-sided inscribed prism) in the oracle's narrowphase, pinned by analytic
contact geometry: MuJoCo's sphere-box and capsule-box colliders
(engine_collision_primitive.c in MuJoCo 3.2.2, not vendored) return the deepest
point (sphere) and the two segment-end points of a capsule lying on a face, with
the contact midway between the surfaces and depth = penetration.  Tolerances:
single-point contacts come from MPR, converged to MuJoCo's mpr_tolerance 1e-6
(as libccd's MPR in MuJoCo); manifold points from face clipping are exact up
to rounding."""
import numpy as np
import pytest

BASE = """
<mujoco><option gravity="0 0 0" cone="elliptic" integrator="implicitfast"/>
<worldbody>
  <body name="floor" pos="0 0 0"><geom name="floor" type="box" size="0.1 0.1 0.02"/></body>
  <body name="b" pos="{pos}" quat="{quat}"><freejoint name="fj"/>{geom}</body>
</worldbody></mujoco>"""


def contacts(geom, pos, quat="1 0 0 0"):
    from mgs.core.mjcf import compile_xml
    from oracle import oracle as O
    cm = compile_xml(BASE.format(geom=geom, pos=pos, quat=quat))
    om = O.OracleModel(cm)
    n, p, fr, dist, g = om.contacts(cm.qpos0, np.zeros(3), np.array([1.0, 0, 0, 0]))
    return n, p, fr, dist


def test_sphere_on_box():
    n, p, fr, dist = contacts('<geom type="sphere" size="0.01"/>', "0.01 -0.02 0.029")
    assert n == 1
    assert np.allclose(dist, [-0.001], atol=1e-6)
    assert np.allclose(np.abs(fr[0, :3]), [0, 0, 1], atol=1e-5)
    assert np.allclose(p[0], [0.01, -0.02, 0.0195], atol=1e-6)


def test_capsule_lying_on_box_two_contacts():
    # capsule axis along world x (rotate local z onto x), 2 mm penetration
    q = f"{np.cos(np.pi / 4)} 0 {np.sin(np.pi / 4)} 0"
    n, p, fr, dist = contacts('<geom type="capsule" size="0.01 0.03"/>', "0 0 0.028", q)
    assert n == 2
    assert np.allclose(dist, [-0.002, -0.002], atol=1e-7)
    assert np.allclose(sorted(p[:, 0]), [-0.03, 0.03], atol=1e-7)
    assert np.allclose(p[:, 2], 0.019, atol=1e-7)


def test_capsule_upright_one_contact():
    n, p, fr, dist = contacts('<geom type="capsule" size="0.01 0.03"/>', "0 0 0.0595")
    assert n == 1 and np.allclose(dist, [-0.0005], atol=1e-6)
    assert np.allclose(p[0], [0, 0, 0.01975], atol=1e-6)


def test_cylinder_standing_on_box_four_contacts():
    # 16-sided prism cap: the manifold keeps 4 rim points, depth 1 mm
    n, p, fr, dist = contacts('<geom type="cylinder" size="0.02 0.03"/>', "0 0 0.049")
    assert n == 4
    assert np.allclose(dist, -0.001, atol=1e-12)
    assert np.allclose(np.hypot(p[:, 0], p[:, 1]), 0.02, atol=1e-12)
    assert np.allclose(p[:, 2], 0.0195, atol=1e-12)


def test_rounded_aabb_includes_radius():
    from mgs.core.mjcf import compile_xml
    cm = compile_xml(BASE.format(geom='<geom type="capsule" size="0.01 0.03"/>', pos="0 0 1", quat="1 0 0 0"))
    assert np.allclose(cm.geom_radius, [0.0, 0.01])
    assert np.allclose(cm.geom_aabb[1, 3:], [0.01, 0.01, 0.04])
