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


# ---- box-box (MuJoCo dispatches box pairs to its dedicated collider, mjc_BoxBox;
# restated in oracle/mgs_oracle.c collide_boxbox): exact separating-axis geometry


def test_box_pair_uses_box_collider():
    from mgs.core.mjcf import compile_xml, PAIR_BOXBOX, PAIR_CONVEX
    cm = compile_xml(BASE.format(geom='<geom type="box" size="0.01 0.01 0.01"/>', pos="0 0 1", quat="1 0 0 0"))
    assert list(cm.pair_kind) == [PAIR_BOXBOX]
    cm = compile_xml(BASE.format(geom='<geom type="sphere" size="0.01"/>', pos="0 0 1", quat="1 0 0 0"))
    assert list(cm.pair_kind) == [PAIR_CONVEX]


def test_box_resting_on_box_four_corners():
    # 2x3x1 cm box, 0.5 mm into the floor's top face (z = 0.02): 4 corner contacts
    n, p, fr, dist = contacts('<geom type="box" size="0.01 0.015 0.005"/>', "0.003 -0.002 0.0245")
    assert n == 4
    assert np.allclose(dist, -0.0005, atol=1e-15)
    assert np.allclose(fr[:, :3], [0, 0, 1], atol=0)
    assert np.allclose(sorted(p[:, 0]), [-0.007, -0.007, 0.013, 0.013], atol=1e-15)
    assert np.allclose(sorted(p[:, 1]), [-0.017, -0.017, 0.013, 0.013], atol=1e-15)
    assert np.allclose(p[:, 2], 0.01975, atol=1e-15)


def test_tilted_box_edge_on_face_two_contacts():
    # box rotated about x by 0.2 rad: its lowest edge (along x) is the contact
    a = 0.2
    hz, hy = 0.005, 0.015
    zlow = -(hy * np.sin(a) + hz * np.cos(a))
    depth = 0.0003
    z = 0.02 - zlow - depth
    q = f"{np.cos(a / 2)} {np.sin(a / 2)} 0 0"
    n, p, fr, dist = contacts('<geom type="box" size="0.01 0.015 0.005"/>', f"0 0 {z}", q)
    assert n == 2
    assert np.allclose(dist, -depth, atol=1e-12)
    assert np.allclose(fr[:, :3], [0, 0, 1], atol=1e-12)
    assert np.allclose(sorted(p[:, 0]), [-0.01, 0.01], atol=1e-12)
    assert np.allclose(p[:, 2], 0.02 - depth / 2, atol=1e-12)


def test_crossed_ridges_edge_edge_contact():
    # a ridge along y (floor-like box turned 45 deg about y) under a ridge along
    # x (cube turned 45 deg about x): the edge-edge axis (z) wins, one contact at
    # the crossing point, midway between the two edges
    from mgs.core.mjcf import compile_xml
    from oracle import oracle as O
    c, s_ = np.cos(np.pi / 8), np.sin(np.pi / 8)
    h = 0.01 * np.sqrt(2)               # half diagonal of a 2 cm cube
    depth = 0.0004
    xml = f"""
<mujoco><option gravity="0 0 0" cone="elliptic" integrator="implicitfast"/>
<worldbody>
  <body name="low" pos="0 0 0" quat="{c} 0 {s_} 0"><geom type="box" size="0.01 0.01 0.01"/></body>
  <body name="b" pos="0.001 0.002 {2 * h - depth}" quat="{c} {s_} 0 0"><freejoint name="fj"/>
    <geom type="box" size="0.01 0.01 0.01"/></body>
</worldbody></mujoco>"""
    cm = compile_xml(xml)
    om = O.OracleModel(cm)
    n, p, fr, dist, g = om.contacts(cm.qpos0, np.zeros(3), np.array([1.0, 0, 0, 0]))
    assert n == 1
    assert np.allclose(fr[0, :3], [0, 0, 1], atol=1e-12)
    assert np.allclose(dist, [-depth], atol=1e-12)
    assert np.allclose(p[0], [0.0, 0.002, h - depth / 2], atol=1e-12)   # lower ridge x = 0, upper ridge y
