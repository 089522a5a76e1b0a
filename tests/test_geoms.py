"""Rounded and cylinder collision geoms (sphere / capsule = hull (+) ball;
cylinder = the exact solid: analytic support in MPR, rim polygons turned onto
the true extreme for the contact features) in the oracle's narrowphase, pinned by analytic
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
    # the cap face: 16 rim points on the true circle, the manifold keeps 4, depth 1 mm
    n, p, fr, dist = contacts('<geom type="cylinder" size="0.02 0.03"/>', "0 0 0.049")
    assert n == 4
    assert np.allclose(dist, -0.001, atol=1e-12)
    assert np.allclose(np.hypot(p[:, 0], p[:, 1]), 0.02, atol=1e-12)
    assert np.allclose(p[:, 2], 0.0195, atol=1e-12)


@pytest.mark.parametrize("spin", [0.0, 0.3, 0.7])
def test_cylinder_lying_on_box_two_generator_contacts(spin):
    # axis along world x, turned about its own axis by `spin` (0.3 / 0.7 rad put
    # no vertex of an inscribed 16-gon at the bottom: a prism would rest up to
    # r (1 - cos(pi / 16)) = 0.38 mm higher), 0.4 mm into the floor: the exact
    # cylinder touches along its bottom generator, contacts at its two ends
    from scipy.spatial.transform import Rotation
    r, h, depth = 0.02, 0.03, 0.0004
    R = Rotation.from_euler("y", np.pi / 2) * Rotation.from_euler("z", spin)
    x, y, z, w = R.as_quat()
    n, p, fr, dist = contacts(f'<geom type="cylinder" size="{r} {h}"/>', f"0 0.003 {0.02 + r - depth}",
                              f"{w} {x} {y} {z}")
    assert n == 2
    # MPR's normal (mpr_tolerance 1e-6) carries into the feature heights, as
    # for the capsule (test_capsule_lying_on_box_two_contacts)
    assert np.allclose(dist, -depth, atol=1e-7)
    assert np.allclose(np.abs(fr[:, 2]), 1.0, atol=1e-6)
    assert np.allclose(sorted(p[:, 0]), [-h, h], atol=1e-7)
    assert np.allclose(p[:, 1], 0.003, atol=1e-6)
    assert np.allclose(p[:, 2], 0.02 - depth / 2, atol=1e-7)


def test_cylinder_tilted_on_box_rim_contact():
    # axis tilted 0.4 rad about x and spun 0.2 rad: one rim point is lowest;
    # exact depth and position (the point midway between it and the face)
    from scipy.spatial.transform import Rotation
    r, h, depth = 0.02, 0.03, 0.0005
    R = Rotation.from_euler("x", 0.4) * Rotation.from_euler("z", 0.2)
    low = R.apply([0.0, -r, -h])            # rim point on the low side: local (0, -r, -h)
    # the lowest point of the tilted solid: rim point towards -y of the bottom cap
    zs = [R.apply([r * np.cos(a), r * np.sin(a), -h])[2] for a in np.linspace(0, 2 * np.pi, 20001)]
    zlow = min(zs)
    assert abs(zlow - low[2]) < 1e-12 or zlow <= low[2]
    c = np.array([0.001, 0.002, 0.02 - zlow - depth])
    x, y, z, w = R.as_quat()
    n, p, fr, dist = contacts(f'<geom type="cylinder" size="{r} {h}"/>', " ".join(map(str, c)), f"{w} {x} {y} {z}")
    assert n == 1
    assert np.allclose(dist, [-depth], atol=1e-8)
    assert np.allclose(np.abs(fr[0, :3]), [0, 0, 1], atol=1e-6)
    lowest = c + R.apply([0.0, -r, -h]) if abs(zlow - low[2]) < 1e-12 else None
    assert np.allclose(p[0, 2], 0.02 - depth / 2, atol=1e-8)
    if lowest is not None:
        assert np.allclose(p[0, :2], lowest[:2], atol=1e-6)


def test_cylinder_support_is_exact():
    # the oracle's MPR support of a cylinder reaches the true surface: a sphere
    # touching the curved side at 45 deg between two prism vertices collides
    # (0.2 mm deep) although it is 0.15 mm clear of the inscribed 16-gon prism
    r, h, rs = 0.02, 0.03, 0.005
    a = np.pi / 16                          # midway between prism vertices
    depth = 0.0002
    dxy = (r + rs - depth) * np.array([np.cos(a), np.sin(a)])
    xml = f"""
<mujoco><option gravity="0 0 0" cone="elliptic" integrator="implicitfast"/>
<worldbody>
  <body name="cyl" pos="0 0 0"><geom type="cylinder" size="{r} {h}"/></body>
  <body name="s" pos="{dxy[0]} {dxy[1]} 0.001"><freejoint name="fj"/><geom type="sphere" size="{rs}"/></body>
</worldbody></mujoco>"""
    from mgs.core.mjcf import compile_xml
    from oracle import oracle as O
    cm = compile_xml(xml)
    assert np.allclose(cm.geom_cyl, [[r, h], [0, 0]])
    om = O.OracleModel(cm)
    n, p, fr, dist, g = om.contacts(cm.qpos0, np.zeros(3), np.array([1.0, 0, 0, 0]))
    assert n == 1
    assert np.allclose(dist, [-depth], atol=2e-6)          # MPR, mpr_tolerance 1e-6
    assert np.allclose(np.abs(fr[0, :2]), [np.cos(a), np.sin(a)], atol=5e-3)   # MPR normal on a curved face


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


def test_tilted_box_edge_on_face_one_contact():
    # box rotated about x by 0.2 rad: its lowest edge (along x) is the contact.
    # An edge on a face (two penetrating clipped vertices) gives one contact at
    # the deeper vertex (round 5: the set that reproduces MuJoCo's recorded
    # Robotiq state_close, tests/test_oracle.py::test_state_close_contact_set_study);
    # both are equally deep here, so the first in clipping order
    a = 0.2
    hz, hy = 0.005, 0.015
    zlow = -(hy * np.sin(a) + hz * np.cos(a))
    depth = 0.0003
    z = 0.02 - zlow - depth
    q = f"{np.cos(a / 2)} {np.sin(a / 2)} 0 0"
    n, p, fr, dist = contacts('<geom type="box" size="0.01 0.015 0.005"/>', f"0 0 {z}", q)
    assert n == 1
    assert np.allclose(dist, -depth, atol=1e-12)
    assert np.allclose(fr[:, :3], [0, 0, 1], atol=1e-12)
    assert np.isclose(abs(p[0, 0]), 0.01, atol=1e-12)
    assert np.allclose(p[:, 2], 0.02 - depth / 2, atol=1e-12)
    # tilted about y as well: the deeper end of the edge
    b = 0.01
    qa = np.array([np.cos(a / 2), np.sin(a / 2), 0, 0])
    qb = np.array([np.cos(b / 2), 0, np.sin(b / 2), 0])
    w1, x1, y1, z1 = qb
    w2, x2, y2, z2 = qa
    qq = [w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2, w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
          w1 * y2 - x1 * z2 + y1 * w2 + z1 * x2, w1 * z2 + x1 * y2 - y1 * x2 + z1 * w2]
    n, p, fr, dist = contacts('<geom type="box" size="0.01 0.015 0.005"/>', f"0 0 {z}", " ".join(map(str, qq)))
    assert n == 1 and dist[0] < -depth and p[0, 0] > 0.0


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
