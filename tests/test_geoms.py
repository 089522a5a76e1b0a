"""Collision geometry of the contact models (mgs_model_desc.ccd_mode).

MuJoCo 3.2.2's collision table restated (ccd_mode 1 with the multiccd flag, 2
without; the envs run 1): analytic sphere / capsule / box / cylinder colliders
(engine_collision_primitive.c: midpoint contacts, depth = penetration, a
capsule lying on a face gives a contact at each end), libccd's MPR for convex
pairs (depth to the final portal triangle, position the tetrahedron
barycentre of the origin -- within the contact patch, not at its deepest
point), multiccd's perturbed extra contacts.  MuJoCo's source is not vendored:
these pin the restated rules (parity unpinned).  Round 5's
contract (ccd_mode 0: face clipping, rounded geoms as hull (+) ball) is kept
for the contact-set study, its tests under contact_model="r5".  Tolerances:
MPR converges to mpr_tolerance 1e-6; analytic and clipped values are exact up
to rounding."""
import numpy as np
import pytest

BASE = """
<mujoco><option gravity="0 0 0" cone="elliptic" integrator="implicitfast">{flag}</option>
<worldbody>
  <body name="floor" pos="0 0 0"><geom name="floor" type="box" size="0.1 0.1 0.02"/></body>
  <body name="b" pos="{pos}" quat="{quat}"><freejoint name="fj"/>{geom}</body>
</worldbody></mujoco>"""
MULTICCD = '<flag multiccd="enable"/>'


def contacts(geom, pos, quat="1 0 0 0", flag="", model="mujoco"):
    from mgs.core.mjcf import compile_xml
    from oracle import oracle as O
    cm = compile_xml(BASE.format(geom=geom, pos=pos, quat=quat, flag=flag))
    cm.options["contact_model"] = model
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


def test_cylinder_standing_on_box_r5_four_contacts():
    # round 5's contract: the cap face, 16 rim points on the true circle, the manifold keeps 4, depth 1 mm
    n, p, fr, dist = contacts('<geom type="cylinder" size="0.02 0.03"/>', "0 0 0.049", model="r5")
    assert n == 4
    assert np.allclose(dist, -0.001, atol=1e-12)
    assert np.allclose(np.hypot(p[:, 0], p[:, 1]), 0.02, atol=1e-12)
    assert np.allclose(p[:, 2], 0.0195, atol=1e-12)


def test_cylinder_standing_on_box_multiccd():
    """mjc_Convex (cylinder-box has no analytic collider): one MPR contact on
    the cap, and with multiccd four more -- each perturbed run tips the cap
    about the first contact onto a rim point (pos within 1 mm of the rim, up
    to r x 2e-3 rad deeper)"""
    n, p, fr, dist = contacts('<geom type="cylinder" size="0.02 0.03"/>', "0 0 0.049")
    assert n == 1 and np.allclose(dist, -0.001, atol=2e-6)
    # geom 1 is the cylinder (MuJoCo type 5 < box 6): the normal points into the floor
    assert np.allclose(fr[0, :3], [0, 0, -1], atol=1e-6)
    n, p, fr, dist = contacts('<geom type="cylinder" size="0.02 0.03"/>', "0 0 0.049", flag=MULTICCD)
    assert n == 5
    assert np.allclose(dist[0], -0.001, atol=2e-6)
    assert np.all(dist[1:] < -0.001) and np.all(dist[1:] > -0.001 - 2 * 0.04 * 1e-3)
    rad = np.hypot(p[1:, 0], p[1:, 1])
    assert np.all(rad > 0.019) and np.all(rad < 0.0201)
    assert np.allclose(fr[:, 2], -1.0, atol=1e-5)
    assert np.all(np.abs(p[:, 2] - 0.0195) < 2e-4)      # libccd positions: within the overlap


@pytest.mark.parametrize("spin", [0.0, 0.3, 0.7])
def test_cylinder_lying_on_box_r5_two_generator_contacts(spin):
    # axis along world x, turned about its own axis by `spin` (0.3 / 0.7 rad put
    # no vertex of an inscribed 16-gon at the bottom: a prism would rest up to
    # r (1 - cos(pi / 16)) = 0.38 mm higher), 0.4 mm into the floor: the exact
    # cylinder touches along its bottom generator, contacts at its two ends
    from scipy.spatial.transform import Rotation
    r, h, depth = 0.02, 0.03, 0.0004
    R = Rotation.from_euler("y", np.pi / 2) * Rotation.from_euler("z", spin)
    x, y, z, w = R.as_quat()
    n, p, fr, dist = contacts(f'<geom type="cylinder" size="{r} {h}"/>', f"0 0.003 {0.02 + r - depth}",
                              f"{w} {x} {y} {z}", model="r5")
    assert n == 2
    # MPR's normal (mpr_tolerance 1e-6) carries into the feature heights, as
    # for the capsule (test_capsule_lying_on_box_two_contacts)
    assert np.allclose(dist, -depth, atol=1e-7)
    assert np.allclose(np.abs(fr[:, 2]), 1.0, atol=1e-6)
    assert np.allclose(sorted(p[:, 0]), [-h, h], atol=1e-7)
    assert np.allclose(p[:, 1], 0.003, atol=1e-6)
    assert np.allclose(p[:, 2], 0.02 - depth / 2, atol=1e-7)


@pytest.mark.parametrize("spin", [0.0, 0.3, 0.7])
def test_cylinder_lying_on_box_multiccd(spin):
    """the exact cylinder along its bottom generator: MPR's contact, then
    multiccd's tilts about the first contact: the two about the tangent across
    the generator find its two ends, the two about the generator roll the
    contact by less than a tenth of a millimetre (distinct at 1e-3 x the
    smaller bounding radius)"""
    from scipy.spatial.transform import Rotation
    r, h, depth = 0.02, 0.03, 0.0004
    R = Rotation.from_euler("y", np.pi / 2) * Rotation.from_euler("z", spin)
    x, y, z, w = R.as_quat()
    n, p, fr, dist = contacts(f'<geom type="cylinder" size="{r} {h}"/>', f"0 0.003 {0.02 + r - depth}",
                              f"{w} {x} {y} {z}", flag=MULTICCD)
    assert n == 5
    assert np.allclose(dist[0], -depth, atol=2e-6)
    assert np.allclose(sorted(p[1:3, 0]), [-h, h], atol=1e-3)
    assert np.allclose(p[3:, 0], p[0, 0], atol=1e-6) and np.all(np.abs(p[3:, 1] - p[0, 1]) < 1e-4)
    assert np.allclose(p[:, 1], 0.003, atol=1e-4)
    assert np.allclose(fr[:, 2], -1.0, atol=1e-5)


def test_cylinder_tilted_on_box_rim_contact():
    # axis tilted 0.4 rad about x and spun 0.2 rad: one rim point is lowest;
    # MPR's depth and normal are exact to the tolerance; libccd's position is
    # the barycentre of the portal's witness points (within the cap's reach)
    from scipy.spatial.transform import Rotation
    r, h, depth = 0.02, 0.03, 0.0005
    R = Rotation.from_euler("x", 0.4) * Rotation.from_euler("z", 0.2)
    zs = [R.apply([r * np.cos(a), r * np.sin(a), -h])[2] for a in np.linspace(0, 2 * np.pi, 20001)]
    zlow = min(zs)
    c = np.array([0.001, 0.002, 0.02 - zlow - depth])
    x, y, z, w = R.as_quat()
    for model in ("mujoco", "r5"):
        n, p, fr, dist = contacts(f'<geom type="cylinder" size="{r} {h}"/>', " ".join(map(str, c)),
                                  f"{w} {x} {y} {z}", model=model)
        assert n == 1
        assert np.allclose(dist, [-depth], atol=1e-6 if model == "mujoco" else 1e-8)
        assert np.allclose(np.abs(fr[0, :3]), [0, 0, 1], atol=1e-6)
        assert np.hypot(*(p[0, :2] - c[:2])) < r + 1e-9
    assert np.allclose(p[0, 2], 0.02 - depth / 2, atol=1e-8)    # r5: midway between the surfaces


def test_capsule_pair_analytic():
    """mjc_CapsuleCapsule: crossed capsules touch at the closest points of their
    segments (1 contact); parallel ones get a contact at each overlapping end"""
    from mgs.core.mjcf import compile_xml, PAIR_CAPSULE_CAPSULE
    from oracle import oracle as O
    xml = """
<mujoco><option gravity="0 0 0" cone="elliptic" integrator="implicitfast"/>
<worldbody>
  <body name="a" pos="0 0 0"><geom type="capsule" size="0.01 0.05" quat="{qa}"/></body>
  <body name="b" pos="0.001 0.002 {z}"><freejoint name="fj"/><geom type="capsule" size="0.01 0.03" quat="{qb}"/></body>
</worldbody></mujoco>"""
    c, s_ = np.cos(np.pi / 4), np.sin(np.pi / 4)
    along_x, along_y = f"{c} 0 {s_} 0", f"{c} {-s_} 0 0"
    cm = compile_xml(xml.format(qa=along_x, qb=along_y, z=0.0197))
    assert cm.pair_table(2)[2].tolist() == [PAIR_CAPSULE_CAPSULE]
    om = O.OracleModel(cm)
    n, p, fr, dist, g = om.contacts(cm.qpos0, np.zeros(3), np.array([1.0, 0, 0, 0]))
    assert n == 1 and np.allclose(dist, [-0.0003], atol=1e-15)
    assert np.allclose(p[0], [0.001, 0.0, 0.0197 / 2], atol=1e-15)
    assert np.allclose(fr[0, :3], [0, 0, 1], atol=1e-15)
    cm = compile_xml(xml.format(qa=along_x, qb=along_x, z=0.0197))
    om = O.OracleModel(cm)
    n, p, fr, dist, g = om.contacts(cm.qpos0, np.zeros(3), np.array([1.0, 0, 0, 0]))
    assert n == 2 and np.allclose(dist, np.hypot(0.002, 0.0197) - 0.02, atol=1e-15)
    assert np.allclose(sorted(p[:, 0]), [0.001 - 0.03, 0.001 + 0.03], atol=1e-15)


def test_sphere_cylinder_analytic():
    """mjc_SphereCylinder: the side, the cap and the rim edge"""
    from mgs.core.mjcf import compile_xml, PAIR_SPHERE_CYLINDER
    from oracle import oracle as O
    xml = """
<mujoco><option gravity="0 0 0" cone="elliptic" integrator="implicitfast"/>
<worldbody>
  <body name="c" pos="0 0 0"><geom type="cylinder" size="0.02 0.03"/></body>
  <body name="s" pos="{pos}"><freejoint name="fj"/><geom type="sphere" size="0.005"/></body>
</worldbody></mujoco>"""
    for pos, depth, normal in [("0.0248 0 0.01", 0.0002, [-1, 0, 0]), ("0.003 0.004 0.0349", 0.0001, [0, 0, -1])]:
        cm = compile_xml(xml.format(pos=pos))
        assert cm.pair_table(2)[2].tolist() == [PAIR_SPHERE_CYLINDER]
        n, p, fr, dist, g = O.OracleModel(cm).contacts(cm.qpos0, np.zeros(3), np.array([1.0, 0, 0, 0]))
        assert n == 1 and np.allclose(dist, [-depth], atol=1e-12)
        assert np.allclose(fr[0, :3], normal, atol=1e-12)       # sphere (geom 1) -> cylinder
    # rim: the sphere centre beyond both the side and the cap, 45 deg
    d = 0.005 - 0.0002
    cm = compile_xml(xml.format(pos=f"{0.02 + d / np.sqrt(2)} 0 {0.03 + d / np.sqrt(2)}"))
    n, p, fr, dist, g = O.OracleModel(cm).contacts(cm.qpos0, np.zeros(3), np.array([1.0, 0, 0, 0]))
    assert n == 1 and np.allclose(dist, [-0.0002], atol=1e-12)
    assert np.allclose(fr[0, :3], [-np.sqrt(0.5), 0, -np.sqrt(0.5)], atol=1e-12)


def test_pair_table_follows_mujoco_types():
    """mj_collideGeoms orders a pair by MuJoCo geom type (geom 1 the smaller);
    the collider comes from the type pair (mjCOLLISIONFUNC)"""
    from mgs.core import mjcf
    from mgs.core.mjcf import compile_xml
    kinds = {"sphere": {"sphere": mjcf.PAIR_SPHERE_SPHERE, "capsule": mjcf.PAIR_SPHERE_CAPSULE,
                        "cylinder": mjcf.PAIR_SPHERE_CYLINDER, "box": mjcf.PAIR_SPHERE_BOX},
             "capsule": {"capsule": mjcf.PAIR_CAPSULE_CAPSULE, "cylinder": mjcf.PAIR_CONVEX,
                         "box": mjcf.PAIR_CAPSULE_BOX},
             "cylinder": {"cylinder": mjcf.PAIR_CONVEX, "box": mjcf.PAIR_CONVEX},
             "box": {"box": mjcf.PAIR_BOXBOX}}
    size = {"sphere": "0.01", "capsule": "0.01 0.02", "cylinder": "0.01 0.02", "box": "0.01 0.01 0.01"}
    for ta, row in kinds.items():
        for tb, kind in row.items():
            # the larger type first in the file: the table swaps it
            xml = f"""<mujoco><option integrator="implicitfast" cone="elliptic"/><worldbody>
  <body name="x"><geom type="{tb}" size="{size[tb]}"/></body>
  <body name="y" pos="0 0 1"><freejoint/><geom type="{ta}" size="{size[ta]}"/></body>
</worldbody></mujoco>"""
            cm = compile_xml(xml)
            g1, g2, k = cm.pair_table(1)
            assert k.tolist() == [kind], (ta, tb)
            assert mjcf.GEOM_TYPES[ta] <= mjcf.GEOM_TYPES[tb]
            if ta != tb:
                assert (g1[0], g2[0]) == (1, 0)
            g1, g2, k = cm.pair_table(0)        # round 5: file order, convex / box-box
            assert (g1[0], g2[0]) == (0, 1)
            assert k.tolist() == [mjcf.PAIR_BOXBOX if ta == tb == "box" else mjcf.PAIR_CONVEX]
    # a mesh pair with a sphere: MPR without multiccd
    cm = compile_xml("""<mujoco><option integrator="implicitfast" cone="elliptic"/><asset><mesh name="m" vertex="0 0 0 1 0 0 0 1 0 0 0 1"/></asset><worldbody>
  <body name="x"><geom type="mesh" mesh="m"/></body>
  <body name="y" pos="0 0 1"><freejoint/><geom type="sphere" size="0.01"/></body></worldbody></mujoco>""")
    assert cm.pair_table(1)[2].tolist() == [mjcf.PAIR_CONVEX_SMOOTH]


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
    cm = compile_xml(BASE.format(geom='<geom type="capsule" size="0.01 0.03"/>', pos="0 0 1", quat="1 0 0 0", flag=""))
    assert np.allclose(cm.geom_radius, [0.0, 0.01])
    assert np.allclose(cm.geom_aabb[1, 3:], [0.01, 0.01, 0.04])


# ---- box-box (MuJoCo dispatches box pairs to its dedicated collider, mjc_BoxBox;
# restated in oracle/mgs_oracle.c collide_boxbox): exact separating-axis geometry


def test_box_pair_uses_box_collider():
    from mgs.core.mjcf import compile_xml, PAIR_BOXBOX, PAIR_CONVEX  # noqa: F401 (pair_kind: the compiled order's)
    cm = compile_xml(BASE.format(geom='<geom type="box" size="0.01 0.01 0.01"/>', pos="0 0 1", quat="1 0 0 0", flag=""))
    assert list(cm.pair_kind) == [PAIR_BOXBOX]
    cm = compile_xml(BASE.format(geom='<geom type="sphere" size="0.01"/>', pos="0 0 1", quat="1 0 0 0", flag=""))
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


def test_mask_without_multiccd_keeps_the_predicate(env, candidates):
    """The collision masks skip multiccd (oracle_collision_free and the
    kernels' forward(full 0), round 6): its contacts repeat a pair that already
    has one, so the any-contact predicate of the full contact set (with
    multiccd, oracle_contacts) is unchanged on the headline's 256 candidates."""
    from oracle import oracle as O
    poses, J = candidates
    q, mp, mq, _ = env.initial_state(poses, J)
    om = O.OracleModel(env.model, ncon_max=128, nefc_max=256)
    free = om.collision_free(q, mp, mq, nthreads=4).astype(bool)
    full = np.array([om.contacts(q[i], mp[i], mq[i], maxc=128)[0] == 0 for i in range(len(q))])
    assert np.array_equal(free, full)
    assert 0 < free.sum() < len(free)
    # and multiccd does add contacts on the colliding ones (the rule is exercised)
    n_full = sum(om.contacts(q[i], mp[i], mq[i], maxc=128)[0] for i in np.nonzero(~free)[0][:32])
    assert n_full > len(np.nonzero(~free)[0][:32])
