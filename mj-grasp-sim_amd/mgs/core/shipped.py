"""The shipped configurations whose model-specialised code objects the build
compiles ahead of time (mgs/core/special.py), and the pile scenes they use.

  * the headline (bench.py): Robotiq 2F-85 x 003_cracker_box, plus its
    capacity-escalation engine (twice the contacts);
  * C3 (tools/bench_configs.py): Panda x every shipped YCB object;
  * C4: Allegro x the GSO-format mug;
  * the DEXEE hand x a YCB can (condim-6 contacts: its object is built with
    -DMGS_MAXDIM=6);
  * C5: the Shadow Hand over the settled 5-object pile (scene state
    tests/golden/clutter_scene_shadow.npz when present, else the pile as
    built);
  * the spread piles of 3 and 4 objects the GPU tests run (nv 32, a dof count
    no library instantiates);
  * the Shadow Hand over spread piles of 7 and 10 objects (nv 70 and 88: two
    dofs per lane, -DMGS_DPL=2).

Nothing here imports the test tree or pytest.
"""
from __future__ import annotations

import os
from typing import List, Sequence, Tuple

import numpy as np

# a pile of 5 YCB objects (gen_scene.yaml:10's num_objects) and the spread
# piles of the GPU tests (tests/test_clutter.py::test_any_pile_size_gpu_parity)
PILE_OBJECTS = ["010_potted_meat_can", "061_foam_brick", "005_tomato_soup_can", "017_orange", "061_foam_brick"]
SPREAD_PILES = [("Robotiq2f85Gripper", ["010_potted_meat_can", "061_foam_brick", "005_tomato_soup_can"]),
                ("PandaGripper", ["010_potted_meat_can", "061_foam_brick", "005_tomato_soup_can", "017_orange"])]

# piles past 64 dofs (tests/test_pile_wide.py): the Shadow Hand over 7 and 10
# objects drawn with repetition, as the reference draws its pile sizes
# (mgs/obj/selector.py:124-130)
WIDE_PILE_OBJECTS = ["010_potted_meat_can", "061_foam_brick", "005_tomato_soup_can", "017_orange", "061_foam_brick",
                     "010_potted_meat_can", "017_orange", "005_tomato_soup_can", "061_foam_brick", "017_orange"]
WIDE_PILES = [("ShadowHand", WIDE_PILE_OBJECTS[:7]), ("ShadowHand", WIDE_PILE_OBJECTS[:10])]

# the dexee x YCB configuration (condim-6 fingertips, mujoco.pid actuators;
# tests/test_dexee.py)
DEXEE_OBJECT = "005_tomato_soup_can"

# gravity compensation under gravity (the dexee's gravcomp="1" bodies in a
# clutter scene): a jointed free body, every body's gravcomp set to {gc}
# (tests/test_dexee.py::test_gravcomp_gpu_parity)
GRAVCOMP_XML = """
<mujoco><option gravity="0 0 -9.81" cone="elliptic" integrator="implicitfast" timestep="0.002"/>
<worldbody><body name="a" pos="0 0 1" gravcomp="{gc}"><freejoint name="fj"/>
  <geom type="box" size="0.05 0.05 0.05" mass="2" contype="0" conaffinity="0"/>
  <body name="b" pos="0.2 0 0" gravcomp="{gc}"><joint name="h" axis="0 1 0"/>
    <geom type="sphere" size="0.03" pos="0.1 0 0" mass="1" contype="0" conaffinity="0"/></body>
</body></worldbody></mujoco>"""

_ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", ".."))
C5_SCENE = os.path.join(_ROOT, "tests", "golden", "clutter_scene_shadow.npz")


def pile_env(gripper_name: str, object_ids: Sequence[str] = PILE_OBJECTS):
    """a ClutterTableEnv over the given objects (the gripper parked out of the
    way, no scene randomisation), as the reference's gen_scene builds one
    (mgs/cli/gen_scene.py:28-45) before dropping the objects"""
    from mgs.env.clutter_table import ClutterTableEnv
    from mgs.gripper.selector import get_gripper
    from mgs.obj.selector import get_object
    from mgs.util.geo.transforms import SE3Pose
    grip = get_gripper({"name": gripper_name},
                       default_pose=SE3Pose(np.array([5.0, 5.0, 1.0]), np.array([1.0, 0, 0, 0]), "wxyz"))
    objs = [get_object(oid, name=f"obj{i}") for i, oid in enumerate(object_ids)]
    return ClutterTableEnv(grip, objs, scene_randomization=False)


def spread_pile(gripper_name: str, object_ids: Sequence[str]):
    """a pile scene of any size with its objects set apart on the table (the
    parity of the kernels does not need a settled pile)"""
    env = pile_env(gripper_name, object_ids)
    parts = env.split_state(env.get_state())
    q = parts["qpos"].copy()
    for i, (n, qs, vs) in enumerate(env._obj_slices()):
        q[qs] = [0.12 * (i - 1.5), 0.06 * (i % 2), 0.06, 1.0, 0.0, 0.0, 0.0]
    env.set_state(env.join_state(dict(parts, qpos=q)))
    return env


def shipped_engines() -> List[Tuple[object, int, object, str]]:
    """(compiled model, ncon_max, nefc_max or None, object role) of the engines
    the shipped configurations and the GPU tests create first (role: see
    mgs.core.special.ROLE_FLAGS)"""
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
    from mgs.gripper.selector import get_gripper
    from mgs.obj.selector import get_object
    from mgs.obj.ycb import ObjectYCB
    out = []
    for grip, objs in (("Robotiq2f85Gripper", ["003_cracker_box"]),
                       ("PandaGripper", ObjectYCB.all_object_ids()),
                       ("AllegroGripper", ["Synthetic_Mug_Body"]),
                       ("DexeeGripper", [DEXEE_OBJECT])):
        for o in objs:
            env = GravitylessObjectGrasping(get_gripper({"name": grip}), get_object(o))
            out.append((env.model, env.ncon_max, env.nefc_max, "main"))
            if grip != "DexeeGripper":
                # the configs' escalation engines (twice the contacts, rows as
                # Engine() sizes them): their re-runs then run specialised too
                # (round 6: multiccd raised the hands' contact counts, so C3 / C4
                # re-run more candidates; on the library kernel without these)
                out.append((env.model, 2 * env.ncon_max, None, "escalation"))
            if grip == "Robotiq2f85Gripper":
                # the rotation fault-injection object of the GPU tests (every
                # ring pop expires: the product must raise, not return labels)
                out.append((env.model, env.ncon_max, env.nefc_max, "fault"))
    env = pile_env("ShadowHand")
    if os.path.isfile(C5_SCENE):
        env.set_state(np.load(C5_SCENE)["state"])
    scenes = [env] + [spread_pile(g, objs) for g, objs in SPREAD_PILES + WIDE_PILES]
    for env in scenes:
        cm = env.model_for(env.get_state())
        out.append((cm, env.ncon_max, env.rows_for(cm, env.ncon_max), "main"))
    from mgs.core.mjcf import compile_xml
    out.append((compile_xml(GRAVCOMP_XML.format(gc=0.5)), 4, None, "main"))
    return out
