"""Build the headline engine's specialised code object from the working tree's
kernel sources into mj-grasp-sim_amd/mgs/_lib/ab/<name>.hsaco (A/B experiments,
tools/ab_special.sh).  Usage: python tools/ab_build.py name [-DFLAG ...]
(name starting with "c5": the C5 pile engine's object instead, for the
c5ab:<names> step of tools/gpu.sh; --ghbm: the main engine's G-rows-in-HBM
object; --drop=FLAG: without one of the planned flags)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mj-grasp-sim_amd")]


def main():
    import numpy as np
    from mgs.core import abi, special
    from mgs.core.engine import library_for
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
    from mgs.gripper.robotiq2f85 import GripperRobotiq2f85
    from mgs.obj.selector import get_object
    from mgs.util.geo.transforms import SE3Pose
    if sys.argv[1].startswith("c5"):
        from mgs.core.shipped import C5_SCENE, pile_env
        env = pile_env("ShadowHand")
        env.set_state(np.load(C5_SCENE)["state"])
        cm = env.model_for(env.get_state())
        fields, _, _ = cm.pack(ncon_max=env.ncon_max, nefc_max=env.rows_for(cm, env.ncon_max))
        lib = library_for(cm.nv, int(fields["nefc_max"]))
    else:
        env = GravitylessObjectGrasping(GripperRobotiq2f85(SE3Pose(np.zeros(3), np.array([1.0, 0, 0, 0]), "wxyz")),
                                        get_object("003_cracker_box"))
        fields, _, _ = env.model.pack(ncon_max=env.ncon_max, nefc_max=env.nefc_max)
        lib = library_for(env.model.nv, int(fields["nefc_max"]))
    args = sys.argv[2:]
    if "--ghbm" in args:
        # the main engine's G-rows-in-HBM object (its desc and flags)
        fields = dict(fields, g_rows_hbm=1)
    header, flags, _ = special.plan(lib, abi.make_desc(fields))
    # --drop=FLAG: leave one of the planned flags out (e.g. -DMGS_WAVES_PER_EU=2)
    drop = {a.split("=", 1)[1] for a in args if a.startswith("--drop=")}
    flags = [f for f in flags if f not in drop] + [a for a in args if a.startswith("-D")]
    out = os.path.join(special.CACHE, "..", "ab")
    os.makedirs(out, exist_ok=True)
    path = os.path.abspath(os.path.join(out, sys.argv[1] + ".hsaco"))
    special.compile_object(header, flags, path)
    print(path)


if __name__ == "__main__":
    main()
