"""python -m mgs.cli.gen_grasp_candidates gripper=<cfg> id=<k> num_grasps=<n>
(reference: mgs/cli/gen_grasp_candidates.py:16-83).

Antipodal candidates (mgs.sampler.antipodal) written to
$MGS_OUTPUT_DIR/<gripper>/<object>/candidates.npz.  Parallel grippers get the
reference's joints (Panda: width_to_joints(_clamp_width(w)), :66-71; Robotiq:
open = zeros).  The Shadow Hand uses the contact-based sampler
(mgs.sampler.contact, the reference's ContactBasedDiff with the Shadow
kinematic model, :33-47, :70-77), which returns its own joints; other
dexterous hands without a kinematic model (Allegro) get antipodal frames with
their open configuration."""
import os

import numpy as np

from mgs.cli._common import grasp_dir, object_id
from mgs.cli._hydra import main
from mgs.gripper.selector import get_gripper
from mgs.obj.selector import get_object
from mgs.sampler import antipodal

CONTACT_SAMPLER_GRIPPERS = ("ShadowHand",)


def sampler_kind(gripper_name):
    """which sampler the reference's CLI picks for a gripper (:33-47): the
    contact sampler for the hands with a kinematic model, antipodal otherwise"""
    return "contact" if gripper_name in CONTACT_SAMPLER_GRIPPERS else "antipodal"


def candidates(gripper, obj, num, seed, sampler="device", gripper_name=None):
    """(pose float32 (num,4,4), joints) for `gripper`; sampler "device" casts the
    rays on the GPU (generate_grasps_device), "host" is the numpy restatement."""
    name = type(gripper).__name__
    if gripper_name is not None and sampler_kind(gripper_name) == "contact":
        from mgs.sampler.contact import ContactBasedDiff
        from mgs.sampler.kin.model import get_kinematics
        H, aux = ContactBasedDiff(obj, rng=np.random.default_rng(seed)).generate_grasps(num,
                                                                                       get_kinematics(gripper_name))
        return H, aux["joints"]
    if sampler == "host":
        if name == "GripperPanda":
            return antipodal.panda_candidates(obj, num, seed=seed, gripper=gripper)[:2]
        if name == "GripperRobotiq2f85":
            return antipodal.robotiq_candidates(obj, num, seed=seed)[:2]
        return antipodal.hand_candidates(obj, num, gripper, seed=seed)[:2]
    gen = antipodal.AntipodalGraspGenerator(obj.obj_file_path, rng=np.random.default_rng(seed))
    H, aux = gen.generate_grasps_device(num)
    H = H.astype(np.float32)
    if name == "GripperPanda":
        j1, j2 = gripper.width_to_joints(gripper._clamp_width(aux["width"]))
        return H, np.stack([j1, j2], axis=-1)
    if name == "GripperRobotiq2f85":
        return H, np.zeros((num, 8))
    site = getattr(gripper, "grasp_site", None)
    if site is not None:
        H[:, :3, 3] -= H[:, :3, :3] @ np.asarray(site, np.float32)
    return H, np.tile(gripper.open_joints(), (num, 1))


@main("gen_grasp_candidates")
def run(cfg):
    print(f"Generating grasp candidates for gripper: {cfg.gripper.name}")
    oid = object_id(cfg)
    obj = get_object(oid)
    gripper = get_gripper(cfg.gripper)
    out = grasp_dir(cfg, oid, "MGS_OUTPUT_DIR")
    os.makedirs(out, exist_ok=True)
    H, J = candidates(gripper, obj, int(cfg.get("num_grasps", 10000)), int(cfg.get("seed", 0)),
                      cfg.get("sampler", "device"), gripper_name=cfg.gripper.name)
    np.savez(os.path.join(out, "candidates.npz"), pose=H, joints=J)
    print("Done!", os.path.join(out, "candidates.npz"))


if __name__ == "__main__":
    run()
