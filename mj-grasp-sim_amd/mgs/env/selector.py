"""Environment factory (reference: mgs/env/selector.py:23-40) and the scene file
format of this build.

The reference stores a scene as `np.savez(scene, scene_definition=<dict of
Python objects>)` and reloads it with `allow_pickle=True` (gen_scene.py:178-185,
eval_grasps.py:68-69), i.e. it pickles gripper and object instances.  This
build writes the same information as plain arrays instead -- gripper name,
object ids and names, the integration-state vector, the removed objects --
and rebuilds the objects on load (`save_scene` / `load_scene`), so no pickle is
ever read."""
import numpy as np

from mgs.env.clutter_table import ClutterTableEnv


def _name(cfg):
    return cfg["name"] if isinstance(cfg, dict) else cfg.name


def get_env(cfg, gripper, obj_list):
    if _name(cfg) == "ClutterTable":
        return ClutterTableEnv(gripper, objects=obj_list)
    raise ValueError(f"Unknown environment {_name(cfg)}")


def get_env_from_dict(cfg, scene_dict, **kw):
    if _name(cfg) == "ClutterTable":
        return ClutterTableEnv.from_dict(scene_dict, **kw)
    raise ValueError(f"Unknown environment {_name(cfg)}")


def save_scene(path, scene_dict):
    """scene dict (ClutterTableEnv.to_dict) -> npz of plain arrays."""
    g = scene_dict["gripper"]
    objs = scene_dict["objects"]
    st = scene_dict["env_state"]
    np.savez(path, gripper=np.array(type(g).__name__), gripper_pos=np.asarray(g.pos, np.float64),
             gripper_quat=np.asarray(g.quat, np.float64), object_ids=np.array([o.object_id for o in objs]),
             object_names=np.array([o.name for o in objs]), state=np.asarray(st["state"], np.float64),
             removed=np.array(list(st.get("removed_objects", [])), dtype=str))


def load_scene(path):
    """npz written by save_scene -> scene dict for get_env_from_dict."""
    from mgs.gripper.selector import gripper_class
    from mgs.obj.selector import get_object
    from mgs.util.geo.transforms import SE3Pose
    z = np.load(path)            # plain arrays only (allow_pickle stays False)
    pose = SE3Pose(z["gripper_pos"], z["gripper_quat"], "wxyz")
    gripper = gripper_class(str(z["gripper"]))(pose)
    objs = [get_object(str(i), name=str(n)) for i, n in zip(z["object_ids"], z["object_names"])]
    return {"gripper": gripper, "objects": objs,
            "env_state": {"state": z["state"], "removed_objects": [str(r) for r in z["removed"]]}}
