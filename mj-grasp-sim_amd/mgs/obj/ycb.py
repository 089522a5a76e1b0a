"""YCB object loader (reference: mgs/obj/ycb.py:28-160).

Reads `<ASSET_PATH>/mj-objects/YCB/<id>/info.yml` and emits the same MJCF
include as the reference: one visual mesh geom (contype/conaffinity 0, density
1000 -- it contributes mass, as in MuJoCo with discardvisual=false) and one
convex collision geom per submesh with mass = weight * prop, condim 4,
friction "1 0.3 0.1", solimp "0.998 0.998 0.001", solref "0.001 1", and a free
joint `<name>:joint` with damping 1e-4 (ycb.py:119-147).
"""
import os
import xml.etree.ElementTree as Et
from typing import Any, Dict, Tuple

import yaml

from mgs.obj.base import CollisionMeshObject
from mgs.util.const import ASSET_PATH
from mgs.util.geo.transforms import SE3Pose


class ObjectYCB(CollisionMeshObject):
    dataset = "YCB"

    def __init__(self, pose: SE3Pose, object_id, name=None):
        v = pose.to_vec(layout="pq", type="wxyz")
        self.pos, self.quat = v[:3], v[3:]
        self.name = object_id if name is None else name
        self.object_id = object_id
        self.file_name = "{}.xml".format(object_id)

    @classmethod
    def dataset_directory(cls):
        return os.path.join(ASSET_PATH, "mj-objects", cls.dataset)

    @property
    def asset_dir(self):
        return os.path.join(self.dataset_directory(), self.object_id)

    @property
    def obj_file_path(self):
        return os.path.join(self.asset_dir, "textured.obj")

    @classmethod
    def all_object_ids(cls):
        d = cls.dataset_directory()
        return sorted(os.listdir(d)) if os.path.isdir(d) else []

    def info(self) -> dict:
        info_file = os.path.join(self.asset_dir, "info.yml")
        if not os.path.isfile(info_file):
            raise AssertionError(f"The file {info_file} was not found. Did you specify the path to the object folder correctly?")
        with open(info_file) as fh:
            return yaml.safe_load(fh)

    def to_xml(self) -> Tuple[str, Dict[str, Any]]:
        key = "{}_{}".format(self.name, self.file_name)
        return '<include file="{}" />'.format(key), {key: self.generate_xml()}

    def generate_xml(self) -> bytes:
        info = self.info()
        root = Et.Element("mujoco", attrib={"model": self.name})
        assets = Et.SubElement(root, "asset")
        world = Et.SubElement(root, "worldbody")
        body = Et.SubElement(world, "body", attrib={
            "name": self.name, "pos": " ".join(map(str, self.pos)),
            "quat": " ".join(map(str, self.quat))})
        Et.SubElement(assets, "mesh", attrib={"name": f"{self.name}_orig",
                                              "file": os.path.join(self.asset_dir, info["original_file"])})
        Et.SubElement(body, "geom", attrib={"mesh": f"{self.name}_orig", "group": "2", "type": "mesh",
                                            "contype": "0", "conaffinity": "0"})
        for i, (sub, prop) in enumerate(zip(info["submesh_files"], info["submesh_props"])):
            Et.SubElement(assets, "mesh", attrib={"name": f"{self.name}_coll_{i}",
                                                  "file": os.path.join(self.asset_dir, sub)})
            Et.SubElement(body, "geom", attrib={
                "mesh": f"{self.name}_coll_{i}", "mass": str(info["weight"] * prop), "group": "3",
                "type": "mesh", "conaffinity": "1", "contype": "1", "condim": "4", "rgba": "1 1 1 1",
                "friction": "1.0 0.3 0.1", "solimp": "0.998 0.998 0.001", "solref": "0.001 1"})
        Et.SubElement(body, "joint", attrib={"damping": "0.0001", "name": f"{self.name}:joint", "type": "free"})
        return Et.tostring(root)
