"""Google Scanned Objects loader (reference: mgs/obj/gso.py:28-160).

Same MJCF include as the YCB loader (visual mesh without contacts, one convex
collision geom per V-HACD submesh with mass = weight * prop, condim 4, the
same friction / solref / solimp, a free joint `<name>:joint`); the dataset
directory is `mj-objects/GoogleScannedObjects/<id>/` and the surface mesh the
samplers use is `model.obj` (gso.py:50-52)."""
import os

from mgs.obj.ycb import ObjectYCB


class ObjectGSO(ObjectYCB):
    dataset = "GoogleScannedObjects"

    @property
    def obj_file_path(self):
        return os.path.join(self.asset_dir, "model.obj")
