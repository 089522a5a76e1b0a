"""Google Scanned Objects loader (reference: mgs/obj/gso.py:28-160, same body as YCB)."""
from mgs.obj.ycb import ObjectYCB


class ObjectGSO(ObjectYCB):
    dataset = "GoogleScannedObjects"
