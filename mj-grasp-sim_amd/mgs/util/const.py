"""Package paths (reference: mgs/util/const.py:23-29).

ASSET_PATH defaults to the package's own asset directory, which holds the
derived Robotiq hulls and the synthetic YCB stand-in objects.  Set
MGS_ASSET_PATH to a directory laid out like the reference's `asset/`
(with `mj-objects/YCB/<id>/info.yml`) to use real object sets.
"""
import os

PACKAGE_PATH = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GIT_PATH = os.path.dirname(PACKAGE_PATH)
ASSET_PATH = os.environ.get("MGS_ASSET_PATH", os.path.join(PACKAGE_PATH, "assets"))
