"""Register / spill records of the headline's specialised rollout object built
with extra -D flags (kernel-source probes such as MGS_REGPROBE_*), compiled
into a scratch directory; CPU only.

    python tools/reg_probe.py [-DFLAG ...] [--lds]      (--lds: the G-rows-in-LDS object)"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mj-grasp-sim_amd")]

import numpy as np  # noqa: E402

from mgs.core import abi, special  # noqa: E402
from mgs.core.engine import auto_capacity, library_for  # noqa: E402

BUNDLER = "/opt/rocm/lib/llvm/bin/clang-offload-bundler"
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def main():
    from mgs.env.gravityless_object_grasping import GravitylessObjectGrasping
    from mgs.gripper.robotiq2f85 import GripperRobotiq2f85
    from mgs.obj.selector import get_object
    from mgs.util.geo.transforms import SE3Pose
    extra = [a for a in sys.argv[1:] if a.startswith("-D")]
    env = GravitylessObjectGrasping(GripperRobotiq2f85(SE3Pose(np.zeros(3), np.array([1.0, 0, 0, 0]), "wxyz")),
                                    get_object("003_cracker_box"))
    nc, ne = auto_capacity(env.model, env.ncon_max)
    fields, _, _ = env.model.pack(ncon_max=nc, nefc_max=ne)
    if "--lds" not in sys.argv:
        fields = dict(fields, g_rows_hbm=1)
    lib = library_for(env.model.nv, int(fields["nefc_max"]))
    header, flags, _ = special.plan(lib, abi.make_desc(fields), role="main")
    d = tempfile.mkdtemp()
    out = os.path.join(d, "probe.hsaco")
    special.compile_object(header, flags + extra, out)
    elf = out + ".elf"
    subprocess.run([BUNDLER, "--unbundle", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                    f"--input={out}", f"--output={elf}"], check=True)
    notes = subprocess.run([READELF, "--notes", elf], capture_output=True, text=True, check=True).stdout
    name = None
    for line in notes.splitlines():
        t = line.strip()
        if t.startswith("- .name:") or t.startswith(".name:"):
            name = t.split(":", 1)[1].strip()
        if name and "rollout" in name and t.startswith((".vgpr_count", ".vgpr_spill_count", ".private_segment",
                                                         ".sgpr_spill_count")):
            print(" ".join(extra) or "(none)", name, t)


if __name__ == "__main__":
    main()
