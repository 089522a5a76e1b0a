"""Build a variant of the headline engine's specialised code object for A/B runs
(bench.py with MGS_SPECIAL_OBJECT=<object>): the working tree's kernel sources
copied to a scratch tree, optionally edited, compiled for the headline model at
a given contact capacity.

  python tools/ab_variant.py NAME [--ncon N] [--nefc N] [--noinline] [--ghbm] [--drop FLAG] [--src DIR]
                             [-DFLAG ...]

--noinline compiles every DEVI helper as a real call (register analysis and the
two-waves-per-SIMD experiment); -D flags go to hipcc (e.g.
-DMGS_WAVES_PER_EU=2).  Output: mj-grasp-sim_amd/mgs/_lib/ab/NAME.hsaco and the
kernel's register / spill counts on stdout."""
import os
import shutil
import subprocess
import sys
import tempfile

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
    args = sys.argv[1:]
    name = args.pop(0)
    ncon, noinline, extra, srcdir, nefc, ghbm, drop = 20, False, [], None, None, False, []
    while args:
        a = args.pop(0)
        if a == "--ncon":
            ncon = int(args.pop(0))
        elif a == "--nefc":
            nefc = int(args.pop(0))
        elif a == "--src":
            srcdir = args.pop(0)      # kernel sources from a scratch directory (experiments)
        elif a == "--noinline":
            noinline = True
        elif a == "--ghbm":
            ghbm = True               # the G-rows-in-HBM object (mgs_model_desc.g_rows_hbm)
        elif a == "--drop":
            drop.append(args.pop(0))  # a planned flag to leave out (e.g. -disable-machine-licm)
        else:
            extra.append(a)
    env = GravitylessObjectGrasping(GripperRobotiq2f85(SE3Pose(np.zeros(3), np.array([1.0, 0, 0, 0]), "wxyz")),
                                    get_object("003_cracker_box"), ncon_max=ncon, nefc_max=nefc)
    fields, _, _ = env.model.pack(ncon_max=env.ncon_max, nefc_max=env.nefc_max)
    lib = library_for(env.model.nv, int(fields["nefc_max"]))
    if ghbm:
        fields["g_rows_hbm"] = 1
    header, flags, _ = special.plan(lib, abi.make_desc(fields))
    for f in drop:
        i = flags.index(f)
        flags = flags[:i - 1] + flags[i + 1:] if i > 0 and flags[i - 1] == "-mllvm" else flags[:i] + flags[i + 1:]
    out_dir = os.path.join(special.CACHE, "..", "ab")
    os.makedirs(out_dir, exist_ok=True)
    path = os.path.abspath(os.path.join(out_dir, name + ".hsaco"))
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "pkg", "csrc")
        os.makedirs(src)
        os.makedirs(os.path.join(td, "include"))
        shutil.copy(abi.HEADER, os.path.join(td, "include"))
        for f in os.listdir(special.CSRC):
            shutil.copy(os.path.join(srcdir or special.CSRC, f), src)
        k = os.path.join(src, "mgs_kernels.hip")
        if noinline:
            s = open(k).read()
            old = "#define DEVI __device__ __attribute__((always_inline)) inline"
            assert old in s
            open(k, "w").write(s.replace(old, "#define DEVI __device__ __attribute__((noinline))"))
        hp = os.path.join(td, "model.h")
        open(hp, "w").write(header)
        cmd = [special._hipcc(), *flags, *extra, f'-DMGS_SPECIAL="{hp}"', os.path.join(src, "mgs_special.hip"),
               "-o", path]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if os.environ.get("AB_REMARKS"):
            print("\n".join(x for x in r.stderr.splitlines() if "remark" in x))
        if r.returncode:
            print(r.stderr[-3000:])
            return 1
        co = os.path.join(td, "obj.co")
        llvm = "/opt/rocm/lib/llvm/bin"
        subprocess.run([f"{llvm}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={path}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes = subprocess.run([f"{llvm}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    print(path, "ncon", env.ncon_max, "nefc", env.nefc_max)
    for line in notes.splitlines():
        t = line.strip()
        if t.startswith((".name:", ".vgpr_count", ".agpr_count", ".vgpr_spill", ".private_segment_fixed")):
            print("  ", t)
    return 0


if __name__ == "__main__":
    sys.exit(main())
