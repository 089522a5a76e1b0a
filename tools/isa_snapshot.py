"""Disassemble the shipped configurations' specialised code objects into a
directory (one .s per engine variant, named by its position in the shipped
list), so that a kernel-source change meant to leave existing builds alone can
be checked instruction for instruction:

    python tools/isa_snapshot.py /tmp/isa_before
    (edit the kernels)
    python tools/isa_snapshot.py /tmp/isa_after
    diff -r /tmp/isa_before /tmp/isa_after

Each variant also gets a .meta file: its kernels' register, spill, scratch and
LDS records from the code object's notes.

Objects missing from the cache are compiled (in parallel) first.  CPU only.
"""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mj-grasp-sim_amd"))

from mgs.core import abi, special  # noqa: E402
from mgs.core.engine import default_rows, library_for  # noqa: E402
from mgs.core.shipped import shipped_engines  # noqa: E402

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
BUNDLER = "/opt/rocm/lib/llvm/bin/clang-offload-bundler"
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def variants():
    out = []
    for k, (cm, nc, ne, role) in enumerate(shipped_engines()):
        if ne is None:
            ne = default_rows(cm, int(cm.pack(ncon_max=nc)[0]["nefc_max"]))
        fields, _, _ = cm.pack(ncon_max=nc, nefc_max=ne)
        lib = library_for(cm.nv, int(fields["nefc_max"]))
        vs = [("", fields)]
        if role == "main" and lib.mgs_rows_per_lane() != 4:
            vs.append(("_ghbm", dict(fields, g_rows_hbm=1)))
        for tag, f in vs:
            header, flags, path = special.plan(lib, abi.make_desc(f), role=role)
            out.append((f"{k:02d}_{role}_nv{cm.nv}{tag}", header, flags, path))
    return out


def main():
    dst = sys.argv[1]
    os.makedirs(dst, exist_ok=True)
    vs = variants()

    def build(v):
        name, header, flags, path = v
        if not os.path.isfile(path):
            special.compile_object(header, flags, path)
        # --genco writes an offload bundle: take the gfx950 code object out first
        elf = os.path.join(dst, name + ".elf")
        subprocess.run([BUNDLER, "--unbundle", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        f"--input={path}", f"--output={elf}"], check=True)
        r = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", elf], capture_output=True, text=True, check=True)
        notes = subprocess.run([READELF, "--notes", elf], capture_output=True, text=True, check=True).stdout
        os.remove(elf)
        # the kernels' resource records (registers, spills, scratch, LDS)
        keep = ("  - .name:", ".vgpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count",
                ".private_segment_fixed_size", ".agpr_count", ".group_segment_fixed_size")
        with open(os.path.join(dst, name + ".meta"), "w") as f:
            f.write("\n".join(l for l in notes.splitlines() if l.strip().startswith(keep) or l.startswith(keep)))
        # drop the file-name line (the object's cache key changes with the sources)
        text = "\n".join(l for l in r.stdout.splitlines() if ".elf" not in l)
        with open(os.path.join(dst, name + ".s"), "w") as f:
            f.write(text)
        return name

    with ThreadPoolExecutor(max_workers=8) as ex:
        for n in ex.map(build, vs):
            print(n)


if __name__ == "__main__":
    main()
