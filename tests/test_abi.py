"""The drop-in boundary: libmgs_gpu.so loads without a GPU, exports every
function include/mgs_gpu.h declares, and the Python mirror of the header
structs matches it.  No compute calls here (CPU container)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "mgs_gpu.h")


def header_functions():
    txt = open(HDR).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w ]*?[\s\*]+(mgs_\w+)\s*\(", txt, flags=re.M)))


@pytest.fixture(scope="module")
def lib():
    from mgs.core import engine
    if not os.path.isfile(engine.LIB_PATH):
        import __graft_entry__
        __graft_entry__.build()
    return ctypes.CDLL(engine.LIB_PATH)


def test_header_declares_the_boundary():
    fns = header_functions()
    for f in ["mgs_abi_version", "mgs_last_error", "mgs_model_create", "mgs_model_free", "mgs_batch_open",
              "mgs_batch_close", "mgs_collision_free", "mgs_collision_free_device", "mgs_rollout",
              "mgs_rollout_device", "mgs_last_kernel_ms", "mgs_last_collision_ms"]:
        assert f in fns, f


def test_library_exports_every_declared_symbol(lib):
    missing = [f for f in header_functions() if not hasattr(lib, f)]
    assert not missing, missing


def test_abi_version(lib):
    from mgs.core import abi
    lib.mgs_abi_version.restype = ctypes.c_int
    assert lib.mgs_abi_version() == abi.MGS["MGS_ABI_VERSION"]


def test_struct_mirror_matches_header():
    from mgs.core import abi
    txt = open(HDR).read()
    body = txt[txt.index("typedef struct mgs_model_desc"):]
    body = body[:body.index("} mgs_model_desc;")]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    names = re.findall(r"(?:int32_t|double|int)\s+(\w+)(?:\[\d+\])?\s*;", body)
    assert [f for f, _ in abi.ModelDesc._fields_] == names


def test_kin_desc_mirror_matches_library(lib):
    """the contact sampler's model struct: ctypes layout == the compiled one"""
    from mgs.core import abi
    lib.mgs_kin_desc_size.restype = ctypes.c_int
    assert lib.mgs_kin_desc_size() == ctypes.sizeof(abi.KinDesc)
    assert abi.KinDesc.perm.size == ctypes.sizeof(ctypes.c_int32) * 120 * 5


def test_pack_fills_every_offset(env):
    from mgs.core import abi
    fields, ib, db = env.model.pack(ncon_max=16)
    d = abi.make_desc(fields)
    for f, _ in abi.ModelDesc._fields_:
        if f.startswith("i_"):
            assert 0 <= getattr(d, f) <= len(ib), f
        if f.startswith("d_"):
            assert 0 <= getattr(d, f) <= len(db), f
    assert d.isize == len(ib) and d.dsize == len(db)


def test_engine_fails_loudly_without_gpu(env, lib):
    """No silent CPU fallback: without a visible device the product raises."""
    from mgs.core import engine
    lib.mgs_device_count.restype = ctypes.c_int
    if lib.mgs_device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(engine.EngineError):
        engine.Engine(env.model)


def test_layout_export_is_consistent(env):
    """mgs_model_layout: offsets ascend, the total matches mgs_model_lds_bytes"""
    from mgs.core.engine import layout_for, lds_bytes_for
    w = layout_for(env.model, env.ncon_max, env.nefc_max)
    nc, ne, nv, total = w[-4:]
    assert (nc, ne, nv) == (env.ncon_max, env.nefc_max, env.model.nv)
    assert total * 8 == lds_bytes_for(env.model, env.ncon_max, env.nefc_max)


def test_specialisation_header(env):
    """mgs.core.special: the generated header names every mgs_model_desc field
    (designated initialisers in declaration order) with the ABI version and
    struct size the kernels static_assert, and the cache key follows the
    description"""
    import ctypes
    from mgs.core import abi, special
    from mgs.core.engine import library_for
    fields, _, _ = env.model.pack(ncon_max=env.ncon_max, nefc_max=env.nefc_max)
    lib = library_for(env.model.nv, int(fields["nefc_max"]))
    desc = abi.make_desc(fields)
    header, flags, path = special.plan(lib, desc)
    names = [n for n, _ in abi.ModelDesc._fields_]
    pos = [header.index(f".{n} = ") for n in names]
    assert pos == sorted(pos)
    assert f"#define MGS_SL_ABI {abi.MGS['MGS_ABI_VERSION']}" in header
    assert f"#define MGS_SL_DESC_BYTES {ctypes.sizeof(abi.ModelDesc)}" in header
    assert f"#define MGS_SL_NV {env.model.nv}" in header
    desc.nefc_max -= 1
    assert special.plan(lib, desc)[2] != path


def test_headline_specialised_object_is_built(env):
    """build() compiles the headline engine's specialised code object into the
    in-tree cache (it travels to the GPU box with the tree), so bench.py's
    headline launches the constant-layout kernels"""
    from mgs.core import abi, special
    from mgs.core.engine import library_for
    fields, _, _ = env.model.pack(ncon_max=env.ncon_max, nefc_max=env.nefc_max)
    lib = library_for(env.model.nv, int(fields["nefc_max"]))
    path = special.plan(lib, abi.make_desc(fields))[2]
    if not os.path.isdir(special.CACHE):
        pytest.skip("build() ran without the specialised objects")
    assert os.path.isfile(path), "headline specialised object missing: run __graft_entry__.build()"
