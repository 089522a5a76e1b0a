"""ctypes binding of libmgs_gpu.so (the MI355X engine).

There is deliberately no CPU fallback: if the HIP library is missing or no
GPU is visible, every entry point raises.  (The CPU restatement under oracle/
is test infrastructure and is never imported from here.)
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from mgs.core import abi
from mgs.core.abi import ptr

LIB_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_lib")
LIB_PATH = os.path.join(LIB_DIR, "libmgs_gpu.so")
# same C-ABI, built with 4 constraint rows per lane and G in HBM (MGS_WIDE) for
# the clutter piles' dof counts and row counts
LIB_WIDE_PATH = os.path.join(LIB_DIR, "libmgs_gpu_wide.so")
_libs = {}


class EngineError(RuntimeError):
    pass


def load_library(wide: bool = False):
    path = LIB_WIDE_PATH if wide else LIB_PATH
    # build-variant experiments (tools/): MGS_LIB_MAIN names another build of the
    # same C-ABI under mgs/_lib to load as the main library
    if not wide and os.environ.get("MGS_LIB_MAIN"):
        path = os.path.join(LIB_DIR, os.environ["MGS_LIB_MAIN"])
    if wide and os.environ.get("MGS_LIB_WIDE"):
        path = os.path.join(LIB_DIR, os.environ["MGS_LIB_WIDE"])
    if path in _libs:
        return _libs[path]
    if not os.path.isfile(path):
        raise EngineError(f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(path)
    P = ctypes.POINTER
    c_i, c_d, c_u8, vp = ctypes.c_int32, ctypes.c_double, ctypes.c_uint8, ctypes.c_void_p
    L.mgs_abi_version.restype = ctypes.c_int
    L.mgs_last_error.restype = ctypes.c_char_p
    L.mgs_model_create.argtypes = [P(abi.ModelDesc), P(c_i), P(c_d), ctypes.c_int, P(vp)]
    L.mgs_model_free.argtypes = [vp]
    L.mgs_batch_open.argtypes = [vp, ctypes.c_int, P(vp)]
    L.mgs_batch_close.argtypes = [vp]
    L.mgs_collision_free.argtypes = [vp, ctypes.c_int, P(c_d), P(c_d), P(c_d), ctypes.c_int, P(c_u8)]
    L.mgs_collision_free_device.argtypes = [vp, ctypes.c_int, vp, vp, vp, ctypes.c_int, vp, vp]
    L.mgs_rollout.argtypes = [vp, P(abi.Schedule), ctypes.c_int, P(c_d), P(c_d), P(c_d), P(c_d),
                              P(abi.RolloutOut)]
    L.mgs_rollout_device.argtypes = [vp, P(abi.Schedule), ctypes.c_int, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp]
    L.mgs_overflow_list_device.argtypes = [ctypes.c_int, vp, ctypes.c_int, vp, vp, vp]
    L.mgs_rollout_list_device.argtypes = [vp, P(abi.Schedule), ctypes.c_int, vp, vp, ctypes.c_int, vp, vp, vp, vp,
                                          vp, vp, vp, vp, vp, vp]
    L.mgs_rollout_resumable_device.argtypes = [vp, P(abi.Schedule), ctypes.c_int] + [vp] * 12
    L.mgs_mask_rollout_device.argtypes = [vp, P(abi.Schedule), ctypes.c_int] + [vp] * 5 + [ctypes.c_int] + [vp] * 8
    L.mgs_rollout_resume.argtypes = [vp, P(abi.Schedule), ctypes.c_int, P(c_d), P(c_d), P(c_d), P(c_d), P(c_d),
                                     P(abi.RolloutOut)]
    L.mgs_queue_stats.argtypes = [vp, P(ctypes.c_uint64)]
    L.mgs_queue_spans.argtypes = [vp, P(c_d), ctypes.c_int, P(ctypes.c_int), P(ctypes.c_int)]
    L.mgs_last_kernel_ms.argtypes = [vp]
    L.mgs_last_kernel_ms.restype = ctypes.c_double
    L.mgs_last_collision_ms.argtypes = [vp]
    L.mgs_last_collision_ms.restype = ctypes.c_double
    L.mgs_arith_probe.argtypes = [P(c_d), P(c_d), ctypes.c_int, P(c_d)]
    L.mgs_tree_probe.argtypes = [P(c_d), P(c_d), ctypes.c_int, ctypes.c_int, P(c_d)]
    L.mgs_lds_bytes.argtypes = [vp]
    L.mgs_device_count.restype = ctypes.c_int
    L.mgs_model_lds_bytes.argtypes = [P(abi.ModelDesc), P(ctypes.c_int64)]
    L.mgs_model_layout.argtypes = [P(abi.ModelDesc), P(ctypes.c_int32), ctypes.c_int, P(ctypes.c_int32)]
    L.mgs_model_attach_special.argtypes = [vp, ctypes.c_char_p]
    L.mgs_model_special.argtypes = [vp]
    L.mgs_rows_per_lane.restype = ctypes.c_int
    L.mgs_max_rows.restype = ctypes.c_int
    L.mgs_antipodal_contacts.argtypes = [ctypes.c_int, P(c_d), ctypes.c_int, ctypes.c_int, P(c_d), P(c_d), P(c_d),
                                         c_d, P(c_d), P(c_i), P(c_d)]
    L.mgs_simulate.argtypes = [vp, P(abi.Schedule), ctypes.c_int, P(c_d), P(c_d), P(c_d), P(c_d), P(c_d), P(c_d),
                               P(c_i)]
    L.mgs_simulate_device.argtypes = [vp, P(abi.Schedule), ctypes.c_int, vp, vp, vp, vp, vp, vp, vp, vp]
    L.mgs_contact_fps.argtypes = [ctypes.c_int, P(c_d), ctypes.c_int, ctypes.c_int, P(c_i), P(c_d)]
    L.mgs_contact_seeds.argtypes = [ctypes.c_int, P(c_d), ctypes.c_int, c_d, ctypes.c_uint64, ctypes.c_int, P(c_i),
                                    P(c_i), P(c_d)]
    L.mgs_contact_optimize.argtypes = [ctypes.c_int, P(abi.KinDesc), ctypes.c_int] + [P(c_d)] * 9
    L.mgs_supports_nv.argtypes = [ctypes.c_int]
    L.mgs_supports_nv.restype = ctypes.c_int
    L.mgs_rollout_grid.argtypes = [vp, ctypes.c_int]
    L.mgs_model_resident.argtypes = [vp]
    L.mgs_model_resident.restype = ctypes.c_int
    L.mgs_rollout_grid.restype = ctypes.c_int
    L.mgs_rollout_queue.argtypes = [ctypes.c_int]
    L.mgs_rollout_queue.restype = ctypes.c_int
    if L.mgs_abi_version() != abi.MGS["MGS_ABI_VERSION"]:
        raise EngineError(f"{os.path.basename(path)} ABI version mismatch with include/mgs_gpu.h")
    _libs[path] = L
    return L


# the main library's flavour (2 rows per lane, G and NV-long operand rows on
# chip) serves dof counts up to this; larger ones use the wide flavour (4 rows
# per lane, G in HBM), instantiated or specialised (mgs.core.special)
MAIN_NV_MAX = 34
# largest dof count: 64 with one dof per lane (the libraries' kernels and most
# specialised objects), 128 with two (specialised objects of the wide flavour,
# mgs.core.special; clutter piles of 7-10 objects)
MAX_NV = 128


def library_for(nv: int, nefc_max: int):
    """the library build (flavour) whose kernels hold this model: the main one
    when it has a kernel for nv, or nv is small enough for its flavour, and the
    rows fit; else the wide one.  A dof count without an instantiation in the
    chosen library runs through a specialised code object."""
    if nv < 1 or nv > MAX_NV:
        raise EngineError(f"nv={nv}: the kernels hold 1 to {MAX_NV} dofs (lanes over dofs, two per lane past 64)")
    L = load_library()
    if nefc_max <= L.mgs_max_rows() and (L.mgs_supports_nv(nv) or nv <= MAIN_NV_MAX):
        return L
    W = load_library(wide=True)
    if nefc_max <= W.mgs_max_rows():
        return W
    raise EngineError(f"nv={nv} with {nefc_max} constraint rows exceeds every library build (mgs_max_rows)")


def supported_nvs():
    """dof counts with a compiled kernel in the main or the wide library
    (MGS_NV_LIST of each build)"""
    libs = [load_library()] + ([load_library(wide=True)] if os.path.isfile(LIB_WIDE_PATH) else [])
    return sorted({nv for L in libs for nv in range(1, 257) if L.mgs_supports_nv(nv)})


LDS_PER_CU = 160 * 1024


def lds_bytes_for(cm, ncon_max, nefc_max=None):
    """Per-candidate LDS bytes of the kernels for this model and capacity (host only)."""
    fields, _, _ = cm.pack(ncon_max=ncon_max, nefc_max=nefc_max)
    L = library_for(cm.nv, int(fields["nefc_max"]))
    desc = abi.make_desc(fields)
    out = ctypes.c_int64()
    _check(L.mgs_model_lds_bytes(ctypes.byref(desc), ctypes.byref(out)), "mgs_model_lds_bytes")
    return int(out.value)


def layout_for(cm, ncon_max, nefc_max=None):
    """The kernels' LDS carve-up for this model and capacity (mgs_model_layout:
    offsets in doubles, then ncon_max, nefc_max, nv, total), host only."""
    fields, _, _ = cm.pack(ncon_max=ncon_max, nefc_max=nefc_max)
    L = library_for(cm.nv, int(fields["nefc_max"]))
    desc = abi.make_desc(fields)
    buf = (ctypes.c_int32 * 256)()
    n = ctypes.c_int32()
    _check(L.mgs_model_layout(ctypes.byref(desc), buf, 256, ctypes.byref(n)), "mgs_model_layout")
    return [int(x) for x in buf[:n.value]]


def default_rows(cm, worst: int) -> int:
    """worst-case constraint rows, capped at what the library flavour that will
    hold this model provides (the main one for nv <= MAIN_NV_MAX or an
    instantiated nv, else the wide one)."""
    main = load_library()
    wide = load_library(wide=True) if os.path.isfile(LIB_WIDE_PATH) else None
    if (main.mgs_supports_nv(cm.nv) or cm.nv <= MAIN_NV_MAX) and (worst <= main.mgs_max_rows() or wide is None):
        return min(worst, main.mgs_max_rows())
    return min(worst, wide.mgs_max_rows()) if wide else worst


def auto_capacity(cm, ncon_max=20):
    """Constraint-row capacity for `ncon_max` contacts that keeps the most
    candidates in flight per CU: rows are shrunk from the worst case (every
    contact at the largest condim) down to 2 rows per contact as long as that
    raises the per-CU occupancy.  Candidates that exceed a capacity are
    flagged by the kernel and re-run wider (GravitylessObjectGrasping.rollout)."""
    fields, _, _ = cm.pack(ncon_max=ncon_max)
    worst = int(fields["nefc_max"])
    fixed = worst - ncon_max * (int(cm.pair_condim.max()) if len(cm.pair_condim) else 1)
    full = default_rows(cm, worst)
    best, best_occ = full, LDS_PER_CU // lds_bytes_for(cm, ncon_max, full)
    # down to 2 rows per contact (a step with more rows than that is rare: the
    # headline averages 26 rows at 4 contacts, and an overflowing candidate is
    # continued wider from that step, GravitylessObjectGrasping.rollout)
    floor = min(full, fixed + 2 * ncon_max)
    for ne in range(full - 1, floor - 1, -1):
        occ = LDS_PER_CU // lds_bytes_for(cm, ncon_max, ne)
        if occ > best_occ:
            best, best_occ = ne, occ
            break
    return ncon_max, best


def _check(rc, what, lib=None):
    if rc != 0:
        msg = (lib or load_library()).mgs_last_error().decode(errors="replace")
        raise EngineError(f"{what} failed ({rc}): {msg}")


def check_no_lost_candidates(fail_step, expired_spins=0):
    """raise if a rotating launch lost a candidate: its fail_step still holds
    the MGS_FAIL_YIELDED sentinel it wrote when it joined the ring (ABI 20), or
    the batch's expired-spin counter grew (mgs_queue_stats out[1]; callers of
    the device entries pass the growth over their launches)"""
    lost = np.nonzero(np.asarray(fail_step) == abi.MGS["MGS_FAIL_YIELDED"])[0]
    if len(lost) or expired_spins:
        raise EngineError(f"in-launch rotation lost {len(lost)} candidate(s) (first {lost[:8].tolist()}), "
                          f"{int(expired_spins)} expired ring spin(s): the launch's outputs are invalid")


class Engine:
    """One compiled model resident on one GPU plus a reusable batch."""

    def __init__(self, cm, device: int = 0, ncon_max: int = 16, nefc_max=None, specialize=None, role="main",
                 g_rows_hbm=None):
        """specialize: True = attach the model-specialised code object, compiling
        it if it is not cached; "cached" = attach it only if cached; False = the
        library's runtime-layout kernels.  Default (None): MGS_SPECIALIZE from the
        environment ("1" / "cached" / "0"), else "cached".  A dof count the
        library has no kernel for always specialises (compiling if needed).
        role: the object's role (mgs.core.special.ROLE_FLAGS): "escalation" for
        the capacity escalation's engines (kernel symbols *_esc in traces).
        g_rows_hbm: keep the constraint rows G in HBM instead of LDS (a main-
        flavour model then runs a specialised object with at most 256
        registers, packed M and the friction read from the model: six headline
        candidates per CU instead of four, +26 % on the driver's command, round
        5).  True / False; "auto" (the envs' primary engines): when that object
        is cached; None: MGS_G_HBM from the environment ("1" / "0"), else
        False.  MGS_G_HBM also overrides "auto"."""
        if nefc_max is None:
            nefc_max = default_rows(cm, int(cm.pack(ncon_max=ncon_max)[0]["nefc_max"]))
        fields, self._ib, self._db = cm.pack(ncon_max=ncon_max, nefc_max=nefc_max)
        self.lib = library_for(cm.nv, int(fields["nefc_max"]))
        env_g = os.environ.get("MGS_G_HBM")
        if g_rows_hbm is None or (g_rows_hbm == "auto" and env_g is not None):
            g_rows_hbm = env_g == "1"
        if g_rows_hbm and self.lib.mgs_rows_per_lane() != 4:
            # main flavour with the G rows in HBM: a specialised object only;
            # "auto" takes it when its object is cached (the shipped engines'
            # are prebuilt), else keeps G in LDS
            g_fields = dict(fields, g_rows_hbm=1)
            from mgs.core import special
            if g_rows_hbm is True or special.code_object(self.lib, abi.make_desc(g_fields), compile=False,
                                                         role=role) is not None:
                fields = g_fields
                specialize = True
        if self.lib.mgs_device_count() <= device:
            raise EngineError("no HIP device visible for the MI355X engine")
        self.desc = abi.make_desc(fields)
        self.cm = cm
        self.device = device
        self._model = ctypes.c_void_p()
        self._ck(self.lib.mgs_model_create(ctypes.byref(self.desc), ptr(self._ib, ctypes.c_int32),
                                         ptr(self._db, ctypes.c_double), device, ctypes.byref(self._model)),
               "mgs_model_create")
        self._batch = ctypes.c_void_p()
        self._cap = 0
        if specialize is None:
            specialize = {"1": True, "0": False}.get(os.environ.get("MGS_SPECIALIZE", "cached"), "cached")
        if not self.lib.mgs_supports_nv(cm.nv) or int(fields["maxcondim"]) > 4:
            # (condim-6 contacts run only in a code object built for them)
            specialize = True
        if specialize and os.environ.get("MGS_SPECIAL_OBJECT"):
            # A/B experiments (tools/ab_bench.sh): explicit objects (':'-separated),
            # each used by the engines whose model and capacity it was made for
            # (the attach checks that)
            for obj in os.environ["MGS_SPECIAL_OBJECT"].split(":"):
                if obj and self.lib.mgs_model_attach_special(self._model, obj.encode()) == 0:
                    specialize = False
                    break
        if specialize:
            from mgs.core import special
            path = special.code_object(self.lib, self.desc, compile=specialize is True, role=role)
            if path is not None:
                self._ck(self.lib.mgs_model_attach_special(self._model, path.encode()), "mgs_model_attach_special")

    def _ck(self, rc, what):
        _check(rc, what, self.lib)

    def close(self):
        if self._batch:
            self.lib.mgs_batch_close(self._batch)
            self._batch = ctypes.c_void_p()
        if self._model:
            self.lib.mgs_model_free(self._model)
            self._model = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def batch(self, n):
        if n > self._cap:
            if self._batch:
                self.lib.mgs_batch_close(self._batch)
            cap = max(n, 256)
            self._batch = ctypes.c_void_p()
            self._ck(self.lib.mgs_batch_open(self._model, cap, ctypes.byref(self._batch)), "mgs_batch_open")
            self._cap = cap
        return self._batch

    def queue_grid(self, n):
        """the rollout_grid of a launch over n candidates under the process's
        current queue mode, from the model's resident workgroup count
        (mgs_model_resident) without opening a batch"""
        mode = int(self.lib.mgs_rollout_queue(-1))
        r = int(self.lib.mgs_model_resident(self._model))
        if mode == 0 or r <= 0:
            return n
        if mode > 1 and r > mode:
            r = mode
        return r if r < n else n

    def rollout_grid(self, n):
        """workgroups a rollout launch over n candidates uses (mgs_rollout_grid:
        the device's resident capacity when the work queue runs, else n)"""
        g = self.lib.mgs_rollout_grid(self.batch(max(1, n)), n)
        if g < 0:
            raise EngineError(f"mgs_rollout_grid: {self.lib.mgs_last_error().decode()}")
        return g

    def collision_free(self, qpos, mocap_pos, mocap_quat, predicate="any"):
        n = len(qpos)
        out = np.zeros(n, np.uint8)
        if n == 0:
            return out.astype(bool)
        pr = abi.predicate_code(predicate)
        q = np.ascontiguousarray(qpos, np.float64)
        mp = np.ascontiguousarray(mocap_pos, np.float64)
        mq = np.ascontiguousarray(mocap_quat, np.float64)
        self._ck(self.lib.mgs_collision_free(self.batch(n), n, ptr(q, ctypes.c_double), ptr(mp, ctypes.c_double),
                                           ptr(mq, ctypes.c_double), pr, ptr(out, ctypes.c_uint8)),
               "mgs_collision_free")
        return out.astype(bool)

    def resume_width(self):
        """doubles per resume record (mgs_rollout_out.resume)"""
        return self.cm.nq + 2 * self.cm.nv + int(self.cm.nact) + abi.MGS["MGS_RESUME_EXTRA"]

    def rollout(self, plan, resumable=False, resume_from=None, pause_step=0, capped_continue=False, yield_every=0):
        """mgs_rollout.  resumable: candidates overflowing the capacity stop at
        that step (fail_step -3) and result["resume"] holds their records;
        resume_from: records of such a capped run, continued here
        (mgs_rollout_resume) instead of restarting from the plan.
        pause_step > 0 (needs resumable): candidates that have run that many
        steps stop there (fail_step -4, MGS_FLAG_PAUSED) with a record, a time
        slice a later call continues; capped_continue: over-capacity candidates
        run on capped and flagged instead of stopping.  yield_every > 0 (needs
        resumable): in-launch rotation (mgs_schedule.yield_every) when the batch
        has more rollouts than the resident grid; outputs are unchanged."""
        n = len(plan.qpos_init)
        sched = abi.make_schedule(plan.nsteps, plan.check_every, plan.check_at_end, plan.ctrl, plan.obj_qposadr,
                                  check_offset=getattr(plan, "check_offset", None))
        sched.pause_step = int(pause_step)
        sched.capped_continue = int(bool(capped_continue))
        sched.yield_every = int(yield_every)
        if yield_every and not resumable:
            raise ValueError("yield_every needs resumable=True (a yielded state goes to the resume records)")
        if pause_step and not resumable:
            raise ValueError("pause_step needs resumable=True (the paused state goes to the resume records)")
        label = np.zeros(n, np.uint8)
        fail = np.zeros(n, np.int32)
        objq = np.zeros((n, 7), np.float64)
        stats = np.zeros((n, abi.MGS["MGS_NSTATS"]), np.int32)
        if n == 0:
            return dict(label=label.astype(bool), fail_step=fail, obj_qpos=objq, stats=stats)
        rec = np.zeros((n, self.resume_width()), np.float64) if resumable else None
        out = abi.RolloutOut(ptr(label, ctypes.c_uint8), ptr(fail, ctypes.c_int32),
                             ptr(objq, ctypes.c_double), ptr(stats, ctypes.c_int32),
                             None if rec is None else ptr(rec, ctypes.c_double))
        q = np.ascontiguousarray(plan.qpos_init, np.float64)
        mq = np.ascontiguousarray(plan.mocap_quat, np.float64)
        ps = np.ascontiguousarray(plan.phase_start, np.float64)
        pt = np.ascontiguousarray(plan.phase_target, np.float64)
        if resume_from is None:
            self._ck(self.lib.mgs_rollout(self.batch(n), ctypes.byref(sched), n, ptr(q, ctypes.c_double),
                                        ptr(mq, ctypes.c_double), ptr(ps, ctypes.c_double),
                                        ptr(pt, ctypes.c_double), ctypes.byref(out)), "mgs_rollout")
        else:
            rs = np.ascontiguousarray(resume_from, np.float64)
            if rs.shape != (n, self.resume_width()):
                raise ValueError(f"resume records have shape {rs.shape}, expected {(n, self.resume_width())}")
            self._ck(self.lib.mgs_rollout_resume(self.batch(n), ctypes.byref(sched), n, ptr(q, ctypes.c_double),
                                               ptr(mq, ctypes.c_double), ptr(ps, ctypes.c_double),
                                               ptr(pt, ctypes.c_double), ptr(rs, ctypes.c_double),
                                               ctypes.byref(out)), "mgs_rollout_resume")
        # (an expired rotation spin already failed the call with MGS_EQUEUE; the
        # sentinel is the second, independent guard against a lost candidate)
        check_no_lost_candidates(fail)
        res = dict(label=label.astype(bool), fail_step=fail, obj_qpos=objq, stats=stats,
                   kernel_ms=self.lib.mgs_last_kernel_ms(self._batch))
        if rec is not None:
            res["resume"] = rec
        return res

    def simulate(self, plan, vstate=None, vclip=0.0):
        """Free simulation (mgs_simulate): final qpos, qvel, qacc_warmstart, act
        (actuator state) and stats of every state.  vstate (n, 2nv + nact):
        initial qvel | qacc_warmstart | act per state (None: the model's qvel0 /
        qacc_ws0, act 0); vclip > 0 clips qvel after each step."""
        n = len(plan.qpos_init)
        nq, nv, na = self.cm.nq, self.cm.nv, int(self.cm.nact)
        out = np.zeros((n, nq + 2 * nv + na))
        stats = np.zeros((n, abi.MGS["MGS_NSTATS"]), np.int32)
        if n:
            npz = [0] * len(plan.nsteps)
            sched = abi.make_schedule(plan.nsteps, npz, npz, plan.ctrl, -1, vclip=vclip)
            q = np.ascontiguousarray(plan.qpos_init, np.float64)
            mq = np.ascontiguousarray(plan.mocap_quat, np.float64)
            ps = np.ascontiguousarray(plan.phase_start, np.float64)
            pt = np.ascontiguousarray(plan.phase_target, np.float64)
            vs = None
            if vstate is not None:
                vs = np.ascontiguousarray(vstate, np.float64)
                if vs.shape != (n, 2 * nv + na):
                    raise ValueError(f"vstate has shape {vs.shape}, expected {(n, 2 * nv + na)}")
            self._ck(self.lib.mgs_simulate(self.batch(n), ctypes.byref(sched), n, ptr(q, ctypes.c_double),
                                         None if vs is None else ptr(vs, ctypes.c_double), ptr(mq, ctypes.c_double),
                                         ptr(ps, ctypes.c_double), ptr(pt, ctypes.c_double),
                                         ptr(out, ctypes.c_double), ptr(stats, ctypes.c_int32)), "mgs_simulate")
        return dict(qpos=out[:, :nq], qvel=out[:, nq:nq + nv], qacc_warmstart=out[:, nq + nv:nq + 2 * nv],
                    act=out[:, nq + 2 * nv:], stats=stats)

    def collision_free_device(self, n, d_qpos, d_mpos, d_mquat, d_out, predicate="any", stream=None):
        """Asynchronous launch on device pointers (ints) with inputs resident in HBM."""
        pr = abi.predicate_code(predicate)
        self._ck(self.lib.mgs_collision_free_device(self.batch(1), n, d_qpos, d_mpos, d_mquat, pr, d_out, stream),
               "mgs_collision_free_device")

    def rollout_device(self, sched, n, d_qpos, d_mquat, d_ps, d_pt, d_label, d_fail, d_objq, d_stats,
                       d_active=None, stream=None):
        """Asynchronous launch on device pointers (ints) with inputs resident in HBM;
        d_active (optional) masks out collision-mask rejects."""
        self._ck(self.lib.mgs_rollout_device(self.batch(1), ctypes.byref(sched), n, d_qpos, d_mquat, d_ps, d_pt,
                                           d_active, d_label, d_fail, d_objq, d_stats, stream),
               "mgs_rollout_device")

    def overflow_list_device(self, n, d_stats, d_count, d_list, stream=None, mask=None):
        """device list of the candidates whose stats flag a capacity overflow
        (d_count: a list header of MGS_LIST_HEADER int32 words)"""
        m = abi.MGS["MGS_FLAG_CAPACITY"] if mask is None else int(mask)
        self._ck(self.lib.mgs_overflow_list_device(n, d_stats, m, d_count, d_list, stream), "mgs_overflow_list_device")

    def rollout_resumable_device(self, sched, n, d_qpos, d_mquat, d_ps, d_pt, d_label, d_fail, d_objq, d_stats,
                                 d_resume_out, d_active=None, stream=None, d_ovf=None):
        """rollout_device whose overflowing candidates stop at the overflowing
        step and leave a resume record (n x resume_width() doubles); d_ovf: a
        zeroed device list (MGS_LIST_HEADER + n int32) the capped candidates
        append themselves to"""
        self._ck(self.lib.mgs_rollout_resumable_device(self.batch(1), ctypes.byref(sched), n, d_qpos, d_mquat, d_ps,
                                                     d_pt, d_active, d_label, d_fail, d_objq, d_stats,
                                                     d_resume_out, d_ovf, stream), "mgs_rollout_resumable_device")

    def mask_rollout_device(self, sched, n, d_qpos, d_mpos, d_mquat, d_ps, d_pt, d_free, d_label, d_fail, d_objq,
                            d_stats, d_resume_out=None, predicate="any", stream=None, d_ovf=None):
        """collision mask and rollout in one launch (mgs_mask_rollout_device):
        d_free gets the mask, the collision-free candidates are rolled out, the
        outputs are those of collision_free_device + rollout_resumable_device
        (d_ovf: the overflow list, as there)"""
        self._ck(self.lib.mgs_mask_rollout_device(self.batch(1), ctypes.byref(sched), n, d_qpos, d_mpos, d_mquat, d_ps,
                                                d_pt, abi.predicate_code(predicate), d_free, d_label, d_fail, d_objq,
                                                d_stats, d_resume_out, d_ovf, stream), "mgs_mask_rollout_device")

    def rollout_list_device(self, sched, n, d_count, d_list, grid, d_qpos, d_mquat, d_ps, d_pt, d_label, d_fail,
                            d_objq, d_stats, stream=None, d_resume_in=None):
        """re-run the candidates of a device list with `grid` workgroups looping
        over it (outputs at their batch indices); d_count is the list header
        (MGS_LIST_HEADER int32: the count ran ends in word 2, words 0-1 are left
        zeroed); d_resume_in: continue each from its resume record instead of
        from the start"""
        self._ck(self.lib.mgs_rollout_list_device(self.batch(grid), ctypes.byref(sched), n, d_count, d_list, grid,
                                                d_qpos, d_mquat, d_ps, d_pt, d_resume_in, d_label, d_fail, d_objq,
                                                d_stats, stream), "mgs_rollout_list_device")

    def queue_stats(self):
        """(yields, expired ring spins) of this engine's batch, cumulative
        (mgs_queue_stats; synchronises the device)"""
        out = (ctypes.c_uint64 * 2)()
        self._ck(self.lib.mgs_queue_stats(self.batch(1), out), "mgs_queue_stats")
        return int(out[0]), int(out[1])

    def queue_spans(self):
        """execution spans (ms, device real-time counter) of this engine's
        work-queue rollout launches completed since the previous call, oldest
        first (mgs_queue_spans; synchronises the device).  self.spans_overwritten:
        the launches since the previous call whose spans the 64-slot ring had
        already overwritten (call at least every 64 launches to keep it 0)"""
        out = (ctypes.c_double * 64)()
        cnt, lost = ctypes.c_int(), ctypes.c_int()
        self._ck(self.lib.mgs_queue_spans(self.batch(1), out, 64, ctypes.byref(cnt), ctypes.byref(lost)),
                 "mgs_queue_spans")
        self.spans_overwritten = int(lost.value)
        return [float(out[i]) for i in range(cnt.value)]

    def last_collision_ms(self):
        return self.lib.mgs_last_collision_ms(self._batch)

    def specialized(self):
        """True if this engine's launches run a model-specialised code object
        (constant LDS layout and model description), False if the runtime-offset
        kernels"""
        return bool(self.lib.mgs_model_special(self._model))

    static_layout = specialized

    def lds_bytes(self):
        return self.lib.mgs_lds_bytes(self._model)

    def last_kernel_ms(self):
        return self.lib.mgs_last_kernel_ms(self._batch)


def antipodal_contacts(tri, origin, direction, u_choice, eps, device=0):
    """GPU ray casting of the antipodal sampler (mgs_antipodal_contacts):
    returns (second contact (n,3), valid-hit count (n,), kernel ms)."""
    L = load_library()
    if L.mgs_device_count() <= device:
        raise EngineError("no HIP device visible for the MI355X engine")
    tri = np.ascontiguousarray(tri, np.float64).reshape(-1, 9)
    o = np.ascontiguousarray(origin, np.float64).reshape(-1, 3)
    d = np.ascontiguousarray(direction, np.float64).reshape(-1, 3)
    u = np.ascontiguousarray(u_choice, np.float64).reshape(-1)
    n = len(o)
    sec = np.zeros((n, 3))
    cnt = np.zeros(n, np.int32)
    ms = ctypes.c_double(0.0)
    _check(L.mgs_antipodal_contacts(device, ptr(tri, ctypes.c_double), len(tri), n, ptr(o, ctypes.c_double),
                                    ptr(d, ctypes.c_double), ptr(u, ctypes.c_double), float(eps),
                                    ptr(sec, ctypes.c_double), ptr(cnt, ctypes.c_int32), ctypes.byref(ms)),
           "mgs_antipodal_contacts", L)
    return sec, cnt, ms.value


def _device_lib(device):
    L = load_library()
    if L.mgs_device_count() <= device:
        raise EngineError("no HIP device visible for the MI355X engine")
    return L


def contact_fps(points, k, device=0):
    """farthest-point seeds on the GPU (mgs_contact_fps): (indices (k,), kernel ms)"""
    L = _device_lib(device)
    x = np.ascontiguousarray(points, np.float64).reshape(-1, 3)
    out = np.zeros(k, np.int32)
    ms = ctypes.c_double(0.0)
    _check(L.mgs_contact_fps(device, ptr(x, ctypes.c_double), len(x), int(k), ptr(out, ctypes.c_int32),
                             ctypes.byref(ms)), "mgs_contact_fps", L)
    return out, ms.value


def contact_seeds(seeds, radius, rng_seed, ntip, device=0):
    """nearest seed and the random admissible picks (mgs_contact_seeds):
    (nn (k,), sel (k, ntip), kernel ms)"""
    L = _device_lib(device)
    s = np.ascontiguousarray(seeds, np.float64).reshape(-1, 3)
    k = len(s)
    nn = np.zeros(k, np.int32)
    sel = np.zeros((k, ntip), np.int32)
    ms = ctypes.c_double(0.0)
    _check(L.mgs_contact_seeds(device, ptr(s, ctypes.c_double), k, float(radius), int(rng_seed) & (2**64 - 1),
                               int(ntip), ptr(nn, ctypes.c_int32), ptr(sel, ctypes.c_int32), ctypes.byref(ms)),
           "mgs_contact_seeds", L)
    return nn, sel, ms.value


def contact_optimize(kin_desc, rot_init, pos_init, targets, normals, device=0):
    """the batched AdamW fit (mgs_contact_optimize): dict of rot (n,3,3) rows,
    pos (n,3), joints (n,ndof), loss (n,), kernel_ms"""
    L = _device_lib(device)
    R0 = np.ascontiguousarray(rot_init, np.float64).reshape(-1, 9)
    n = len(R0)
    nt = kin_desc.ntip
    p0 = np.ascontiguousarray(pos_init, np.float64).reshape(n, 3)
    T = np.ascontiguousarray(targets, np.float64).reshape(n, nt, 3)
    N = np.ascontiguousarray(normals, np.float64).reshape(n, nt, 3)
    oR, oP = np.zeros((n, 3, 3)), np.zeros((n, 3))
    oJ, oL = np.zeros((n, kin_desc.ndof)), np.zeros(n)
    ms = ctypes.c_double(0.0)
    d = ctypes.c_double
    _check(L.mgs_contact_optimize(device, ctypes.byref(kin_desc), n, ptr(R0, d), ptr(p0, d), ptr(T, d), ptr(N, d),
                                  ptr(oR, d), ptr(oP, d), ptr(oJ, d), ptr(oL, d), ctypes.byref(ms)),
           "mgs_contact_optimize", L)
    return dict(rot=oR, pos=oP, joints=oJ, loss=oL, kernel_ms=ms.value)


def tree_probe(a, c, n):
    """Device pairwise-tree reduction of a*c over the first n of 64 lanes, per row."""
    L = load_library()
    a = np.ascontiguousarray(a, np.float64).reshape(-1, 64)
    c = np.ascontiguousarray(c, np.float64).reshape(-1, 64)
    out = np.zeros(len(a))
    _check(L.mgs_tree_probe(ptr(a, ctypes.c_double), ptr(c, ctypes.c_double), n, len(a), ptr(out, ctypes.c_double)),
           "mgs_tree_probe")
    return out


def arith_probe(x, y):
    L = load_library()
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    out = np.zeros((len(x), 4))
    _check(L.mgs_arith_probe(ptr(x, ctypes.c_double), ptr(y, ctypes.c_double), len(x), ptr(out, ctypes.c_double)),
           "mgs_arith_probe")
    return out
