"""ctypes wrapper of oracle/libmgs_oracle.so -- TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg (see mgs_oracle.c's header for what the oracle restates and its parity
status).  The product (mj-grasp-sim_amd/) never imports this module.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from mgs.core import abi
from mgs.core.abi import ptr

_HERE = os.path.dirname(os.path.abspath(__file__))
# MGS_ORACLE_LIB: another build of the same sources (the sanitizer build of
# `make asan`, tools/asan_oracle.sh)
_LIB = os.environ.get("MGS_ORACLE_LIB") or os.path.join(_HERE, "libmgs_oracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        srcs = [os.path.join(_HERE, f) for f in ("mgs_oracle.c", "mgs_contact_oracle.c")]
        if not os.path.isfile(_LIB) or os.path.getmtime(_LIB) < max(os.path.getmtime(f) for f in srcs):
            build()
        L = ctypes.CDLL(_LIB)
        c_i, c_d, c_u8 = ctypes.c_int32, ctypes.c_double, ctypes.c_uint8
        P = ctypes.POINTER
        L.oracle_collision_free.argtypes = [P(abi.ModelDesc), P(c_i), P(c_d), ctypes.c_int, P(c_d), P(c_d),
                                            P(c_d), ctypes.c_int, P(c_u8), ctypes.c_int]
        L.oracle_rollout.argtypes = [P(abi.ModelDesc), P(c_i), P(c_d), P(abi.Schedule), ctypes.c_int, P(c_d),
                                     P(c_d), P(c_d), P(c_d), P(c_u8), P(c_i), P(c_d), P(c_i), ctypes.c_int]
        L.oracle_trace.argtypes = [P(abi.ModelDesc), P(c_i), P(c_d), P(c_d), P(c_d), P(c_d), P(c_d),
                                   ctypes.c_int, P(c_d), P(c_i), P(c_d)]
        L.oracle_contacts.argtypes = [P(abi.ModelDesc), P(c_i), P(c_d), P(c_d), P(c_d), P(c_d), ctypes.c_int,
                                      P(c_d), P(c_d), P(c_d), P(c_i)]
        L.oracle_sincos.argtypes = [P(c_d), ctypes.c_int, P(c_d), P(c_d)]
        L.oracle_tree_dot.argtypes = [P(c_d), P(c_d), ctypes.c_int]
        L.oracle_tree_dot.restype = c_d
        L.oracle_set_bbmode.argtypes = [ctypes.c_int]
        L.oracle_set_eqimp.argtypes = [ctypes.c_int]
        _lib = L
    return _lib


class OracleModel:
    def __init__(self, cm, ncon_max=16, nefc_max=None):
        fields, self.ib, self.db = cm.pack(ncon_max=ncon_max, nefc_max=nefc_max)
        self.desc = abi.make_desc(fields)
        self.cm = cm

    def _args(self):
        return (ctypes.byref(self.desc), ptr(self.ib, ctypes.c_int32), ptr(self.db, ctypes.c_double))

    def collision_free(self, qpos, mocap_pos, mocap_quat, predicate="any", nthreads=1):
        n = len(qpos)
        out = np.zeros(n, np.uint8)
        pr = abi.predicate_code(predicate)
        q = np.ascontiguousarray(qpos, np.float64)
        mp = np.ascontiguousarray(mocap_pos, np.float64)
        mq = np.ascontiguousarray(mocap_quat, np.float64)
        lib().oracle_collision_free(*self._args(), n, ptr(q, ctypes.c_double), ptr(mp, ctypes.c_double),
                                    ptr(mq, ctypes.c_double), pr, ptr(out, ctypes.c_uint8), nthreads)
        return out.astype(bool)

    def rollout(self, plan, nthreads=1):
        n = len(plan.qpos_init)
        sched = abi.make_schedule(plan.nsteps, plan.check_every, plan.check_at_end, plan.ctrl, plan.obj_qposadr,
                                  check_offset=getattr(plan, "check_offset", None))
        label = np.zeros(n, np.uint8)
        fail = np.zeros(n, np.int32)
        objq = np.zeros((n, 7), np.float64)
        stats = np.zeros((n, abi.MGS["MGS_NSTATS"]), np.int32)
        q = np.ascontiguousarray(plan.qpos_init, np.float64)
        mq = np.ascontiguousarray(plan.mocap_quat, np.float64)
        ps = np.ascontiguousarray(plan.phase_start, np.float64)
        pt = np.ascontiguousarray(plan.phase_target, np.float64)
        lib().oracle_rollout(*self._args(), ctypes.byref(sched), n, ptr(q, ctypes.c_double),
                             ptr(mq, ctypes.c_double), ptr(ps, ctypes.c_double), ptr(pt, ctypes.c_double),
                             ptr(label, ctypes.c_uint8), ptr(fail, ctypes.c_int32), ptr(objq, ctypes.c_double),
                             ptr(stats, ctypes.c_int32), nthreads)
        return dict(label=label.astype(bool), fail_step=fail, obj_qpos=objq, stats=stats)

    def simulate_batch(self, plan, vstate=None, vclip=0.0, nthreads=1):
        """mgs_simulate restated: final qpos, qvel, qacc_warmstart, act and stats of
        every state; vstate (n, 2nv + nact): initial qvel | warmstart | act."""
        n = len(plan.qpos_init)
        cm = self.cm
        sched = abi.make_schedule(plan.nsteps, plan.check_every, plan.check_at_end, plan.ctrl, plan.obj_qposadr,
                                  check_offset=getattr(plan, "check_offset", None), vclip=vclip)
        na = int(cm.nact)
        out = np.zeros((n, cm.nq + 2 * cm.nv + na))
        stats = np.zeros((n, abi.MGS["MGS_NSTATS"]), np.int32)
        q = np.ascontiguousarray(plan.qpos_init, np.float64)
        mq = np.ascontiguousarray(plan.mocap_quat, np.float64)
        ps = np.ascontiguousarray(plan.phase_start, np.float64)
        pt = np.ascontiguousarray(plan.phase_target, np.float64)
        vs = None if vstate is None else np.ascontiguousarray(vstate, np.float64)
        if vs is not None and vs.shape != (n, 2 * cm.nv + na):
            raise ValueError(f"vstate has shape {vs.shape}, expected {(n, 2 * cm.nv + na)}")
        lib().oracle_simulate_batch(*self._args(), ctypes.byref(sched), n, ptr(q, ctypes.c_double),
                                    None if vs is None else ptr(vs, ctypes.c_double), ptr(mq, ctypes.c_double),
                                    ptr(ps, ctypes.c_double), ptr(pt, ctypes.c_double), ptr(out, ctypes.c_double),
                                    ptr(stats, ctypes.c_int32), nthreads)
        nq, nv = cm.nq, cm.nv
        return dict(qpos=out[:, :nq], qvel=out[:, nq:nq + nv], qacc_warmstart=out[:, nq + nv:nq + 2 * nv],
                    act=out[:, nq + 2 * nv:], stats=stats)

    def trace(self, qpos, mocap_pos, mocap_quat, ctrl, nsteps):
        nq = self.cm.nq
        tr = np.zeros((nsteps, nq))
        nc = np.zeros(nsteps, np.int32)
        qv = np.zeros(self.cm.nv)
        args = [np.ascontiguousarray(a, np.float64) for a in (qpos, mocap_pos, mocap_quat, ctrl)]
        lib().oracle_trace(*self._args(), *[ptr(a, ctypes.c_double) for a in args], nsteps,
                           ptr(tr, ctypes.c_double), ptr(nc, ctypes.c_int32), ptr(qv, ctypes.c_double))
        return tr, nc, qv

    def simulate(self, qpos, mocap_pos, mocap_quat, ctrl, nsteps, vclip=0.0):
        """free simulation from qpos and the model's qvel0 / qacc_ws0; returns the
        final (qpos, qvel, qacc_warmstart)."""
        from types import SimpleNamespace
        mp = np.asarray(mocap_pos, np.float64).reshape(1, 1, 3)
        plan = SimpleNamespace(nsteps=[int(nsteps)], check_every=[0], check_at_end=[0],
                               ctrl=[np.asarray(ctrl, np.float64)], obj_qposadr=-1, check_offset=None,
                               qpos_init=np.asarray(qpos, np.float64).reshape(1, -1),
                               mocap_quat=np.asarray(mocap_quat, np.float64).reshape(1, 4),
                               phase_start=mp, phase_target=mp)
        r = self.simulate_batch(plan, vclip=vclip)
        return r["qpos"][0], r["qvel"][0], r["qacc_warmstart"][0]

    def forward_debug(self, qpos, mocap_pos, mocap_quat, ctrl, qvel=None, qacc_ws=None, solver=2):
        """one forward() at a state (oracle_forward_debug): the constraint rows'
        forces, types (efc_type), dims, R, b, aref, and qacc"""
        L = lib()
        P, d, i32 = ctypes.POINTER, ctypes.c_double, ctypes.c_int32
        L.oracle_forward_debug.argtypes = [P(abi.ModelDesc), P(i32), P(d)] + [P(d)] * 6 + [ctypes.c_int] + \
            [P(d), P(d), P(i32), P(i32), P(d), P(d), P(d), P(d)]
        nv, cap = self.cm.nv, int(self.desc.nefc_max)
        f, qa, ty, it = np.zeros(cap), np.zeros(nv), np.zeros(cap, np.int32), np.zeros(1, np.int32)
        R, ar, pm = np.zeros(2 * cap), np.zeros(cap), np.zeros(4 * cap)
        z = np.zeros(nv)
        a = [np.ascontiguousarray(x, np.float64) for x in
             (qpos, z if qvel is None else qvel, z if qacc_ws is None else qacc_ws, mocap_pos, mocap_quat, ctrl)]
        ne = L.oracle_forward_debug(*self._args(), *[ptr(x, d) for x in a], int(solver), ptr(f, d), ptr(qa, d),
                                    ptr(ty, i32), ptr(it, i32), None, ptr(ar, d), ptr(R, d), ptr(pm, d))
        return dict(nefc=ne, force=f[:ne], type=ty[:ne] // 16, dim=ty[:ne] % 16, R=R[:ne], b=R[ne:2 * ne],
                    aref=ar[:ne], pos=pm[:ne], margin=pm[ne:2 * ne], diag=pm[2 * ne:3 * ne],
                    vel=pm[3 * ne:4 * ne], qacc=qa, iters=int(it[0]))

    def contacts(self, qpos, mocap_pos, mocap_quat, maxc=64):
        pos = np.zeros((maxc, 3)); fr = np.zeros((maxc, 9)); dist = np.zeros(maxc); g = np.zeros((maxc, 2), np.int32)
        args = [np.ascontiguousarray(a, np.float64) for a in (qpos, mocap_pos, mocap_quat)]
        n = lib().oracle_contacts(*self._args(), *[ptr(a, ctypes.c_double) for a in args], maxc,
                                  ptr(pos, ctypes.c_double), ptr(fr, ctypes.c_double), ptr(dist, ctypes.c_double),
                                  ptr(g, ctypes.c_int32))
        k = min(n, maxc)
        return n, pos[:k], fr[:k], dist[:k], g[:k]


def antipodal_contacts(tri, origin, direction, u_choice, eps, nthreads=8):
    """CPU restatement of mgs_antipodal_contacts (checker)."""
    tri = np.ascontiguousarray(tri, np.float64).reshape(-1, 9)
    o = np.ascontiguousarray(origin, np.float64).reshape(-1, 3)
    d = np.ascontiguousarray(direction, np.float64).reshape(-1, 3)
    u = np.ascontiguousarray(u_choice, np.float64).reshape(-1)
    n = len(o)
    sec = np.zeros((n, 3))
    cnt = np.zeros(n, np.int32)
    L = lib()
    L.oracle_antipodal_contacts.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.c_int] + \
        [ctypes.POINTER(ctypes.c_double)] * 3 + [ctypes.c_double, ctypes.POINTER(ctypes.c_double),
                                                 ctypes.POINTER(ctypes.c_int32), ctypes.c_int]
    L.oracle_antipodal_contacts(ptr(tri, ctypes.c_double), len(tri), n, ptr(o, ctypes.c_double),
                                ptr(d, ctypes.c_double), ptr(u, ctypes.c_double), float(eps),
                                ptr(sec, ctypes.c_double), ptr(cnt, ctypes.c_int32), nthreads)
    return sec, cnt


def contact_predicate(om, pairs, predicate):
    """oracle_contact_predicate: the kernels' contact predicate on a given list
    of (geom1, geom2) collision-geom index pairs"""
    L = lib()
    L.oracle_contact_predicate.argtypes = [ctypes.POINTER(abi.ModelDesc), ctypes.POINTER(ctypes.c_int32),
                                           ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int32),
                                           ctypes.c_int, ctypes.c_int]
    pr = np.ascontiguousarray(np.asarray(pairs, np.int32).reshape(-1, 2))
    return bool(L.oracle_contact_predicate(*om._args(), ptr(pr, ctypes.c_int32), len(pr),
                                           abi.predicate_code(predicate)))


def sincos(x):
    x = np.ascontiguousarray(x, np.float64)
    s = np.zeros_like(x)
    c = np.zeros_like(x)
    lib().oracle_sincos(ptr(x, ctypes.c_double), len(x), ptr(s, ctypes.c_double), ptr(c, ctypes.c_double))
    return s, c


def tree_dot(a, b, n):
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    return lib().oracle_tree_dot(ptr(a, ctypes.c_double), ptr(b, ctypes.c_double), n)


# ---------------------------------------------------------------------------
# contact-based dexterous-hand sampler (oracle/mgs_contact_oracle.c; checker)
def _contact_lib():
    L = lib()
    P, d, i32 = ctypes.POINTER, ctypes.c_double, ctypes.c_int32
    L.oracle_contact_fps.argtypes = [P(d), ctypes.c_int, ctypes.c_int, P(i32)]
    L.oracle_contact_seeds.argtypes = [P(d), ctypes.c_int, d, ctypes.c_uint64, ctypes.c_int, P(i32), P(i32),
                                       ctypes.c_int]
    L.oracle_contact_optimize.argtypes = [P(abi.KinDesc), ctypes.c_int] + [P(d)] * 8 + [ctypes.c_int]
    L.oracle_contact_fk.argtypes = [P(abi.KinDesc), P(d), P(d), P(d)]
    L.oracle_contact_loss_grad.argtypes = [P(abi.KinDesc), P(d), P(d), P(d), P(d)]
    L.oracle_contact_loss_grad.restype = d
    return L


def contact_fps(points, k):
    x = np.ascontiguousarray(points, np.float64).reshape(-1, 3)
    out = np.zeros(k, np.int32)
    _contact_lib().oracle_contact_fps(ptr(x, ctypes.c_double), len(x), int(k), ptr(out, ctypes.c_int32))
    return out


def contact_seeds(seeds, radius, rng_seed, ntip, nthreads=8):
    s = np.ascontiguousarray(seeds, np.float64).reshape(-1, 3)
    k = len(s)
    nn = np.zeros(k, np.int32)
    sel = np.zeros((k, ntip), np.int32)
    _contact_lib().oracle_contact_seeds(ptr(s, ctypes.c_double), k, float(radius), int(rng_seed) & (2**64 - 1),
                                        int(ntip), ptr(nn, ctypes.c_int32), ptr(sel, ctypes.c_int32), nthreads)
    return nn, sel


def contact_optimize(desc, rot_init, pos_init, targets, normals, nthreads=8):
    d = ctypes.c_double
    R0 = np.ascontiguousarray(rot_init, np.float64).reshape(-1, 9)
    n = len(R0)
    p0 = np.ascontiguousarray(pos_init, np.float64).reshape(n, 3)
    T = np.ascontiguousarray(targets, np.float64).reshape(n, desc.ntip, 3)
    N = np.ascontiguousarray(normals, np.float64).reshape(n, desc.ntip, 3)
    oR, oP, oJ, oL = np.zeros((n, 3, 3)), np.zeros((n, 3)), np.zeros((n, desc.ndof)), np.zeros(n)
    _contact_lib().oracle_contact_optimize(ctypes.byref(desc), n, ptr(R0, d), ptr(p0, d), ptr(T, d), ptr(N, d),
                                           ptr(oR, d), ptr(oP, d), ptr(oJ, d), ptr(oL, d), nthreads)
    return dict(rot=oR, pos=oP, joints=oJ, loss=oL)


def contact_fk(desc, theta):
    """hand-frame tip points (ntip, 3 points, 3) and their chain derivatives
    (ntip, MAXCHAIN, 3, 3)"""
    d = ctypes.c_double
    th = np.ascontiguousarray(theta, np.float64)
    mc = abi.MGS["MGS_KIN_MAXCHAIN"]
    X = np.zeros((desc.ntip, 3, 3))
    dX = np.zeros((desc.ntip, mc, 3, 3))
    _contact_lib().oracle_contact_fk(ctypes.byref(desc), ptr(th, d), ptr(X, d), ptr(dX, d))
    return X, dX


def contact_loss_grad(desc, prm, targets, normals):
    d = ctypes.c_double
    p = np.ascontiguousarray(prm, np.float64)
    T = np.ascontiguousarray(targets, np.float64)
    N = np.ascontiguousarray(normals, np.float64)
    g = np.zeros(len(p))
    loss = _contact_lib().oracle_contact_loss_grad(ctypes.byref(desc), ptr(p, d), ptr(T, d), ptr(N, d), ptr(g, d))
    return loss, g


def set_study_variant(bbmode=0, eqimp=0):
    """the state_close study's model variants (mgs_oracle.c oracle_set_bbmode /
    oracle_set_eqimp); (0, 0) is the contract the kernels follow"""
    lib().oracle_set_bbmode(int(bbmode))
    lib().oracle_set_eqimp(int(eqimp))
