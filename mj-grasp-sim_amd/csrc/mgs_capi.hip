// mgs_capi.hip -- host side of libmgs_gpu.so: the C-ABI declared in
// include/mgs_gpu.h (model upload, batch buffers, kernel launches, timing).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#ifdef MGS_WIDE
#define MGS_RPL 4
#ifndef MGS_G_LDS          /* -DMGS_G_LDS: the wide build with G kept in LDS (experiments) */
#define MGS_G_GLOBAL 1
#endif
#endif
#include "mgs_kernels.hip"
#include "mgs_launch.h"
#include "mgs_sampler.hip"
#include "mgs_contact.hip"

#include <cstdlib>

#define MGS_QUEUE_RING 64

namespace {
thread_local std::string g_err;

int fail(int code, const char* fmt, const char* what = "") {
  char buf[512];
  snprintf(buf, sizeof(buf), fmt, what);
  g_err = buf;
  return code;
}

#define HIPCHK(expr)                                                                  \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess) return fail(MGS_EHIP, "HIP error: %s", hipGetErrorString(_e)); \
  } while (0)

// whether a model's G rows live in HBM
#ifdef MGS_G_GLOBAL
bool g_in_hbm(const mgs_model_desc&) { return true; }
#else
bool g_in_hbm(const mgs_model_desc& m) { return m.g_rows_hbm != 0; }
#endif

// main-library objects with G in HBM also pack M / the Newton Hessian and read
// the contacts' friction from the model (-DMGS_PACKED=1 -DMGS_MU_MODEL=1,
// mgs/core/special.py), so that six headline candidates fit a CU
int m_square_size(const mgs_model_desc& m) {
  const int nv = m.nv;
  return (MGS_PACKED || m.g_rows_hbm) ? nv * (nv + 1) / 2 : nv * nv;
}
bool mu_from_model(const mgs_model_desc& m) { return !MGS_PACKED && m.g_rows_hbm; }
// ... and keep certificates, contact frames and contact blocks in the HBM
// slice (-DMGS_HBM_EXTRA=1): seven headline candidates per CU
bool hbm_extra(const mgs_model_desc& m) { return !MGS_PACKED && m.g_rows_hbm; }
int layout_maxdim(const mgs_model_desc& m);
size_t hbm_slice_doubles(const mgs_model_desc& m) {
  const int md = layout_maxdim(m);
  return (size_t)m.nefc_max * m.nv +
         (hbm_extra(m) ? (size_t)(K_CERT * CERT_W + 9 * m.ncon_max + md * md * m.ncon_max) : 0);
}

// the contact dimension the kernels for this model are built for (MGS_MAXDIM)
int layout_maxdim(const mgs_model_desc& m) { return m.maxcondim > 4 ? 6 : 4; }

// LDS carve-up of one candidate's working set (doubles, then int counters and
// index arrays).  U is time-multiplexed: collision scratch, then composite
// inertias / RNE temporaries, then constraint rows (G) + solver scratch, then
// the integrator's derivative matrix.
Lay make_layout(const mgs_model_desc& m, size_t* bytes) {
  Lay l;
  memset(&l, 0, sizeof(l));
  int nq = m.nq, nv = m.nv, nb = m.nbody, ng = m.ngeom, nu = m.nu > 0 ? m.nu : 1;
  int nj = m.njnt > 0 ? m.njnt : 1, nc = m.ncon_max, ne = m.nefc_max;
  int sizes[L_COUNT];
  sizes[L_qpos] = nq; sizes[L_qvel] = nv; sizes[L_qacc_ws] = nv; sizes[L_ctrl] = nu;
  sizes[L_mocap_pos] = 3 * m.nmocap + 3; sizes[L_mocap_quat] = 4 * m.nmocap + 4; sizes[L_time] = 1;
  sizes[L_act] = m.nact; sizes[L_act_dot] = m.nact;
  sizes[L_xpos] = 3 * nb; sizes[L_xquat] = 4 * nb; sizes[L_xmat] = 9 * nb; sizes[L_subtree_com] = 3 * nb;
  sizes[L_cinert] = 10 * nb; sizes[L_cdof] = 6 * nv;
  sizes[L_M] = m_square_size(m); sizes[L_Dv] = nv; sizes[L_Dinv] = nv; sizes[L_sD] = nv; sizes[L_isD] = nv;
  sizes[L_tmp] = nv; sizes[L_tmp2] = nv;
  sizes[L_qfrc_smooth] = nv; sizes[L_qacc_smooth] = nv; sizes[L_qfrc_constraint] = nv;
  // (the wide build reads the actuator moment rows from the model)
  sizes[L_act_force] = nu; sizes[L_act_moment] = MGS_PACKED ? 0 : nu * nv; sizes[L_act_length] = nu; sizes[L_act_vel] = nu;
  sizes[L_con_pos] = 3 * nc; sizes[L_con_frame] = hbm_extra(m) ? 0 : 9 * nc; sizes[L_con_dist] = nc; sizes[L_con_mu] = mu_from_model(m) ? 0 : 5 * nc;
  // contact blocks (and Newton cone Hessians): maxdim^2 per contact, maxdim 6
  // for models with condim-6 pairs (their code objects: -DMGS_MAXDIM=6)
  const int maxdim = layout_maxdim(m);
  sizes[L_con_blk] = hbm_extra(m) ? 0 : maxdim * maxdim * nc;
  sizes[L_efc_R] = ne; sizes[L_efc_b] = ne; sizes[L_cert] = hbm_extra(m) ? 0 : K_CERT * CERT_W;
  // U: per-stage sub-layouts, each packed from offset 0 (see the kernel's Lay comment)
  int us[U_COUNT];
  for (int k = 0; k < U_COUNT; k++) us[k] = 0;
  us[U_poly] = K_POLY_POINTS * 3; us[U_pdep] = K_MAXPOLY; us[U_geom_xpos] = 3 * ng; us[U_geom_xmat] = 9 * ng;
  us[U_xipos] = 3 * nb; us[U_xanchor] = 3 * nj; us[U_xaxis] = 3 * nj; us[U_subtree_mass] = nb;
  us[U_comacc] = 4 * nb;
  us[U_cvel] = 6 * nb; us[U_cacc] = 6 * nb; us[U_cfrc] = 6 * nb; us[U_cdof_dot] = 6 * nv;
  us[U_qfrc_bias] = nv; us[U_qfrc_passive] = nv; us[U_qfrc_actuator] = nv;
  // G in HBM (batch buffer, see bind()): the wide library always, the main
  // library's specialised objects on request (mgs_model_desc.g_rows_hbm)
  us[U_G] = g_in_hbm(m) ? 0 : ne * (nv + MGS_GPAD);   // row stride: GS in the kernel
  us[U_aref] = ne;
  us[U_scratch] = (2 * ne > nv ? 2 * ne : nv);
  // {vel, pos, margin} (make_constraints) | Newton Hessian, which may run on into
  // the scratch slot (scratch is idle while the Hessian is live)
  // (the Hessian's weight table, (maxdim + 1) ne, runs on into scratch too)
  int xreg = 3 * ne;
  if (xreg + us[U_scratch] < (maxdim + 1) * ne) xreg = (maxdim + 1) * ne - us[U_scratch];
  if (xreg + us[U_scratch] < m_square_size(m)) xreg = m_square_size(m) - us[U_scratch];
  us[U_jar] = ne; us[U_jv] = ne; us[U_f] = ne; us[U_Dr] = ne; us[U_isR] = ne;
  us[U_nw] = nv; us[U_nw0] = nv; us[U_ng] = nv; us[U_ndir] = nv;
  int U = 0, off;
  // kin / collision stage
  off = 0;
  for (int k = U_poly; k <= U_comacc; k++) { l.u[k] = off; off += us[k]; }
  if (off > U) U = off;
  // dynamics: crb alone, then rne arrays (crb is dead by then) + qfrc parts
  l.u[U_crb] = 0;
  if (10 * nb > U) U = 10 * nb;
  off = 0;
  for (int k = U_cvel; k <= U_qfrc_actuator; k++) { l.u[k] = off; off += us[k]; }
  if (off > U) U = off;
  // constraints + solver
  off = 0;
  l.u[U_G] = off; off += us[U_G];
  l.u[U_aref] = off; off += us[U_aref];
  l.u[U_vel] = off; l.u[U_pos] = off + ne; l.u[U_margin] = off + 2 * ne; l.u[U_nH] = off; off += xreg;
  for (int k = U_scratch; k <= U_ndir; k++) { l.u[k] = off; off += us[k]; }
  if (off > U) U = off;
  // integration: M - dt qDeriv is formed in place in M (the qDeriv view is
  // not stored)
  l.u[U_qDeriv] = 0;
  sizes[L_U] = U;
  sizes[L_ints] = (16 + 3 * nc + 4 * ne + 1) / 2;
  off = 0;
  for (int k = 0; k < L_COUNT; k++) {
    l.o[k] = off;
    off += sizes[k];
  }
  l.ncon_max = nc;
  l.nefc_max = ne;
  l.nv = nv;
  l.total_doubles = off;
  *bytes = (size_t)off * sizeof(double);
  return l;
}
}  // namespace

// dof counts with a compiled kernel instantiation (mgs_inst.hip, one translation
// unit each).  Main library: Panda + free object = 14, Robotiq 2F-85 + free
// object = 20, Allegro + free object = 28, Shadow + free object = 34.  Wide
// library (MGS_WIDE: 4 rows per lane, G in HBM) for clutter piles of 5 free
// objects: Panda 38, Robotiq 44, Allegro 52, Shadow 58.  Any other dof count
// (up to 64) runs through a model-specialised code object
// (mgs_model_attach_special).  The list is MGS_NV_LIST from the build
// (__graft_entry__.py), here the default.
#ifndef MGS_NV_LIST
#ifdef MGS_WIDE
#define MGS_NV_LIST(X) X(38) X(44) X(52) X(58)
#else
#define MGS_NV_LIST(X) X(14) X(20) X(28) X(34)
#endif
#endif

#define MGS_DECL(NV_) template <> const KernelSet* mgs_kernels_nv<NV_>();
MGS_NV_LIST(MGS_DECL)
#undef MGS_DECL

static const KernelSet* kernels_for(int nv) {
  switch (nv) {
#define MGS_CASE(NV_) case NV_: return mgs_kernels_nv<NV_>();
    MGS_NV_LIST(MGS_CASE)
#undef MGS_CASE
    default: return nullptr;
  }
}

static bool nv_supported(int nv) { return kernels_for(nv) != nullptr; }

// static LDS of the kernels (the diagnostic stage timers of the MGS_PROFILE build)
#ifdef MGS_PROFILE
#define MGS_STATIC_LDS (65 * 8)
#else
#define MGS_STATIC_LDS 0
#endif

static hipError_t set_lds_limit(int nv, int bytes) {
  const KernelSet* k = kernels_for(nv);
  if (!k) return hipSuccess;     // specialised-only dof count: nothing to set here
  hipError_t e = hipFuncSetAttribute(k->rollout_fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute(k->collision_fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

struct mgs_model {
  mgs_model_desc desc;
  int device;
  int32_t* dI;
  double* dD;
  Lay lay;
  size_t lds_bytes;
  // model-specialised code object (mgs_special.hip), if attached
  hipModule_t special_mod;
  hipFunction_t special_collision, special_rollout;
  int resident;     // rollout workgroups the device holds at once (work-queue grid), 0 = not computed yet
};

struct mgs_batch {
  mgs_model* m;
  int cap;
  double *d_qpos, *d_mpos, *d_mquat, *d_ps, *d_pt, *d_objq;
  uint8_t *d_label, *d_free;
  int32_t *d_fail, *d_stats;
  double* d_G;      // MGS_G_GLOBAL: per-candidate constraint rows (HBM)
  size_t g_elems;
  double* d_resume; // resume records (n * (nq + 2 nv + nact + MGS_RESUME_EXTRA)), allocated on first use
  uint32_t* d_queue;                // work-queue headers (MGS_QHDR words: next index, exits, rotation
  int qslot;                        // ring head / tail, ring address), one per launch in a ring of
                                    // MGS_QUEUE_RING (launches in flight on other streams keep their
                                    // own); each launch's last workgroup returns its counters to zero
  uint32_t* d_rings;                // rotation rings (ABI 19), MGS_QRING_F(ring_n) words per header,
  int ring_n;                       // allocated on the first launch with yield_every > 0 and grown
                                    // when a launch's n exceeds ring_n (the kernel indexes a ring by
                                    // its launch's n, which may exceed the batch capacity: ADVICE r4)
  int qslot_drained;                // qslot at the last mgs_queue_spans (spans older than 64 launches are lost)
  uint64_t spins_seen;              // expired ring spins already reported (mgs_queue_stats word 7)
  hipEvent_t e0, e1, e2, e3;
  double last_ms;
};

extern "C" {

int mgs_abi_version(void) { return MGS_ABI_VERSION; }
const char* mgs_last_error(void) { return g_err.c_str(); }

int mgs_model_create(const mgs_model_desc* desc, const int32_t* ibuf, const double* dbuf, int device,
                     mgs_model** out) {
  if (!desc || !ibuf || !dbuf || !out) return fail(MGS_EINVAL, "mgs_model_create: null argument%s");
  if (desc->nv < 1) return fail(MGS_EINVAL, "nv must be >= 1%s");
  if (desc->cone != 1 || desc->integrator != 2)
    return fail(MGS_EINVAL, "only elliptic cones and implicitfast are supported%s");
  if (desc->nu > 32) return fail(MGS_EINVAL, "at most 32 actuators%s");
  if (desc->nmocap > 1) return fail(MGS_EINVAL, "at most one mocap body%s");
  if (desc->nefc_max > 64 * MGS_RPL) return fail(MGS_EINVAL, "nefc_max exceeds this library's rows (mgs_max_rows)%s");
  // more than 64 dofs: the model's specialised code object runs it (two dofs
  // per lane); the library's kernels refuse it at launch (no instantiation)
  if (desc->nv > MGS_MAX_NV) return fail(MGS_EINVAL, "nv must be <= 128 (two dofs per lane)%s");
  if (desc->nbody > 64) return fail(MGS_EINVAL, "at most 64 bodies (lanes over bodies)%s");
  if (desc->njnt > 64) return fail(MGS_EINVAL, "at most 64 joints (lanes over joints)%s");
  if (desc->maxcondim != 1 && desc->maxcondim != 3 && desc->maxcondim != 4 && desc->maxcondim != 6)
    return fail(MGS_EINVAL, "maxcondim must be 1, 3, 4 or 6%s");
  for (int p = 0; p < desc->npair; p++) {
    int cd = ibuf[desc->i_pair_condim + p];
    if (cd != 1 && cd != 3 && cd != 4 && cd != 6) return fail(MGS_EINVAL, "condim must be 1, 3, 4 or 6%s");
    if (cd > desc->maxcondim) return fail(MGS_EINVAL, "a pair's condim exceeds maxcondim%s");
  }
  if (desc->nact < 0 || desc->nact > 4 * 32) return fail(MGS_EINVAL, "bad nact%s");
  for (int u = 0, used = 0; u < desc->nu; u++) {
    const int adr = ibuf[desc->i_actuator_actadr + u];
    int need = 0;
    if (ibuf[desc->i_actuator_gaintype + u] == MGS_GAIN_PID) {
      const double* pp = dbuf + desc->d_actuator_pidprm + 5 * u;
      need = (pp[4] >= 0.0) + (pp[1] != 0.0);
    }
    if (need == 0 ? adr != -1 : adr != used)
      return fail(MGS_EINVAL, "actuator_actadr: a mujoco.pid actuator's act entries are its slew and integral "
                              "states, packed in actuator order%s");
    used += need;
    if (u == desc->nu - 1 && used != desc->nact) return fail(MGS_EINVAL, "nact differs from the actuators' act entries%s");
  }
  if (desc->nu == 0 && desc->nact != 0) return fail(MGS_EINVAL, "nact without actuators%s");
  HIPCHK(hipSetDevice(device));
  mgs_model* m = new mgs_model();
  m->desc = *desc;
  m->device = device;
  size_t ib = sizeof(int32_t) * (desc->isize > 0 ? desc->isize : 1);
  size_t db = sizeof(double) * (desc->dsize > 0 ? desc->dsize : 1);
  if (hipMalloc(&m->dI, ib) != hipSuccess || hipMalloc(&m->dD, db) != hipSuccess) {
    delete m;
    return fail(MGS_ENOMEM, "device allocation failed%s");
  }
  HIPCHK(hipMemcpy(m->dI, ibuf, sizeof(int32_t) * desc->isize, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(m->dD, dbuf, sizeof(double) * desc->dsize, hipMemcpyHostToDevice));
  m->lay = make_layout(*desc, &m->lds_bytes);
  if (m->lds_bytes > 160 * 1024 - MGS_STATIC_LDS) {
    size_t need = m->lds_bytes;
    mgs_model_free(m);
    char buf[64];
    snprintf(buf, sizeof(buf), "%zu", need);
    return fail(MGS_ECAPACITY, "per-candidate working set %s B exceeds 160 KiB LDS; lower ncon_max", buf);
  }
  // the attribute is per kernel function, shared by every model of this nv: set it
  // to the CU's whole LDS so a later, smaller model cannot lower it under an
  // earlier, wider one (occupancy follows each launch's own dynamic size)
  HIPCHK(set_lds_limit(desc->nv, 160 * 1024 - MGS_STATIC_LDS));
  *out = m;
  return MGS_OK;
}

void mgs_model_free(mgs_model* m) {
  if (!m) return;
  if (m->special_mod) hipModuleUnload(m->special_mod);
  hipFree(m->dI);
  hipFree(m->dD);
  delete m;
}

int mgs_batch_open(mgs_model* model, int capacity, mgs_batch** out) {
  if (!model || capacity <= 0 || !out) return fail(MGS_EINVAL, "mgs_batch_open: bad argument%s");
  HIPCHK(hipSetDevice(model->device));
  mgs_batch* b = new mgs_batch();
  memset(b, 0, sizeof(*b));
  b->m = model;
  b->cap = capacity;
  const mgs_model_desc& d = model->desc;
  size_t n = (size_t)capacity;
  bool ok = hipMalloc(&b->d_qpos, sizeof(double) * n * d.nq) == hipSuccess &&
            hipMalloc(&b->d_mpos, sizeof(double) * n * 3) == hipSuccess &&
            hipMalloc(&b->d_mquat, sizeof(double) * n * 4) == hipSuccess &&
            hipMalloc(&b->d_ps, sizeof(double) * n * 3 * MGS_MAX_PHASES) == hipSuccess &&
            hipMalloc(&b->d_pt, sizeof(double) * n * 3 * MGS_MAX_PHASES) == hipSuccess &&
            hipMalloc(&b->d_objq, sizeof(double) * n * 7) == hipSuccess &&
            hipMalloc(&b->d_label, n) == hipSuccess && hipMalloc(&b->d_free, n) == hipSuccess &&
            hipMalloc(&b->d_fail, sizeof(int32_t) * n) == hipSuccess &&
            hipMalloc(&b->d_stats, sizeof(int32_t) * n * MGS_NSTATS) == hipSuccess &&
            hipMalloc(&b->d_queue, MGS_QHDR * sizeof(uint32_t) * MGS_QUEUE_RING) == hipSuccess &&
            hipMemset(b->d_queue, 0, MGS_QHDR * sizeof(uint32_t) * MGS_QUEUE_RING) == hipSuccess &&
            // the counters must be zero before any stream's launch reads them
            // (hipMemset may still be in flight on the null stream otherwise)
            hipDeviceSynchronize() == hipSuccess;
  if (!ok) {
    mgs_batch_close(b);
    return fail(MGS_ENOMEM, "device allocation failed%s");
  }
  HIPCHK(hipEventCreate(&b->e0));
  HIPCHK(hipEventCreate(&b->e1));
  HIPCHK(hipEventCreate(&b->e2));
  HIPCHK(hipEventCreate(&b->e3));
  *out = b;
  return MGS_OK;
}

void mgs_batch_close(mgs_batch* b) {
  if (!b) return;
  hipFree(b->d_qpos); hipFree(b->d_mpos); hipFree(b->d_mquat); hipFree(b->d_ps); hipFree(b->d_pt);
  hipFree(b->d_objq); hipFree(b->d_label); hipFree(b->d_free); hipFree(b->d_fail); hipFree(b->d_stats);
  if (b->d_G) hipFree(b->d_G);
  if (b->d_resume) hipFree(b->d_resume);
  if (b->d_queue) hipFree(b->d_queue);
  if (b->d_rings) hipFree(b->d_rings);
  if (b->e0) hipEventDestroy(b->e0);
  if (b->e1) hipEventDestroy(b->e1);
  if (b->e2) hipEventDestroy(b->e2);
  if (b->e3) hipEventDestroy(b->e3);
  delete b;
}

// the layout a launch over n candidates uses: in the wide library the G rows of
// every candidate live in a batch-owned HBM buffer, grown on demand
static int launch_layout(mgs_batch* b, int n, Lay* lay) {
  *lay = b->m->lay;
  lay->gmem = nullptr;
  if (g_in_hbm(b->m->desc)) {
    size_t need = (size_t)n * hbm_slice_doubles(b->m->desc);
    if (need > b->g_elems) {
      if (b->d_G) HIPCHK(hipFree(b->d_G));
      b->d_G = nullptr;
      b->g_elems = 0;
      if (hipMalloc(&b->d_G, need * sizeof(double)) != hipSuccess)
        return fail(MGS_ENOMEM, "G buffer allocation failed%s");
      b->g_elems = need;
    }
    lay->gmem = b->d_G;
  }
  return MGS_OK;
}

// Rollout launches run as a work queue by default: the grid is the number of
// rollout workgroups the device holds at once (occupancy of the launched
// function at this model's LDS size x CUs) and each workgroup pulls candidate
// indices from a counter (reset by the launch's last workgroup, see rollout_entry).  Mode (mgs_rollout_queue; MGS_QUEUE in the
// environment sets the initial one): 0 one workgroup per candidate, 1 the
// queue on the resident grid, k >= 2 the queue on at most k workgroups (tests).
static int g_queue_mode = -1;

static int queue_mode() {
  if (g_queue_mode < 0) {
    const char* e = getenv("MGS_QUEUE");
    g_queue_mode = e ? atoi(e) : 1;
    if (g_queue_mode < 0) g_queue_mode = 1;
  }
  return g_queue_mode;
}

static int resident_workgroups(mgs_model* m) {
  if (m->resident) return m->resident;
  int per_cu = 0, cus = 0;
  hipError_t e;
  if (m->special_rollout) {
    e = hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, m->special_rollout, 64, m->lds_bytes);
  } else {
    const KernelSet* k = kernels_for(m->desc.nv);
    e = k ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k->rollout_fn, 64, m->lds_bytes) : hipErrorInvalidValue;
  }
  if (e != hipSuccess || per_cu < 1 ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, m->device) != hipSuccess || cus < 1) {
    (void)hipGetLastError();
    m->resident = -1;       // unknown: one workgroup per candidate
    return -1;
  }
  m->resident = per_cu * cus;
  return m->resident;
}

int mgs_model_resident(mgs_model* model) {
  if (!model) return fail(MGS_EINVAL, "mgs_model_resident: null model%s");
  HIPCHK(hipSetDevice(model->device));
  return resident_workgroups(model);
}

static Mdl device_model(const mgs_model* m) {
  Mdl md;
  md.m = m->desc;
  md.I = m->dI;
  md.D = m->dD;
  return md;
}

int mgs_collision_free_device(mgs_batch* b, int n, const double* d_qpos_init, const double* d_mocap_pos,
                              const double* d_mocap_quat, int predicate, uint8_t* d_out_free, void* stream) {
  if (!b || n < 0) return fail(MGS_EINVAL, "mgs_collision_free_device: bad argument%s");
  if (n == 0) return MGS_OK;
  if (!d_qpos_init || !d_mocap_pos || !d_mocap_quat || !d_out_free) return fail(MGS_EINVAL, "null argument%s");
  if (predicate != MGS_PRED_ANY_CONTACT && predicate != MGS_PRED_PARTITION && predicate != MGS_PRED_PARTITION_INCL)
    return fail(MGS_EINVAL, "unknown contact predicate%s");
  HIPCHK(hipSetDevice(b->m->device));
  hipStream_t st = (hipStream_t)stream;
  Mdl md = device_model(b->m);
  Lay lay;
  int lrc = launch_layout(b, n, &lay);
  if (lrc) return lrc;
  HIPCHK(hipEventRecord(b->e2, st));
  CollisionArgs a{md, lay, n, d_qpos_init, d_mocap_pos, d_mocap_quat, predicate, d_out_free};
  if (b->m->special_collision) {
    const int32_t* I = md.I;
    const double* D = md.D;
    void* p[] = {&a.md, &I, &D, &a.lay, &a.n, &a.qpos_init, &a.mocap_pos, &a.mocap_quat, &a.predicate, &a.out};
    HIPCHK(hipModuleLaunchKernel(b->m->special_collision, n, 1, 1, 64, 1, 1, b->m->lds_bytes, st, p, nullptr));
  } else {
    const KernelSet* k = kernels_for(md.m.nv);
    if (!k) return fail(MGS_EINVAL, "no kernel for this nv in this library and no specialised code object attached%s");
    k->collision(dim3(n), b->m->lds_bytes, st, a);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(b->e3, st));
  return MGS_OK;
}

int mgs_collision_free(mgs_batch* b, int n, const double* qpos_init, const double* mocap_pos,
                       const double* mocap_quat, int predicate, uint8_t* out_free) {
  if (!b || n < 0 || n > b->cap) return fail(MGS_EINVAL, "mgs_collision_free: n exceeds batch capacity%s");
  if (n == 0) return MGS_OK;
  if (!qpos_init || !mocap_pos || !mocap_quat || !out_free) return fail(MGS_EINVAL, "null argument%s");
  const mgs_model_desc& d = b->m->desc;
  HIPCHK(hipSetDevice(b->m->device));
  HIPCHK(hipMemcpy(b->d_qpos, qpos_init, sizeof(double) * n * d.nq, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(b->d_mpos, mocap_pos, sizeof(double) * n * 3, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(b->d_mquat, mocap_quat, sizeof(double) * n * 4, hipMemcpyHostToDevice));
  int rc = mgs_collision_free_device(b, n, b->d_qpos, b->d_mpos, b->d_mquat, predicate, b->d_free, nullptr);
  if (rc) return rc;
  HIPCHK(hipMemcpy(out_free, b->d_free, n, hipMemcpyDeviceToHost));
  return MGS_OK;
}

// the rotation rings of every queue header for launches of up to n
// candidates (zeroed; each header's words 4-5 get its ring's address; a
// launch over n indexes MGS_QRING_F(n) words of its ring).  Synchronous: on
// the first rotating launch, and again whenever a launch's n exceeds the n the
// rings were sized for (the old rings are freed once no launch uses them).
static int alloc_rings(mgs_batch* b, int n) {
  if (b->d_rings && b->ring_n >= n) return MGS_OK;
  const size_t per = MGS_QRING_F(n);
  HIPCHK(hipDeviceSynchronize());   // no launch holds a header or a ring while they are replaced
  if (b->d_rings) {
    HIPCHK(hipFree(b->d_rings));
    b->d_rings = nullptr;
    b->ring_n = 0;
  }
  if (hipMalloc(&b->d_rings, sizeof(uint32_t) * per * MGS_QUEUE_RING) != hipSuccess) {
    b->d_rings = nullptr;
    uint64_t z = 0;
    for (int k = 0; k < MGS_QUEUE_RING; k++)      // no header may point at the freed rings
      HIPCHK(hipMemcpy(b->d_queue + MGS_QHDR * k + 4, &z, sizeof(z), hipMemcpyHostToDevice));
    return fail(MGS_ENOMEM, "rotation ring allocation failed%s");
  }
  HIPCHK(hipMemset(b->d_rings, 0, sizeof(uint32_t) * per * MGS_QUEUE_RING));
  for (int k = 0; k < MGS_QUEUE_RING; k++) {
    uint64_t a = (uint64_t)(uintptr_t)(b->d_rings + per * k);
    HIPCHK(hipMemcpy(b->d_queue + MGS_QHDR * k + 4, &a, sizeof(a), hipMemcpyHostToDevice));
  }
  HIPCHK(hipDeviceSynchronize());
  b->ring_n = n;
  return MGS_OK;
}

// the expired-spin counters (word 7 of every queue header), summed
static int expired_spins(mgs_batch* b, uint64_t* out) {
  uint32_t h[MGS_QHDR * MGS_QUEUE_RING];
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(h, b->d_queue, sizeof(h), hipMemcpyDeviceToHost));
  uint64_t e = 0;
  for (int k = 0; k < MGS_QUEUE_RING; k++) e += h[MGS_QHDR * k + 7];
  *out = e;
  return MGS_OK;
}

// after a rotating launch of a synchronous entry: an expired ring spin (a
// candidate possibly lost, a ring slot possibly written after its launch
// ended) fails the call with MGS_EQUEUE and resets every ring and ring
// head / tail, so the next launch starts from a clean protocol state
// before a synchronous rotating launch: expired spins left by earlier launches
// (the device entries', which their callers audit) are acknowledged here and
// the rings they may have left dirty are reset, so the check after this launch
// counts only its own
static int sync_rotation(mgs_batch* b) {
  if (!b->d_rings) return MGS_OK;
  uint64_t e = 0;
  int rc = expired_spins(b, &e);
  if (rc) return rc;
  if (e == b->spins_seen) return MGS_OK;
  b->spins_seen = e;
  HIPCHK(hipMemset(b->d_rings, 0, sizeof(uint32_t) * MGS_QRING_F(b->ring_n) * MGS_QUEUE_RING));
  for (int k = 0; k < MGS_QUEUE_RING; k++)
    HIPCHK(hipMemset(b->d_queue + MGS_QHDR * k + 2, 0, 2 * sizeof(uint32_t)));
  HIPCHK(hipDeviceSynchronize());
  return MGS_OK;
}

static int check_rotation(mgs_batch* b) {
  if (!b->d_rings) return MGS_OK;
  uint64_t e = 0;
  int rc = expired_spins(b, &e);
  if (rc) return rc;
  if (e == b->spins_seen) return MGS_OK;
  b->spins_seen = e;
  HIPCHK(hipMemset(b->d_rings, 0, sizeof(uint32_t) * MGS_QRING_F(b->ring_n) * MGS_QUEUE_RING));
  for (int k = 0; k < MGS_QUEUE_RING; k++)
    HIPCHK(hipMemset(b->d_queue + MGS_QHDR * k + 2, 0, 2 * sizeof(uint32_t)));
  HIPCHK(hipDeviceSynchronize());
  return fail(MGS_EQUEUE, "rotation ring protocol timed out (expired spin): a candidate may have been lost; "
                          "the launch's outputs are invalid%s");
}

static int launch_rollout(mgs_batch* b, const mgs_schedule* sched, int n, const double* d_qpos_init,
                          const double* d_mocap_quat, const double* d_phase_start, const double* d_phase_target,
                          const uint8_t* d_active, uint8_t* d_label, int32_t* d_fail_step, double* d_obj_qpos,
                          int32_t* d_stats, const double* d_vstate, double* d_state_out, void* stream,
                          const int32_t* d_list = nullptr, int32_t* d_count = nullptr, int grid = 0,
                          double* d_resume_out = nullptr, const double* d_resume_in = nullptr,
                          const double* d_mask_mpos = nullptr, int mask_pred = 0, uint8_t* d_mask_out = nullptr,
                          int32_t* d_ovf = nullptr) {
  if (!b || !sched || n < 0) return fail(MGS_EINVAL, "mgs_rollout_device: bad argument%s");
  if (sched->nphase < 1 || sched->nphase > MGS_MAX_PHASES) return fail(MGS_EINVAL, "bad phase count%s");
  if (n == 0) return MGS_OK;
  HIPCHK(hipSetDevice(b->m->device));
  hipStream_t st = (hipStream_t)stream;
  Mdl md = device_model(b->m);
  Lay lay;
  int nwg = d_list ? grid : n;
  uint32_t* q = nullptr;
  int slot = 0;
  if (!d_list && queue_mode() > 0) {
    int r = resident_workgroups(b->m);
    if (queue_mode() > 1 && r > queue_mode()) r = queue_mode();
    if (r > 0 && r < n) {
      nwg = r;
      slot = b->qslot++ % MGS_QUEUE_RING;
      q = b->d_queue + MGS_QHDR * slot;
      if (sched->yield_every > 0 && d_resume_out) {
        int rrc = alloc_rings(b, n);
        if (rrc) return rrc;
      }
    }
  }
  int lrc = launch_layout(b, nwg, &lay);
  if (lrc) return lrc;
  HIPCHK(hipEventRecord(b->e0, st));
  RolloutArgs a{md, lay, *sched, n, d_qpos_init, d_mocap_quat, d_phase_start, d_phase_target, d_active, d_label,
                d_fail_step, d_obj_qpos, d_stats, d_vstate, d_state_out, d_list, d_count, d_resume_out, d_resume_in,
                d_mask_mpos, mask_pred, d_mask_out, q, d_ovf, d_ovf ? d_ovf + MGS_LIST_HEADER : nullptr};
  if (b->m->special_rollout) {
    const int32_t* I = md.I;
    const double* D = md.D;
    void* p[] = {&a.md, &I, &D, &a.lay, &a.sc, &a.n, &a.qpos_init, &a.mocap_quat, &a.phase_start, &a.phase_target,
                 &a.active, &a.label, &a.fail_step, &a.obj_qpos, &a.stats, &a.vstate_init, &a.state_out, &a.list,
                 &a.list_count, &a.resume_out, &a.resume_in, &a.mask_mpos, &a.mask_pred, &a.mask_out, &a.queue,
                 &a.ovf_count, &a.ovf_list};
    HIPCHK(hipModuleLaunchKernel(b->m->special_rollout, nwg, 1, 1, 64, 1, 1, b->m->lds_bytes, st, p, nullptr));
  } else {
    const KernelSet* k = kernels_for(md.m.nv);
    if (!k) return fail(MGS_EINVAL, "no kernel for this nv in this library and no specialised code object attached%s");
    if (layout_maxdim(md.m) > MGS_MAXDIM)
      return fail(MGS_EINVAL, "condim-6 contacts run through the model's specialised code object only "
                              "(mgs.core.special); none is attached%s");
#ifndef MGS_G_GLOBAL
    if (md.m.g_rows_hbm)
      return fail(MGS_EINVAL, "g_rows_hbm: G rows in HBM need the model's specialised code object%s");
#endif
    k->rollout(dim3(nwg), b->m->lds_bytes, st, a);
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipEventRecord(b->e1, st));
  return MGS_OK;
}

int mgs_rollout_device(mgs_batch* b, const mgs_schedule* sched, int n, const double* d_qpos_init,
                       const double* d_mocap_quat, const double* d_phase_start, const double* d_phase_target,
                       const uint8_t* d_active, uint8_t* d_label, int32_t* d_fail_step, double* d_obj_qpos,
                       int32_t* d_stats, void* stream) {
  return launch_rollout(b, sched, n, d_qpos_init, d_mocap_quat, d_phase_start, d_phase_target, d_active, d_label,
                        d_fail_step, d_obj_qpos, d_stats, nullptr, nullptr, stream);
}

int mgs_queue_stats(mgs_batch* b, uint64_t* out) {
  if (!b || !out) return fail(MGS_EINVAL, "mgs_queue_stats: null argument%s");
  HIPCHK(hipSetDevice(b->m->device));
  uint32_t h[MGS_QHDR * MGS_QUEUE_RING];
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(h, b->d_queue, sizeof(h), hipMemcpyDeviceToHost));
  out[0] = out[1] = 0;
  for (int k = 0; k < MGS_QUEUE_RING; k++) {
    out[0] += h[MGS_QHDR * k + 6];
    out[1] += h[MGS_QHDR * k + 7];
  }
  return MGS_OK;
}

int mgs_queue_spans(mgs_batch* b, double* out_ms, int cap, int* count, int* overwritten) {
  if (!b || !out_ms || !count || cap < 0) return fail(MGS_EINVAL, "mgs_queue_spans: bad argument%s");
  // launches since the previous call beyond the ring's 64 headers: their spans
  // were overwritten before they could be read
  const int since = b->qslot - b->qslot_drained;
  if (overwritten) *overwritten = since > MGS_QUEUE_RING ? since - MGS_QUEUE_RING : 0;
  b->qslot_drained = b->qslot;
  HIPCHK(hipSetDevice(b->m->device));
  uint32_t h[MGS_QHDR * MGS_QUEUE_RING];
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(h, b->d_queue, sizeof(h), hipMemcpyDeviceToHost));
  int k = 0;
  for (int i = 0; i < MGS_QUEUE_RING; i++) {
    // oldest first: the slot after the last one handed out
    const int s = (b->qslot + i) % MGS_QUEUE_RING;
    uint64_t t0, t1;
    memcpy(&t0, h + MGS_QHDR * s + 8, sizeof(t0));
    memcpy(&t1, h + MGS_QHDR * s + 10, sizeof(t1));
    if (t0 == 0 || t1 <= t0) continue;
    if (k < cap) out_ms[k++] = (double)(t1 - t0) * 1e-5;   // 100 MHz ticks
    HIPCHK(hipMemset(b->d_queue + MGS_QHDR * s + 8, 0, 4 * sizeof(uint32_t)));
  }
  HIPCHK(hipDeviceSynchronize());
  *count = k;
  return MGS_OK;
}

int mgs_overflow_list_device(int n, const int32_t* d_stats, int flag_mask, int32_t* d_count, int32_t* d_list,
                             void* stream) {
  if (n < 0 || !d_stats || !d_count || !d_list) return fail(MGS_EINVAL, "mgs_overflow_list_device: bad argument%s");
  hipStream_t st = (hipStream_t)stream;
  HIPCHK(hipMemsetAsync(d_count, 0, 2 * sizeof(int32_t), st));   // count and exits of the list header
  if (n == 0) return MGS_OK;
  hipLaunchKernelGGL(mgs_overflow_list_kernel, dim3((n + 255) / 256), dim3(256), 0, st, d_stats, n, flag_mask, d_count,
                     d_list);
  HIPCHK(hipGetLastError());
  return MGS_OK;
}

int mgs_rollout_list_device(mgs_batch* b, const mgs_schedule* sched, int n, int32_t* d_count,
                            const int32_t* d_list, int grid, const double* d_qpos_init, const double* d_mocap_quat,
                            const double* d_phase_start, const double* d_phase_target, const double* d_resume_in,
                            uint8_t* d_label, int32_t* d_fail_step, double* d_obj_qpos, int32_t* d_stats,
                            void* stream) {
  if (!b || !d_count || !d_list || grid < 1 || grid > b->cap)
    return fail(MGS_EINVAL, "mgs_rollout_list_device: bad argument (1 <= grid <= batch capacity)%s");
  return launch_rollout(b, sched, n, d_qpos_init, d_mocap_quat, d_phase_start, d_phase_target, nullptr, d_label,
                        d_fail_step, d_obj_qpos, d_stats, nullptr, nullptr, stream, d_list, d_count, grid, nullptr,
                        d_resume_in);
}

int mgs_rollout_resumable_device(mgs_batch* b, const mgs_schedule* sched, int n, const double* d_qpos_init,
                                 const double* d_mocap_quat, const double* d_phase_start,
                                 const double* d_phase_target, const uint8_t* d_active, uint8_t* d_label,
                                 int32_t* d_fail_step, double* d_obj_qpos, int32_t* d_stats, double* d_resume_out,
                                 int32_t* d_ovf, void* stream) {
  if (!d_resume_out) return fail(MGS_EINVAL, "mgs_rollout_resumable_device: null resume buffer%s");
  return launch_rollout(b, sched, n, d_qpos_init, d_mocap_quat, d_phase_start, d_phase_target, d_active, d_label,
                        d_fail_step, d_obj_qpos, d_stats, nullptr, nullptr, stream, nullptr, nullptr, 0,
                        d_resume_out, nullptr, nullptr, 0, nullptr, d_ovf);
}

int mgs_mask_rollout_device(mgs_batch* b, const mgs_schedule* sched, int n, const double* d_qpos_init,
                            const double* d_mocap_pos, const double* d_mocap_quat, const double* d_phase_start,
                            const double* d_phase_target, int predicate, uint8_t* d_free_out, uint8_t* d_label,
                            int32_t* d_fail_step, double* d_obj_qpos, int32_t* d_stats, double* d_resume_out,
                            int32_t* d_ovf, void* stream) {
  if (!d_mocap_pos || !d_free_out) return fail(MGS_EINVAL, "mgs_mask_rollout_device: mocap_pos and free_out are required%s");
  if (predicate < MGS_PRED_ANY_CONTACT || predicate > MGS_PRED_PARTITION_INCL)
    return fail(MGS_EINVAL, "mgs_mask_rollout_device: bad predicate%s");
  return launch_rollout(b, sched, n, d_qpos_init, d_mocap_quat, d_phase_start, d_phase_target, nullptr, d_label,
                        d_fail_step, d_obj_qpos, d_stats, nullptr, nullptr, stream, nullptr, nullptr, 0,
                        d_resume_out, nullptr, d_mocap_pos, predicate, d_free_out, d_ovf);
}

int mgs_simulate_device(mgs_batch* b, const mgs_schedule* sched, int n, const double* d_qpos_init,
                        const double* d_vstate_init, const double* d_mocap_quat, const double* d_phase_start,
                        const double* d_phase_target, double* d_state_out, int32_t* d_stats, void* stream) {
  if (!b || !sched || !d_state_out || n < 0 || n > b->cap) return fail(MGS_EINVAL, "mgs_simulate_device: bad argument%s");
  mgs_schedule s = *sched;   // no contact checks: a free simulation never stops early
  for (int p = 0; p < MGS_MAX_PHASES; p++) { s.check_every[p] = 0; s.check_at_end[p] = 0; }
  return launch_rollout(b, &s, n, d_qpos_init, d_mocap_quat, d_phase_start, d_phase_target, nullptr, b->d_label,
                        b->d_fail, b->d_objq, d_stats ? d_stats : b->d_stats, d_vstate_init, d_state_out, stream);
}

int mgs_simulate(mgs_batch* b, const mgs_schedule* sched, int n, const double* qpos_init,
                 const double* vstate_init, const double* mocap_quat, const double* phase_start,
                 const double* phase_target, double* state_out, int32_t* stats) {
  if (!b || !sched || n < 0 || n > b->cap) return fail(MGS_EINVAL, "mgs_simulate: bad argument%s");
  if (n == 0) return MGS_OK;
  if (!qpos_init || !mocap_quat || !phase_start || !phase_target || !state_out)
    return fail(MGS_EINVAL, "mgs_simulate: null argument%s");
  const mgs_model_desc& d = b->m->desc;
  int np = sched->nphase;
  HIPCHK(hipSetDevice(b->m->device));
  double *dv = nullptr, *ds = nullptr;
  size_t nst = (size_t)n * (d.nq + 2 * d.nv + d.nact);
  if (hipMalloc(&ds, nst * sizeof(double)) != hipSuccess) return fail(MGS_ENOMEM, "state buffer allocation failed%s");
  if (vstate_init && hipMalloc(&dv, (size_t)n * (2 * d.nv + d.nact) * sizeof(double)) != hipSuccess) {
    hipFree(ds);
    return fail(MGS_ENOMEM, "state buffer allocation failed%s");
  }
  int rc = MGS_OK;
  if (hipMemcpy(b->d_qpos, qpos_init, sizeof(double) * n * d.nq, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(b->d_mquat, mocap_quat, sizeof(double) * n * 4, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(b->d_ps, phase_start, sizeof(double) * n * 3 * np, hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(b->d_pt, phase_target, sizeof(double) * n * 3 * np, hipMemcpyHostToDevice) != hipSuccess ||
      (dv && hipMemcpy(dv, vstate_init, (size_t)n * (2 * d.nv + d.nact) * sizeof(double), hipMemcpyHostToDevice) != hipSuccess))
    rc = fail(MGS_EHIP, "host to device copy failed%s");
  if (!rc) rc = mgs_simulate_device(b, sched, n, b->d_qpos, dv, b->d_mquat, b->d_ps, b->d_pt, ds, nullptr, nullptr);
  if (!rc && hipMemcpy(state_out, ds, nst * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
    rc = fail(MGS_EHIP, "device to host copy failed%s");
  if (!rc && stats &&
      hipMemcpy(stats, b->d_stats, sizeof(int32_t) * n * MGS_NSTATS, hipMemcpyDeviceToHost) != hipSuccess)
    rc = fail(MGS_EHIP, "device to host copy failed%s");
  hipFree(ds);
  if (dv) hipFree(dv);
  return rc;
}

double mgs_last_collision_ms(mgs_batch* b) {
  if (!b) return -1.0;
  float ms = 0.f;
  if (hipEventSynchronize(b->e3) != hipSuccess) return -1.0;
  if (hipEventElapsedTime(&ms, b->e2, b->e3) != hipSuccess) return -1.0;
  return ms;
}

double mgs_last_kernel_ms(mgs_batch* b) {
  if (!b) return -1.0;
  float ms = 0.f;
  if (hipEventSynchronize(b->e1) != hipSuccess) return -1.0;
  if (hipEventElapsedTime(&ms, b->e0, b->e1) != hipSuccess) return -1.0;
  b->last_ms = ms;
  return ms;
}

static int rollout_host(mgs_batch* b, const mgs_schedule* sched, int n, const double* qpos_init,
                        const double* mocap_quat, const double* phase_start, const double* phase_target,
                        const double* resume_in, mgs_rollout_out* out) {
  if (!b || !sched || !out || n < 0 || n > b->cap) return fail(MGS_EINVAL, "mgs_rollout: bad argument%s");
  if (n == 0) return MGS_OK;
  if (!qpos_init || !mocap_quat || !phase_start || !phase_target || !out->label)
    return fail(MGS_EINVAL, "mgs_rollout: null argument%s");
  const mgs_model_desc& d = b->m->desc;
  int np = sched->nphase;
  HIPCHK(hipSetDevice(b->m->device));
  const size_t rs = (size_t)d.nq + 2 * (size_t)d.nv + (size_t)d.nact + MGS_RESUME_EXTRA;
  // resume records: one buffer serves as the output of a resumable run or the
  // input of a resumed one
  if ((out->resume || resume_in) && !b->d_resume &&
      hipMalloc(&b->d_resume, sizeof(double) * rs * (size_t)b->cap) != hipSuccess)
    return fail(MGS_ENOMEM, "resume buffer allocation failed%s");
  HIPCHK(hipMemcpy(b->d_qpos, qpos_init, sizeof(double) * n * d.nq, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(b->d_mquat, mocap_quat, sizeof(double) * n * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(b->d_ps, phase_start, sizeof(double) * n * 3 * np, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(b->d_pt, phase_target, sizeof(double) * n * 3 * np, hipMemcpyHostToDevice));
  if (resume_in) HIPCHK(hipMemcpy(b->d_resume, resume_in, sizeof(double) * rs * n, hipMemcpyHostToDevice));
  int rc;
  if (sched->yield_every > 0 && (rc = sync_rotation(b))) return rc;
  rc = launch_rollout(b, sched, n, b->d_qpos, b->d_mquat, b->d_ps, b->d_pt, nullptr, b->d_label, b->d_fail,
                          b->d_objq, b->d_stats, nullptr, nullptr, nullptr, nullptr, nullptr, 0,
                          out->resume ? b->d_resume : nullptr, resume_in ? b->d_resume : nullptr);
  if (rc) return rc;
  if (sched->yield_every > 0 && (rc = check_rotation(b))) return rc;
  HIPCHK(hipMemcpy(out->label, b->d_label, n, hipMemcpyDeviceToHost));
  if (out->fail_step) HIPCHK(hipMemcpy(out->fail_step, b->d_fail, sizeof(int32_t) * n, hipMemcpyDeviceToHost));
  if (out->obj_qpos) HIPCHK(hipMemcpy(out->obj_qpos, b->d_objq, sizeof(double) * n * 7, hipMemcpyDeviceToHost));
  if (out->stats) HIPCHK(hipMemcpy(out->stats, b->d_stats, sizeof(int32_t) * n * MGS_NSTATS, hipMemcpyDeviceToHost));
  if (out->resume) HIPCHK(hipMemcpy(out->resume, b->d_resume, sizeof(double) * rs * n, hipMemcpyDeviceToHost));
  return MGS_OK;
}

int mgs_rollout(mgs_batch* b, const mgs_schedule* sched, int n, const double* qpos_init,
                const double* mocap_quat, const double* phase_start, const double* phase_target,
                mgs_rollout_out* out) {
  return rollout_host(b, sched, n, qpos_init, mocap_quat, phase_start, phase_target, nullptr, out);
}

int mgs_rollout_resume(mgs_batch* b, const mgs_schedule* sched, int n, const double* qpos_init,
                       const double* mocap_quat, const double* phase_start, const double* phase_target,
                       const double* resume, mgs_rollout_out* out) {
  if (!resume) return fail(MGS_EINVAL, "mgs_rollout_resume: null resume records%s");
  return rollout_host(b, sched, n, qpos_init, mocap_quat, phase_start, phase_target, resume, out);
}

// test hook: device arithmetic on n inputs (out: n*4 = sqrt|x|, x/y, sin, cos)
int mgs_arith_probe(const double* x, const double* y, int n, double* out) {
  double *dx, *dy, *dout;
  HIPCHK(hipMalloc(&dx, sizeof(double) * n));
  HIPCHK(hipMalloc(&dy, sizeof(double) * n));
  HIPCHK(hipMalloc(&dout, sizeof(double) * n * 4));
  HIPCHK(hipMemcpy(dx, x, sizeof(double) * n, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dy, y, sizeof(double) * n, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(mgs_arith_probe_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, dx, dy, n, dout);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(out, dout, sizeof(double) * n * 4, hipMemcpyDeviceToHost));
  hipFree(dx); hipFree(dy); hipFree(dout);
  return MGS_OK;
}

// test hook: pairwise-tree wave reduction, nb blocks of 64 lanes
int mgs_tree_probe(const double* a, const double* c, int n, int nb, double* out) {
  double *da, *dc, *dout;
  HIPCHK(hipMalloc(&da, sizeof(double) * nb * 64));
  HIPCHK(hipMalloc(&dc, sizeof(double) * nb * 64));
  HIPCHK(hipMalloc(&dout, sizeof(double) * nb));
  HIPCHK(hipMemcpy(da, a, sizeof(double) * nb * 64, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dc, c, sizeof(double) * nb * 64, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(mgs_tree_probe_kernel, dim3(nb), dim3(64), 0, 0, da, dc, n, dout);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(out, dout, sizeof(double) * nb, hipMemcpyDeviceToHost));
  hipFree(da); hipFree(dc); hipFree(dout);
  return MGS_OK;
}

// diagnostic build only: read and clear the stage timers (s_memtime ticks) of
// every dof count's kernels of this library
int mgs_prof_read(unsigned long long* out) {
#ifdef MGS_PROFILE
  for (int k = 0; k < 64; k++) out[k] = 0;
#define MGS_CASE(NV_) if (mgs_kernels_nv<NV_>()->prof_read(out)) return fail(MGS_EHIP, "stage timer read failed%s");
  MGS_NV_LIST(MGS_CASE)
#undef MGS_CASE
  return MGS_OK;
#else
  (void)out;
  return MGS_EINVAL;
#endif
}

// the same for a model's specialised code object (built with -DMGS_PROFILE)
int mgs_model_prof_read(mgs_model* m, unsigned long long* out) {
  if (!m || !m->special_mod || !out) return fail(MGS_EINVAL, "mgs_model_prof_read: no specialised code object%s");
  hipDeviceptr_t p;
  size_t sz = 0;
  unsigned long long z[64] = {0};
  if (hipModuleGetGlobal(&p, &sz, m->special_mod, "g_prof") != hipSuccess || sz != sizeof(z))
    return fail(MGS_EINVAL, "the specialised code object has no stage timers (not an MGS_PROFILE build)%s");
  HIPCHK(hipMemcpyDtoH(out, p, sizeof(z)));
  HIPCHK(hipMemcpyHtoD(p, z, sizeof(z)));
  return MGS_OK;
}

int mgs_lds_bytes(mgs_model* m) { return m ? (int)m->lds_bytes : -1; }

int mgs_antipodal_contacts(int device, const double* tri, int ntri, int n, const double* origin,
                           const double* dir, const double* u_choice, double eps, double* out_second,
                           int32_t* out_nvalid, double* kernel_ms) {
  if (n < 0 || ntri < 0) return fail(MGS_EINVAL, "mgs_antipodal_contacts: negative size%s");
  if (n == 0) return MGS_OK;
  if (!tri || !origin || !dir || !u_choice || !out_second || !out_nvalid)
    return fail(MGS_EINVAL, "mgs_antipodal_contacts: null argument%s");
  HIPCHK(hipSetDevice(device));
  double *dT = nullptr, *dO = nullptr, *dD = nullptr, *dU = nullptr, *dS = nullptr;
  int32_t* dN = nullptr;
  size_t nt = (size_t)(ntri > 0 ? ntri : 1) * 9;
  bool ok = hipMalloc(&dT, nt * sizeof(double)) == hipSuccess && hipMalloc(&dO, 3 * n * sizeof(double)) == hipSuccess &&
            hipMalloc(&dD, 3 * n * sizeof(double)) == hipSuccess && hipMalloc(&dU, n * sizeof(double)) == hipSuccess &&
            hipMalloc(&dS, 3 * n * sizeof(double)) == hipSuccess && hipMalloc(&dN, n * sizeof(int32_t)) == hipSuccess;
  int rc = MGS_OK;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (!ok) {
    rc = fail(MGS_ENOMEM, "device allocation failed%s");
  } else {
    if (ntri > 0) hipMemcpy(dT, tri, (size_t)ntri * 9 * sizeof(double), hipMemcpyHostToDevice);
    hipMemcpy(dO, origin, 3 * n * sizeof(double), hipMemcpyHostToDevice);
    hipMemcpy(dD, dir, 3 * n * sizeof(double), hipMemcpyHostToDevice);
    hipMemcpy(dU, u_choice, n * sizeof(double), hipMemcpyHostToDevice);
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, nullptr);
    hipLaunchKernelGGL(mgs_antipodal_kernel, dim3((n + 255) / 256), dim3(256), 0, nullptr, dT, ntri, n, dO, dD, dU,
                       eps, dS, dN);
    hipEventRecord(e1, nullptr);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    if (e != hipSuccess) {
      rc = fail(MGS_EHIP, "HIP error: %s", hipGetErrorString(e));
    } else {
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      if (kernel_ms) *kernel_ms = ms;
      hipMemcpy(out_second, dS, 3 * n * sizeof(double), hipMemcpyDeviceToHost);
      hipMemcpy(out_nvalid, dN, n * sizeof(int32_t), hipMemcpyDeviceToHost);
    }
  }
  if (e0) hipEventDestroy(e0);
  if (e1) hipEventDestroy(e1);
  hipFree(dT); hipFree(dO); hipFree(dD); hipFree(dU); hipFree(dS); hipFree(dN);
  return rc;
}

// ---------------------------------------------------------------------------
// contact-based dexterous-hand sampler (csrc/mgs_contact.hip)
}  // extern "C"
namespace {
struct DevBufs {
  std::vector<void*> p;
  bool ok = true;
  template <class T>
  T* get(size_t n) {
    void* q = nullptr;
    if (hipMalloc(&q, (n > 0 ? n : 1) * sizeof(T)) != hipSuccess) { ok = false; return nullptr; }
    p.push_back(q);
    return (T*)q;
  }
  ~DevBufs() { for (void* q : p) hipFree(q); }
};
struct EvTimer {
  hipEvent_t e0 = nullptr, e1 = nullptr;
  EvTimer() { hipEventCreate(&e0); hipEventCreate(&e1); hipEventRecord(e0, nullptr); }
  int finish(double* ms) {
    hipEventRecord(e1, nullptr);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    if (e != hipSuccess) return fail(MGS_EHIP, "HIP error: %s", hipGetErrorString(e));
    float f = 0.f;
    hipEventElapsedTime(&f, e0, e1);
    if (ms) *ms = f;
    return MGS_OK;
  }
  ~EvTimer() { hipEventDestroy(e0); hipEventDestroy(e1); }
};
}  // namespace
extern "C" {

int mgs_kin_desc_size(void) { return (int)sizeof(mgs_kin_desc); }

int mgs_contact_fps(int device, const double* points, int n, int k, int32_t* out_idx, double* kernel_ms) {
  if (n < 0 || k < 0 || (k > 0 && n == 0) || k > n) return fail(MGS_EINVAL, "mgs_contact_fps: need 0 <= k <= n%s");
  if (k == 0) return MGS_OK;
  if (!points || !out_idx) return fail(MGS_EINVAL, "mgs_contact_fps: null argument%s");
  HIPCHK(hipSetDevice(device));
  DevBufs b;
  double* dX = b.get<double>(3 * (size_t)n);
  double* dD = b.get<double>((size_t)n);
  int32_t* dO = b.get<int32_t>((size_t)k);
  if (!b.ok) return fail(MGS_ENOMEM, "device allocation failed%s");
  HIPCHK(hipMemcpy(dX, points, 3 * (size_t)n * sizeof(double), hipMemcpyHostToDevice));
  EvTimer t;
  hipLaunchKernelGGL(mgs_fps_kernel, dim3(1), dim3(MGS_FPS_THREADS), 0, nullptr, dX, n, k, dD, dO);
  int rc = t.finish(kernel_ms);
  if (rc == MGS_OK) HIPCHK(hipMemcpy(out_idx, dO, (size_t)k * sizeof(int32_t), hipMemcpyDeviceToHost));
  return rc;
}

int mgs_contact_seeds(int device, const double* seeds, int k, double radius, uint64_t rng_seed, int ntip,
                      int32_t* out_nn, int32_t* out_sel, double* kernel_ms) {
  if (k < 0 || ntip < 1 || ntip > MGS_KIN_MAXTIP) return fail(MGS_EINVAL, "mgs_contact_seeds: bad size%s");
  if (k == 0) return MGS_OK;
  if (!seeds || !out_nn || !out_sel) return fail(MGS_EINVAL, "mgs_contact_seeds: null argument%s");
  HIPCHK(hipSetDevice(device));
  DevBufs b;
  double* dS = b.get<double>(3 * (size_t)k);
  int32_t* dN = b.get<int32_t>((size_t)k);
  int32_t* dL = b.get<int32_t>((size_t)k * ntip);
  if (!b.ok) return fail(MGS_ENOMEM, "device allocation failed%s");
  HIPCHK(hipMemcpy(dS, seeds, 3 * (size_t)k * sizeof(double), hipMemcpyHostToDevice));
  EvTimer t;
  hipLaunchKernelGGL(mgs_seeds_kernel, dim3((k + MGS_SEED_TILE - 1) / MGS_SEED_TILE), dim3(MGS_SEED_TILE), 0,
                     nullptr, dS, k, radius, rng_seed, ntip, dN, dL);
  int rc = t.finish(kernel_ms);
  if (rc == MGS_OK) {
    HIPCHK(hipMemcpy(out_nn, dN, (size_t)k * sizeof(int32_t), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(out_sel, dL, (size_t)k * ntip * sizeof(int32_t), hipMemcpyDeviceToHost));
  }
  return rc;
}

int mgs_contact_optimize(int device, const mgs_kin_desc* kin, int n, const double* rot_init, const double* pos_init,
                         const double* targets, const double* normals, double* out_rot, double* out_pos,
                         double* out_joints, double* out_loss, double* kernel_ms) {
  if (!kin || n < 0) return fail(MGS_EINVAL, "mgs_contact_optimize: bad argument%s");
  if (kin->ndof < 1 || kin->ndof > MGS_KIN_MAXDOF || kin->ntip < 1 || kin->ntip > MGS_KIN_MAXTIP ||
      kin->nperm < 1 || kin->nperm > MGS_KIN_MAXPERM || kin->iters < 0)
    return fail(MGS_EINVAL, "mgs_contact_optimize: kinematic model out of range%s");
  for (int a = 0; a < kin->ntip; a++) {
    if (kin->chain_len[a] < 1 || kin->chain_len[a] > MGS_KIN_MAXCHAIN)
      return fail(MGS_EINVAL, "mgs_contact_optimize: chain length out of range%s");
    for (int s = 0; s < kin->chain_len[a]; s++)
      if (kin->chain[a][s] < 0 || kin->chain[a][s] >= kin->ndof)
        return fail(MGS_EINVAL, "mgs_contact_optimize: chain dof out of range%s");
  }
  for (int q = 0; q < kin->nperm; q++)
    for (int a = 0; a < kin->ntip; a++)
      if (kin->perm[q][a] < 0 || kin->perm[q][a] >= kin->ntip)
        return fail(MGS_EINVAL, "mgs_contact_optimize: permutation entry out of range%s");
  if (n == 0) return MGS_OK;
  if (!rot_init || !pos_init || !targets || !normals || !out_rot || !out_pos || !out_joints)
    return fail(MGS_EINVAL, "mgs_contact_optimize: null argument%s");
  HIPCHK(hipSetDevice(device));
  const size_t nt = (size_t)kin->ntip, nd = (size_t)kin->ndof, nn = (size_t)n;
  DevBufs b;
  mgs_kin_desc* dK = b.get<mgs_kin_desc>(1);
  double* dR = b.get<double>(9 * nn);
  double* dP = b.get<double>(3 * nn);
  double* dT = b.get<double>(3 * nt * nn);
  double* dN = b.get<double>(3 * nt * nn);
  double* oR = b.get<double>(9 * nn);
  double* oP = b.get<double>(3 * nn);
  double* oJ = b.get<double>(nd * nn);
  double* oL = b.get<double>(nn);
  if (!b.ok) return fail(MGS_ENOMEM, "device allocation failed%s");
  HIPCHK(hipMemcpy(dK, kin, sizeof(mgs_kin_desc), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dR, rot_init, 9 * nn * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dP, pos_init, 3 * nn * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dT, targets, 3 * nt * nn * sizeof(double), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dN, normals, 3 * nt * nn * sizeof(double), hipMemcpyHostToDevice));
  EvTimer t;
  hipLaunchKernelGGL(mgs_contact_opt_kernel, dim3((n + 63) / 64), dim3(64), 0, nullptr, dK, n, dR, dP, dT, dN,
                     oR, oP, oJ, oL);
  int rc = t.finish(kernel_ms);
  if (rc == MGS_OK) {
    HIPCHK(hipMemcpy(out_rot, oR, 9 * nn * sizeof(double), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(out_pos, oP, 3 * nn * sizeof(double), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(out_joints, oJ, nd * nn * sizeof(double), hipMemcpyDeviceToHost));
    if (out_loss) HIPCHK(hipMemcpy(out_loss, oL, nn * sizeof(double), hipMemcpyDeviceToHost));
  }
  return rc;
}

int mgs_max_rows(void) { return 64 * MGS_RPL; }

int mgs_supports_nv(int nv) { return nv_supported(nv) ? 1 : 0; }

int mgs_rows_per_lane(void) { return MGS_RPL; }

int mgs_model_lds_bytes(const mgs_model_desc* desc, int64_t* out_bytes) {
  if (!desc || !out_bytes) return fail(MGS_EINVAL, "mgs_model_lds_bytes: null argument%s");
  size_t b = 0;
  make_layout(*desc, &b);
  *out_bytes = (int64_t)b;
  return MGS_OK;
}

int mgs_model_layout(const mgs_model_desc* desc, int32_t* out, int cap, int32_t* nwords) {
  if (!desc || !out || !nwords) return fail(MGS_EINVAL, "mgs_model_layout: null argument%s");
  size_t b = 0;
  Lay l = make_layout(*desc, &b);
  int32_t w[L_COUNT + U_COUNT + 4];
  int k = 0;
  for (int i = 0; i < L_COUNT; i++) w[k++] = l.o[i];
  for (int i = 0; i < U_COUNT; i++) w[k++] = l.u[i];
  w[k++] = l.ncon_max; w[k++] = l.nefc_max; w[k++] = l.nv; w[k++] = l.total_doubles;
  if (cap < k) return fail(MGS_EINVAL, "mgs_model_layout: output too small%s");
  for (int i = 0; i < k; i++) out[i] = w[i];
  *nwords = k;
  return MGS_OK;
}

int mgs_model_special(const mgs_model* m) { return m && m->special_rollout ? 1 : 0; }

int mgs_model_attach_special(mgs_model* m, const char* path) {
  if (!m || !path) return fail(MGS_EINVAL, "mgs_model_attach_special: null argument%s");
  HIPCHK(hipSetDevice(m->device));
  hipModule_t mod = nullptr;
  if (hipModuleLoad(&mod, path) != hipSuccess) return fail(MGS_EINVAL, "cannot load code object %s", path);
  // the object's baked ABI version, description and layout must be this model's
  auto check = [&]() -> int {
    hipDeviceptr_t p;
    size_t sz = 0;
    int abi = 0, rpl = 0;
    mgs_model_desc dsc;
    int32_t w[L_COUNT + U_COUNT + 4];
    if (hipModuleGetGlobal(&p, &sz, mod, "mgs_special_abi") != hipSuccess || sz != sizeof(int) ||
        hipMemcpyDtoH(&abi, p, sizeof(int)) != hipSuccess || abi != MGS_ABI_VERSION)
      return fail(MGS_EINVAL, "code object %s is of another ABI version", path);
    if (hipModuleGetGlobal(&p, &sz, mod, "mgs_special_rows_per_lane") != hipSuccess || sz != sizeof(int) ||
        hipMemcpyDtoH(&rpl, p, sizeof(int)) != hipSuccess || rpl != MGS_RPL)
      return fail(MGS_EINVAL, "code object %s is of the other library flavour (rows per lane)", path);
    int mxd = 0;
    if (hipModuleGetGlobal(&p, &sz, mod, "mgs_special_maxdim") != hipSuccess || sz != sizeof(int) ||
        hipMemcpyDtoH(&mxd, p, sizeof(int)) != hipSuccess || mxd != layout_maxdim(m->desc))
      return fail(MGS_EINVAL, "code object %s was built for another contact dimension (MGS_MAXDIM)", path);
    int mxnv = 0;
    if (hipModuleGetGlobal(&p, &sz, mod, "mgs_special_max_nv") != hipSuccess || sz != sizeof(int) ||
        hipMemcpyDtoH(&mxnv, p, sizeof(int)) != hipSuccess || mxnv < m->desc.nv)
      return fail(MGS_EINVAL, "code object %s holds fewer dofs per lane than the model needs (MGS_DPL)", path);
    if (hipModuleGetGlobal(&p, &sz, mod, "mgs_special_desc") != hipSuccess || sz != sizeof(dsc) ||
        hipMemcpyDtoH(&dsc, p, sizeof(dsc)) != hipSuccess || memcmp(&dsc, &m->desc, sizeof(dsc)) != 0)
      return fail(MGS_EINVAL, "code object %s was specialised for another model description", path);
    const Lay& l = m->lay;
    int k = 0;
    int32_t mine[L_COUNT + U_COUNT + 4];
    for (int i = 0; i < L_COUNT; i++) mine[k++] = l.o[i];
    for (int i = 0; i < U_COUNT; i++) mine[k++] = l.u[i];
    mine[k++] = l.ncon_max; mine[k++] = l.nefc_max; mine[k++] = l.nv; mine[k++] = l.total_doubles;
    if (hipModuleGetGlobal(&p, &sz, mod, "mgs_special_words") != hipSuccess || sz != sizeof(w) ||
        hipMemcpyDtoH(w, p, sizeof(w)) != hipSuccess || memcmp(w, mine, sizeof(w)) != 0)
      return fail(MGS_EINVAL, "code object %s was specialised for another LDS layout", path);
    return MGS_OK;
  };
  int rc = check();
  hipFunction_t fc = nullptr, fr = nullptr;
  // main-role objects name their kernels mgs_special_*, escalation-role ones
  // mgs_special_*_esc (mgs_special.hip).  The lookup of the naming an object
  // does not use fails by design: its error is cleared here, or the next
  // launch's hipGetLastError would report it
  if (rc == MGS_OK) {
    bool found = (hipModuleGetFunction(&fc, mod, "mgs_special_collision") == hipSuccess &&
                  hipModuleGetFunction(&fr, mod, "mgs_special_rollout") == hipSuccess) ||
                 (hipModuleGetFunction(&fc, mod, "mgs_special_collision_esc") == hipSuccess &&
                  hipModuleGetFunction(&fr, mod, "mgs_special_rollout_esc") == hipSuccess);
    (void)hipGetLastError();
    if (!found) rc = fail(MGS_EINVAL, "code object %s lacks the specialised kernels", path);
  }
  if (rc != MGS_OK) {
    hipModuleUnload(mod);
    return rc;
  }
  if (m->special_mod) hipModuleUnload(m->special_mod);
  m->special_mod = mod;
  m->special_collision = fc;
  m->special_rollout = fr;
  m->resident = 0;          // occupancy of the new rollout function, computed at its first launch
  return MGS_OK;
}

int mgs_rollout_grid(mgs_batch* b, int n) {
  if (!b || n < 0) return fail(MGS_EINVAL, "mgs_rollout_grid: bad argument%s");
  if (hipSetDevice(b->m->device) != hipSuccess) return fail(MGS_EHIP, "mgs_rollout_grid: hipSetDevice failed%s");
  if (queue_mode() == 0) return n;
  int r = resident_workgroups(b->m);
  if (queue_mode() > 1 && r > queue_mode()) r = queue_mode();
  return (r > 0 && r < n) ? r : n;
}

int mgs_rollout_queue(int mode) {
  int prev = queue_mode();
  if (mode >= 0) g_queue_mode = mode;
  return prev;
}

int mgs_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

}  // extern "C"
