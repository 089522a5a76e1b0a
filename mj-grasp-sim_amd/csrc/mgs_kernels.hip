// mgs_kernels.hip -- batched grasp-candidate physics for MI355X (gfx950).
//
// One 64-lane wavefront owns one grasp candidate for its whole rollout
// (close -> lift -> shake, reference mgs/env/gravityless_object_grasping.py:
// 127-295): the candidate's state lives in LDS for all steps, the model
// (hulls, bodies, pairs) is read through the L1/L2 from HBM, and only the
// initial state and the outputs cross HBM.  Lanes parallelise the wide loops
// of a step:
//   * convex-hull support mapping (lanes over hull vertices, wave argmax),
//   * contact-feature extraction (ballot compaction in vertex order),
//   * constraint Jacobians, K = M^-1 J^T, efc velocities / diagonals
//     (lanes over dofs or constraint rows),
//   * LDL^T columns of the mass matrix (lanes over rows),
//   * the PGS row residuals J_r . w (lanes over dofs, pairwise tree reduction).
// The remaining scalar control logic (kinematic tree walk, MPR portal logic,
// polygon clipping, QCQP friction projection) runs lane-uniform.
//
// Numerical contract (see oracle/mgs_oracle.c): compiled with
// -ffp-contract=off; every expression below evaluates in the same order as the
// oracle restatement, and the only cross-lane reduction is the pairwise tree
// of tree_dot(), so fp64 results are bit-identical to the oracle.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mgs_gpu.h"

#define K_MINVAL 1e-15
#define K_MAXF 16
#define K_MAXPOLY 40
#define K_POLY_POINTS (4 * K_MAXF + 3 * K_MAXPOLY)   // collide_manifold's polygon scratch
#define K_MPR_MAXIT 64
#define K_FEAT_EPS 1e-5
#define K_BB_MERGE 1e-6     // box-box: merge distance of manifold points, x face half size (oracle BB_MERGE)
// separation certificates (cert_check): slots per candidate, doubles per slot,
// the least margin worth keeping and the safety margin of the validity test
#define K_CERT 8
#define CERT_W 17
#define CERT_STORE 1e-6
#define CERT_EPS 1e-10
#define WAVE 64
// row stride of the constraint matrix G (doubles).  An odd stride (NV + 1) makes
// row walks bank-conflict free but measured no faster and costs 680 B of LDS
// G row stride (doubles): NV + MGS_GPAD.  With lanes over rows reading G[r * GS + k],
// an odd stride spreads the 32 lanes of a ds_read_b64 group over distinct banks
#ifndef MGS_GPAD
#ifdef MGS_G_GLOBAL
#define MGS_GPAD 0
#else
#define MGS_GPAD 1
#endif
#endif
#define GS (NV + MGS_GPAD)
#if defined(MGS_G_GLOBAL) && MGS_GPAD != 0
#error "G rows in HBM are unpadded (launch_layout sizes them nefc_max * nv)"
#endif
#define DEVI __device__ __attribute__((always_inline)) inline

struct P2 { double x, y, h; };

// ---------------------------------------------------------------------------
// model access
struct Mdl {
  mgs_model_desc m;
  const int32_t* I;
  const double* D;
};
#define IA(md, f) ((md).I + (md).m.i_##f)
#define DA(md, f) ((md).D + (md).m.d_##f)

// per-candidate working set in LDS (see make_layout in mgs_capi.hip for the
// carve-up; the U region is time-multiplexed between pipeline stages)
struct Dat {
  double *qpos, *qvel, *qacc_ws, *ctrl, *mocap_pos, *mocap_quat, *time;
  double *act, *act_dot;   // actuator state (mujoco.pid setpoint / integral) and its rate (ABI 21)
  double *xpos, *xquat, *xmat, *xipos, *xanchor, *xaxis;
  double *subtree_com, *subtree_mass, *cinert, *cdof;
  double *geom_xpos, *geom_xmat;
  double *M, *Dv, *Dinv, *sD, *isD, *tmp, *tmp2;
  double *qfrc_bias, *qfrc_passive, *qfrc_actuator, *qfrc_smooth, *qacc_smooth, *qfrc_constraint;
  double *act_force, *act_moment, *act_length, *act_vel;
  double *con_pos, *con_frame, *con_dist;
  double *efc_R, *efc_b, *con_mu, *con_blk;
  double* cert;     // separation certificates (K_CERT slots of CERT_W doubles, see cert_check)
  // U region views
  double *crb, *cvel, *cacc, *cfrc, *cdof_dot;          // dynamics stage
  P2* poly;                                           // collision stage
  double* pdep;                                       // collision stage
  double *comacc;                                     // comPos stage
  double *G, *efc_aref, *efc_vel, *efc_pos, *efc_margin, *scratch;  // constraint + solver stage
  double* qDeriv;                                     // integration stage
  // Newton solver workspace (U region, after the constraint stage views)
  double *efc_jar, *efc_jv, *efc_f, *efc_Dr, *efc_isR, *nH, *nw, *nw0, *ng, *ndir, *con_hb;
  int *con_pair, *con_g1, *con_g2, *efc_type, *efc_dim, *efc_con, *efc_state, *ints;
  int gs;   // row stride of G (nv + 1)
};
// ints[]: 0 ncon, 1 nefc, 2 overflow, 3 iters, 6 cr0, 7 cr1, 8 neq rows, 9 fr0, 10 fr1, 11 lr0, 12 lr1
#define NCON ints[0]
#define NEFC ints[1]
#define OVERFLOW ints[2]
#define ITERS ints[3]
// largest contact dimension the kernels handle: 4 (frictionless, sliding,
// torsional) in the libraries and most specialised objects; 6 (rolling too)
// in the objects of models with condim-6 pairs (mgs/core/special.py,
// -DMGS_MAXDIM=6).  Per-contact block storage is MGS_MAXDIM^2 doubles.
#ifndef MGS_MAXDIM
#define MGS_MAXDIM 4
#endif
static_assert(MGS_MAXDIM == 4 || MGS_MAXDIM == 6, "MGS_MAXDIM is 4 or 6");
#define BLKSTRIDE (MGS_MAXDIM * MGS_MAXDIM)
#ifndef MGS_RPL
#define MGS_RPL 2   // constraint rows per lane (nefc_max <= 64 * MGS_RPL)
#endif
// NV-long operand rows of the factor, the triangular solves and the G
// products held in registers, or read from LDS at each use.  Registers in
// every build of one dof per lane: the wide flavour's pile objects (nv 38-58,
// one wave per SIMD) hold them in 424 VGPRs without spilling, and the C5 pile
// rollout runs 6 % faster for it (round 5, profiles/r05w_c5_register_rows_ab.txt);
// with two dofs per lane (MGS_DPL 2) each lane has two rows: LDS.  Same values
// either way.
#ifndef MGS_REG_ROWS
#if defined(MGS_DPL) && MGS_DPL > 1
#define MGS_REG_ROWS 0
#else
#define MGS_REG_ROWS 1
#endif
#endif

// Packed storage of the mass matrix / its LDL factor and of the Newton
// Hessian (symmetric; only the lower triangle is ever read): row i of the
// lower triangle at i (i + 1) / 2 instead of i nv.  The wide build (clutter
// piles, nv up to 58, whose row loops read M and H from LDS anyway) packs
// them: 2 x 1653 doubles less at nv 58 (round 5, two pile workgroups per CU);
// the main build keeps the square layout its register-row factor loads.
#ifndef MGS_PACKED
#ifdef MGS_WIDE
#define MGS_PACKED 1
#else
#define MGS_PACKED 0
#endif
#endif
#if MGS_PACKED
#define TRI(i, k, n) ((((i) * ((i) + 1)) >> 1) + (k))
#define TRI_SIZE(n) (((n) * ((n) + 1)) >> 1)
#else
#define TRI(i, k, n) ((i) * (n) + (k))
#define TRI_SIZE(n) ((n) * (n))
#endif
// (the register-row factor and solves load row i's lower entries by TRI too;
// the upper ones they load are never used, and TRI keeps them in bounds)
// the friction coefficients of a contact: its pair's row of the model instead
// of a per-contact copy in LDS (main-library objects with G in HBM, round 5:
// the same values -- the copy's one extra slot, mu[dim - 1] = 0, is never read)
#ifndef MGS_MU_MODEL
#define MGS_MU_MODEL 0
#endif

// the lane index through an opaque move at every use: index arithmetic and
// lane masks derived from it are recomputed where they are used instead of
// being hoisted out of the step loop and held (in VGPRs, AGPRs and SGPR
// spill lanes) for the whole rollout (round 5: the headline rollout 430 ->
// 328 registers with this alone; profiles/r05c_ab.txt)
DEVI int lane_id() {
  int l = (int)__lane_id();
  asm volatile("" : "+v"(l));
  return l;
}
// values that are uniform across the wave but come from LDS: move to SGPRs so
// control flow on them is scalar
DEVI int uni(int x) { return __builtin_amdgcn_readfirstlane(x); }

// wave-wide shuffle from lane src (0..63): HIP's __shfl(x, src) with width 64
// (ds_bpermute at byte address 4 src), without its lane-index term, so no
// per-lane address is derived from the lane index and held across the step loop
DEVI int shfl(int x, int src) { return __builtin_amdgcn_ds_bpermute(src << 2, x); }
DEVI double shfl(double x, int src) {
  const int a = src << 2;
  const int lo = __builtin_amdgcn_ds_bpermute(a, __double2loint(x));
  const int hi = __builtin_amdgcn_ds_bpermute(a, __double2hiint(x));
  return __hiloint2double(hi, lo);
}

// Diagnostic stage timers (built only with -DMGS_PROFILE; never in the product build)
#ifdef MGS_PROFILE
#ifdef MGS_SPECIAL
// a specialised code object's timers, read by the host with hipModuleGetGlobal
extern "C" {
__device__ unsigned long long g_prof[64];
}
#else
// one copy per translation unit (each dof count's kernels, mgs_inst.hip)
static __device__ unsigned long long g_prof[64];
#endif
// per-workgroup accumulators in static LDS; PT(k) at wave-uniform points only
__shared__ unsigned long long s_prof[67];
#define PT(k) do { unsigned long long _n = __builtin_amdgcn_s_memtime(); \
    if (__lane_id() == 0) { s_prof[k] += _n - s_prof[64]; s_prof[64] = _n; } } while (0)
// slots 61 / 62 at the flush: the workgroup's shader-clock and 100 MHz
// real-time spans (their ratio is the clock the chip held, MI355X_MICROARCH.md
// "DVFS give-back" item 6)
#define PROF_DECL if (__lane_id() == 0) { for (int _k = 0; _k < 64; _k++) s_prof[_k] = 0; \
    s_prof[64] = s_prof[65] = __builtin_amdgcn_s_memtime(); s_prof[66] = __builtin_amdgcn_s_memrealtime(); }
#define PROF(k) PT(k)
#define PCNT(k, v) do { if (__lane_id() == 0) s_prof[k] += (v); } while (0)
#define PROF_FLUSH if (lane_id() == 0) { \
    s_prof[61] = __builtin_amdgcn_s_memtime() - s_prof[65]; \
    s_prof[62] = __builtin_amdgcn_s_memrealtime() - s_prof[66]; \
    for (int _k = 0; _k < 64; _k++) atomicAdd(&g_prof[_k], s_prof[_k]); }
#else
#define PT(k)
#define PROF_DECL
#define PROF(k)
#define PCNT(k, v)
#define PROF_FLUSH
#endif
// Lane-to-lane hand-off inside the one-wave workgroup.  Main build: every
// such hand-off goes through LDS, whose operations a wave issues and the LDS
// processes in order, so a wavefront-scope fence (it keeps the compiler from
// moving memory operations across it) is enough: +1 % on the bench, -1 % on
// one API launch (profiles/r04v_wavefront_fence_ab.txt).  Wide build (G in
// HBM: rows written by lanes over rows and read by lanes over dofs through
// global memory): the workgroup barrier, which waits for the stores.
#if defined(MGS_WSYNC_FENCE) || (!defined(MGS_G_GLOBAL) && !defined(MGS_WSYNC_BARRIER))
DEVI void wsync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }
#else
DEVI void wsync() { __syncthreads(); }
#endif

// ---------------------------------------------------------------------------
// math primitives: identical expressions to the oracle
DEVI void k_sincos(double x, double* s, double* c) {
  const double inv_pio2 = 6.36619772367581382433e-01;
  const double pio2_1 = 1.57079632673412561417e+00;
  const double pio2_1t = 6.07710050650619224932e-11;
  const double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
               S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
               S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
  const double C1 = 4.16666666666666019037e-02, C2 = -1.38888888888741095749e-03,
               C3 = 2.48015872894767294178e-05, C4 = -2.75573143513906633035e-07,
               C5 = 2.08757232129817482790e-09, C6 = -1.13596475577881948265e-11;
  double kd = x * inv_pio2;
  kd = (kd >= 0.0) ? floor(kd + 0.5) : -floor(0.5 - kd);
  double r = (x - kd * pio2_1) - kd * pio2_1t;
  double z = r * r;
  double ps = S1 + z * (S2 + z * (S3 + z * (S4 + z * (S5 + z * S6))));
  double sr = r + (r * z) * ps;
  double pc = C1 + z * (C2 + z * (C3 + z * (C4 + z * (C5 + z * C6))));
  double cr = (1.0 - 0.5 * z) + (z * z) * pc;
  long k = (long)kd;
  int q = (int)(k & 3);
  if (q == 0) { *s = sr; *c = cr; }
  else if (q == 1) { *s = cr; *c = -sr; }
  else if (q == 2) { *s = -sr; *c = -cr; }
  else { *s = -cr; *c = sr; }
}

DEVI double dot3(const double* a, const double* b) {
  return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2];
}
DEVI void cross3(double* r, const double* a, const double* b) {
  double r0 = a[1] * b[2] - a[2] * b[1];
  double r1 = a[2] * b[0] - a[0] * b[2];
  double r2 = a[0] * b[1] - a[1] * b[0];
  r[0] = r0; r[1] = r1; r[2] = r2;
}
DEVI void sub3(double* r, const double* a, const double* b) {
  r[0] = a[0] - b[0]; r[1] = a[1] - b[1]; r[2] = a[2] - b[2];
}
DEVI void add3(double* r, const double* a, const double* b) {
  r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2];
}
DEVI void mulmv3(double* r, const double* m, const double* v) {
  double r0 = (m[0] * v[0] + m[1] * v[1]) + m[2] * v[2];
  double r1 = (m[3] * v[0] + m[4] * v[1]) + m[5] * v[2];
  double r2 = (m[6] * v[0] + m[7] * v[1]) + m[8] * v[2];
  r[0] = r0; r[1] = r1; r[2] = r2;
}
DEVI void mulmtv3(double* r, const double* m, const double* v) {
  double r0 = (m[0] * v[0] + m[3] * v[1]) + m[6] * v[2];
  double r1 = (m[1] * v[0] + m[4] * v[1]) + m[7] * v[2];
  double r2 = (m[2] * v[0] + m[5] * v[1]) + m[8] * v[2];
  r[0] = r0; r[1] = r1; r[2] = r2;
}
DEVI void quatmul(double* r, const double* a, const double* b) {
  double r0 = ((a[0] * b[0] - a[1] * b[1]) - a[2] * b[2]) - a[3] * b[3];
  double r1 = ((a[0] * b[1] + a[1] * b[0]) + a[2] * b[3]) - a[3] * b[2];
  double r2 = ((a[0] * b[2] - a[1] * b[3]) + a[2] * b[0]) + a[3] * b[1];
  double r3 = ((a[0] * b[3] + a[1] * b[2]) - a[2] * b[1]) + a[3] * b[0];
  r[0] = r0; r[1] = r1; r[2] = r2; r[3] = r3;
}
DEVI void quat2mat(double* m, const double* q) {
  double q00 = q[0] * q[0], q01 = q[0] * q[1], q02 = q[0] * q[2], q03 = q[0] * q[3];
  double q11 = q[1] * q[1], q12 = q[1] * q[2], q13 = q[1] * q[3];
  double q22 = q[2] * q[2], q23 = q[2] * q[3], q33 = q[3] * q[3];
  m[0] = ((q00 + q11) - q22) - q33;
  m[1] = 2.0 * (q12 - q03);
  m[2] = 2.0 * (q13 + q02);
  m[3] = 2.0 * (q12 + q03);
  m[4] = ((q00 - q11) + q22) - q33;
  m[5] = 2.0 * (q23 - q01);
  m[6] = 2.0 * (q13 - q02);
  m[7] = 2.0 * (q23 + q01);
  m[8] = ((q00 - q11) - q22) + q33;
}
DEVI void normalize4(double* q) {
  double n = sqrt(((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3]);
  if (n < K_MINVAL) { q[0] = 1.0; q[1] = q[2] = q[3] = 0.0; return; }
  double inv = 1.0 / n;
  q[0] = q[0] * inv; q[1] = q[1] * inv; q[2] = q[2] * inv; q[3] = q[3] * inv;
}
DEVI double normalize3(double* v) {
  double n = sqrt(dot3(v, v));
  if (n < K_MINVAL) { v[0] = 1.0; v[1] = v[2] = 0.0; return 0.0; }
  double inv = 1.0 / n;
  v[0] = v[0] * inv; v[1] = v[1] * inv; v[2] = v[2] * inv;
  return n;
}
DEVI void axisangle2quat(double* q, const double* axis, double angle) {
  double s, c;
  k_sincos(0.5 * angle, &s, &c);
  q[0] = c; q[1] = axis[0] * s; q[2] = axis[1] * s; q[3] = axis[2] * s;
}
DEVI void mul_inert_vec(double* r, const double* i, const double* v) {
  double r0 = ((i[0] * v[0] + i[3] * v[1]) + i[4] * v[2]) - i[8] * v[4] + i[7] * v[5];
  double r1 = ((i[3] * v[0] + i[1] * v[1]) + i[5] * v[2]) + i[8] * v[3] - i[6] * v[5];
  double r2 = ((i[4] * v[0] + i[5] * v[1]) + i[2] * v[2]) - i[7] * v[3] + i[6] * v[4];
  double r3 = (i[8] * v[1] - i[7] * v[2]) + i[9] * v[3];
  double r4 = (i[6] * v[2] - i[8] * v[0]) + i[9] * v[4];
  double r5 = (i[7] * v[0] - i[6] * v[1]) + i[9] * v[5];
  r[0] = r0; r[1] = r1; r[2] = r2; r[3] = r3; r[4] = r4; r[5] = r5;
}
DEVI double dot6(const double* a, const double* b) {
  return ((((a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]) + a[3] * b[3]) + a[4] * b[4]) + a[5] * b[5];
}
DEVI void cross_motion(double* r, const double* v, const double* u) {
  double r0 = v[1] * u[2] - v[2] * u[1];
  double r1 = v[2] * u[0] - v[0] * u[2];
  double r2 = v[0] * u[1] - v[1] * u[0];
  double r3 = (v[1] * u[5] - v[2] * u[4]) + (v[4] * u[2] - v[5] * u[1]);
  double r4 = (v[2] * u[3] - v[0] * u[5]) + (v[5] * u[0] - v[3] * u[2]);
  double r5 = (v[0] * u[4] - v[1] * u[3]) + (v[3] * u[1] - v[4] * u[0]);
  r[0] = r0; r[1] = r1; r[2] = r2; r[3] = r3; r[4] = r4; r[5] = r5;
}
DEVI void cross_force(double* r, const double* v, const double* f) {
  double r0 = (v[1] * f[2] - v[2] * f[1]) + (v[4] * f[5] - v[5] * f[4]);
  double r1 = (v[2] * f[0] - v[0] * f[2]) + (v[5] * f[3] - v[3] * f[5]);
  double r2 = (v[0] * f[1] - v[1] * f[0]) + (v[3] * f[4] - v[4] * f[3]);
  double r3 = v[1] * f[5] - v[2] * f[4];
  double r4 = v[2] * f[3] - v[0] * f[5];
  double r5 = v[0] * f[4] - v[1] * f[3];
  r[0] = r0; r[1] = r1; r[2] = r2; r[3] = r3; r[4] = r4; r[5] = r5;
}

// Pairwise tree reduction over lanes, identical to the oracle's tree_dot():
// level s (s = 1, 2, 4, ... < P) adds lane k^s to lane k.  Within a 16-lane row
// the levels are DPP moves (xor 1 and xor 2 by quad permutes; xor 4 and xor 8 by
// the half-row / row mirrors, which equal xor on values already uniform over
// the lower levels); the last two levels combine the four row sums read with
// v_readlane in the same pairing ((r0 + r1) + (r2 + r3)).  Result is uniform.
DEVI double dpp_d(double x, int ctrl_sel) {
  int lo = __double2loint(x), hi = __double2hiint(x);
  switch (ctrl_sel) {
    case 0: lo = __builtin_amdgcn_mov_dpp(lo, 0xB1, 0xF, 0xF, false); hi = __builtin_amdgcn_mov_dpp(hi, 0xB1, 0xF, 0xF, false); break;
    case 1: lo = __builtin_amdgcn_mov_dpp(lo, 0x4E, 0xF, 0xF, false); hi = __builtin_amdgcn_mov_dpp(hi, 0x4E, 0xF, 0xF, false); break;
    case 2: lo = __builtin_amdgcn_mov_dpp(lo, 0x141, 0xF, 0xF, false); hi = __builtin_amdgcn_mov_dpp(hi, 0x141, 0xF, 0xF, false); break;
    default: lo = __builtin_amdgcn_mov_dpp(lo, 0x140, 0xF, 0xF, false); hi = __builtin_amdgcn_mov_dpp(hi, 0x140, 0xF, 0xF, false); break;
  }
  return __hiloint2double(hi, lo);
}
DEVI double readlane_d(double x, int l) {
  int lo = __builtin_amdgcn_readlane(__double2loint(x), l);
  int hi = __builtin_amdgcn_readlane(__double2hiint(x), l);
  return __hiloint2double(hi, lo);
}
DEVI double tree_sum(double leaf, int P) {
  if (P > 1) leaf = leaf + dpp_d(leaf, 0);
  if (P > 2) leaf = leaf + dpp_d(leaf, 1);
  if (P > 4) leaf = leaf + dpp_d(leaf, 2);
  if (P > 8) leaf = leaf + dpp_d(leaf, 3);
  if (P > 16) {
    double r0 = readlane_d(leaf, 0), r1 = readlane_d(leaf, 16);
    if (P > 32) {
      double r2 = readlane_d(leaf, 32), r3 = readlane_d(leaf, 48);
      return (r0 + r1) + (r2 + r3);
    }
    return r0 + r1;
  }
  return readlane_d(leaf, 0);
}
DEVI int next_pow2(int n) {
  int P = 1;
  while (P < n) P <<= 1;
  return P;
}

// Dofs per lane.  Lanes over dofs is the unit of the dynamics, the solves and
// the solver sweeps: lane l owns dof l (MGS_DPL 1, every library build and
// every model of at most 64 dofs) or dofs l and l + 64 (MGS_DPL 2: the
// specialised objects of models with 65-128 dofs, clutter piles of 7-10
// objects).  A dof-indexed value held in registers is a DofV; with MGS_DPL 1
// every helper below is the single-slot expression it replaces.
#ifndef MGS_DPL
#define MGS_DPL 1
#endif
static_assert(MGS_DPL == 1 || MGS_DPL == 2, "MGS_DPL is 1 or 2");
static_assert(MGS_DPL == 1 || (MGS_PACKED && !MGS_REG_ROWS), "two dofs per lane: the wide flavour (MGS_WIDE)");
#define MGS_MAXNV (WAVE * MGS_DPL)
struct DofV {
  double v[MGS_DPL];
};
DEVI DofV dof_zero() {
  DofV x;
#pragma unroll
  for (int h = 0; h < MGS_DPL; h++) x.v[h] = 0.0;
  return x;
}
// p[dof] on the dof's lane, 0 past nv
DEVI DofV dof_load(const double* p, int nv, int lane) {
  DofV x;
#pragma unroll
  for (int h = 0; h < MGS_DPL; h++) x.v[h] = (lane + h * WAVE < nv) ? p[lane + h * WAVE] : 0.0;
  return x;
}
DEVI DofV dof_mul(const DofV& a, const DofV& b) {
  DofV x;
#pragma unroll
  for (int h = 0; h < MGS_DPL; h++) x.v[h] = a.v[h] * b.v[h];
  return x;
}
// the oracle's tree_dot over the dof leaves (P = next_pow2(nv)): a tree over
// 128 leaves is the tree over dofs 0-63 plus the tree over dofs 64-127 (its
// last level adds leaf 64 to leaf 0)
DEVI double dof_tree(const DofV& x, int P) {
  if (MGS_DPL == 1 || P <= WAVE) return tree_sum(x.v[0], P);
  return tree_sum(x.v[0], WAVE) + tree_sum(x.v[MGS_DPL - 1], WAVE);
}
// u += g delta on the lanes' dofs below nv (the others keep their value)
DEVI void dof_axpy(DofV& u, const DofV& g, double delta, int nv, int lane) {
#pragma unroll
  for (int h = 0; h < MGS_DPL; h++) {
    double s = u.v[h] + g.v[h] * delta;
    if (lane + h * WAVE < nv) u.v[h] = s;
  }
}
// `DOF_SLOTS(i, nv) stmt;`: stmt for each dof i < nv of this lane (lane, lane + 64)
#define DOF_SLOTS(i, nv) \
  _Pragma("unroll") for (int _h = 0, i = lane + 0; _h < MGS_DPL; _h++, i += WAVE) if (i < (nv))
// dof k's value, uniform (k uniform)
DEVI double dof_readlane(const DofV& x, int k) {
  if (MGS_DPL == 1) return readlane_d(x.v[0], k);
  return readlane_d((k >> 6) ? x.v[MGS_DPL - 1] : x.v[0], k & (WAVE - 1));
}
// dof col moves body b: the model's body_dofmask, bit col of the body's words
// (2 words per body, 4 for models of more than 64 dofs; mgs_gpu.h)
DEVI int dof_moves(const Mdl& md, int b, int col) {
  if (MGS_DPL == 1) {
    const int32_t* mask = IA(md, body_dofmask) + 2 * b;
    return (col < 32) ? ((mask[0] >> col) & 1) : ((mask[1] >> (col - 32)) & 1);
  }
  const int32_t* mask = IA(md, body_dofmask) + (md.m.nv > 64 ? 4 : 2) * b;
  return (mask[col >> 5] >> (col & 31)) & 1;
}

// ---------------------------------------------------------------------------
// Tree-level parallel forward kinematics (oracle kinematics()): lane b owns
// body b; bodies of one tree depth are independent given their parents, so the
// levels run in order and the bodies of a level in parallel.  Per-body
// arithmetic is the oracle's.
// a body's static model data (and its first joint's), loaded into registers
// once per kinematics pass before the level loop: the global loads of every
// level are then in flight together instead of one dependent round trip per
// tree level
struct BodyStatic {
  int parent, mocap, jn, j0, jt, qa;
  double bpos[3], bquat[4], ipos[3], jpos[3], jaxis[3], q0;
};
DEVI void body_static(const Mdl& md, int b, BodyStatic& s) {
  s.parent = IA(md, body_parentid)[b];
  s.mocap = IA(md, body_mocapid)[b];
  s.jn = IA(md, body_jntnum)[b];
  s.j0 = IA(md, body_jntadr)[b];
  int j = s.jn > 0 ? s.j0 : 0;
  s.jt = IA(md, jnt_type)[j];
  s.qa = IA(md, jnt_qposadr)[j];
  const double *bpos = DA(md, body_pos) + 3 * b, *bquat = DA(md, body_quat) + 4 * b, *ipos = DA(md, body_ipos) + 3 * b;
  const double *jpos = DA(md, jnt_pos) + 3 * j, *jaxis = DA(md, jnt_axis) + 3 * j;
  for (int k = 0; k < 3; k++) { s.bpos[k] = bpos[k]; s.ipos[k] = ipos[k]; s.jpos[k] = jpos[k]; s.jaxis[k] = jaxis[k]; }
  for (int k = 0; k < 4; k++) s.bquat[k] = bquat[k];
  s.q0 = DA(md, qpos0)[s.qa];
}

DEVI void body_kin(const Mdl& md, Dat& d, int b, const BodyStatic& bs) {
  const int32_t *jtype = IA(md, jnt_type), *qadr = IA(md, jnt_qposadr);
  const double *jposA = DA(md, jnt_pos), *jaxisA = DA(md, jnt_axis), *qpos0 = DA(md, qpos0);
  double pos[3], quat[4], mat[9];
  if (bs.mocap >= 0) {
    const double* mp = d.mocap_pos + 3 * bs.mocap;
    const double* mq = d.mocap_quat + 4 * bs.mocap;
    pos[0] = mp[0]; pos[1] = mp[1]; pos[2] = mp[2];
    quat[0] = mq[0]; quat[1] = mq[1]; quat[2] = mq[2]; quat[3] = mq[3];
    normalize4(quat);
  } else {
    int p = bs.parent;
    double t[3];
    mulmv3(t, d.xmat + 9 * p, bs.bpos);
    add3(pos, d.xpos + 3 * p, t);
    quatmul(quat, d.xquat + 4 * p, bs.bquat);
    for (int k = 0; k < bs.jn; k++) {
      int j = bs.j0 + k;
      // the first joint's data are preloaded; further joints of the body load here
      int jt = k == 0 ? bs.jt : jtype[j];
      int a = k == 0 ? bs.qa : qadr[j];
      const double* jpos = k == 0 ? bs.jpos : jposA + 3 * j;
      const double* jaxis = k == 0 ? bs.jaxis : jaxisA + 3 * j;
      double q0 = k == 0 ? bs.q0 : qpos0[a];
      if (jt == MGS_JNT_FREE) {
        pos[0] = d.qpos[a]; pos[1] = d.qpos[a + 1]; pos[2] = d.qpos[a + 2];
        quat[0] = d.qpos[a + 3]; quat[1] = d.qpos[a + 4]; quat[2] = d.qpos[a + 5]; quat[3] = d.qpos[a + 6];
        normalize4(quat);
        d.xanchor[3 * j] = pos[0]; d.xanchor[3 * j + 1] = pos[1]; d.xanchor[3 * j + 2] = pos[2];
        d.xaxis[3 * j] = 0.0; d.xaxis[3 * j + 1] = 0.0; d.xaxis[3 * j + 2] = 1.0;
      } else {
        double anc[3], axw[3];
        quat2mat(mat, quat);
        mulmv3(axw, mat, jaxis);
        mulmv3(t, mat, jpos);
        add3(anc, t, pos);
        d.xaxis[3 * j] = axw[0]; d.xaxis[3 * j + 1] = axw[1]; d.xaxis[3 * j + 2] = axw[2];
        d.xanchor[3 * j] = anc[0]; d.xanchor[3 * j + 1] = anc[1]; d.xanchor[3 * j + 2] = anc[2];
        if (jt == MGS_JNT_HINGE) {
          double ql[4], qn[4];
          axisangle2quat(ql, jaxis, d.qpos[a] - q0);
          quatmul(qn, quat, ql);
          quat[0] = qn[0]; quat[1] = qn[1]; quat[2] = qn[2]; quat[3] = qn[3];
          quat2mat(mat, quat);
          mulmv3(t, mat, jpos);
          sub3(pos, anc, t);
        } else {
          double dq = d.qpos[a] - q0;
          pos[0] = pos[0] + axw[0] * dq;
          pos[1] = pos[1] + axw[1] * dq;
          pos[2] = pos[2] + axw[2] * dq;
        }
      }
    }
    normalize4(quat);
  }
  d.xpos[3 * b] = pos[0]; d.xpos[3 * b + 1] = pos[1]; d.xpos[3 * b + 2] = pos[2];
  d.xquat[4 * b] = quat[0]; d.xquat[4 * b + 1] = quat[1]; d.xquat[4 * b + 2] = quat[2]; d.xquat[4 * b + 3] = quat[3];
  quat2mat(mat, quat);
  for (int k = 0; k < 9; k++) d.xmat[9 * b + k] = mat[k];
  double t[3];
  mulmv3(t, mat, bs.ipos);
  add3(d.xipos + 3 * b, pos, t);
}

DEVI int max_depth(const Mdl& md) { return IA(md, body_depth)[md.m.nbody]; }

DEVI void kinematics(const Mdl& md, Dat& d) {
  int lane = lane_id(), nb = md.m.nbody;
  const int32_t* depth = IA(md, body_depth);
  if (lane == 0) {
    d.xpos[0] = d.xpos[1] = d.xpos[2] = 0.0;
    d.xquat[0] = 1.0; d.xquat[1] = d.xquat[2] = d.xquat[3] = 0.0;
    quat2mat(d.xmat, d.xquat);
  }
  wsync();
  int maxd = max_depth(md);
  int myd = (lane < nb) ? depth[lane] : -1;
  BodyStatic bs;
  body_static(md, (lane < nb && lane > 0) ? lane : (nb > 1 ? 1 : 0), bs);
  for (int L = 1; L <= maxd; L++) {
    if (myd == L) body_kin(md, d, lane, bs);
    wsync();
  }
  const int32_t* gbody = IA(md, geom_bodyid);
  const double *gpos = DA(md, geom_pos), *gquat = DA(md, geom_quat);
  for (int g = lane; g < md.m.ngeom; g += WAVE) {
    int b = gbody[g];
    double t[3], q[4];
    mulmv3(t, d.xmat + 9 * b, gpos + 3 * g);
    add3(d.geom_xpos + 3 * g, d.xpos + 3 * b, t);
    quatmul(q, d.xquat + 4 * b, gquat + 4 * g);
    quat2mat(d.geom_xmat + 9 * g, q);
  }
  wsync();
}

// arr[p] += arr[c] over the tree from the leaves up, children of each parent in
// decreasing body index (the oracle's `for b = nb-1..1: arr[parent] += arr[b]`
// order per parent); W doubles per body; world included iff with_world.
// The child list (first ACC_KIDS entries) is loaded into registers before the
// level loop, so the levels do not each wait on a dependent global load.
#define ACC_KIDS 4
template <int W>
DEVI void accumulate_up(const Mdl& md, double* arr, int with_world) {
  int lane = lane_id(), nb = md.m.nbody;
  const int32_t* depth = IA(md, body_depth);
  int maxd = max_depth(md);
  int lb = lane < nb ? lane : 0;
  int myd = (lane < nb) ? depth[lane] : -1;
  const int32_t* kids = IA(md, body_child) + IA(md, body_childadr)[lb];
  int nk = IA(md, body_childnum)[lb];
  int kr[ACC_KIDS];
#pragma unroll
  for (int q = 0; q < ACC_KIDS; q++) kr[q] = kids[q < nk ? q : 0];
  for (int L = maxd; L >= 1; L--) {
    if (myd == L - 1 && (with_world || lane > 0)) {
      double acc[W];
#pragma unroll
      for (int k = 0; k < W; k++) acc[k] = arr[W * lane + k];
      for (int q = 0; q < nk; q++) {   // children in decreasing body index
        int c;
        if (q < ACC_KIDS) {
          c = kr[0];
#pragma unroll
          for (int r = 1; r < ACC_KIDS; r++)
            if (q == r) c = kr[r];
        } else {
          c = kids[q];
        }
#pragma unroll
        for (int k = 0; k < W; k++) acc[k] = acc[k] + arr[W * c + k];
      }
#pragma unroll
      for (int k = 0; k < W; k++) arr[W * lane + k] = acc[k];
    }
    wsync();
  }
}

// mj_comPos (oracle com_pos()), lanes over bodies / dofs
DEVI void com_pos(const Mdl& md, Dat& d) {
  int lane = lane_id(), nb = md.m.nbody;
  const int32_t *rootid = IA(md, body_rootid);
  const int32_t *jntnum = IA(md, body_jntnum), *jntadr = IA(md, body_jntadr);
  const int32_t *jtype = IA(md, jnt_type), *dadr = IA(md, jnt_dofadr);
  const double *mass = DA(md, body_mass), *inertia = DA(md, body_inertia);
  // subtree mass + mass-weighted com packed as 4 doubles per body
  double* sc = d.comacc;
  for (int b = lane; b < nb; b += WAVE) {
    sc[4 * b] = mass[b];
    sc[4 * b + 1] = mass[b] * d.xipos[3 * b];
    sc[4 * b + 2] = mass[b] * d.xipos[3 * b + 1];
    sc[4 * b + 3] = mass[b] * d.xipos[3 * b + 2];
  }
  wsync();
  accumulate_up<4>(md, sc, 1);
  for (int b = lane; b < nb; b += WAVE) {
    double m = sc[4 * b];
    d.subtree_mass[b] = m;
    if (m < K_MINVAL) {
      d.subtree_com[3 * b] = d.xipos[3 * b];
      d.subtree_com[3 * b + 1] = d.xipos[3 * b + 1];
      d.subtree_com[3 * b + 2] = d.xipos[3 * b + 2];
    } else {
      double inv = 1.0 / m;
      d.subtree_com[3 * b] = sc[4 * b + 1] * inv;
      d.subtree_com[3 * b + 1] = sc[4 * b + 2] * inv;
      d.subtree_com[3 * b + 2] = sc[4 * b + 3] * inv;
    }
  }
  wsync();
  for (int b = lane; b < nb; b += WAVE) {
    double* ci = d.cinert + 10 * b;
    double qi[4], R[9];
    quatmul(qi, d.xquat + 4 * b, DA(md, body_iquat) + 4 * b);
    quat2mat(R, qi);
    const double* in = inertia + 3 * b;
    double mm = mass[b];
    double off[3];
    sub3(off, d.xipos + 3 * b, d.subtree_com + 3 * rootid[b]);
    double t[9];
    for (int i = 0; i < 3; i++)
      for (int j = 0; j < 3; j++)
        t[3 * i + j] = ((R[3 * i] * in[0]) * R[3 * j] + (R[3 * i + 1] * in[1]) * R[3 * j + 1]) +
                       (R[3 * i + 2] * in[2]) * R[3 * j + 2];
    ci[0] = t[0] + mm * (off[1] * off[1] + off[2] * off[2]);
    ci[1] = t[4] + mm * (off[0] * off[0] + off[2] * off[2]);
    ci[2] = t[8] + mm * (off[0] * off[0] + off[1] * off[1]);
    ci[3] = t[1] - mm * (off[0] * off[1]);
    ci[4] = t[2] - mm * (off[0] * off[2]);
    ci[5] = t[5] - mm * (off[1] * off[2]);
    ci[6] = mm * off[0];
    ci[7] = mm * off[1];
    ci[8] = mm * off[2];
    ci[9] = mm;
    if (b == 0) continue;
    const double* c = d.subtree_com + 3 * rootid[b];
    for (int k = 0; k < jntnum[b]; k++) {
      int j = jntadr[b] + k;
      int da = dadr[j];
      double off2[3];
      sub3(off2, c, d.xanchor + 3 * j);
      if (jtype[j] == MGS_JNT_FREE) {
        for (int i = 0; i < 3; i++) {
          double* cd = d.cdof + 6 * (da + i);
          cd[0] = cd[1] = cd[2] = 0.0;
          cd[3] = (i == 0) ? 1.0 : 0.0; cd[4] = (i == 1) ? 1.0 : 0.0; cd[5] = (i == 2) ? 1.0 : 0.0;
        }
        const double* Rb = d.xmat + 9 * b;
        for (int i = 0; i < 3; i++) {
          double* cd = d.cdof + 6 * (da + 3 + i);
          double ax[3] = {Rb[i], Rb[3 + i], Rb[6 + i]};
          cd[0] = ax[0]; cd[1] = ax[1]; cd[2] = ax[2];
          cross3(cd + 3, ax, off2);
        }
      } else if (jtype[j] == MGS_JNT_HINGE) {
        double* cd = d.cdof + 6 * da;
        const double* ax = d.xaxis + 3 * j;
        cd[0] = ax[0]; cd[1] = ax[1]; cd[2] = ax[2];
        cross3(cd + 3, ax, off2);
      } else {
        double* cd = d.cdof + 6 * da;
        const double* ax = d.xaxis + 3 * j;
        cd[0] = cd[1] = cd[2] = 0.0;
        cd[3] = ax[0]; cd[4] = ax[1]; cd[5] = ax[2];
      }
    }
  }
  wsync();
}

// composite rigid bodies + mass matrix (oracle crb()), tree-parallel
DEVI void crb(const Mdl& md, Dat& d) {
  int nb = md.m.nbody, nv = md.m.nv, lane = lane_id();
  const int32_t *dbody = IA(md, dof_bodyid), *dpar = IA(md, dof_parentid);
  const double* arm = DA(md, dof_armature);
  for (int k = lane; k < 10 * nb; k += WAVE) d.crb[k] = d.cinert[k];
  wsync();
  accumulate_up<10>(md, d.crb, 0);
  for (int k = lane; k < TRI_SIZE(nv); k += WAVE) d.M[k] = 0.0;
  wsync();
  if (nv <= WAVE) {
    // lane i walks dof i's ancestors; the walk reads a lane-resident copy of
    // dof_parentid through cross-lane permutes (in wave-uniform control flow,
    // every lane participating) instead of one dependent global load per step
    int dp_lane = lane < nv ? dpar[lane] : -1;
    int i = lane < nv ? lane : 0;
    double buf[6];
    mul_inert_vec(buf, d.crb + 10 * dbody[i], d.cdof + 6 * i);
    if (lane < nv) d.M[TRI(i, i, nv)] = dot6(d.cdof + 6 * i, buf) + arm[i];
    int j = dp_lane;
    while (__ballot(j >= 0)) {
      if (j >= 0) {
        double v = dot6(d.cdof + 6 * j, buf);
        d.M[TRI(i, j, nv)] = v;
#if !MGS_PACKED
        d.M[j * nv + i] = v;
#endif
      }
      int jn = shfl(dp_lane, j >= 0 ? j : 0);
      j = j >= 0 ? jn : -1;
    }
  } else {
    for (int i = lane; i < nv; i += WAVE) {
      double buf[6];
      mul_inert_vec(buf, d.crb + 10 * dbody[i], d.cdof + 6 * i);
      d.M[TRI(i, i, nv)] = dot6(d.cdof + 6 * i, buf) + arm[i];
      int j = dpar[i];
      while (j >= 0) {
        double v = dot6(d.cdof + 6 * j, buf);
        d.M[TRI(i, j, nv)] = v;
#if !MGS_PACKED
        d.M[j * nv + i] = v;
#endif
        j = dpar[j];
      }
    }
  }
  wsync();
}

// Dense LDL^T, register resident: lane i holds row i (NV doubles);
// column j's row L[j, 0:j] is broadcast from lane j with v_readlane, so a column
// costs j scalar reads and 2j FMAs-worth of VALU with no LDS round trip.  The
// per-element expressions are the oracle's ldl_factor():
//   W_k = L_jk Dv_k,  D_j = A_jj - sum_k W_k L_jk,  L_ij = (A_ij - sum_k L_ik W_k) / D_j.
// On exit the strict lower triangle of A (row-major in LDS) holds L, Dv/Dinv
// the diagonal.
// NV: the model's dof count as a compile-time constant (kernels are
// instantiated per supported nv, see MGS_NV_LIST in mgs_capi.hip), so the
// register rows and their loops are fully static.
// column broadcasts of the register factor through LDS (1) or v_readlane (0);
// default (-1): LDS up to 20 dofs, where it measured faster (the headline
// +1.2 %, profiles/r05b_ldl_broadcast_ab.txt), v_readlane above: the LDS
// form's unrolled loads are hoisted into registers, and past 20 dofs that
// spills (nv 28 under the 256-register cap: 94 -> 1305 VGPR spills, C4 -21 %;
// nv 58: 9 k, C5 -20 %)
#ifndef MGS_LDL_LDS_BCAST
#define MGS_LDL_LDS_BCAST -1
#endif
template <int NV>
DEVI void ldl_factor_regs(double (&r)[NV], double* Dv, double* Dinv) {
  // right-looking: after pivot j is scaled, every later column c takes its
  // update r_i[c] -= l_ij (l_cj d_j) at once.  Each entry receives the same
  // products in the same ascending-pivot order as the oracle's left-looking
  // loop (l_ij w with w = l_cj d_j; the diagonal w l_jj commutes), so the
  // factor is bit-identical while the pivot chain shrinks to one column.
  int lane = lane_id();
#pragma unroll
  for (int j = 0; j < NV; j++) {
    double dj = readlane_d(r[j], j);
    double inv = 1.0 / dj;
    if (lane > j) r[j] = r[j] * inv;
    if (lane == 0) { Dv[j] = dj; Dinv[j] = inv; }
    double v = r[j] * dj;   // lane c: l_cj d_j
    if constexpr (MGS_LDL_LDS_BCAST > 0 || (MGS_LDL_LDS_BCAST < 0 && NV <= 20)) {
      // the column's l_cj d_j to every lane through LDS: lane c parks it in
      // Dv[c], a slot column c itself writes later (the wave's LDS operations
      // complete in order), and every lane reads them at uniform addresses --
      // no SGPR per broadcast (the readlane form spills them)
      if (lane > j && lane < NV) Dv[lane] = v;
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
      for (int c = j + 1; c < NV; c++) r[c] = __builtin_fma(-r[j], Dv[c], r[c]);
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    } else {
#pragma unroll
      for (int c = j + 1; c < NV; c++) {
        double w = readlane_d(v, c);
        r[c] = __builtin_fma(-r[j], w, r[c]);
      }
    }
  }
}
// The same factor without register rows (two dofs per lane, nv 65-128):
// left-looking, lane i keeps row i in LDS; column c of
// every row takes sum_{k<c} l_ik (l_ck d_k) in ascending k -- the products and
// order of the right-looking loop above, so the factor is bit-identical.  The
// l_ck d_k are parked in the (dead) upper triangle, V[c][k] at A[k][c].  The
// diagonal keeps the original entries (meaninertia reads them).
template <int NV>
DEVI void ldl_factor_lds(double* A, double* Dv, double* Dinv) {
  const int lane = lane_id();
  for (int c = 0; c < NV; c++) {
    DofV sv;
#pragma unroll
    for (int h = 0; h < MGS_DPL; h++) {
      // row lane + 64 h (MGS_DPL 2: each lane factors its two rows in turn)
      const int li = lane + h * WAVE < NV ? lane + h * WAVE : 0;
      double s = A[TRI(li, c, NV)];
      // four products' operands loaded ahead of their FMAs (the LDS latency is
      // paid once per four terms instead of once per term); the FMA chain and
      // its ascending-k order are unchanged.  V_ck = l_ck d_k: parked in the
      // dead upper triangle (square layout), or formed again from l_ck and
      // Dv[k] (packed layout: the same product of the same operands)
#if MGS_PACKED
#define LDL_V(k) (A[TRI(c, (k), NV)] * Dv[k])
#else
#define LDL_V(k) A[(k) * NV + c]
#endif
      int k = 0;
      // eight at a time first (one LDS latency per eight terms), then four
      for (; k + 8 <= c; k += 8) {
        double a[8], b[8];
#pragma unroll
        for (int q = 0; q < 8; q++) { a[q] = A[TRI(li, k + q, NV)]; b[q] = LDL_V(k + q); }
#pragma unroll
        for (int q = 0; q < 8; q++) s = __builtin_fma(-a[q], b[q], s);
      }
      for (; k + 4 <= c; k += 4) {
        const double a0 = A[TRI(li, k, NV)], a1 = A[TRI(li, k + 1, NV)], a2 = A[TRI(li, k + 2, NV)],
                     a3 = A[TRI(li, k + 3, NV)];
        const double b0 = LDL_V(k), b1 = LDL_V(k + 1), b2 = LDL_V(k + 2), b3 = LDL_V(k + 3);
        s = __builtin_fma(-a0, b0, s);
        s = __builtin_fma(-a1, b1, s);
        s = __builtin_fma(-a2, b2, s);
        s = __builtin_fma(-a3, b3, s);
      }
      for (; k < c; k++) s = __builtin_fma(-A[TRI(li, k, NV)], LDL_V(k), s);
#undef LDL_V
      sv.v[h] = s;
    }
    double dc = dof_readlane(sv, c);
    double inv = 1.0 / dc;
    if (lane == 0) { Dv[c] = dc; Dinv[c] = inv; }
#pragma unroll
    for (int h = 0; h < MGS_DPL; h++) {
      const int i = lane + h * WAVE;
      if (i > c && i < NV) {
        double l = sv.v[h] * inv;
        A[TRI(i, c, NV)] = l;
#if !MGS_PACKED
        A[c * NV + i] = l * dc;
#endif
      }
    }
    wsync();
  }
}

template <int NV>
DEVI void store_lower(double* A, const double (&r)[NV]) {
  int lane = lane_id();
  if (lane < NV) {
#pragma unroll
    for (int k = 0; k < NV; k++)
      if (k < lane) A[TRI(lane, k, NV)] = r[k];
  }
  wsync();
}
template <int NV>
DEVI void ldl_factor(double* A, double* Dv, double* Dinv) {
#if MGS_REG_ROWS
  int lane = lane_id();
  int li = lane < NV ? lane : 0;
  double r[NV];
#pragma unroll
  for (int k = 0; k < NV; k++) r[k] = A[TRI(li, k, NV)];
  ldl_factor_regs<NV>(r, Dv, Dinv);
  store_lower<NV>(A, r);
#else
  ldl_factor_lds<NV>(A, Dv, Dinv);
#endif
}

// x = (L D L^T)^-1 b, all lanes (lane i owns x_i).  Forward substitution
// column by column (y_k broadcast, lanes i > k subtract L_ik y_k: the oracle's
// ascending-k order per row), then backward with k descending (oracle order).
// b and x may alias.
template <int NV>
DEVI void ldl_solve(const double* L, const double* Dinv, const double* b, double* x) {
  int lane = lane_id();
  // lane's row in slot h (rows past NV: row 0, never stored)
#define LS_ROW(h) (lane + (h) * WAVE < NV ? lane + (h) * WAVE : 0)
#if MGS_REG_ROWS
  static_assert(MGS_DPL == 1, "register rows hold one dof per lane");
  int li = LS_ROW(0);
  double Lr[NV], Lc[NV];
#pragma unroll
  for (int k = 0; k < NV; k++) { Lr[k] = L[TRI(li, k, NV)]; Lc[k] = L[TRI(k, li, NV)]; }
#define LS_LR(h, k) Lr[k]
#define LS_LC(h, k) Lc[k]
#else
#define LS_LR(h, k) L[TRI(LS_ROW(h), (k), NV)]
#define LS_LC(h, k) L[TRI((k), LS_ROW(h), NV)]
#endif
  DofV acc;
#pragma unroll
  for (int h = 0; h < MGS_DPL; h++) acc.v[h] = b[LS_ROW(h)];
#pragma unroll
  for (int k = 0; k < NV; k++) {
    double yk = dof_readlane(acc, k);
#pragma unroll
    for (int h = 0; h < MGS_DPL; h++)
      if (lane + h * WAVE > k) acc.v[h] = __builtin_fma(-LS_LR(h, k), yk, acc.v[h]);
  }
#pragma unroll
  for (int h = 0; h < MGS_DPL; h++) acc.v[h] = acc.v[h] * Dinv[LS_ROW(h)];
#pragma unroll
  for (int k = NV - 1; k >= 0; k--) {
    double xk = dof_readlane(acc, k);
#pragma unroll
    for (int h = 0; h < MGS_DPL; h++)
      if (lane + h * WAVE < k) acc.v[h] = __builtin_fma(-LS_LC(h, k), xk, acc.v[h]);
  }
#undef LS_LR
#undef LS_LC
#undef LS_ROW
  wsync();
#pragma unroll
  for (int h = 0; h < MGS_DPL; h++)
    if (lane + h * WAVE < NV) x[lane + h * WAVE] = acc.v[h];
  wsync();
}

// mujoco.pid actuator force (mgs_gpu.h d_actuator_pidprm; oracle pid_force):
// setpoint = the clamped ctrl, slew-limited against the previous setpoint (act
// entry 0 with slewmax), error = setpoint - length; force = kp error + kd
// (setpoint rate - velocity) + ki integral (the next act entry with ki != 0).
// The act rates for the step's advance go to act_dot (lane 0).  Restated from
// MuJoCo's documented plugin semantics; parity unpinned (its source is not here).
DEVI double pid_force(const Mdl& md, Dat& d, int u, double c, double len, double vel, int lane) {
  const double* pp = DA(md, actuator_pidprm) + 5 * u;
  const double dt = md.m.timestep;
  int k = IA(md, actuator_actadr)[u];
  double cdot = 0.0;
  if (pp[4] >= 0.0) {
    const double prev = d.act[k];
    const double lo = prev - pp[4] * dt, hi = prev + pp[4] * dt;
    if (c < lo) c = lo;
    if (c > hi) c = hi;
    cdot = (c - prev) / dt;
    if (lane == 0) d.act_dot[k] = cdot;
    k++;
  }
  const double err = c - len;
  double f = pp[0] * err + pp[2] * (cdot - vel);
  if (pp[1] != 0.0) {
    f = f + pp[1] * d.act[k];
    if (lane == 0) d.act_dot[k] = err;
  }
  return f;
}

// actuation (oracle actuation()), lanes over dofs: each lane builds its entry of
// every moment row (tendon wraps in order), the actuator length / velocity are
// the oracle's sequential sums evaluated uniformly, forces applied per dof.
DEVI void actuation(const Mdl& md, Dat& d) {
  int nv = md.m.nv, lane = lane_id();
  const int32_t *trntype = IA(md, actuator_trntype), *trnid = IA(md, actuator_trnid);
  const int32_t *gtype = IA(md, actuator_gaintype), *btype = IA(md, actuator_biastype);
  const int32_t *clim = IA(md, actuator_ctrllimited), *flim = IA(md, actuator_forcelimited);
  const double *gain = DA(md, actuator_gainprm), *bias = DA(md, actuator_biasprm);
  const double *crange = DA(md, actuator_ctrlrange), *frange = DA(md, actuator_forcerange);
  const double* gear = DA(md, actuator_gear);
  const int32_t *tadr = IA(md, tendon_adr), *tnum = IA(md, tendon_num);
  const int32_t *wdof = IA(md, wrap_dofid), *wq = IA(md, wrap_qposadr);
  const double* wcoef = DA(md, wrap_coef);
  const int32_t *jq = IA(md, jnt_qposadr), *jd = IA(md, jnt_dofadr);
  DofV qfa = dof_zero();
  for (int u = 0; u < md.m.nu; u++) {
#if MGS_PACKED
    // the wide build reads the moment rows from the model (joint and fixed-
    // tendon transmissions: constant; mgs_model_desc.d_actuator_moment, the
    // same sums formed on the host) instead of keeping nu x nv of them in LDS
    const double* mom = DA(md, actuator_moment) + u * nv;
    DofV m = dof_load(mom, nv, lane);
    double len;
    if (trntype[u] == MGS_TRN_JOINT) {
      len = d.qpos[jq[trnid[u]]] * gear[u];
    } else {
      int t = trnid[u];
      double tl = 0.0;
      for (int w = tadr[t]; w < tadr[t] + tnum[t]; w++) tl = tl + wcoef[w] * d.qpos[wq[w]];
      len = tl * gear[u];
    }
    (void)jd;
    (void)wdof;
#else
    static_assert(MGS_DPL == 1, "two dofs per lane read the moment rows from the model (MGS_PACKED)");
    double* mom = d.act_moment + u * nv;
    DofV m = dof_zero();
    double len;
    if (trntype[u] == MGS_TRN_JOINT) {
      int j = trnid[u];
      len = d.qpos[jq[j]] * gear[u];
      if (lane == jd[j]) m.v[0] = gear[u];
    } else {
      int t = trnid[u];
      double tl = 0.0;
      for (int w = tadr[t]; w < tadr[t] + tnum[t]; w++) {
        tl = tl + wcoef[w] * d.qpos[wq[w]];
        if (lane == wdof[w]) m.v[0] = m.v[0] + wcoef[w] * gear[u];
      }
      len = tl * gear[u];
    }
    if (lane < nv) mom[lane] = m.v[0];
    wsync();
#endif
    double vel = 0.0;
    for (int k = 0; k < nv; k++) vel = vel + mom[k] * d.qvel[k];
    double c = d.ctrl[u];
    if (clim[u]) {
      if (c < crange[2 * u]) c = crange[2 * u];
      if (c > crange[2 * u + 1]) c = crange[2 * u + 1];
    }
    double f;
    if (md.m.npid > 0 && gtype[u] == MGS_GAIN_PID) {
      f = pid_force(md, d, u, c, len, vel, lane);
    } else {
      double g = gain[3 * u];
      if (gtype[u] == MGS_GAIN_AFFINE) g = (gain[3 * u] + gain[3 * u + 1] * len) + gain[3 * u + 2] * vel;
      f = g * c;
      if (btype[u] == MGS_BIAS_AFFINE) f = f + ((bias[3 * u] + bias[3 * u + 1] * len) + bias[3 * u + 2] * vel);
    }
    if (flim[u]) {
      if (f < frange[2 * u]) f = frange[2 * u];
      if (f > frange[2 * u + 1]) f = frange[2 * u + 1];
    }
    if (lane == 0) { d.act_length[u] = len; d.act_vel[u] = vel; d.act_force[u] = f; }
#pragma unroll
    for (int h = 0; h < MGS_DPL; h++) qfa.v[h] = qfa.v[h] + m.v[h] * f;
  }
#pragma unroll
  for (int h = 0; h < MGS_DPL; h++)
    if (lane + h * WAVE < nv) d.qfrc_actuator[lane + h * WAVE] = qfa.v[h];
}

// passive forces (oracle passive()), one dof per lane
DEVI void passive(const Mdl& md, Dat& d) {
  const int32_t *jtype = IA(md, jnt_type), *jq = IA(md, jnt_qposadr), *djnt = IA(md, dof_jntid);
  const double *stiff = DA(md, jnt_stiffness), *qspring = DA(md, qpos_spring), *damp = DA(md, dof_damping);
  const int lane = lane_id();
#pragma unroll
  for (int h = 0; h < MGS_DPL; h++) {
    const int i = lane + h * WAVE;   // this slot's dof
    if (i >= md.m.nv) continue;
    int j = djnt[i];
    double v = 0.0;
    if (stiff[j] != 0.0 && (jtype[j] == MGS_JNT_HINGE || jtype[j] == MGS_JNT_SLIDE))
      v = -stiff[j] * (d.qpos[jq[j]] - qspring[jq[j]]);
    v = v - damp[i] * d.qvel[i];
    // gravity compensation (oracle passive(): MuJoCo mj_gravcomp with the
    // force's moment arm from cinert, bodies in order)
    const double* g = md.m.gravity;
    if (g[0] != 0.0 || g[1] != 0.0 || g[2] != 0.0) {
      const double* gc = DA(md, body_gravcomp);
      double acc = 0.0;
      int any = 0;
      for (int b = 1; b < md.m.nbody; b++) {
        if (gc[b] == 0.0) continue;
        if (!dof_moves(md, b, i)) continue;
        const double* ci = d.cinert + 10 * b;
        const double* cd = d.cdof + 6 * i;
        double cr[3];
        cross3(cr, cd, ci + 6);
        double t = ((g[0] * cd[3] + g[1] * cd[4]) + g[2] * cd[5]) * ci[9] + ((g[0] * cr[0] + g[1] * cr[1]) + g[2] * cr[2]);
        acc = acc + (-gc[b]) * t;
        any = 1;
      }
      if (any) v = v + acc;
    }
    d.qfrc_passive[i] = v;
  }
}

// recursive Newton-Euler bias forces (oracle rne()): forward velocity /
// acceleration pass by tree level (lane per body), cfrc accumulated up the tree
// in the oracle's child order, then one dof per lane.
// p, nd, da: the body's parent, dof count and first dof (preloaded by rne)
DEVI void rne_body(Dat& d, int b, int p, int nd, int da) {
  double cv[6], ca[6];
  for (int k = 0; k < 6; k++) { cv[k] = d.cvel[6 * p + k]; ca[k] = d.cacc[6 * p + k]; }
  for (int i = 0; i < nd; i++) {
    int dd = da + i;
    cross_motion(d.cdof_dot + 6 * dd, cv, d.cdof + 6 * dd);
    for (int k = 0; k < 6; k++) cv[k] = cv[k] + d.cdof[6 * dd + k] * d.qvel[dd];
  }
  for (int i = 0; i < nd; i++) {
    int dd = da + i;
    for (int k = 0; k < 6; k++) ca[k] = ca[k] + d.cdof_dot[6 * dd + k] * d.qvel[dd];
  }
  for (int k = 0; k < 6; k++) { d.cvel[6 * b + k] = cv[k]; d.cacc[6 * b + k] = ca[k]; }
  double f1[6], f2[6], f3[6];
  mul_inert_vec(f1, d.cinert + 10 * b, ca);
  mul_inert_vec(f2, d.cinert + 10 * b, cv);
  cross_force(f3, cv, f2);
  for (int k = 0; k < 6; k++) d.cfrc[6 * b + k] = f1[k] + f3[k];
}

DEVI void rne(const Mdl& md, Dat& d) {
  int lane = lane_id(), nb = md.m.nbody;
  const int32_t *dbody = IA(md, dof_bodyid), *depth = IA(md, body_depth);
  if (lane == 0) {
    for (int k = 0; k < 6; k++) { d.cvel[k] = 0.0; d.cacc[k] = 0.0; }
    d.cacc[3] = -md.m.gravity[0]; d.cacc[4] = -md.m.gravity[1]; d.cacc[5] = -md.m.gravity[2];
  }
  wsync();
  int maxd = max_depth(md);
  int lb = lane < nb ? lane : 0;
  int myd = (lane < nb) ? depth[lane] : -1;
  int bp = IA(md, body_parentid)[lb], bnd = IA(md, body_dofnum)[lb], bda = IA(md, body_dofadr)[lb];
  for (int L = 1; L <= maxd; L++) {
    if (myd == L) rne_body(d, lane, bp, bnd, bda);
    wsync();
  }
  accumulate_up<6>(md, d.cfrc, 0);
#pragma unroll
  for (int h = 0; h < MGS_DPL; h++) {
    const int i = lane + h * WAVE;
    if (i < md.m.nv) d.qfrc_bias[i] = dot6(d.cdof + 6 * i, d.cfrc + 6 * dbody[i]);
  }
  wsync();
}

// ---------------------------------------------------------------------------
// collision
struct SupPt { double v[3], a[3], b[3]; };

// wave-parallel support mapping (oracle support_geom()): argmax over hull
// vertices of v.dl, ties -> smallest index.  Lanes stride the vertices and keep
// their best vertex in registers; the (value, index) pair is reduced with DPP
// inside each 16-lane row (max with index tie-break is order independent), the
// four row winners are combined uniformly, and the winning vertex is read from
// its lane (index & 63) -- no shuffle through LDS, no dependent global reload.
struct SupAcc {
  double best, vx, vy, vz;
  int bi;
};
DEVI void sup_init(SupAcc& a) { a.best = -INFINITY; a.bi = 0x7fffffff; a.vx = a.vy = a.vz = 0.0; }
// reduce and return the winning local-frame vertex (uniform).  Only lanes
// < min(n, 64) hold candidates, so the reduction stops at the smallest power of
// two covering them (8-vertex boxes: three DPP levels).  The value alone is
// reduced (one v_max_f64 per DPP level; lane values are never NaN: they only
// change on a strict '>'), then the lanes holding it are found with a ballot
// and the smallest vertex index among them wins -- the (value, index) order of
// the oracle's ascending scan.  Lane l holds vertices l, l+64, ..., so for a
// hull of <= 64 vertices the lowest tied lane is the answer; larger hulls
// compare the tied lanes' indices (exact ties only).
// v_max_f64 without the operand canonicalisation __builtin_fmax adds (two
// extra v_max per use): the support values are never signalling NaNs (they
// come from arithmetic), for which both give the same result.  The s_nop
// covers the VALU-write -> DPP-read wait states of the next reduction level
// (the hazard recognizer does not look into inline asm).
DEVI double max_f64(double a, double b) {
  double r;
  asm("v_max_f64 %0, %1, %2\n\ts_nop 1" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
DEVI void sup_finish(SupAcc& a, double* v, int n) {
  int P = n < WAVE ? next_pow2(n) : WAVE;
  double m = a.best;
  if (P > 1) m = max_f64(m, dpp_d(m, 0));
  if (P > 2) m = max_f64(m, dpp_d(m, 1));
  if (P > 4) m = max_f64(m, dpp_d(m, 2));
  if (P > 8) m = max_f64(m, dpp_d(m, 3));
  double M = readlane_d(m, 0);
  if (P > 16) {
    M = max_f64(M, readlane_d(m, 16));
    if (P > 32) {
      M = max_f64(M, readlane_d(m, 32));
      M = max_f64(M, readlane_d(m, 48));
    }
  }
  unsigned long long tied = __ballot(a.bi != 0x7fffffff && a.best == M);
  int bi = 0;
  if (tied) {
    int l = __ffsll((long long)tied) - 1;
    bi = __builtin_amdgcn_readlane(a.bi, l);
    if (n > WAVE) {
      tied &= tied - 1ull;
      while (tied) {
        int l2 = __ffsll((long long)tied) - 1;
        tied &= tied - 1ull;
        int b2 = __builtin_amdgcn_readlane(a.bi, l2);
        if (b2 < bi) bi = b2;
      }
    }
  }
  int wl = bi & (WAVE - 1);
  v[0] = readlane_d(a.vx, wl);
  v[1] = readlane_d(a.vy, wl);
  v[2] = readlane_d(a.vz, wl);
  a.bi = bi;
}

// Per-pair narrowphase context: both geoms' poses in registers (uniform) and,
// for hulls of at most 64 vertices, this lane's vertex (lane i holds vertex i)
// so the support mappings of a small hull never touch memory.
struct PairCtx {
  int n1, n2;
  const double *V1, *V2;
  double R1[9], R2[9], x1[3], x2[3];
  double c1[3], c2[3];
  double r1, r2;   // rounding radii (sphere / capsule: hull (+) ball), 0 for hulls
  double cy1[2], cy2[2];   // cylinder radius / half-height (exact solid), 0 0 for others
};
// the context with the geoms' poses read from R1 / x1 / R2 / x2 (LDS)
DEVI void pair_ctx_pose(const Mdl& md, int g1, int g2, const double* R1, const double* x1, const double* R2,
                        const double* x2, PairCtx& c) {
  int lane = lane_id();
  const int32_t *ghull = IA(md, geom_hullid), *hadr = IA(md, hull_vertadr), *hnum = IA(md, hull_vertnum);
  int h1 = ghull[g1], h2 = ghull[g2];
  c.n1 = hnum[h1];
  c.n2 = hnum[h2];
  c.V1 = DA(md, hull_vert) + 3 * hadr[h1];
  c.V2 = DA(md, hull_vert) + 3 * hadr[h2];
  for (int k = 0; k < 9; k++) { c.R1[k] = R1[k]; c.R2[k] = R2[k]; }
  for (int k = 0; k < 3; k++) { c.x1[k] = x1[k]; c.x2[k] = x2[k]; }
  int i1 = (lane < c.n1) ? lane : 0, i2 = (lane < c.n2) ? lane : 0;
  for (int k = 0; k < 3; k++) { c.c1[k] = c.V1[k * c.n1 + i1]; c.c2[k] = c.V2[k * c.n2 + i2]; }
  c.r1 = DA(md, geom_radius)[g1];
  c.r2 = DA(md, geom_radius)[g2];
  const double* cy = DA(md, geom_cyl);
  c.cy1[0] = cy[2 * g1]; c.cy1[1] = cy[2 * g1 + 1];
  c.cy2[0] = cy[2 * g2]; c.cy2[1] = cy[2 * g2 + 1];
}
DEVI void pair_ctx(const Mdl& md, const Dat& d, int g1, int g2, PairCtx& c) {
  pair_ctx_pose(md, g1, g2, d.geom_xmat + 9 * g1, d.geom_xpos + 3 * g1, d.geom_xmat + 9 * g2, d.geom_xpos + 3 * g2, c);
}

// exact cylinder support in the geom frame (oracle cyl_support; MuJoCo's ccd
// support of mjGEOM_CYLINDER): the rim point along dl's radial part on the cap
// dl points to, (0, 0, +-h) along the axis; dl is uniform, so is the result
DEVI void cyl_support(double* v, const double* cy, const double* dl) {
  // MuJoCo's operation order (dir / length * size) and mju_sign (0 at 0)
  double rho = sqrt(dl[0] * dl[0] + dl[1] * dl[1]);
  if (rho > K_MINVAL) {
    v[0] = dl[0] / rho * cy[0];
    v[1] = dl[1] / rho * cy[0];
  } else {
    v[0] = 0.0;
    v[1] = 0.0;
  }
  v[2] = dl[2] > 0.0 ? cy[1] : (dl[2] < 0.0 ? -cy[1] : 0.0);
}

DEVI void sup_cached(SupAcc& a, int n, const double* cached, const double* dl) {
  int lane = lane_id();
  if (lane < n) {
    double sc = (cached[0] * dl[0] + cached[1] * dl[1]) + cached[2] * dl[2];
    if (sc > a.best) { a.best = sc; a.bi = lane; a.vx = cached[0]; a.vy = cached[1]; a.vz = cached[2]; }
  }
}
// vertices [base, base + SUP_CH * 64) of a large hull: every load issued before
// the first compare, so a round costs one memory latency, not one per vertex
// stride; each lane still visits its vertices in ascending order (strict >,
// ties keep the smaller index)
#define SUP_CH 4
struct SupChunk { double x[SUP_CH], y[SUP_CH], z[SUP_CH]; };
DEVI void sup_load(SupChunk& c, const double* V, int n, int base) {
  int lane = lane_id();
#pragma unroll
  for (int u = 0; u < SUP_CH; u++) {
    int i = base + u * WAVE + lane;
    int ii = i < n ? i : 0;
    c.x[u] = V[ii]; c.y[u] = V[n + ii]; c.z[u] = V[2 * n + ii];
  }
}
DEVI void sup_take_chunk(SupAcc& a, const SupChunk& c, int n, int base, const double* dl) {
  int lane = lane_id();
#pragma unroll
  for (int u = 0; u < SUP_CH; u++) {
    int i = base + u * WAVE + lane;
    double sc = (c.x[u] * dl[0] + c.y[u] * dl[1]) + c.z[u] * dl[2];
    if (i < n && sc > a.best) { a.best = sc; a.bi = i; a.vx = c.x[u]; a.vy = c.y[u]; a.vz = c.z[u]; }
  }
}

// supports of g1 along dir and g2 along -dir (world frame), oracle support_geom()
DEVI void support_pair(const PairCtx& c, const double* dir, double* out1, double* out2) {
  double nd[3] = {-dir[0], -dir[1], -dir[2]};
  double dl1[3], dl2[3];
  mulmtv3(dl1, c.R1, dir);
  mulmtv3(dl2, c.R2, nd);
  SupAcc a1, a2;
  sup_init(a1);
  sup_init(a2);
  if (c.n1 <= WAVE) sup_cached(a1, c.n1, c.c1, dl1);
  if (c.n2 <= WAVE) sup_cached(a2, c.n2, c.c2, dl2);
  int big1 = c.n1 > WAVE, big2 = c.n2 > WAVE;
  if (big1 | big2) {
    int nmax = big1 ? c.n1 : 0;
    if (big2 && c.n2 > nmax) nmax = c.n2;
    for (int base = 0; base < nmax; base += SUP_CH * WAVE) {
      SupChunk k1, k2;
      int t1 = big1 && base < c.n1, t2 = big2 && base < c.n2;
      if (t1) sup_load(k1, c.V1, c.n1, base);
      if (t2) sup_load(k2, c.V2, c.n2, base);
      if (t1) sup_take_chunk(a1, k1, c.n1, base, dl1);
      if (t2) sup_take_chunk(a2, k2, c.n2, base, dl2);
    }
  }
  double v1[3], v2[3], t[3];
  sup_finish(a1, v1, c.n1);
  sup_finish(a2, v2, c.n2);
  if (c.cy1[0] > 0.0) cyl_support(v1, c.cy1, dl1);
  if (c.cy2[0] > 0.0) cyl_support(v2, c.cy2, dl2);
  mulmv3(t, c.R1, v1);
  add3(out1, c.x1, t);
  mulmv3(t, c.R2, v2);
  add3(out2, c.x2, t);
  // rounded geoms (oracle support_geom): + r * unit direction
  if (c.r1 > 0.0) { out1[0] = out1[0] + c.r1 * dir[0]; out1[1] = out1[1] + c.r1 * dir[1]; out1[2] = out1[2] + c.r1 * dir[2]; }
  if (c.r2 > 0.0) { out2[0] = out2[0] + c.r2 * nd[0]; out2[1] = out2[1] + c.r2 * nd[1]; out2[2] = out2[2] + c.r2 * nd[2]; }
}

DEVI void mink_support(const PairCtx& c, const double* dir, SupPt* p) {
  PT(4);
  PCNT(28, 1);
  PCNT(29, (c.n1 > WAVE) + (c.n2 > WAVE));
  support_pair(c, dir, p->a, p->b);
  sub3(p->v, p->a, p->b);
  if (c.n1 > WAVE || c.n2 > WAVE) PT(39); else PT(22);
}

// Two narrowphase pairs at once (collide_pair2): the MPR of pair A runs on
// lanes 0-31 and that of pair B on lanes 32-63, each half computing exactly
// what a whole wave computes for one pair (the MPR's control flow depends only
// on values that are uniform within a half).  The support mappings use one
// 16-lane row per hull: row 0 pair A's geom 1, row 1 A's geom 2, rows 2 / 3
// B's (lane 16 s + i of a half holds vertex i), so one row-local reduction
// serves all four hulls -- pairs whose four hulls have at most 16 vertices.
struct PairCtx2 {
  int n;               // this lane's hull: its vertex count,
  double R[9], x[3];   // its geom's pose,
  double c[3];         // the lane's vertex (lane & 15 < n)
  double r;            // and rounding radius
  int P;               // reduction width: next_pow2 of the largest of the four counts (<= 16)
};
DEVI void pair_ctx2(const Mdl& md, const Dat& d, int gA1, int gA2, int gB1, int gB2, PairCtx2& c) {
  const int lane = lane_id(), row = lane >> 4;
  const int32_t *ghull = IA(md, geom_hullid), *hadr = IA(md, hull_vertadr), *hnum = IA(md, hull_vertnum);
  const int g = row == 0 ? gA1 : (row == 1 ? gA2 : (row == 2 ? gB1 : gB2));
  const int h = ghull[g];
  c.n = hnum[h];
  const double* V = DA(md, hull_vert) + 3 * hadr[h];
#pragma unroll
  for (int k = 0; k < 9; k++) c.R[k] = d.geom_xmat[9 * g + k];
#pragma unroll
  for (int k = 0; k < 3; k++) c.x[k] = d.geom_xpos[3 * g + k];
  const int li = lane & 15, i = li < c.n ? li : 0;
#pragma unroll
  for (int k = 0; k < 3; k++) c.c[k] = V[k * c.n + i];
  c.r = DA(md, geom_radius)[g];
  int nm = __builtin_amdgcn_readlane(c.n, 0);
  int t = __builtin_amdgcn_readlane(c.n, 16);
  nm = t > nm ? t : nm;
  t = __builtin_amdgcn_readlane(c.n, 32);
  nm = t > nm ? t : nm;
  t = __builtin_amdgcn_readlane(c.n, 48);
  nm = t > nm ? t : nm;
  c.P = next_pow2(nm);
}

// support_pair for both pairs: the oracle's support_geom per hull (same
// expressions as sup_cached / sup_finish / support_pair), dir per half
DEVI void support_pair2(const PairCtx2& c, const double* dir, double* out1, double* out2) {
  const int lane = lane_id(), row = lane >> 4, li = lane & 15;
  const bool second = row & 1;    // geom 2 of the pair: support along -dir
  double sd[3] = {second ? -dir[0] : dir[0], second ? -dir[1] : dir[1], second ? -dir[2] : dir[2]};
  double dl[3];
  mulmtv3(dl, c.R, sd);
  SupAcc a;
  sup_init(a);
  if (li < c.n) {
    double sc = (c.c[0] * dl[0] + c.c[1] * dl[1]) + c.c[2] * dl[2];
    if (sc > a.best) { a.best = sc; a.bi = li; a.vx = c.c[0]; a.vy = c.c[1]; a.vz = c.c[2]; }
  }
  const int P = c.P;
  double m = a.best;
  if (P > 1) m = max_f64(m, dpp_d(m, 0));
  if (P > 2) m = max_f64(m, dpp_d(m, 1));
  if (P > 4) m = max_f64(m, dpp_d(m, 2));
  if (P > 8) m = max_f64(m, dpp_d(m, 3));
  const double M0 = readlane_d(m, 0), M1 = readlane_d(m, 16), M2 = readlane_d(m, 32), M3 = readlane_d(m, 48);
  const double M = row == 0 ? M0 : (row == 1 ? M1 : (row == 2 ? M2 : M3));
  const unsigned long long tied = __ballot(a.bi != 0x7fffffff && a.best == M);
  // each row's winner: its lowest tied lane (none: the row's first lane, as
  // sup_finish falls back to lane 0)
  int w[4];
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const unsigned tr = (unsigned)(tied >> (16 * q)) & 0xffffu;
    w[q] = 16 * q + (tr ? __ffs(tr) - 1 : 0);
  }
  const int src = row == 0 ? w[0] : (row == 1 ? w[1] : (row == 2 ? w[2] : w[3]));
  double v[3] = {shfl(a.vx, src), shfl(a.vy, src), shfl(a.vz, src)};
  double t[3], wv[3];
  mulmv3(t, c.R, v);
  add3(wv, c.x, t);
  if (c.r > 0.0) { wv[0] = wv[0] + c.r * sd[0]; wv[1] = wv[1] + c.r * sd[1]; wv[2] = wv[2] + c.r * sd[2]; }
  const int s1 = lane & 32, s2 = s1 + 16;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    out1[k] = shfl(wv[k], s1);
    out2[k] = shfl(wv[k], s2);
  }
}

DEVI void mink_support(const PairCtx2& c, const double* dir, SupPt* p) {
  PT(4);
  PCNT(28, 1);
  support_pair2(c, dir, p->a, p->b);
  sub3(p->v, p->a, p->b);
  PT(22);
}

DEVI void portal_normal(double* n, const SupPt* p1, const SupPt* p2, const SupPt* p3) {
  double e1[3], e2[3];
  sub3(e1, p2->v, p1->v);
  sub3(e2, p3->v, p1->v);
  cross3(n, e1, e2);
  normalize3(n);
}
DEVI int portal_reach_tol(const SupPt* p1, const SupPt* p2, const SupPt* p3, const SupPt* p4,
                                const double* n, double tol) {
  double dv4 = dot3(p4->v, n);
  double t1 = dv4 - dot3(p1->v, n);
  double t2 = dv4 - dot3(p2->v, n);
  double t3 = dv4 - dot3(p3->v, n);
  double mn = t1 < t2 ? t1 : t2;
  mn = mn < t3 ? mn : t3;
  return mn <= tol;
}
// which portal vertex p4 replaces (1, 2 or 3); value semantics keep the
// support points in registers (pointer-selected stores spilled them to scratch)
DEVI int portal_choose(const SupPt& p0, const SupPt& p1, const SupPt& p2, const SupPt& p3, const SupPt& p4) {
  double c[3];
  cross3(c, p4.v, p0.v);
  if (dot3(p1.v, c) > 0.0) return (dot3(p2.v, c) > 0.0) ? 1 : 3;
  return (dot3(p3.v, c) > 0.0) ? 2 : 1;
}
#define PORTAL_EXPAND(p0, p1, p2, p3, p4)             \
  do {                                                \
    int _k = portal_choose(p0, p1, p2, p3, p4);       \
    if (_k == 1) p1 = p4;                             \
    else if (_k == 2) p2 = p4;                        \
    else p3 = p4;                                     \
  } while (0)

// On a miss that is certified by a separating direction (the support of the
// Minkowski difference along dir is <= 0), *cm = -h(dir) >= 0 and dir (the
// caller's array, the search direction throughout) is left at that unit world
// direction; else *cm = -1.  (dir is the caller's so that no exit path stores a
// copy of it: the compiler would merge those stores with the contact point's
// into one store through a selected pointer and keep both arrays in scratch.)
#define MPR_CERT(P) do { *cm = -dot3((P).v, dir); } while (0)
// (Ctx: PairCtx for one pair on the whole wave, PairCtx2 for two pairs on the
// two halves; g1 / g2 are then the half's geoms)
template <class Ctx>
DEVI int mpr_penetration(const Mdl& md, const Dat& d, const Ctx& pc, int g1, int g2, double* n, double* depth,
                         double* pos, double* dir, double* cm) {
  *cm = -1.0;
  const double tol = md.m.mpr_tolerance;
  const int32_t* ghull = IA(md, geom_hullid);
  const double* HC = DA(md, hull_center);
  SupPt p0, p1, p2, p3, p4;
  double t[3];
  mulmv3(t, d.geom_xmat + 9 * g1, HC + 3 * ghull[g1]);
  add3(p0.a, d.geom_xpos + 3 * g1, t);
  mulmv3(t, d.geom_xmat + 9 * g2, HC + 3 * ghull[g2]);
  add3(p0.b, d.geom_xpos + 3 * g2, t);
  sub3(p0.v, p0.a, p0.b);
  if (p0.v[0] == 0.0 && p0.v[1] == 0.0 && p0.v[2] == 0.0) p0.v[0] = 1e-9;
  dir[0] = -p0.v[0]; dir[1] = -p0.v[1]; dir[2] = -p0.v[2];
  normalize3(dir);
  mink_support(pc, dir, &p1);
  if (dot3(p1.v, dir) <= 0.0) { MPR_CERT(p1); return 0; }
  cross3(dir, p0.v, p1.v);
  if (dot3(dir, dir) < 1e-30) {
    double nn = sqrt(dot3(p1.v, p1.v));
    if (nn < K_MINVAL) return 0;
    n[0] = p1.v[0] / nn; n[1] = p1.v[1] / nn; n[2] = p1.v[2] / nn;
    *depth = nn;
    pos[0] = 0.5 * (p1.a[0] + p1.b[0]); pos[1] = 0.5 * (p1.a[1] + p1.b[1]); pos[2] = 0.5 * (p1.a[2] + p1.b[2]);
    return 1;
  }
  normalize3(dir);
  mink_support(pc, dir, &p2);
  if (dot3(p2.v, dir) <= 0.0) { MPR_CERT(p2); return 0; }
  {
    double e1[3], e2[3];
    sub3(e1, p1.v, p0.v);
    sub3(e2, p2.v, p0.v);
    cross3(dir, e1, e2);
    normalize3(dir);
  }
  if (dot3(dir, p0.v) > 0.0) {
    SupPt tmp = p1; p1 = p2; p2 = tmp;
    dir[0] = -dir[0]; dir[1] = -dir[1]; dir[2] = -dir[2];
  }
  int it;
  for (it = 0; it < K_MPR_MAXIT; it++) {
    mink_support(pc, dir, &p3);
    if (dot3(p3.v, dir) <= 0.0) { MPR_CERT(p3); return 0; }
    double c[3];
    int cont = 0;
    cross3(c, p1.v, p3.v);
    if (dot3(c, p0.v) < 0.0) { p2 = p3; cont = 1; }
    else {
      cross3(c, p3.v, p2.v);
      if (dot3(c, p0.v) < 0.0) { p1 = p3; cont = 1; }
    }
    if (!cont) break;
    double e1[3], e2[3];
    sub3(e1, p1.v, p0.v);
    sub3(e2, p2.v, p0.v);
    cross3(dir, e1, e2);
    normalize3(dir);
  }
  if (it == K_MPR_MAXIT) return 0;
  for (it = 0; it < K_MPR_MAXIT; it++) {
    portal_normal(dir, &p1, &p2, &p3);
    if (dot3(dir, p1.v) >= 0.0) break;
    mink_support(pc, dir, &p4);
    if (dot3(p4.v, dir) < 0.0) { MPR_CERT(p4); return 0; }
    if (portal_reach_tol(&p1, &p2, &p3, &p4, dir, tol)) return 0;
    PORTAL_EXPAND(p0, p1, p2, p3, p4);
  }
  if (it == K_MPR_MAXIT) return 0;
  for (it = 0;; it++) {
    portal_normal(dir, &p1, &p2, &p3);
    mink_support(pc, dir, &p4);
    if (it >= K_MPR_MAXIT || portal_reach_tol(&p1, &p2, &p3, &p4, dir, tol)) {
      double dep = dot3(dir, p1.v);
      if (!(dep > 0.0)) return 0;
      n[0] = dir[0]; n[1] = dir[1]; n[2] = dir[2];
      *depth = dep;
      double q[3] = {dir[0] * dep, dir[1] * dep, dir[2] * dep};
      double a1[3], a2[3], a3[3], c[3];
      sub3(a1, p1.v, q); sub3(a2, p2.v, q); sub3(a3, p3.v, q);
      cross3(c, a2, a3); double u1 = dot3(c, dir);
      cross3(c, a3, a1); double u2 = dot3(c, dir);
      cross3(c, a1, a2); double u3 = dot3(c, dir);
      double su = (u1 + u2) + u3;
      if (fabs(su) < 1e-30) { u1 = u2 = u3 = 1.0 / 3.0; }
      else { double inv = 1.0 / su; u1 = u1 * inv; u2 = u2 * inv; u3 = u3 * inv; }
#pragma unroll
      for (int k = 0; k < 3; k++) {
        double pa = (u1 * p1.a[k] + u2 * p2.a[k]) + u3 * p3.a[k];
        double pb = (u1 * p1.b[k] + u2 * p2.b[k]) + u3 * p3.b[k];
        pos[k] = 0.5 * (pa + pb);
      }
      return 1;
    }
    PORTAL_EXPAND(p0, p1, p2, p3, p4);
  }
}

#undef MPR_CERT

DEVI void make_frame(const double* n, double* t1, double* t2) {
  double a[3];
  /* mju_makeFrame: tangent seed (0,1,0) unless |n_y| >= 0.5, then (0,0,1) */
  if (n[1] < 0.5 && n[1] > -0.5) { a[0] = 0.0; a[1] = 1.0; a[2] = 0.0; }
  else { a[0] = 0.0; a[1] = 0.0; a[2] = 1.0; }
  double an = dot3(a, n);
  t1[0] = a[0] - n[0] * an; t1[1] = a[1] - n[1] * an; t1[2] = a[2] - n[2] * an;
  normalize3(t1);
  cross3(t2, n, t1);
}

// feature extraction: wave max over heights, then ballot compaction in vertex
// feature extraction on geom 1 or 2 of the pair (oracle feature()): extreme of
// the signed height along n over the hull (wave reduction sized to the hull),
// then, if collect, the vertices within tol of it, compacted with a ballot in
// vertex order (<= K_MAXF) into out[] (LDS).  Small hulls use the lane-cached
// vertex of the pair context.
DEVI int feature(const PairCtx& c, int which, const double* n, const double* t1, const double* t2, int sign,
                 double tol, int collect, P2* out, double* ext) {
  int lane = lane_id();
  const double* R = which == 1 ? c.R1 : c.R2;
  const double* x = which == 1 ? c.x1 : c.x2;
  const double* V = which == 1 ? c.V1 : c.V2;
  const double* cv = which == 1 ? c.c1 : c.c2;
  int num = which == 1 ? c.n1 : c.n2;
  double rr = which == 1 ? c.r1 : c.r2;
  const double* cy = which == 1 ? c.cy1 : c.cy2;
  double nl[3];
  mulmtv3(nl, R, n);
  double base = dot3(x, n);
  if (rr > 0.0) base = (sign > 0) ? base + rr : base - rr;   // rounded: surface = hull (+) ball
  // exact cylinder (oracle feature()): its rim polygons turned about the axis
  // so that vertex 0 of each cap is the true rim extreme along n; n along the
  // axis keeps the prism (a cap face).  The prism has 32 <= WAVE vertices, so
  // every vertex comes from the lane cache and is turned in registers
  const bool cyl = cy[0] > 0.0;
  double c0 = 1.0, s0 = 0.0;
  if (cyl) {
    double rho = sqrt(nl[0] * nl[0] + nl[1] * nl[1]);
    if (rho > K_MINVAL) {
      double sg = (sign > 0) ? 1.0 : -1.0;
      c0 = sg * (nl[0] / rho);
      s0 = sg * (nl[1] / rho);
    }
  }
  double cvx = cv[0], cvy = cv[1];
  if (cyl) { double tx = c0 * cvx - s0 * cvy; cvy = s0 * cvx + c0 * cvy; cvx = tx; }
  // the collecting pass takes the extreme its first pass computed (*ext): the
  // same expressions over the same vertices, so the same value
  double best = (sign > 0) ? -INFINITY : INFINITY;
  if (collect) {
    best = *ext;
  } else {
  if (num <= WAVE) {
    if (lane < num) best = base + ((cvx * nl[0] + cvy * nl[1]) + cv[2] * nl[2]);
  } else {
    for (int b0 = 0; b0 < num; b0 += SUP_CH * WAVE) {
      SupChunk k;
      sup_load(k, V, num, b0);
#pragma unroll
      for (int u = 0; u < SUP_CH; u++) {
        int i = b0 + u * WAVE + lane;
        double s = base + ((k.x[u] * nl[0] + k.y[u] * nl[1]) + k.z[u] * nl[2]);
        if (i < num && (sign > 0 ? (s > best) : (s < best))) best = s;
      }
    }
  }
  int P = num < WAVE ? next_pow2(num) : WAVE;
#pragma unroll
  for (int sel = 0; sel < 4; sel++) {
    if (P > (1 << sel)) {
      double ob = dpp_d(best, sel);
      if (sign > 0 ? (ob > best) : (ob < best)) best = ob;
    }
  }
  {
    double b0 = readlane_d(best, 0);
    if (P > 16) {
      double r1 = readlane_d(best, 16);
      if (sign > 0 ? (r1 > b0) : (r1 < b0)) b0 = r1;
      if (P > 32) {
        double r2 = readlane_d(best, 32), r3 = readlane_d(best, 48);
        if (sign > 0 ? (r2 > b0) : (r2 < b0)) b0 = r2;
        if (sign > 0 ? (r3 > b0) : (r3 < b0)) b0 = r3;
      }
    }
    best = b0;
  }
  *ext = best;
  return 0;
  }
  double lim = (sign > 0) ? best - tol : best + tol;
  int cnt = 0;
  for (int c0 = 0; c0 < num && cnt < K_MAXF; c0 += WAVE) {
    int i = c0 + lane;
    double s = 0.0, vx = 0.0, vy = 0.0, vz = 0.0;
    int pred = 0;
    if (i < num) {
      if (num <= WAVE) { vx = cvx; vy = cvy; vz = cv[2]; }
      else { vx = V[i]; vy = V[num + i]; vz = V[2 * num + i]; }
      s = base + ((vx * nl[0] + vy * nl[1]) + vz * nl[2]);
      pred = sign > 0 ? (s >= lim) : (s <= lim);
    }
    unsigned long long mask = __ballot(pred);
    int before = __popcll(mask & ((1ull << lane) - 1ull));
    int pos = cnt + before;
    if (pred && pos < K_MAXF) {
      double vv[3] = {vx, vy, vz}, t[3], Pw[3];
      mulmv3(t, R, vv);
      add3(Pw, x, t);
      out[pos].x = dot3(Pw, t1);
      out[pos].y = dot3(Pw, t2);
      out[pos].h = s;
    }
    cnt += __popcll(mask);
  }
  wsync();
  return cnt < K_MAXF ? cnt : K_MAXF;
}

DEVI double cross2(const P2* o, const P2* a, const P2* b) {
  return (a->x - o->x) * (b->y - o->y) - (a->y - o->y) * (b->x - o->x);
}

// monotone-chain half of hull2d on points already sorted and deduplicated
DEVI int hull_chain(const P2* pts, int n, P2* out) {
  if (n <= 2) {
    for (int i = 0; i < n; i++) out[i] = pts[i];
    return n;
  }
  int k = 0;
  for (int i = 0; i < n; i++) {
    while (k >= 2 && cross2(&out[k - 2], &out[k - 1], &pts[i]) <= 0.0) k--;
    out[k++] = pts[i];
  }
  int lo = k + 1;
  for (int i = n - 2; i >= 0; i--) {
    while (k >= lo && cross2(&out[k - 2], &out[k - 1], &pts[i]) <= 0.0) k--;
    out[k++] = pts[i];
  }
  return k - 1;
}

// hull_chain with the stack held across lanes (lane k keeps out[k] in
// registers) and the points broadcast from their lanes: the same pushes, pops
// and cross2 tests as the sequential loop, in the same order, but every access
// is a readlane instead of a dependent LDS round trip.  All lanes run it
// (uniform k); n <= K_MAXF, so the stack (< 2n entries) fits one wave.
DEVI int hull_chain_wave(const P2* pts, int n, P2* out) {
  int lane = lane_id();
  P2 me;
  me.x = me.y = me.h = 0.0;
  if (lane < n) me = pts[lane];
  if (n <= 2) {
    if (lane < n) out[lane] = me;
    return n;
  }
  P2 st;
  st.x = st.y = st.h = 0.0;
  int k = 0;
  for (int i = 0; i < n; i++) {
    P2 b;
    b.x = readlane_d(me.x, i); b.y = readlane_d(me.y, i); b.h = readlane_d(me.h, i);
    while (k >= 2) {
      P2 o, a;
      o.x = readlane_d(st.x, k - 2); o.y = readlane_d(st.y, k - 2);
      a.x = readlane_d(st.x, k - 1); a.y = readlane_d(st.y, k - 1);
      if (cross2(&o, &a, &b) <= 0.0) k--;
      else break;
    }
    if (lane == k) st = b;
    k++;
  }
  int lo = k + 1;
  for (int i = n - 2; i >= 0; i--) {
    P2 b;
    b.x = readlane_d(me.x, i); b.y = readlane_d(me.y, i); b.h = readlane_d(me.h, i);
    while (k >= lo) {
      P2 o, a;
      o.x = readlane_d(st.x, k - 2); o.y = readlane_d(st.y, k - 2);
      a.x = readlane_d(st.x, k - 1); a.y = readlane_d(st.y, k - 1);
      if (cross2(&o, &a, &b) <= 0.0) k--;
      else break;
    }
    if (lane == k) st = b;
    k++;
  }
  if (lane < k) out[lane] = st;
  return k - 1;
}

// hull2d's stable (x, y) insertion sort and duplicate removal, across lanes:
// lane i ranks point i against all n (ties by index: the stable order),
// scatters it, then keeps the first of each run of equal (x, y) with a ballot
// compaction -- the same array the sequential code leaves.  Returns the count
// (uniform), or -1 when a coordinate is NaN (the caller then runs hull2d).
DEVI int sort_dedup_wave(P2* pts, int n) {
  int lane = lane_id();
  P2 me;
  me.x = me.y = me.h = 0.0;
  if (lane < n) me = pts[lane];
  if (__ballot(lane < n && (me.x != me.x || me.y != me.y))) return -1;
  int rank = 0;
  for (int j = 0; j < n; j++) {
    double xj = readlane_d(me.x, j), yj = readlane_d(me.y, j);
    int before = (xj < me.x) || (xj == me.x && (yj < me.y || (yj == me.y && j < lane)));
    rank += before;
  }
  wsync();
  if (lane < n) pts[rank] = me;
  wsync();
  P2 cur, prv;
  cur.x = cur.y = cur.h = 0.0;
  prv = cur;
  if (lane < n) cur = pts[lane];
  if (lane > 0 && lane < n) prv = pts[lane - 1];
  int keep = lane < n && (lane == 0 || cur.x != prv.x || cur.y != prv.y);
  unsigned long long mk = __ballot(keep);
  unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (WAVE - lane));
  int pos = __popcll(mk & lt);
  wsync();
  if (keep) pts[pos] = cur;
  wsync();
  return __popcll(mk);
}

DEVI int hull2d(P2* pts, int n, P2* out) {
  for (int i = 1; i < n; i++) {
    P2 key = pts[i];
    int j = i - 1;
    while (j >= 0 && (pts[j].x > key.x || (pts[j].x == key.x && pts[j].y > key.y))) {
      pts[j + 1] = pts[j];
      j--;
    }
    pts[j + 1] = key;
  }
  int m = 0;
  for (int i = 0; i < n; i++)
    if (m == 0 || pts[i].x != pts[m - 1].x || pts[i].y != pts[m - 1].y) pts[m++] = pts[i];
  return hull_chain(pts, m, out);
}

DEVI P2 lerp2(const P2* a, const P2* b, double t) {
  P2 r;
  r.x = a->x + t * (b->x - a->x);
  r.y = a->y + t * (b->y - a->y);
  r.h = a->h + t * (b->h - a->h);
  return r;
}

DEVI int clip_poly(const P2* P, int np, P2* Q, int nq, P2* buf) {
  if (nq == 1) {
    for (int e = 0; e < np; e++) {
      const P2* a = &P[e];
      const P2* b = &P[(e + 1) % np];
      if (cross2(a, b, &Q[0]) < 0.0) return 0;
    }
    return 1;
  }
  if (nq == 2) {
    double t0 = 0.0, t1 = 1.0;
    for (int e = 0; e < np; e++) {
      const P2* a = &P[e];
      const P2* b = &P[(e + 1) % np];
      double d0 = cross2(a, b, &Q[0]);
      double d1 = cross2(a, b, &Q[1]);
      if (d0 < 0.0 && d1 < 0.0) return 0;
      if (d0 < 0.0) { double t = d0 / (d0 - d1); if (t > t0) t0 = t; }
      else if (d1 < 0.0) { double t = d0 / (d0 - d1); if (t < t1) t1 = t; }
    }
    if (t0 > t1) return 0;
    P2 a = lerp2(&Q[0], &Q[1], t0);
    P2 b = lerp2(&Q[0], &Q[1], t1);
    Q[0] = a; Q[1] = b;
    return 2;
  }
  for (int e = 0; e < np && nq > 0; e++) {
    const P2* a = &P[e];
    const P2* b = &P[(e + 1) % np];
    int no = 0;
    for (int i = 0; i < nq; i++) {
      const P2* cur = &Q[i];
      const P2* prv = &Q[(i + nq - 1) % nq];
      double dc = cross2(a, b, cur);
      double dp = cross2(a, b, prv);
      if (dc >= 0.0) {
        if (dp < 0.0 && no < K_MAXPOLY) buf[no++] = lerp2(prv, cur, dp / (dp - dc));
        if (no < K_MAXPOLY) buf[no++] = *cur;
      } else if (dp >= 0.0) {
        if (no < K_MAXPOLY) buf[no++] = lerp2(prv, cur, dp / (dp - dc));
      }
    }
    for (int i = 0; i < no; i++) Q[i] = buf[i];
    nq = no;
  }
  return nq;
}

// clip_poly across lanes (lanes over the clipped polygon's vertices, np
// reference edges in order): per edge each vertex emits the entry intersection
// and / or itself exactly as the sequential pass does, a ballot prefix places
// them, points past K_MAXPOLY are dropped as there.  Degenerate subjects (1 or
// 2 points) run the sequential code on lane 0.  Returns the count (uniform).
DEVI int clip_poly_wave(const P2* P, int np, P2* Q, int nq, P2* buf) {
  int lane = lane_id();
  if (nq <= 2) {
    int r = 0;
    if (lane == 0) r = clip_poly(P, np, Q, nq, buf);
    r = shfl(r, 0);
    wsync();
    return r;
  }
  unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (WAVE - lane));
  // the reference polygon across lanes (np <= K_MAXPOLY < WAVE): its edges are
  // readlane broadcasts; the clipped polygon stays in registers (cur, prv)
  // between edges and only the compaction goes through LDS, ping-ponging
  // between buf and Q
  P2 pe;
  pe.x = pe.y = pe.h = 0.0;
  if (lane < np) pe = P[lane];
  P2 cur, prv;
  cur.x = cur.y = cur.h = 0.0;
  prv = cur;
  if (lane < nq) {
    cur = Q[lane];
    prv = Q[(lane + nq - 1) % nq];
  }
  P2* out = buf;
  for (int e = 0; e < np && nq > 0; e++) {
    int en = (e + 1) % np;
    P2 a, b;
    a.x = readlane_d(pe.x, e); a.y = readlane_d(pe.y, e); a.h = 0.0;
    b.x = readlane_d(pe.x, en); b.y = readlane_d(pe.y, en); b.h = 0.0;
    double dc = cross2(&a, &b, &cur);
    double dp = cross2(&a, &b, &prv);
    int e1 = lane < nq && ((dc >= 0.0 && dp < 0.0) || (dc < 0.0 && dp >= 0.0));
    int e2 = lane < nq && dc >= 0.0;
    unsigned long long m1 = __ballot(e1), m2 = __ballot(e2);
    int pos = __popcll(m1 & lt) + __popcll(m2 & lt);
    int total = __popcll(m1) + __popcll(m2);
    // out was last read two edges ago, before the previous edge's barrier
    if (e1 && pos < K_MAXPOLY) out[pos] = lerp2(&prv, &cur, dp / (dp - dc));
    if (e2 && pos + e1 < K_MAXPOLY) out[pos + e1] = cur;
    nq = total < K_MAXPOLY ? total : K_MAXPOLY;
    wsync();
    if (lane < nq) {
      cur = out[lane];
      prv = out[(lane + nq - 1) % nq];
    }
    out = (out == buf) ? Q : buf;
  }
  if (out == Q) {   // the last compaction went to buf: the caller reads Q
    wsync();
    if (lane < nq) Q[lane] = cur;
  }
  wsync();
  return nq;
}

DEVI double dist2d(const P2* a, const P2* b) {
  double dx = a->x - b->x, dy = a->y - b->y;
  return dx * dx + dy * dy;
}

// keep <= 4 of np manifold points (oracle select4): the deepest, the farthest
// from it, the one spanning the largest triangle with those, the one farthest
// from all three
DEVI void select4(const P2* pts, const double* dep, int np, int* sel, int* ns) {
  if (np <= 4) {
    for (int i = 0; i < np; i++) sel[i] = i;
    *ns = np;
    return;
  }
  int i0 = 0;
  for (int i = 1; i < np; i++) if (dep[i] > dep[i0]) i0 = i;
  int i1 = -1; double bd = -1.0;
  for (int i = 0; i < np; i++) { if (i == i0) continue; double v = dist2d(&pts[i], &pts[i0]); if (v > bd) { bd = v; i1 = i; } }
  int i2 = -1; bd = -1.0;
  for (int i = 0; i < np; i++) {
    if (i == i0 || i == i1) continue;
    double v = fabs(cross2(&pts[i0], &pts[i1], &pts[i]));
    if (v > bd) { bd = v; i2 = i; }
  }
  int i3 = -1; bd = -1.0;
  for (int i = 0; i < np; i++) {
    if (i == i0 || i == i1 || i == i2) continue;
    double v0 = dist2d(&pts[i], &pts[i0]), v1 = dist2d(&pts[i], &pts[i1]), v2 = dist2d(&pts[i], &pts[i2]);
    double v = v0 < v1 ? v0 : v1;
    v = v < v2 ? v : v2;
    if (v > bd) { bd = v; i3 = i; }
  }
  sel[0] = i0; sel[1] = i1; sel[2] = i2; sel[3] = i3;
  *ns = 4;
}

DEVI void add_contact(Dat& d, int ncon_max, int pair, int g1, int g2, const double* pos, const double* n,
                            const double* t1, const double* t2, double dist) {
  if (d.NCON >= ncon_max) { d.OVERFLOW |= 1; return; }
  int c = d.NCON++;
  d.con_pos[3 * c] = pos[0]; d.con_pos[3 * c + 1] = pos[1]; d.con_pos[3 * c + 2] = pos[2];
  double* f = d.con_frame + 9 * c;
  f[0] = n[0]; f[1] = n[1]; f[2] = n[2];
  f[3] = t1[0]; f[4] = t1[1]; f[5] = t1[2];
  f[6] = t2[0]; f[7] = t2[1]; f[8] = t2[2];
  d.con_dist[c] = dist;
  d.con_pair[c] = pair;
  d.con_g1[c] = g1;
  d.con_g2[c] = g2;
}

// ---------------------------------------------------------------------------
// Separation certificates (oracle cert_*).  A convex pair whose MPR missed
// with a separating direction d (world, unit) -- the Minkowski difference
// g1 - g2 has support -m < 0 along d -- stays separated while the motion of g1
// relative to g2 cannot close the margin: in g2's frame the supports of g2 do
// not change and those of g1 along d_B (d in g2's frame) grow by at most
// d_B . dp + ||dR||_F rho_1 (dp, dR: change of g1's origin and rotation in
// g2's frame since the certifying step, rho_1 the largest vertex norm of g1's
// hull; a rounding ball adds the same term before and after).  A certified pair
// is skipped by the narrowphase: MPR would miss it again, so the contacts are
// the ones MuJoCo finds.  Slot (CERT_W doubles): pair, m, d_B (3), g1's origin
// (3) and rotation (9) in g2's frame at the certifying step; pair -1 = free.
DEVI void rel_pose(const Dat& d, int g1, int g2, double* p, double* R) {
  const double *R1 = d.geom_xmat + 9 * g1, *R2 = d.geom_xmat + 9 * g2;
  double dx[3];
  sub3(dx, d.geom_xpos + 3 * g1, d.geom_xpos + 3 * g2);
  mulmtv3(p, R2, dx);
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) R[3 * i + j] = (R2[i] * R1[j] + R2[3 + i] * R1[3 + j]) + R2[6 + i] * R1[6 + j];
}

DEVI int cert_ok(const Mdl& md, const Dat& d, const double* c) {
  int pair = (int)c[0];
  int g1 = IA(md, pair_geom1)[pair], g2 = IA(md, pair_geom2)[pair];
  double p[3], R[9], dp[3];
  rel_pose(d, g1, g2, p, R);
  sub3(dp, p, c + 5);
  double f = 0.0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
    double e = R[k] - c[8 + k];
    f = f + e * e;
  }
  double grow = dot3(c + 2, dp) + sqrt(f) * DA(md, geom_rbound)[g1];
  return c[1] - grow > CERT_EPS;
}

// before a pair chunk's narrowphase (lanes < K_CERT over the slots): slots of
// the chunk's pairs that left the broadphase set are freed, the others tested;
// returns the chunk bits of the certified pairs
DEVI unsigned long long cert_check(const Mdl& md, Dat& d, int c0, unsigned long long ov) {
  int lane = lane_id();
  int ok = 0, bit = 0;
  if (lane < K_CERT) {
    double* c = d.cert + CERT_W * lane;
    int pr = (int)c[0];
    if (pr >= c0 && pr < c0 + WAVE) {
      bit = pr - c0;
      if (!((ov >> bit) & 1ull)) c[0] = -1.0;
      else ok = cert_ok(md, d, c);
    }
  }
  unsigned long long okm = __ballot(ok), skip = 0ull;
  while (okm) {
    int l = __ffsll((long long)okm) - 1;
    okm &= okm - 1ull;
    skip |= 1ull << __builtin_amdgcn_readlane(bit, l);
  }
  wsync();
  PCNT(58, __popcll(skip));
#ifdef MGS_NO_CERT
  skip = 0ull;      // A/B experiments: certificates kept but not used
#endif
  return skip;
}

// after a convex pair's MPR: a certified miss (margin > CERT_STORE) goes to
// the pair's slot or the first free one; a hit or an uncertified miss frees the
// pair's slot
DEVI void cert_update(const Mdl& md, Dat& d, int pair, int g1, int g2, int hit, const double* cd, double cm) {
  int lane = lane_id();
  int pr = lane < K_CERT ? (int)d.cert[CERT_W * lane] : 0;
  unsigned long long mine = __ballot(lane < K_CERT && pr == pair);
  unsigned long long freem = __ballot(lane < K_CERT && pr < 0);
  int keep = !hit && cm > CERT_STORE;
  int sl = mine ? __ffsll((long long)mine) - 1 : ((keep && freem) ? __ffsll((long long)freem) - 1 : -1);
  if (sl < 0) return;
  wsync();
  if (lane == 0) {
    double* c = d.cert + CERT_W * sl;
    if (!keep) {
      c[0] = -1.0;
    } else {
      double p[3], R[9], db[3];
      rel_pose(d, g1, g2, p, R);
      mulmtv3(db, d.geom_xmat + 9 * g2, cd);
      c[0] = (double)pair;
      c[1] = cm;
      c[2] = db[0]; c[3] = db[1]; c[4] = db[2];
      c[5] = p[0]; c[6] = p[1]; c[7] = p[2];
      for (int k = 0; k < 9; k++) c[8 + k] = R[k];
    }
  }
  wsync();
}

DEVI void collide_manifold(const Mdl& md, Dat& d, const PairCtx& pc, int pair, int g1, int g2, const double* n,
                           const double* mpos);

// narrowphase of one admissible pair, all lanes participate
DEVI void collide_pair(const Mdl& md, Dat& d, int pair) {
  int g1 = IA(md, pair_geom1)[pair], g2 = IA(md, pair_geom2)[pair];
  double n[3], depth, mpos[3];
  PairCtx pc;
#ifdef MGS_PROFILE
  // diagnostic split of the narrowphase between missed and hit pairs: ticks
  // from here to the MPR verdict (54 miss / 55 hit) and support calls (56 / 57)
  unsigned long long t_pair = __builtin_amdgcn_s_memtime();
  unsigned long long sc0 = s_prof[28];
#endif
  pair_ctx(md, d, g1, g2, pc);
  double cd[3], cm;
  int hit = mpr_penetration(md, d, pc, g1, g2, n, &depth, mpos, cd, &cm);
  cert_update(md, d, pair, g1, g2, hit, cd, cm);
  PT(4);
  PCNT(26, 1);
  PCNT(27, hit);
  PCNT(30, (pc.n1 > WAVE) + (pc.n2 > WAVE));
#ifdef MGS_PROFILE
  PCNT(hit ? 55 : 54, __builtin_amdgcn_s_memtime() - t_pair);
  PCNT(hit ? 57 : 56, s_prof[28] - sc0);
#endif
  if (!hit) return;
  collide_manifold(md, d, pc, pair, g1, g2, n, mpos);
}

// contact manifold of a pair MPR found penetrating (normal n, MPR point mpos)
DEVI void collide_manifold(const Mdl& md, Dat& d, const PairCtx& pc, int pair, int g1, int g2, const double* n,
                           const double* mpos) {
  int lane = lane_id();
  double t1[3], t2[3];
  make_frame(n, t1, t2);
  // the polygon scratch (K_POLY_POINTS points): each buffer sized for what
  // reaches it -- features <= K_MAXF points, the reference hull <= 2 K_MAXF
  // (the monotone chain's stack), the clipped polygon and its kept points
  // <= K_MAXPOLY (the clip's cap)
  P2* fa = d.poly;
  P2* fb = fa + K_MAXF;
  P2* refpoly = fb + K_MAXF;
  P2* inc = refpoly + 2 * K_MAXF;
  P2* buf = inc + K_MAXPOLY;
  P2* pts = buf + K_MAXPOLY;
  double* dep = d.pdep;
  double s1, s2;
  // first pass: only the extremes are used (the oracle's first feature() pass
  // output is overwritten by the second); the collecting pass starts from them
  feature(pc, 1, n, t1, t2, +1, 0.0, 0, fa, &s1);
  feature(pc, 2, n, t1, t2, -1, 0.0, 0, fb, &s2);
  double dn = s1 - s2;
  if (!(dn > 0.0)) return;
  double tol = dn + K_FEAT_EPS;
  int na = feature(pc, 1, n, t1, t2, +1, tol, 1, fa, &s1);
  int nb = feature(pc, 2, n, t1, t2, -1, tol, 1, fb, &s2);
  PT(40);
  const int refB = (nb >= na);
  // sort + dedup of both feature sets across lanes (uniform counts), the
  // monotone chains with a lane-held stack, clipping and the depth filter
  // across lanes (lanes over polygon vertices), selection on lane 0
  int mr = sort_dedup_wave(refB ? fb : fa, refB ? nb : na);
  int mi = sort_dedup_wave(refB ? fa : fb, refB ? na : nb);
  PT(47);
  int nr = mr >= 0 ? hull_chain_wave(refB ? fb : fa, mr, refpoly) : -1;
  int ni = mi >= 0 ? hull_chain_wave(refB ? fa : fb, mi, inc) : -1;
  if (nr < 0 || ni < 0) {   // a NaN coordinate: the sequential hull2d on lane 0
    wsync();
    if (lane == 0) {
      if (nr < 0) nr = refB ? hull2d(fb, nb, refpoly) : hull2d(fa, na, refpoly);
      if (ni < 0) ni = refB ? hull2d(fa, na, inc) : hull2d(fb, nb, inc);
    }
    nr = shfl(nr, 0);
    ni = shfl(ni, 0);
  }
  wsync();
  PT(48);
  int np = 0;
  if (nr >= 3) {
    int nc = clip_poly_wave(refpoly, nr, inc, ni, buf);
    P2 q;
    q.x = q.y = q.h = 0.0;
    double dd = 0.0;
    if (lane < nc) {
      q = inc[lane];
      dd = refB ? (q.h - s2) : (s1 - q.h);
    }
    int keep = lane < nc && dd > 0.0;
    unsigned long long mk = __ballot(keep);
    unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (WAVE - lane));
    int pos = __popcll(mk & lt);
    if (keep) { pts[pos] = q; dep[pos] = dd; }
    np = __popcll(mk);
    wsync();
  }
  PT(49);
  if (lane == 0) {
    int ncmax = md.m.ncon_max;
    if (np == 0) {
      add_contact(d, ncmax, pair, g1, g2, mpos, n, t1, t2, -dn);
    } else {
      int sel[4], ns;
      select4(pts, dep, np, sel, &ns);
      double sref = refB ? s2 : s1;
      for (int k = 0; k < ns; k++) {
        const P2* p = &pts[sel[k]];
        double hm = 0.5 * (p->h + sref);
        double pos[3];
        for (int c = 0; c < 3; c++) pos[c] = (p->x * t1[c] + p->y * t2[c]) + hm * n[c];
        add_contact(d, ncmax, pair, g1, g2, pos, n, t1, t2, -dep[sel[k]]);
      }
    }
  }
  wsync();
  PT(41);
}

// two admissible convex pairs whose hulls all have <= 16 vertices, A before B:
// both MPRs at once on the two halves (PairCtx2), then per pair in order the
// certificate update and, for a hit, the manifold on the whole wave -- the
// operations and order of collide_pair(A); collide_pair(B)
DEVI void collide_pair2(const Mdl& md, Dat& d, int pairA, int pairB) {
  const int lane = lane_id();
  const int32_t *p1 = IA(md, pair_geom1), *p2 = IA(md, pair_geom2);
  const int gA1 = p1[pairA], gA2 = p2[pairA], gB1 = p1[pairB], gB2 = p2[pairB];
  PairCtx2 q;
  pair_ctx2(md, d, gA1, gA2, gB1, gB2, q);
  const int g1 = lane < 32 ? gA1 : gB1, g2 = lane < 32 ? gA2 : gB2;
  double n[3], depth, mpos[3], cd[3], cm;
  int hit = mpr_penetration(md, d, q, g1, g2, n, &depth, mpos, cd, &cm);
  PT(4);
#pragma unroll
  for (int k = 0; k < 2; k++) {
    const int src = 32 * k, pair = k ? pairB : pairA, G1 = k ? gB1 : gA1, G2 = k ? gB2 : gA2;
    const int hk = __builtin_amdgcn_readlane(hit, src);
    double nk[3], mk[3], ck[3];
#pragma unroll
    for (int i = 0; i < 3; i++) {
      nk[i] = readlane_d(n[i], src);
      mk[i] = readlane_d(mpos[i], src);
      ck[i] = readlane_d(cd[i], src);
    }
    cert_update(md, d, pair, G1, G2, hk, ck, readlane_d(cm, src));
    PCNT(26, 1);
    PCNT(27, hk);
    if (hk) {
      PairCtx pc;
      pair_ctx(md, d, G1, G2, pc);
      collide_manifold(md, d, pc, pair, G1, G2, nk, mk);
    }
  }
}

// Box-box pair (oracle collide_boxbox; MuJoCo's dedicated mjc_BoxBox collider
// takes box pairs instead of the convex path).  The 15 separating axes are
// evaluated one per lane; lane 0 then picks the axis in the oracle's order
// (box 1 faces, box 2 faces, edge-edge only if shallower by > 5 %) and builds
// the manifold: the incident face clipped to the reference face rectangle, or
// one point at the closest points of two edges.
DEVI int bb_clip(P2* Q, int nq, int axis, double lim, double sgn, P2* buf) {
  int no = 0;
  for (int i = 0; i < nq; i++) {
    const P2* cur = &Q[i];
    const P2* prv = &Q[(i + nq - 1) % nq];
    double dc = lim - sgn * (axis ? cur->y : cur->x);
    double dp = lim - sgn * (axis ? prv->y : prv->x);
    if (dc >= 0.0) {
      if (dp < 0.0 && no < 16) buf[no++] = lerp2(prv, cur, dp / (dp - dc));
      if (no < 16) buf[no++] = *cur;
    } else if (dp >= 0.0 && no < 16) {
      buf[no++] = lerp2(prv, cur, dp / (dp - dc));
    }
  }
  for (int i = 0; i < no; i++) Q[i] = buf[i];
  return no;
}

// column k (a box axis) of a geom rotation matrix held in LDS, for a k that
// differs between lanes or is only known in lane 0: a per-lane LDS read, where
// indexing a register copy with it would go through scratch memory
DEVI void lds_col(const double* R, int k, double* r) {
  r[0] = R[k];
  r[1] = R[3 + k];
  r[2] = R[6 + k];
}

DEVI void collide_boxbox(const Mdl& md, Dat& d, int pair) {
  int lane = lane_id();
  int g1 = IA(md, pair_geom1)[pair], g2 = IA(md, pair_geom2)[pair];
  const double *R1 = d.geom_xmat + 9 * g1, *R2 = d.geom_xmat + 9 * g2;
  const double *x1 = d.geom_xpos + 3 * g1, *x2 = d.geom_xpos + 3 * g2;
  const double *h1 = DA(md, geom_aabb) + 6 * g1 + 3, *h2 = DA(md, geom_aabb) + 6 * g2 + 3;
  const double margin = DA(md, pair_margin)[pair];
  double A1[9], A2[9], D[3];
  for (int k = 0; k < 3; k++)
    for (int i = 0; i < 3; i++) { A1[3 * k + i] = R1[3 * i + k]; A2[3 * k + i] = R2[3 * i + k]; }
  sub3(D, x2, x1);
  // lane q < 15 evaluates axis q: 0-2 box 1 faces, 3-5 box 2 faces, 6-14 edge pairs
  double s = -INFINITY, L[3] = {0.0, 0.0, 0.0};
  int valid = 0;
  if (lane < 3) {
    double Lf[3];
    lds_col(R1, lane, Lf);
    double r2 = (h2[0] * fabs(dot3(A2, Lf)) + h2[1] * fabs(dot3(A2 + 3, Lf))) + h2[2] * fabs(dot3(A2 + 6, Lf));
    s = fabs(dot3(D, Lf)) - (h1[lane] + r2);
    valid = 1;
  } else if (lane < 6) {
    int k = lane - 3;
    double Lf[3];
    lds_col(R2, k, Lf);
    double r1 = (h1[0] * fabs(dot3(A1, Lf)) + h1[1] * fabs(dot3(A1 + 3, Lf))) + h1[2] * fabs(dot3(A1 + 6, Lf));
    s = fabs(dot3(D, Lf)) - (h2[k] + r1);
    valid = 1;
  } else if (lane < 15) {
    int a = (lane - 6) / 3, b = (lane - 6) % 3;
    double Ra[3], Rb[3];
    lds_col(R1, a, Ra);
    lds_col(R2, b, Rb);
    cross3(L, Ra, Rb);
    double ll = sqrt(dot3(L, L));
    if (!(ll < 1e-6)) {
      L[0] = L[0] / ll; L[1] = L[1] / ll; L[2] = L[2] / ll;
      double r1 = (h1[0] * fabs(dot3(A1, L)) + h1[1] * fabs(dot3(A1 + 3, L))) + h1[2] * fabs(dot3(A1 + 6, L));
      double r2 = (h2[0] * fabs(dot3(A2, L)) + h2[1] * fabs(dot3(A2 + 3, L))) + h2[2] * fabs(dot3(A2 + 6, L));
      s = fabs(dot3(D, L)) - (r1 + r2);
      valid = 1;
    }
  }
  if (__ballot(valid && s > margin)) return;     // a separating axis: no contact
  // lane 0 gathers the 15 values in axis order
  double sv[15], lx[15], ly[15], lz[15];
  int vv[15];
#pragma unroll
  for (int q = 0; q < 15; q++) {
    sv[q] = shfl(s, q);
    lx[q] = shfl(L[0], q);
    ly[q] = shfl(L[1], q);
    lz[q] = shfl(L[2], q);
    vv[q] = shfl(valid, q);
  }
  if (lane == 0) {
    double best = -INFINITY;
    int code = -1;
    for (int q = 0; q < 6; q++) if (sv[q] > best) { best = sv[q]; code = q; }
    double ebest = -INFINITY, eL[3] = {0.0, 0.0, 0.0};
    int ecode = -1;
    for (int q = 6; q < 15; q++)
      if (vv[q] && sv[q] > ebest) { ebest = sv[q]; ecode = q - 6; eL[0] = lx[q]; eL[1] = ly[q]; eL[2] = lz[q]; }
    int ncmax = md.m.ncon_max;
    double t1[3], t2[3];
    if (ecode >= 0 && 1.05 * ebest > best) {
      int a = ecode / 3, b = ecode % 3;
      double n[3] = {eL[0], eL[1], eL[2]};
      if (dot3(n, D) < 0.0) { n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2]; }
      double e1[3] = {x1[0], x1[1], x1[2]}, e2[3] = {x2[0], x2[1], x2[2]};
#pragma unroll
      for (int k = 0; k < 3; k++) {
        if (k != a) {
          double sg = dot3(A1 + 3 * k, n) >= 0.0 ? h1[k] : -h1[k];
          for (int i = 0; i < 3; i++) e1[i] = e1[i] + sg * A1[3 * k + i];
        }
        if (k != b) {
          double sg = dot3(A2 + 3 * k, n) >= 0.0 ? -h2[k] : h2[k];
          for (int i = 0; i < 3; i++) e2[i] = e2[i] + sg * A2[3 * k + i];
        }
      }
      double U[3], V[3];
      lds_col(R1, a, U);
      lds_col(R2, b, V);
      double w[3];
      sub3(w, e1, e2);
      double bu = dot3(U, V), du = dot3(U, w), ev = dot3(V, w);
      double den = 1.0 - bu * bu;
      double ss = (bu * ev - du) / den, tt = (ev - bu * du) / den;
      if (ss < -h1[a]) ss = -h1[a];
      if (ss > h1[a]) ss = h1[a];
      if (tt < -h2[b]) tt = -h2[b];
      if (tt > h2[b]) tt = h2[b];
      double pos[3];
      for (int i = 0; i < 3; i++) pos[i] = 0.5 * ((e1[i] + ss * U[i]) + (e2[i] + tt * V[i]));
      make_frame(n, t1, t2);
      add_contact(d, ncmax, pair, g1, g2, pos, n, t1, t2, ebest);
    } else {
      int ref1 = code < 3, k = code % 3;
      // reference / incident box rotations (LDS) and their axes by column reads
      const double *RA = ref1 ? R1 : R2, *RB = ref1 ? R2 : R1;
      const double *hA = ref1 ? h1 : h2, *hB = ref1 ? h2 : h1;
      const double *xA = ref1 ? x1 : x2, *xB = ref1 ? x2 : x1;
      double DAB[3];
      sub3(DAB, xB, xA);
      double nr[3];
      lds_col(RA, k, nr);
      if (dot3(DAB, nr) < 0.0) { nr[0] = -nr[0]; nr[1] = -nr[1]; nr[2] = -nr[2]; }
      double n[3] = {nr[0], nr[1], nr[2]};
      if (!ref1) { n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2]; }
      int ku = (k + 1) % 3, kv = (k + 2) % 3;
      double u[3], v[3];
      lds_col(RA, ku, u);
      lds_col(RA, kv, v);
      double cA[3];
      for (int i = 0; i < 3; i++) cA[i] = xA[i] + hA[k] * nr[i];
      int j = 0;
      double Bc[3];
      lds_col(RB, 0, Bc);
      double bj = fabs(dot3(Bc, nr));
      for (int q = 1; q < 3; q++) {
        lds_col(RB, q, Bc);
        double c = fabs(dot3(Bc, nr));
        if (c > bj) { bj = c; j = q; }
      }
      double Bj[3], Bp[3], Bq[3];
      int jp = (j + 1) % 3, jq = (j + 2) % 3;
      lds_col(RB, j, Bj);
      lds_col(RB, jp, Bp);
      lds_col(RB, jq, Bq);
      double sB = dot3(Bj, nr) > 0.0 ? -hB[j] : hB[j];
      P2* poly = d.poly;
      P2* buf = d.poly + 16;
      P2* pts = d.poly + 32;
      double* dep = d.pdep;
      double deep = INFINITY, deep_c[3] = {0.0, 0.0, 0.0};
      for (int c = 0; c < 4; c++) {
        double cp = (c == 0 || c == 3) ? 1.0 : -1.0, cq = (c < 2) ? 1.0 : -1.0;
        double P[3], rel[3];
        for (int i = 0; i < 3; i++)
          P[i] = ((xB[i] + sB * Bj[i]) + (cp * hB[jp]) * Bp[i]) + (cq * hB[jq]) * Bq[i];
        sub3(rel, P, cA);
        poly[c].x = dot3(rel, u);
        poly[c].y = dot3(rel, v);
        poly[c].h = dot3(rel, nr);
        if (poly[c].h < deep) { deep = poly[c].h; deep_c[0] = P[0]; deep_c[1] = P[1]; deep_c[2] = P[2]; }
      }
      int nq = 4;
      nq = bb_clip(poly, nq, 0, hA[ku], 1.0, buf);
      if (nq) nq = bb_clip(poly, nq, 0, hA[ku], -1.0, buf);
      if (nq) nq = bb_clip(poly, nq, 1, hA[kv], 1.0, buf);
      if (nq) nq = bb_clip(poly, nq, 1, hA[kv], -1.0, buf);
      double mtol = K_BB_MERGE * (hA[ku] > hA[kv] ? hA[ku] : hA[kv]);
      mtol = mtol * mtol;
      int np = 0;
      for (int i = 0; i < nq; i++) {
        if (!(poly[i].h < margin)) continue;
        int dup = 0;
        for (int q = 0; q < np; q++) if (dist2d(&pts[q], &poly[i]) < mtol) dup = 1;
        if (!dup) { pts[np] = poly[i]; dep[np] = -poly[i].h; np++; }
      }
      make_frame(n, t1, t2);
      if (np == 0) {
        double pos[3];
        for (int i = 0; i < 3; i++) pos[i] = deep_c[i] - (0.5 * deep) * nr[i];
        add_contact(d, ncmax, pair, g1, g2, pos, n, t1, t2, deep);
      } else {
        // an edge on a face (exactly two penetrating vertices): one contact at
        // the deeper vertex (oracle collide_boxbox, round 5: the set that
        // reproduces MuJoCo's recorded Robotiq state_close)
        int sel[4], ns;
        if (np == 2) {
          ns = 1;
          sel[0] = dep[1] > dep[0] ? 1 : 0;
        } else {
          select4(pts, dep, np, sel, &ns);
        }
        for (int q = 0; q < ns; q++) {
          const P2* p = &pts[sel[q]];
          double pos[3];
          for (int i = 0; i < 3; i++) pos[i] = ((cA[i] + p->x * u[i]) + p->y * v[i]) + (0.5 * p->h) * nr[i];
          add_contact(d, ncmax, pair, g1, g2, pos, n, t1, t2, p->h);
        }
      }
    }
  }
  wsync();
}

// ---------------------------------------------------------------------------
// MuJoCo 3.2.2's collision table (ccd_mode 1 / 2, ABI 23): the oracle's
// collide_convex_mj / collide_prim, same expressions in the same order.
// Convex pairs: libccd's ccdMPRPenetration (libccd's ccdIsZero / ccdEq tests,
// the depth as the distance from the origin to the final portal triangle, the
// position as the tetrahedron barycentre of the origin); with multiccd four more
// MPRs with the geoms turned by -+1e-3 rad about the first contact's tangents.
// Primitive pairs: the analytic colliders.  Parity vs MuJoCo unpinned
// (DESIGN.md §2); GPU == oracle bit for bit.
#define CCD_EPS 2.2204460492503131e-16
// multiccd's four perturbations on 16-lane groups at once (1, ccd_mpr_q) or
// one after another on the whole wave (0: A/B builds)
#ifndef MGS_MCCD_Q
#define MGS_MCCD_Q 1
#endif
#define MCCD_RELTOL 1e-3
#define MCCD_C 0.9999998750000026       // cos(5e-4): half the perturbation angle
#define MCCD_S 4.999999791666669e-04    // sin(5e-4)
#define CCD_MAXLOOP 64
#define MGS_CB_NCAND 49

DEVI int ccd_iszero(double x) { return fabs(x) < CCD_EPS; }
DEVI int ccd_eq(double a, double b) {
  double ab = fabs(a - b);
  if (ab < CCD_EPS) return 1;
  double fa = fabs(a), fb = fabs(b);
  return fb > fa ? (ab < CCD_EPS * fb) : (ab < CCD_EPS * fa);
}
DEVI int ccd_vzero(const double* a) { return ccd_eq(a[0], 0.0) && ccd_eq(a[1], 0.0) && ccd_eq(a[2], 0.0); }
DEVI void ccd_normalize(double* v) {
  double k = 1.0 / sqrt(dot3(v, v));
  v[0] = v[0] * k; v[1] = v[1] * k; v[2] = v[2] * k;
}
DEVI void mulmm3(double* r, const double* a, const double* b) {
  double t[9];
#pragma unroll
  for (int i = 0; i < 3; i++)
#pragma unroll
    for (int j = 0; j < 3; j++) t[3 * i + j] = (a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j]) + a[3 * i + 2] * b[6 + j];
#pragma unroll
  for (int k = 0; k < 9; k++) r[k] = t[k];
}
DEVI int ccd_reach_tol(const SupPt& p1, const SupPt& p2, const SupPt& p3, const SupPt& p4, const double* n,
                       double tol) {
  double dv4 = dot3(p4.v, n);
  double t1 = dv4 - dot3(p1.v, n);
  double t2 = dv4 - dot3(p2.v, n);
  double t3 = dv4 - dot3(p3.v, n);
  double mn = t1 < t2 ? t1 : t2;
  mn = mn < t3 ? mn : t3;
  return ccd_eq(mn, tol) || mn < tol;
}
DEVI void ccd_portal_dir(double* n, const SupPt& p1, const SupPt& p2, const SupPt& p3) {
  double e1[3], e2[3];
  sub3(e1, p2.v, p1.v);
  sub3(e2, p3.v, p1.v);
  cross3(n, e1, e2);
  ccd_normalize(n);
}
DEVI double ccd_seg_dist2(const double* x0, const double* b, double* w) {
  double dd[3], a[3] = {x0[0], x0[1], x0[2]};
  sub3(dd, b, x0);
  double t = -dot3(a, dd);
  t = t / dot3(dd, dd);
  if (t < 0.0 || ccd_iszero(t)) {
    w[0] = x0[0]; w[1] = x0[1]; w[2] = x0[2];
  } else if (t > 1.0 || ccd_eq(t, 1.0)) {
    w[0] = b[0]; w[1] = b[1]; w[2] = b[2];
  } else {
    w[0] = dd[0] * t + x0[0]; w[1] = dd[1] * t + x0[1]; w[2] = dd[2] * t + x0[2];
  }
  return dot3(w, w);
}
DEVI double ccd_tri_dist2(const double* x0, const double* B, const double* C, double* w) {
  double d1[3], d2[3];
  sub3(d1, B, x0);
  sub3(d2, C, x0);
  const double* a = x0;
  double v = dot3(d1, d1), ww = dot3(d2, d2), p = dot3(a, d1), q = dot3(a, d2), r = dot3(d1, d2);
  double dt = ww * v - r * r, s, t;
  if (ccd_iszero(dt)) {
    s = -1.0; t = -1.0;
  } else {
    s = (q * r - ww * p) / dt;
    t = (-s * r - q) / ww;
  }
  if ((ccd_iszero(s) || s > 0.0) && (ccd_eq(s, 1.0) || s < 1.0) && (ccd_iszero(t) || t > 0.0) &&
      (ccd_eq(t, 1.0) || t < 1.0) && (ccd_eq(t + s, 1.0) || t + s < 1.0)) {
#pragma unroll
    for (int k = 0; k < 3; k++) w[k] = (x0[k] + d1[k] * s) + d2[k] * t;
    return dot3(w, w);
  }
  double w2[3];
  double dist = ccd_seg_dist2(x0, B, w);
  double d2b = ccd_seg_dist2(x0, C, w2);
  if (d2b < dist) { dist = d2b; w[0] = w2[0]; w[1] = w2[1]; w[2] = w2[2]; }
  d2b = ccd_seg_dist2(B, C, w2);
  if (d2b < dist) { dist = d2b; w[0] = w2[0]; w[1] = w2[1]; w[2] = w2[2]; }
  return dist;
}
DEVI void ccd_find_pos(const SupPt& p0, const SupPt& p1, const SupPt& p2, const SupPt& p3, double* pos) {
  double dir[3], c[3], b0, b1, b2, b3;
  ccd_portal_dir(dir, p1, p2, p3);
  cross3(c, p1.v, p2.v); b0 = dot3(c, p3.v);
  cross3(c, p3.v, p2.v); b1 = dot3(c, p0.v);
  cross3(c, p0.v, p1.v); b2 = dot3(c, p3.v);
  cross3(c, p2.v, p1.v); b3 = dot3(c, p0.v);
  double sum = ((b0 + b1) + b2) + b3;
  if (ccd_iszero(sum) || sum < 0.0) {
    b0 = 0.0;
    cross3(c, p2.v, p3.v); b1 = dot3(c, dir);
    cross3(c, p3.v, p1.v); b2 = dot3(c, dir);
    cross3(c, p1.v, p2.v); b3 = dot3(c, dir);
    sum = (b1 + b2) + b3;
  }
  double inv = 1.0 / sum;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    double a1 = (((0.0 + p0.a[k] * b0) + p1.a[k] * b1) + p2.a[k] * b2) + p3.a[k] * b3;
    double a2 = (((0.0 + p0.b[k] * b0) + p1.b[k] * b1) + p2.b[k] * b2) + p3.b[k] * b3;
    pos[k] = (a1 * inv + a2 * inv) * 0.5;
  }
}

// oracle ccd_mpr (Ctx: PairCtx, or PairCtx2 for two pairs on the two halves;
// g1 / g2 the half's geoms, whose centres are their geom_xpos); dir is the
// caller's array as in mpr_penetration (the certificate's direction on a miss)
#define CCD_CERT(P) do { *cm = -dot3((P).v, dir); } while (0)
// the MPR's interior point: the two geoms' centres (mjccd_center: geom_xpos,
// or the perturbed centre of a multiccd run, which the context holds)
DEVI void mpr_centres(const PairCtx& c, const Dat&, int, int, double* a, double* b) {
#pragma unroll
  for (int k = 0; k < 3; k++) { a[k] = c.x1[k]; b[k] = c.x2[k]; }
}
DEVI void mpr_centres(const PairCtx2&, const Dat& d, int g1, int g2, double* a, double* b) {
#pragma unroll
  for (int k = 0; k < 3; k++) { a[k] = d.geom_xpos[3 * g1 + k]; b[k] = d.geom_xpos[3 * g2 + k]; }
}
template <class Ctx>
DEVI int ccd_mpr(const Mdl& md, const Dat& d, const Ctx& pc, int g1, int g2, double* n, double* depth, double* pos,
                 double* dir, double* cm) {
  *cm = -1.0;
  const double tol = md.m.mpr_tolerance;
  const int maxit = md.m.ccd_iterations;
  SupPt p0, p1, p2, p3, p4;
  double dt;
  mpr_centres(pc, d, g1, g2, p0.a, p0.b);
  sub3(p0.v, p0.a, p0.b);
  if (ccd_vzero(p0.v)) p0.v[0] = p0.v[0] + CCD_EPS * 10.0;
  dir[0] = -p0.v[0]; dir[1] = -p0.v[1]; dir[2] = -p0.v[2];
  ccd_normalize(dir);
  mink_support(pc, dir, &p1);
  dt = dot3(p1.v, dir);
  if (ccd_iszero(dt) || dt < 0.0) { CCD_CERT(p1); return 0; }
  cross3(dir, p0.v, p1.v);
  if (ccd_iszero(dot3(dir, dir))) {
    if (ccd_vzero(p1.v)) return 0;
#pragma unroll
    for (int k = 0; k < 3; k++) { n[k] = p1.v[k]; pos[k] = (p1.a[k] + p1.b[k]) * 0.5; }
    *depth = sqrt(dot3(n, n));
    ccd_normalize(n);
    return 1;
  }
  ccd_normalize(dir);
  mink_support(pc, dir, &p2);
  dt = dot3(p2.v, dir);
  if (ccd_iszero(dt) || dt < 0.0) { CCD_CERT(p2); return 0; }
  {
    double e1[3], e2[3];
    sub3(e1, p1.v, p0.v);
    sub3(e2, p2.v, p0.v);
    cross3(dir, e1, e2);
    ccd_normalize(dir);
  }
  if (dot3(dir, p0.v) > 0.0) {
    SupPt tmp = p1; p1 = p2; p2 = tmp;
    dir[0] = -dir[0]; dir[1] = -dir[1]; dir[2] = -dir[2];
  }
  int it;
  for (it = 0; it < CCD_MAXLOOP; it++) {
    mink_support(pc, dir, &p3);
    dt = dot3(p3.v, dir);
    if (ccd_iszero(dt) || dt < 0.0) { CCD_CERT(p3); return 0; }
    double c[3];
    int cont = 0;
    cross3(c, p1.v, p3.v);
    dt = dot3(c, p0.v);
    if (dt < 0.0 && !ccd_iszero(dt)) { p2 = p3; cont = 1; }
    if (!cont) {
      cross3(c, p3.v, p2.v);
      dt = dot3(c, p0.v);
      if (dt < 0.0 && !ccd_iszero(dt)) { p1 = p3; cont = 1; }
    }
    if (!cont) break;
    double e1[3], e2[3];
    sub3(e1, p1.v, p0.v);
    sub3(e2, p2.v, p0.v);
    cross3(dir, e1, e2);
    ccd_normalize(dir);
  }
  if (it == CCD_MAXLOOP) return 0;
  for (it = 0; it < CCD_MAXLOOP; it++) {
    ccd_portal_dir(dir, p1, p2, p3);
    dt = dot3(dir, p1.v);
    if (ccd_iszero(dt) || dt > 0.0) break;
    mink_support(pc, dir, &p4);
    dt = dot3(p4.v, dir);
    if (!(ccd_iszero(dt) || dt > 0.0)) { CCD_CERT(p4); return 0; }
    if (ccd_reach_tol(p1, p2, p3, p4, dir, tol)) return 0;
    PORTAL_EXPAND(p0, p1, p2, p3, p4);
  }
  if (it == CCD_MAXLOOP) return 0;
  for (it = 0;; it++) {
    ccd_portal_dir(dir, p1, p2, p3);
    mink_support(pc, dir, &p4);
    if (ccd_reach_tol(p1, p2, p3, p4, dir, tol) || it > maxit) {
      double w[3];
      double dep = sqrt(ccd_tri_dist2(p1.v, p2.v, p3.v, w));
      if (ccd_iszero(dep)) return 0;
      n[0] = w[0]; n[1] = w[1]; n[2] = w[2];
      ccd_normalize(n);
      *depth = dep;
      ccd_find_pos(p0, p1, p2, p3, pos);
      return 1;
    }
    PORTAL_EXPAND(p0, p1, p2, p3, p4);
  }
}
#undef CCD_CERT

// multiccd (oracle collide_convex_mj after its first contact): the pair's
// first contact (n, pos) is in; four more MPRs with geom 1 turned by -+angle
// and geom 2 by the opposite angle about the frame's tangents, each new
// contact farther than MCCD_RELTOL x the smaller bounding radius from the
// pair's contacts so far added (all lanes; lane 0 writes)
// the pair's contacts so far, for multiccd's distinctness test: in the
// collision stage's polygon scratch (unused by the ccd_mode 1 / 2 colliders),
// uniform addresses, lane 0 writes (registers here spilled the object)
DEVI void mccd_list_init(Dat& d, const double* pos) {
  double* cp = (double*)d.poly;
  if (lane_id() == 0) { cp[0] = pos[0]; cp[1] = pos[1]; cp[2] = pos[2]; }
  wsync();
}
DEVI int mccd_is_new(const Dat& d, int nc, const double* p, double tolr) {
  const double* cp = (const double*)d.poly;
  int isnew = 1;
  for (int k = 0; k < nc; k++) {
    double dx[3] = {p[0] - cp[3 * k], p[1] - cp[3 * k + 1], p[2] - cp[3 * k + 2]};
    if (sqrt(dot3(dx, dx)) < tolr) isnew = 0;
  }
  return isnew;
}
DEVI void mccd_list_add(Dat& d, int nc, const double* p) {
  double* cp = (double*)d.poly;
  wsync();
  if (lane_id() == 0) { cp[3 * nc] = p[0]; cp[3 * nc + 1] = p[1]; cp[3 * nc + 2] = p[2]; }
  wsync();
}
DEVI double mccd_tol(const Mdl& md, int g1, int g2) {
  const double* rb = DA(md, geom_rbound);
  const double* rr = DA(md, geom_radius);
  double rb1 = rb[g1] + rr[g1], rb2 = rb[g2] + rr[g2];
  return MCCD_RELTOL * (rb1 < rb2 ? rb1 : rb2);
}

// multiccd's four perturbed MPRs of one pair at once (round 6): groups of
// 2 x HW lanes each run one perturbation's MPR, HW lanes per hull (lane
// HW * side + i of a group holds vertex i of geom 1 or 2), for pairs whose
// two hulls have at most HW vertices: HW 8 -> four MPRs per pass, HW 16 ->
// two.  Each group computes exactly what the whole wave computes for its
// perturbation (the MPR's control flow depends only on values uniform within
// a group), so the contacts are multiccd()'s, bit for bit.
template <int HW>
struct PairCtxQ {
  int n;               // this lane's hull: its vertex count,
  double R[9], x[3];   // its geom's pose (the group's perturbation about the first contact),
  double cx1[3], cx2[3];   // the group's two perturbed centres (the MPR's interior point)
  double c[3];         // the lane's vertex (lane % HW < n)
  double r;            // and rounding radius
  int P;               // reduction width: next_pow2 of the larger count (<= HW)
};
// the perturbation q = 2 ax + sg of a group (oracle collide_convex_mj's loop order)
template <int HW>
DEVI void pair_ctxq(const Mdl& md, const Dat& d, int g1, int g2, const double* t1, const double* t2,
                    const double* pv, int q0, PairCtxQ<HW>& c) {
  const int lane = lane_id(), grp = lane / (2 * HW), side = (lane / HW) & 1, li = lane % HW;
  const int q = q0 + grp, ax = q >> 1, sg = q & 1;
  const int g = side ? g2 : g1;
  const int32_t *ghull = IA(md, geom_hullid), *hadr = IA(md, hull_vertadr), *hnum = IA(md, hull_vertnum);
  const int h = ghull[g];
  c.n = hnum[h];
  const double* V = DA(md, hull_vert) + 3 * hadr[h];
  const int i = li < c.n ? li : 0;
#pragma unroll
  for (int k = 0; k < 3; k++) c.c[k] = V[k * c.n + i];
  c.r = DA(md, geom_radius)[g];
  double axis[3] = {ax ? t2[0] : t1[0], ax ? t2[1] : t1[1], ax ? t2[2] : t1[2]};
  double s = sg ? MCCD_S : -MCCD_S;
  double qq[4];
  qq[0] = MCCD_C;
  if (side) { qq[1] = -(axis[0] * s); qq[2] = -(axis[1] * s); qq[3] = -(axis[2] * s); }
  else { qq[1] = axis[0] * s; qq[2] = axis[1] * s; qq[3] = axis[2] * s; }
  double M[9], Rg[9], xg[3], r[3], t[3];
  quat2mat(M, qq);
#pragma unroll
  for (int k = 0; k < 9; k++) Rg[k] = d.geom_xmat[9 * g + k];
#pragma unroll
  for (int k = 0; k < 3; k++) xg[k] = d.geom_xpos[3 * g + k];
  // mjc_rotateFrame about the first contact pv (oracle collide_convex_mj)
  mulmm3(c.R, M, Rg);
  sub3(r, xg, pv);
  mulmv3(t, M, r);
  add3(c.x, t, pv);
  // the group's centres: geom 1's from its first lane, geom 2's from lane HW
  const int gb = lane - (lane % (2 * HW));
#pragma unroll
  for (int k = 0; k < 3; k++) {
    c.cx1[k] = shfl(c.x[k], gb);
    c.cx2[k] = shfl(c.x[k], gb + HW);
  }
  const int n1 = hnum[ghull[g1]], n2 = hnum[ghull[g2]];
  c.P = next_pow2(n1 > n2 ? n1 : n2);
}
template <int HW>
DEVI void mpr_centres(const PairCtxQ<HW>& c, const Dat&, int, int, double* a, double* b) {
#pragma unroll
  for (int k = 0; k < 3; k++) { a[k] = c.cx1[k]; b[k] = c.cx2[k]; }
}
template <int HW>
DEVI void support_pairq(const PairCtxQ<HW>& c, const double* dir, double* out1, double* out2) {
  const int lane = lane_id(), side = (lane / HW) & 1, li = lane % HW, hb = lane - li;
  double sd[3] = {side ? -dir[0] : dir[0], side ? -dir[1] : dir[1], side ? -dir[2] : dir[2]};
  double dl[3];
  mulmtv3(dl, c.R, sd);
  SupAcc a;
  sup_init(a);
  if (li < c.n) {
    double sc = (c.c[0] * dl[0] + c.c[1] * dl[1]) + c.c[2] * dl[2];
    if (sc > a.best) { a.best = sc; a.bi = li; a.vx = c.c[0]; a.vy = c.c[1]; a.vz = c.c[2]; }
  }
  const int P = c.P;
  double m = a.best;
  if (P > 1) m = max_f64(m, dpp_d(m, 0));
  if (P > 2) m = max_f64(m, dpp_d(m, 1));
  if (P > 4) m = max_f64(m, dpp_d(m, 2));
  if (HW > 8 && P > 8) m = max_f64(m, dpp_d(m, 3));
  // this lane's hull maximum: the reduced value of the hull's first lane
  const double M = shfl(m, hb);
  const unsigned long long tied = __ballot(a.bi != 0x7fffffff && a.best == M);
  const unsigned tr = (unsigned)(tied >> hb) & ((1u << HW) - 1u);
  const int src = hb + (tr ? __ffs(tr) - 1 : 0);
  double v[3] = {shfl(a.vx, src), shfl(a.vy, src), shfl(a.vz, src)};
  double t[3], wv[3];
  mulmv3(t, c.R, v);
  add3(wv, c.x, t);
  if (c.r > 0.0) { wv[0] = wv[0] + c.r * sd[0]; wv[1] = wv[1] + c.r * sd[1]; wv[2] = wv[2] + c.r * sd[2]; }
  const int s1 = lane - (lane % (2 * HW)), s2 = s1 + HW;
#pragma unroll
  for (int k = 0; k < 3; k++) {
    out1[k] = shfl(wv[k], s1);
    out2[k] = shfl(wv[k], s2);
  }
}
template <int HW>
DEVI void mink_support(const PairCtxQ<HW>& c, const double* dir, SupPt* p, unsigned long long) {
  PT(4);
  PCNT(28, 1);
  support_pairq<HW>(c, dir, p->a, p->b);
  sub3(p->v, p->a, p->b);
  PT(22);
}
// multiccd_q's MPR: ccd_mpr's arithmetic step for step, with every group in
// lockstep -- one support call per pass for the whole wave, each group
// advancing its own phase (first two supports, portal discovery, refinement,
// penetration) with its own counter; a group that is done keeps its state and
// the loop ends when no group is left.  (ccd_mpr's own loops diverge per group
// here, and in the register-capped object the compiler spilled inside those
// divergent loops: 39 of 41 parity rollouts left the oracle, round 6.)  The
// normal, depth and position of a hit; no certificate (multiccd has none).
#define MQ_P1 0
#define MQ_P2 1
#define MQ_DISC 2
#define MQ_REF 3
#define MQ_PEN 4
#define MQ_FIN 5
#define MQ_DONE 6
template <class QC>
DEVI int ccd_mpr_q(const Mdl& md, const Dat& d, const QC& pc, double* n, double* depth, double* pos) {
  const double tol = md.m.mpr_tolerance;
  const int maxit = md.m.ccd_iterations;
  SupPt p0, p1, p2, p3, ps;
  double dir[3];
  int ph = MQ_P1, it = 0, hit = 0;
  mpr_centres(pc, d, 0, 0, p0.a, p0.b);
  sub3(p0.v, p0.a, p0.b);
  if (ccd_vzero(p0.v)) p0.v[0] = p0.v[0] + CCD_EPS * 10.0;
  dir[0] = -p0.v[0]; dir[1] = -p0.v[1]; dir[2] = -p0.v[2];
  ccd_normalize(dir);
  p1 = p0; p2 = p0; p3 = p0;
  for (;;) {
    if (ph == MQ_REF || ph == MQ_PEN) {
      ccd_portal_dir(dir, p1, p2, p3);
      if (ph == MQ_REF) {
        const double dt = dot3(dir, p1.v);
        if (ccd_iszero(dt) || dt > 0.0) { ph = MQ_PEN; it = 0; }
      }
    }
    const unsigned long long act = __ballot(ph < MQ_FIN);
    if (!act) break;
    mink_support(pc, dir, &ps, act);
    const double dt = dot3(ps.v, dir);
    if (ph == MQ_P1) {
      if (ccd_iszero(dt) || dt < 0.0) {
        ph = MQ_DONE;
      } else {
        p1 = ps;
        cross3(dir, p0.v, p1.v);
        if (ccd_iszero(dot3(dir, dir))) {
          if (!ccd_vzero(p1.v)) {
#pragma unroll
            for (int k = 0; k < 3; k++) { n[k] = p1.v[k]; pos[k] = (p1.a[k] + p1.b[k]) * 0.5; }
            *depth = sqrt(dot3(n, n));
            ccd_normalize(n);
            hit = 1;
          }
          ph = MQ_DONE;
        } else {
          ccd_normalize(dir);
          ph = MQ_P2;
        }
      }
    } else if (ph == MQ_P2) {
      if (ccd_iszero(dt) || dt < 0.0) {
        ph = MQ_DONE;
      } else {
        p2 = ps;
        double e1[3], e2[3];
        sub3(e1, p1.v, p0.v);
        sub3(e2, p2.v, p0.v);
        cross3(dir, e1, e2);
        ccd_normalize(dir);
        if (dot3(dir, p0.v) > 0.0) {
          SupPt tmp = p1; p1 = p2; p2 = tmp;
          dir[0] = -dir[0]; dir[1] = -dir[1]; dir[2] = -dir[2];
        }
        ph = MQ_DISC;
        it = 0;
      }
    } else if (ph == MQ_DISC) {
      if (ccd_iszero(dt) || dt < 0.0) {
        ph = MQ_DONE;
      } else {
        p3 = ps;
        double c[3];
        int cont = 0;
        cross3(c, p1.v, p3.v);
        double dc = dot3(c, p0.v);
        if (dc < 0.0 && !ccd_iszero(dc)) { p2 = p3; cont = 1; }
        if (!cont) {
          cross3(c, p3.v, p2.v);
          dc = dot3(c, p0.v);
          if (dc < 0.0 && !ccd_iszero(dc)) { p1 = p3; cont = 1; }
        }
        if (!cont) {
          ph = MQ_REF;
          it = 0;
        } else {
          double e1[3], e2[3];
          sub3(e1, p1.v, p0.v);
          sub3(e2, p2.v, p0.v);
          cross3(dir, e1, e2);
          ccd_normalize(dir);
          if (++it == CCD_MAXLOOP) ph = MQ_DONE;
        }
      }
    } else if (ph == MQ_REF) {
      if (!(ccd_iszero(dt) || dt > 0.0) || ccd_reach_tol(p1, p2, p3, ps, dir, tol)) {
        ph = MQ_DONE;
      } else {
        PORTAL_EXPAND(p0, p1, p2, p3, ps);
        if (++it == CCD_MAXLOOP) ph = MQ_DONE;
      }
    } else if (ph == MQ_PEN) {
      if (ccd_reach_tol(p1, p2, p3, ps, dir, tol) || it > maxit) {
        ph = MQ_FIN;
      } else {
        PORTAL_EXPAND(p0, p1, p2, p3, ps);
        it++;
      }
    }
  }
  // the penetration's end (ccd_mpr's last block), every lane computing it; the
  // groups that stopped there take it
  double w[3], fp[3];
  const double dep = sqrt(ccd_tri_dist2(p1.v, p2.v, p3.v, w));
  ccd_normalize(w);
  ccd_find_pos(p0, p1, p2, p3, fp);
  if (ph == MQ_FIN && !ccd_iszero(dep)) {
#pragma unroll
    for (int k = 0; k < 3; k++) { n[k] = w[k]; pos[k] = fp[k]; }
    *depth = dep;
    hit = 1;
  }
  return hit;
}

// scratch after the perturbed poses: the first contact's normal (MCCD_N), an
// MPR's results (MCCD_RES + 12 k: n pos dir depth cm hit; k the group of
// multiccd_q) and the two-pair MPR's per pair (MCCD_RES2 + 12 k: they must
// outlive pair A's multiccd)
#define MCCD_N 40
#define MCCD_RES 48
#define MCCD_RES2 96
DEVI void mccd_store(Dat& d, int at, int hit, const double* n, const double* pos, const double* cd, double depth,
                     double cm) {
  double* o = (double*)d.poly + at;
#pragma unroll
  for (int i = 0; i < 3; i++) { o[i] = n[i]; o[3 + i] = pos[i]; o[6 + i] = cd[i]; }
  o[9] = depth;
  o[10] = cm;
  o[11] = hit ? 1.0 : 0.0;
}
// each group's MPR result (multiccd_q's and multiccd_w's, MCCD_RES + 12 group)
// taken in perturbation order: distinct ones added to the pair's contacts
DEVI void mccd_take_groups(const Mdl& md, Dat& d, int pair, int g1, int g2, int ngroups, int& nc) {
  const double* cp = (const double*)d.poly;
  const int ncmax = md.m.ncon_max;
#pragma unroll 1
  for (int k = 0; k < ngroups; k++) {
    const double* r = cp + MCCD_RES + 12 * k;
    if (r[11] == 0.0) continue;
    double pk[3] = {r[3], r[4], r[5]};
    if (!mccd_is_new(d, nc, pk, mccd_tol(md, g1, g2))) continue;
    double nk[3] = {r[0], r[1], r[2]};
    const double dk = r[9];
    mccd_list_add(d, nc, pk);
    nc++;
    double u1[3], u2[3];
    make_frame(nk, u1, u2);
    if (lane_id() == 0) add_contact(d, ncmax, pair, g1, g2, pk, nk, u1, u2, -dk);
  }
  wsync();
}
// multiccd() with its four perturbed MPRs on groups of 2 x HW lanes (pairs
// whose hulls have at most HW vertices and no cylinder): the same contacts in
// the same order
template <int HW>
DEVI void multiccd_q(const Mdl& md, Dat& d, int pair, int g1, int g2, const double* n, const double* pos) {
  constexpr int G = WAVE / (2 * HW);      // perturbations per pass
  mccd_list_init(d, pos);
  int nc = 1;
#pragma unroll 1
  for (int q0 = 0; q0 < 4; q0 += G) {
    {
      double t1[3], t2[3];
      make_frame(n, t1, t2);
      PairCtxQ<HW> pc;
      pair_ctxq<HW>(md, d, g1, g2, t1, t2, pos, q0, pc);
      double nn[3], dd = 0.0, pp[3], dir[3] = {0.0, 0.0, 0.0}, cmx = -1.0;
      const int hit = ccd_mpr_q(md, d, pc, nn, &dd, pp);
      // each group's result through LDS (MCCD_RES + 12 group)
      const int lane = lane_id();
      if (lane % (2 * HW) == 0) mccd_store(d, MCCD_RES + 12 * (lane / (2 * HW)), hit, nn, pp, dir, dd, cmx);
      wsync();
    }
    mccd_take_groups(md, d, pair, g1, g2, G, nc);
  }
  wsync();
}

// the perturbed poses go to the collision stage's polygon scratch after the
// contact list (R1 R2 x1 x2 at MCCD_POSE), lane 0 writing: the context is then
// read back like an unperturbed one (perturbed poses held in registers across
// the MPR spilled the eight-per-CU object)
#define MCCD_POSE 16
DEVI void mccd_perturb(const Dat& d, Dat& dw, int g1, int g2, const double* n, const double* pv, int q, int at) {
  const int ax = q >> 1, sg = q & 1;
  double t1[3], t2[3];
  make_frame(n, t1, t2);
  double axis[3] = {ax ? t2[0] : t1[0], ax ? t2[1] : t1[1], ax ? t2[2] : t1[2]};
  double s = sg ? MCCD_S : -MCCD_S;
  double* out = (double*)dw.poly + at;
#pragma unroll 1
  for (int side = 0; side < 2; side++) {
    const int g = side ? g2 : g1;
    double qq[4];
    qq[0] = MCCD_C;
    if (side) { qq[1] = -(axis[0] * s); qq[2] = -(axis[1] * s); qq[3] = -(axis[2] * s); }
    else { qq[1] = axis[0] * s; qq[2] = axis[1] * s; qq[3] = axis[2] * s; }
    double M[9], R[9], xg[3], r[3], t[3], xo[3];
#pragma unroll
    for (int k = 0; k < 9; k++) R[k] = d.geom_xmat[9 * g + k];
#pragma unroll
    for (int k = 0; k < 3; k++) xg[k] = d.geom_xpos[3 * g + k];
    quat2mat(M, qq);
    mulmm3(R, M, R);
    sub3(r, xg, pv);
    mulmv3(t, M, r);
    add3(xo, t, pv);
    if (lane_id() == 0) {
#pragma unroll
      for (int k = 0; k < 9; k++) out[9 * side + k] = R[k];
#pragma unroll
      for (int k = 0; k < 3; k++) out[18 + 3 * side + k] = xo[k];
    }
  }
  wsync();
}

// multiccd's four perturbed MPRs of a pair that multiccd_q cannot take (a hull
// of more than 8 vertices, or a cylinder: the gripper's link meshes on the
// object), in lockstep on four 16-lane groups as there (ccd_mpr_q), each
// support of the four perturbations computed by the whole wave in turn
// (support_pair over the pair's hulls, the group's perturbed poses from LDS,
// only for the groups still running): four MPR scalar chains at once instead
// of one after another, the same supports, the same contacts in the same order
#ifndef MGS_MCCD_W
#define MGS_MCCD_W 1   // 0: these perturbations one after another (A/B builds)
#endif
#define MCCD_POSEW 128   // the four perturbed poses (24 doubles each: R1 R2 x1 x2)
struct PairCtxW {
  PairCtx base;          // the pair's hulls, radii and cylinder sizes (its poses unused)
  const double* pose;    // the four perturbed poses
  double cx1[3], cx2[3];  // this lane's group's perturbed centres
};
DEVI void mpr_centres(const PairCtxW& c, const Dat&, int, int, double* a, double* b) {
#pragma unroll
  for (int k = 0; k < 3; k++) { a[k] = c.cx1[k]; b[k] = c.cx2[k]; }
}
DEVI void mink_support(const PairCtxW& c, const double* dir, SupPt* p, unsigned long long act) {
  const int grp = lane_id() >> 4;
#pragma unroll 1
  for (int g = 0; g < 4; g++) {
    if (!((act >> (16 * g)) & 1ull)) continue;
    double dg[3] = {readlane_d(dir[0], 16 * g), readlane_d(dir[1], 16 * g), readlane_d(dir[2], 16 * g)};
    PairCtx q = c.base;
    const double* P = c.pose + 24 * g;
#pragma unroll
    for (int k = 0; k < 9; k++) { q.R1[k] = P[k]; q.R2[k] = P[9 + k]; }
#pragma unroll
    for (int k = 0; k < 3; k++) { q.x1[k] = P[18 + k]; q.x2[k] = P[21 + k]; }
    SupPt t;
    mink_support(q, dg, &t);
    if (grp == g) {
#pragma unroll
      for (int k = 0; k < 3; k++) { p->a[k] = t.a[k]; p->b[k] = t.b[k]; }
    }
  }
  sub3(p->v, p->a, p->b);
}
DEVI void multiccd_w(const Mdl& md, Dat& d, int pair, int g1, int g2, const double* n, const double* pos) {
  mccd_list_init(d, pos);
#pragma unroll 1
  for (int q = 0; q < 4; q++) mccd_perturb(d, d, g1, g2, n, pos, q, MCCD_POSEW + 24 * q);
  const int lane = lane_id(), grp = lane >> 4;
  {
    PairCtxW pc;
    pair_ctx(md, d, g1, g2, pc.base);
    pc.pose = (const double*)d.poly + MCCD_POSEW;
    const double* P = pc.pose + 24 * grp;
#pragma unroll
    for (int k = 0; k < 3; k++) { pc.cx1[k] = P[18 + k]; pc.cx2[k] = P[21 + k]; }
    double nn[3], dd = 0.0, pp[3], dir[3] = {0.0, 0.0, 0.0};
    const int hit = ccd_mpr_q(md, d, pc, nn, &dd, pp);
    if ((lane & 15) == 0) mccd_store(d, MCCD_RES + 12 * grp, hit, nn, pp, dir, dd, -1.0);
    wsync();
  }
  int nc = 1;
  mccd_take_groups(md, d, pair, g1, g2, 4, nc);
}

// convex pairs (ccd_mode 1 / 2; oracle collide_convex_mj): one pair on the
// whole wave, or two pairs whose hulls fit 16-lane rows at once on the two
// halves (pairB >= 0); then per pair in order its certificate, first contact
// and multiccd -- four perturbed MPRs on 16-lane groups when both hulls have
// at most 8 vertices and no cylinder, else one after another through the
// whole-wave MPR call site the single pair's first MPR uses (each MPR
// instance inlined once: more copies spilled the eight-per-CU object)
DEVI void collide_convex_mj(const Mdl& md, Dat& d, int pairA, int pairB, int mccd) {
  const int lane = lane_id();
  const int32_t *p1 = IA(md, pair_geom1), *p2 = IA(md, pair_geom2);
  const int32_t *ghull = IA(md, geom_hullid), *hnum = IA(md, hull_vertnum);
  const double* cy = DA(md, geom_cyl);
  const int ncmax = md.m.ncon_max;
  if (pairB >= 0) {
    // both pairs' first MPRs at once, results through LDS (held in registers
    // across the per-pair stage below they spilled the object)
    const int gA1 = p1[pairA], gA2 = p2[pairA], gB1 = p1[pairB], gB2 = p2[pairB];
    PairCtx2 q;
    pair_ctx2(md, d, gA1, gA2, gB1, gB2, q);
    const int g1 = lane < 32 ? gA1 : gB1, g2 = lane < 32 ? gA2 : gB2;
    double n[3], depth, pos[3], cd[3], cm;
    const int hit = ccd_mpr(md, d, q, g1, g2, n, &depth, pos, cd, &cm);
    if ((lane & 31) == 0) mccd_store(d, MCCD_RES2 + 12 * (lane >> 5), hit, n, pos, cd, depth, cm);
    wsync();
  }
  const int np = pairB >= 0 ? 2 : 1;
  const double* cp = (const double*)d.poly;
#pragma unroll 1
  for (int k = 0; k < np; k++) {
    const int pair = k ? pairB : pairA;
    const int G1 = p1[pair], G2 = p2[pair];
    const bool multi = mccd && md.m.ccd_mode == MGS_CCD_MULTI && IA(md, pair_kind)[pair] == MGS_PAIR_CONVEX;
    int nc = 0;
#pragma unroll 1
    for (int it = 0; it < 5; it++) {
      if (it > 0 || pairB < 0) {
        PairCtx pc;
        if (it > 0) {
          mccd_perturb(d, d, G1, G2, cp + MCCD_N, cp, it - 1, MCCD_POSE);
          const double* pz = cp + MCCD_POSE;
          pair_ctx_pose(md, G1, G2, pz, pz + 18, pz + 9, pz + 21, pc);
        } else {
          pair_ctx(md, d, G1, G2, pc);
        }
        double n[3], depth, pos[3], cd[3], cm;
        const int hit = ccd_mpr(md, d, pc, G1, G2, n, &depth, pos, cd, &cm);
        wsync();
        if (lane == 0) mccd_store(d, MCCD_RES, hit, n, pos, cd, depth, cm);
        wsync();
      }
      const double* r = it == 0 && pairB >= 0 ? cp + MCCD_RES2 + 12 * k : cp + MCCD_RES;
      const int hk = r[11] != 0.0;
      if (it == 0) {
        PT(4);
        cert_update(md, d, pair, G1, G2, hk, r + 6, r[10]);
        PCNT(26, 1);
        PCNT(27, hk);
        if (!hk) break;
        double t1[3], t2[3];
        make_frame(r, t1, t2);
        if (lane == 0) add_contact(d, ncmax, pair, G1, G2, r + 3, r, t1, t2, -r[9]);
        wsync();
        if (!multi) break;
        const int nm1 = hnum[ghull[G1]], nm2 = hnum[ghull[G2]];
        const bool cyl = cy[2 * G1] > 0.0 || cy[2 * G2] > 0.0;
        if (MGS_MCCD_Q && !cyl && nm1 <= 8 && nm2 <= 8) {
          double n0[3] = {r[0], r[1], r[2]}, p0[3] = {r[3], r[4], r[5]};
          multiccd_q<8>(md, d, pair, G1, G2, n0, p0);
          break;
        }
        if (MGS_MCCD_W) {
          double n0[3] = {r[0], r[1], r[2]}, p0[3] = {r[3], r[4], r[5]};
          multiccd_w(md, d, pair, G1, G2, n0, p0);
          break;
        }
        // the first contact: the list's first entry and the perturbation frame
        if (lane == 0) {
          double* w = (double*)d.poly;
#pragma unroll
          for (int i = 0; i < 3; i++) { w[i] = r[3 + i]; w[MCCD_N + i] = r[i]; }
        }
        wsync();
        nc = 1;
      } else {
        if (!hk) continue;
        double pk[3] = {r[3], r[4], r[5]};
        if (!mccd_is_new(d, nc, pk, mccd_tol(md, G1, G2))) continue;
        double nk[3] = {r[0], r[1], r[2]};
        const double dk = r[9];
        mccd_list_add(d, nc, pk);
        nc++;
        double u1[3], u2[3];
        make_frame(nk, u1, u2);
        if (lane == 0) add_contact(d, ncmax, pair, G1, G2, pk, nk, u1, u2, -dk);
      }
    }
    wsync();
  }
  PT(41);
}

// analytic primitive colliders (oracle collide_prim): every lane computes the
// same values (the capsule-box candidates: one per lane), lane 0 adds them
DEVI double kdist3(const double* a, const double* b) {
  double dx[3];
  sub3(dx, a, b);
  return sqrt(dot3(dx, dx));
}
DEVI int raw_sphere_sphere(const double* p1, const double* z1, double r1, const double* p2, const double* z2,
                           double r2, double margin, double* pos, double* n, double* dist) {
  double dd = (kdist3(p1, p2) - r1) - r2;
  if (dd > margin) return 0;
  sub3(n, p2, p1);
  if (normalize3(n) < K_MINVAL) {
    cross3(n, z1, z2);
    normalize3(n);
  }
  double s = r1 + 0.5 * dd;
#pragma unroll
  for (int k = 0; k < 3; k++) pos[k] = p1[k] + n[k] * s;
  *dist = dd;
  return 1;
}
DEVI int raw_sphere_box(const double* c, double r, const double* x, const double* R, const double* s, double margin,
                        double* pos, double* n, double* dist) {
  double t[3], cl[3], q[3], df[3], nl[3], pl[3];
  sub3(t, c, x);
  mulmtv3(cl, R, t);
#pragma unroll
  for (int k = 0; k < 3; k++) q[k] = cl[k] < -s[k] ? -s[k] : (cl[k] > s[k] ? s[k] : cl[k]);
  sub3(df, q, cl);
  double dc = sqrt(dot3(df, df));
  if (dc - r > margin) return 0;
  double dd;
  if (dc > K_MINVAL) {
#pragma unroll
    for (int k = 0; k < 3; k++) nl[k] = df[k] / dc;
    dd = dc - r;
  } else {
    int kk = 0;
    double a = s[0] - fabs(cl[0]);
    double a1 = s[1] - fabs(cl[1]);
    if (a1 < a) { a = a1; kk = 1; }
    double a2 = s[2] - fabs(cl[2]);
    if (a2 < a) { a = a2; kk = 2; }
    double sgn = (kk == 0 ? cl[0] : (kk == 1 ? cl[1] : cl[2])) >= 0.0 ? -1.0 : 1.0;
    nl[0] = kk == 0 ? sgn : 0.0;
    nl[1] = kk == 1 ? sgn : 0.0;
    nl[2] = kk == 2 ? sgn : 0.0;
    dd = -(a + r);
  }
  double h = r + 0.5 * dd;
#pragma unroll
  for (int k = 0; k < 3; k++) pl[k] = cl[k] + nl[k] * h;
  mulmv3(n, R, nl);
  mulmv3(t, R, pl);
  add3(pos, x, t);
  *dist = dd;
  return 1;
}
DEVI double box_phi(const double* p, const double* s) {
  double o0 = fabs(p[0]) - s[0], o1 = fabs(p[1]) - s[1], o2 = fabs(p[2]) - s[2];
  if (o0 > 0.0 || o1 > 0.0 || o2 > 0.0) {
    double a = o0 > 0.0 ? o0 : 0.0, b = o1 > 0.0 ? o1 : 0.0, c = o2 > 0.0 ? o2 : 0.0;
    return sqrt((a * a + b * b) + c * c);
  }
  double m = o0 > o1 ? o0 : o1;
  return m > o2 ? m : o2;
}
// oracle capbox_cand: candidate k of the segment parameter (0 if it does not exist)
DEVI int capbox_cand(int k, const double* c, const double* a, const double* s, double* tout) {
  double t;
  if (k < 2) { *tout = k ? 1.0 : -1.0; return 1; }
  if (k < 8) {
    int i = (k - 2) >> 1;
    double sg = ((k - 2) & 1) ? 1.0 : -1.0;
    double ai = i == 0 ? a[0] : (i == 1 ? a[1] : a[2]);
    double ci = i == 0 ? c[0] : (i == 1 ? c[1] : c[2]);
    double si = i == 0 ? s[0] : (i == 1 ? s[1] : s[2]);
    if (fabs(ai) < K_MINVAL) return 0;
    t = (sg * si - ci) / ai;
  } else if (k < 34) {
    int code = k - 8 + 1;
    double num = 0.0, den = 0.0;
#pragma unroll
    for (int i = 0; i < 3; i++) {
      int dgt = code % 3;
      code /= 3;
      if (dgt != 0) {
        double sg = dgt == 1 ? -1.0 : 1.0;
        num = num + (c[i] - sg * s[i]) * a[i];
        den = den + a[i] * a[i];
      }
    }
    if (den < K_MINVAL) return 0;
    t = -num / den;
    t = t < -1.0 ? -1.0 : (t > 1.0 ? 1.0 : t);
    *tout = t;
    return 1;
  } else {
    int q = k - 34, l1 = 0, l2 = 1;
    for (int x = 0; x < 6; x++)
      for (int y = x + 1; y < 6; y++) {
        if (q == 0) { l1 = x; l2 = y; }
        q--;
      }
    int i = l1 >> 1, j = l2 >> 1;
    double si = (l1 & 1) ? 1.0 : -1.0, sj = (l2 & 1) ? 1.0 : -1.0;
    double ai = i == 0 ? a[0] : (i == 1 ? a[1] : a[2]), aj = j == 0 ? a[0] : (j == 1 ? a[1] : a[2]);
    double ci = i == 0 ? c[0] : (i == 1 ? c[1] : c[2]), cj = j == 0 ? c[0] : (j == 1 ? c[1] : c[2]);
    double Si = i == 0 ? s[0] : (i == 1 ? s[1] : s[2]), Sj = j == 0 ? s[0] : (j == 1 ? s[1] : s[2]);
    double coef = si * ai - sj * aj;
    if (fabs(coef) < K_MINVAL) return 0;
    t = ((Si - Sj) - (si * ci - sj * cj)) / coef;
  }
  if (!(t >= -1.0 && t <= 1.0)) return 0;
  *tout = t;
  return 1;
}
DEVI void collide_prim(const Mdl& md, Dat& d, int pair, int kind) {
  const int lane = lane_id();
  int g1 = IA(md, pair_geom1)[pair], g2 = IA(md, pair_geom2)[pair];
  double R1[9], R2[9], x1[3], x2[3], s1[3], s2[3];
#pragma unroll
  for (int k = 0; k < 9; k++) { R1[k] = d.geom_xmat[9 * g1 + k]; R2[k] = d.geom_xmat[9 * g2 + k]; }
#pragma unroll
  for (int k = 0; k < 3; k++) {
    x1[k] = d.geom_xpos[3 * g1 + k]; x2[k] = d.geom_xpos[3 * g2 + k];
    s1[k] = DA(md, geom_size)[3 * g1 + k]; s2[k] = DA(md, geom_size)[3 * g2 + k];
  }
  const double margin = DA(md, pair_margin)[pair];
  double z1[3] = {R1[2], R1[5], R1[8]}, z2[3] = {R2[2], R2[5], R2[8]};
  double pos0[3], n0[3], dist0, pos1[3] = {0.0, 0.0, 0.0}, n1[3] = {1.0, 0.0, 0.0}, dist1 = 0.0;
  int nc = 0;
  if (kind == MGS_PAIR_SPHERE_SPHERE) {
    nc = raw_sphere_sphere(x1, z1, s1[0], x2, z2, s2[0], margin, pos0, n0, &dist0);
  } else if (kind == MGS_PAIR_SPHERE_CAPSULE) {
    double v[3], q[3];
    sub3(v, x1, x2);
    double xx = dot3(z2, v);
    xx = xx < -s2[1] ? -s2[1] : (xx > s2[1] ? s2[1] : xx);
#pragma unroll
    for (int k = 0; k < 3; k++) q[k] = x2[k] + z2[k] * xx;
    nc = raw_sphere_sphere(x1, z1, s1[0], q, z2, s2[0], margin, pos0, n0, &dist0);
  } else if (kind == MGS_PAIR_CAPSULE_CAPSULE) {
    double a1[3], a2[3], df[3];
#pragma unroll
    for (int k = 0; k < 3; k++) { a1[k] = z1[k] * s1[1]; a2[k] = z2[k] * s2[1]; }
    sub3(df, x1, x2);
    double ma = dot3(a1, a1), mb = -dot3(a1, a2), mc = dot3(a2, a2);
    double u = -dot3(a1, df), v = dot3(a2, df);
    double det = ma * mc - mb * mb;
    double v1[3], v2[3];
    if (fabs(det) >= K_MINVAL) {
      double xa = (mc * u - mb * v) / det, xb = (ma * v - mb * u) / det;
      if (xa > 1.0) { xa = 1.0; xb = (v - mb) / mc; }
      else if (xa < -1.0) { xa = -1.0; xb = (v + mb) / mc; }
      if (xb > 1.0) {
        xb = 1.0;
        xa = (u - mb) / ma;
        xa = xa < -1.0 ? -1.0 : (xa > 1.0 ? 1.0 : xa);
      } else if (xb < -1.0) {
        xb = -1.0;
        xa = (u + mb) / ma;
        xa = xa < -1.0 ? -1.0 : (xa > 1.0 ? 1.0 : xa);
      }
#pragma unroll
      for (int k = 0; k < 3; k++) { v1[k] = x1[k] + a1[k] * xa; v2[k] = x2[k] + a2[k] * xb; }
      nc = raw_sphere_sphere(v1, z1, s1[0], v2, z2, s2[0], margin, pos0, n0, &dist0);
    } else {
      for (int e = 0; e < 4 && nc < 2; e++) {
        double sg = (e & 1) ? -1.0 : 1.0, xx;
        if (e < 2) {
          xx = (sg > 0.0 ? (v - mb) : (v + mb)) / mc;
          xx = xx < -1.0 ? -1.0 : (xx > 1.0 ? 1.0 : xx);
#pragma unroll
          for (int k = 0; k < 3; k++) { v1[k] = x1[k] + sg * a1[k]; v2[k] = x2[k] + a2[k] * xx; }
        } else {
          xx = (sg > 0.0 ? (u - mb) : (u + mb)) / ma;
          xx = xx < -1.0 ? -1.0 : (xx > 1.0 ? 1.0 : xx);
#pragma unroll
          for (int k = 0; k < 3; k++) { v2[k] = x2[k] + sg * a2[k]; v1[k] = x1[k] + a1[k] * xx; }
        }
        double pp[3], nn[3], dd;
        if (raw_sphere_sphere(v1, z1, s1[0], v2, z2, s2[0], margin, pp, nn, &dd)) {
          if (nc == 0) {
#pragma unroll
            for (int k = 0; k < 3; k++) { pos0[k] = pp[k]; n0[k] = nn[k]; }
            dist0 = dd;
          } else {
#pragma unroll
            for (int k = 0; k < 3; k++) { pos1[k] = pp[k]; n1[k] = nn[k]; }
            dist1 = dd;
          }
          nc++;
        }
      }
    }
  } else if (kind == MGS_PAIR_SPHERE_BOX) {
    nc = raw_sphere_box(x1, s1[0], x2, R2, s2, margin, pos0, n0, &dist0);
  } else if (kind == MGS_PAIR_CAPSULE_BOX) {
    double t[3], c[3], a[3], hz[3];
    sub3(t, x1, x2);
    mulmtv3(c, R2, t);
#pragma unroll
    for (int k = 0; k < 3; k++) hz[k] = z1[k] * s1[1];
    mulmtv3(a, R2, hz);
    // candidate k on lane k, then the first (lowest k) of the smallest phi
    double tk = 0.0, ph = INFINITY;
    if (lane < MGS_CB_NCAND && capbox_cand(lane, c, a, s2, &tk)) {
      double p[3] = {c[0] + a[0] * tk, c[1] + a[1] * tk, c[2] + a[2] * tk};
      ph = box_phi(p, s2);
    }
    double m = ph;
#pragma unroll
    for (int sel = 0; sel < 4; sel++) { double o = dpp_d(m, sel); m = o < m ? o : m; }
    double M = readlane_d(m, 0);
    double r1 = readlane_d(m, 16), r2 = readlane_d(m, 32), r3 = readlane_d(m, 48);
    M = r1 < M ? r1 : M;
    M = r2 < M ? r2 : M;
    M = r3 < M ? r3 : M;
    unsigned long long tied = __ballot(ph == M);
    int wl = tied ? __ffsll((long long)tied) - 1 : 0;
    double tb = readlane_d(tk, wl);
    double ctr[3];
#pragma unroll
    for (int k = 0; k < 3; k++) ctr[k] = x1[k] + hz[k] * tb;
    nc = raw_sphere_box(ctr, s1[0], x2, R2, s2, margin, pos0, n0, &dist0);
    if (nc) {
      double pe0[3], ne0[3], de0, pe1[3], ne1[3], de1, ce[3];
#pragma unroll
      for (int k = 0; k < 3; k++) ce[k] = x1[k] - hz[k];
      int ok = raw_sphere_box(ce, s1[0], x2, R2, s2, margin, pe0, ne0, &de0) && ne0[0] == n0[0] &&
               ne0[1] == n0[1] && ne0[2] == n0[2];
      if (ok) {
#pragma unroll
        for (int k = 0; k < 3; k++) ce[k] = x1[k] + hz[k];
        ok = raw_sphere_box(ce, s1[0], x2, R2, s2, margin, pe1, ne1, &de1) && ne1[0] == n0[0] &&
             ne1[1] == n0[1] && ne1[2] == n0[2];
      }
      if (ok) {
#pragma unroll
        for (int k = 0; k < 3; k++) { pos0[k] = pe0[k]; n0[k] = ne0[k]; pos1[k] = pe1[k]; n1[k] = ne1[k]; }
        dist0 = de0;
        dist1 = de1;
        nc = 2;
      }
    }
  } else if (kind == MGS_PAIR_SPHERE_CYLINDER) {
    double t[3], cl[3], q[3], df[3], nl[3], pl[3];
    const double r = s1[0], cr = s2[0], ch = s2[1];
    sub3(t, x1, x2);
    mulmtv3(cl, R2, t);
    double rho = sqrt(cl[0] * cl[0] + cl[1] * cl[1]);
    if (rho > cr) { q[0] = cl[0] / rho * cr; q[1] = cl[1] / rho * cr; }
    else { q[0] = cl[0]; q[1] = cl[1]; }
    q[2] = cl[2] < -ch ? -ch : (cl[2] > ch ? ch : cl[2]);
    sub3(df, q, cl);
    double dc = sqrt(dot3(df, df)), dd;
    if (dc - r <= margin) {
      if (dc > K_MINVAL) {
#pragma unroll
        for (int k = 0; k < 3; k++) nl[k] = df[k] / dc;
        dd = dc - r;
      } else {
        double side = cr - rho, cap = ch - fabs(cl[2]), a;
        if (side < cap && rho > K_MINVAL) {
          nl[0] = -(cl[0] / rho); nl[1] = -(cl[1] / rho); nl[2] = 0.0;
          a = side;
        } else {
          nl[0] = nl[1] = 0.0;
          nl[2] = cl[2] >= 0.0 ? -1.0 : 1.0;
          a = cap;
        }
        dd = -(a + r);
      }
      double h = r + 0.5 * dd;
#pragma unroll
      for (int k = 0; k < 3; k++) pl[k] = cl[k] + nl[k] * h;
      mulmv3(n0, R2, nl);
      mulmv3(t, R2, pl);
      add3(pos0, x2, t);
      dist0 = dd;
      nc = 1;
    }
  }
  if (lane == 0) {
    const int ncmax = md.m.ncon_max;
    double t1[3], t2[3];
    if (nc > 0) {
      make_frame(n0, t1, t2);
      add_contact(d, ncmax, pair, g1, g2, pos0, n0, t1, t2, dist0);
    }
    if (nc > 1) {
      make_frame(n1, t1, t2);
      add_contact(d, ncmax, pair, g1, g2, pos1, n1, t1, t2, dist1);
    }
  }
  wsync();
}

/* Second broadphase stage: separating-axis test between the geoms' oriented
 * bounding boxes (their local AABBs posed in the world; 15 axes).  Each convex
 * hull lies inside its box, so separated boxes cannot produce a contact and the
 * narrowphase is skipped (MuJoCo would run MPR and find nothing; on the round-1
 * benchmark this removes ~55% of narrowphase calls).  The oracle's
 * obb_separated tests the axes in turn; here a pair is separated iff one of its
 * 15 axis tests is, so the axes run on lanes: one pass takes up to 4 pairs,
 * 16 lanes each (lane q of a group = axis q; q = 15 idles).
 *
 * One axis test, the expressions of the oracle's loop body for axis q: D = c2 -
 * c1 (the posed box centres), h1 / h2 the half widths, A1 / A2 the box axes
 * (columns of R1 / R2, read from LDS).  The axis is chosen by selects with
 * constant indices (a computed index into a register array would go through
 * scratch). */
DEVI int obb_axis_separated(int q, const double* R1, const double* R2, const double* D, const double* h1,
                            const double* h2, double margin) {
  double A1[9], A2[9];  /* box axes as rows: A[k] = column k of R */
#pragma unroll
  for (int k = 0; k < 3; k++)
#pragma unroll
    for (int i = 0; i < 3; i++) { A1[3 * k + i] = R1[3 * i + k]; A2[3 * k + i] = R2[3 * i + k]; }
  // the axis' vectors straight from LDS by per-lane column (a select between
  // register values would be folded into a select of addresses and put A1 / A2
  // in scratch)
  const int qa = q < 6 ? 0 : (q - 6) / 3, qb = q < 6 ? 0 : (q - 6) % 3;
  const double* Rf = q < 3 ? R1 : R2;
  const int kf = q < 3 ? q : (q < 6 ? q - 3 : 0);
  double e1[3], e2[3], L[3], cx[3];
#pragma unroll
  for (int i = 0; i < 3; i++) {
    e1[i] = R1[3 * i + qa];
    e2[i] = R2[3 * i + qb];
  }
  cross3(cx, e1, e2);
#pragma unroll
  for (int i = 0; i < 3; i++) L[i] = q < 6 ? Rf[3 * i + kf] : cx[i];
  double ll = dot3(L, L);
  if (ll < 1e-20) return 0;
  double r1 = (h1[0] * fabs(dot3(A1, L)) + h1[1] * fabs(dot3(A1 + 3, L))) + h1[2] * fabs(dot3(A1 + 6, L));
  double r2 = (h2[0] * fabs(dot3(A2, L)) + h2[1] * fabs(dot3(A2 + 3, L))) + h2[2] * fabs(dot3(A2 + 6, L));
  return fabs(dot3(D, L)) > (r1 + r2) + (margin + 1e-12) * sqrt(ll);
}

/* the chunk's pairs in `am` (AABB-overlapping) whose boxes are separated; lane
 * b of the chunk holds pair b's g1, g2, D, half widths and margin */
DEVI unsigned long long obb_separated_wave(const Dat& d, unsigned long long am, int g1, int g2, const double* D,
                                           const double* h1, const double* h2, double margin) {
  const int lane = lane_id(), grp = lane >> 4, q = lane & 15;
  unsigned long long sep = 0ull;
  while (am) {
    unsigned long long m = am;      // this group's pair: the grp-th lowest bit
    for (int t = 0; t < grp; t++) m &= m - 1ull;
    int b = m ? __ffsll((long long)m) - 1 : 0;
    int G1 = shfl(g1, b), G2 = shfl(g2, b);
    double Db[3], h1b[3], h2b[3];
#pragma unroll
    for (int i = 0; i < 3; i++) {
      Db[i] = shfl(D[i], b);
      h1b[i] = shfl(h1[i], b);
      h2b[i] = shfl(h2[i], b);
    }
    double mb = shfl(margin, b);
    int s = 0;
    if (m && q < 15) s = obb_axis_separated(q, d.geom_xmat + 9 * G1, d.geom_xmat + 9 * G2, Db, h1b, h2b, mb);
    unsigned long long sm = __ballot(s);
#pragma unroll
    for (int k = 0; k < 4; k++) {
      if (!am) break;
      int bk = __ffsll((long long)am) - 1;
      if ((sm >> (16 * k)) & 0x7fffull) sep |= 1ull << bk;
      am &= am - 1ull;
    }
  }
  return sep;
}

// broadphase over all admissible pairs (lanes over pairs), then narrowphase in
// pair order.  mccd 0 (the collision masks: forward(full 0)): no multiccd --
// its contacts repeat a pair that already has one, so no mask predicate can
// change, and they cannot crowd a later pair's first contact out of the
// capacity (oracle_collision_free, the same rule)
DEVI void collision(const Mdl& md, Dat& d, int mccd = 1) {
  int lane = lane_id();
  const int32_t *p1 = IA(md, pair_geom1), *p2 = IA(md, pair_geom2);
  const double *aabb = DA(md, geom_aabb), *pm = DA(md, pair_margin);
  if (lane == 0) d.NCON = 0;
  wsync();
  int npair = md.m.npair;
  for (int c0 = 0; c0 < npair; c0 += WAVE) {
    int p = c0 + lane;
    int ov = 0;
    int g[2] = {0, 0};
    double c[2][3], hw[2][3], D[3] = {0.0, 0.0, 0.0}, h[2][3] = {{0.0, 0.0, 0.0}, {0.0, 0.0, 0.0}}, mp = 0.0;
    if (p < npair) {
      g[0] = p1[p];
      g[1] = p2[p];
      mp = pm[p];
      for (int s = 0; s < 2; s++) {
        const double* R = d.geom_xmat + 9 * g[s];
        const double* lc = aabb + 6 * g[s];
        const double* lh = lc + 3;
        double t[3];
        mulmv3(t, R, lc);
        add3(c[s], d.geom_xpos + 3 * g[s], t);
        for (int k = 0; k < 3; k++) {
          h[s][k] = lh[k];
          hw[s][k] = (fabs(R[3 * k]) * lh[0] + fabs(R[3 * k + 1]) * lh[1]) + fabs(R[3 * k + 2]) * lh[2];
        }
      }
      ov = 1;
      for (int k = 0; k < 3; k++)
        if (fabs(c[0][k] - c[1][k]) > (hw[0][k] + hw[1][k]) + mp) ov = 0;
      sub3(D, c[1], c[0]);
    }
    PT(59);
    // convex pairs whose four hulls fit 16-lane rows may go two at a time
    int small2 = 0;
    const int pk = p < npair ? IA(md, pair_kind)[p] : MGS_PAIR_BOXBOX;
    const bool mpr_pair = md.m.ccd_mode == MGS_CCD_R5 ? pk != MGS_PAIR_BOXBOX
                                                       : (pk == MGS_PAIR_CONVEX || pk == MGS_PAIR_CONVEX_SMOOTH);
    if (ov && mpr_pair) {
      const int32_t *ghull = IA(md, geom_hullid), *hnum = IA(md, hull_vertnum);
      small2 = hnum[ghull[g[0]]] <= 16 && hnum[ghull[g[1]]] <= 16;
    }
    const unsigned long long smallm = __ballot(small2);
    unsigned long long mask = __ballot(ov);
    mask &= ~obb_separated_wave(d, mask, g[0], g[1], D, h[0], h[1], mp);
    PT(60);
    mask &= ~cert_check(md, d, c0, mask);
    PT(3);
    while (mask) {
      int b = __ffsll((long long)mask) - 1;
      mask &= mask - 1ull;
      const int kind = IA(md, pair_kind)[c0 + b];
      if (((smallm >> b) & 1ull) && mask && ((smallm >> (__ffsll((long long)mask) - 1)) & 1ull)) {
        int b2 = __ffsll((long long)mask) - 1;
        mask &= mask - 1ull;
        if (md.m.ccd_mode == MGS_CCD_R5) collide_pair2(md, d, c0 + b, c0 + b2);
        else collide_convex_mj(md, d, c0 + b, c0 + b2, mccd);
      } else if (kind == MGS_PAIR_BOXBOX) {
        collide_boxbox(md, d, c0 + b);
      } else if (md.m.ccd_mode == MGS_CCD_R5) {
        collide_pair(md, d, c0 + b);
      } else if (kind == MGS_PAIR_CONVEX || kind == MGS_PAIR_CONVEX_SMOOTH) {
        collide_convex_mj(md, d, c0 + b, -1, mccd);
      } else {
        collide_prim(md, d, c0 + b, kind);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// LDS layout (offsets in doubles; computed on the host by make_layout)
// LDS carve-up (make_layout in mgs_capi.hip).  Persistent arrays live for the
// whole step; the U region is time-multiplexed between stages:
//   kin/collision: polygon buffers, geom poses, xipos/xanchor/xaxis, comPos sums
//   dynamics:      crb | cvel, cacc, cfrc, cdof_dot, qfrc_bias/passive/actuator
//   constraints:   G, aref, {vel,pos,margin | Newton Hessian}, scratch, Newton rows
//   integration:   qDeriv
enum {
  L_qpos, L_qvel, L_qacc_ws, L_ctrl, L_mocap_pos, L_mocap_quat, L_time, L_act, L_act_dot,
  L_xpos, L_xquat, L_xmat, L_subtree_com, L_cinert, L_cdof,
  L_M, L_Dv, L_Dinv, L_sD, L_isD, L_tmp, L_tmp2,
  L_qfrc_smooth, L_qacc_smooth, L_qfrc_constraint,
  L_act_force, L_act_moment, L_act_length, L_act_vel,
  L_con_pos, L_con_frame, L_con_dist, L_con_mu, L_con_blk,
  L_efc_R, L_efc_b, L_cert,
  L_U, L_ints, L_COUNT
};
enum {
  U_poly, U_pdep, U_geom_xpos, U_geom_xmat, U_xipos, U_xanchor, U_xaxis, U_subtree_mass, U_comacc,
  U_crb, U_cvel, U_cacc, U_cfrc, U_cdof_dot, U_qfrc_bias, U_qfrc_passive, U_qfrc_actuator,
  U_G, U_aref, U_vel, U_pos, U_margin, U_nH, U_scratch, U_jar, U_jv, U_f, U_Dr, U_isR, U_nw, U_nw0, U_ng,
  U_ndir, U_qDeriv, U_COUNT
};
// doubles of one candidate's HBM slice (G rows, and with MGS_HBM_EXTRA the
// certificates, contact frames and contact blocks); mgs_capi.hip's hbm_slice
// allocates the same
#ifndef MGS_HBM_EXTRA
#define MGS_HBM_EXTRA 0
#endif
DEVI size_t hbm_slice(int ne, int nv, int nc) {
  return (size_t)ne * nv + (MGS_HBM_EXTRA ? (size_t)(K_CERT * CERT_W + 9 * nc + BLKSTRIDE * nc) : 0);
}
struct Lay {
  int o[L_COUNT];
  int u[U_COUNT];   // offsets relative to o[L_U]
  int ncon_max, nefc_max, nv;
  int total_doubles;
  double* gmem;     // MGS_G_GLOBAL: per-candidate G rows in HBM (nefc_max * nv doubles each)
};

// Model specialisation: a code object compiled for one model (mgs_special.hip
// with the header mgs.core.special generates for it, -DMGS_SPECIAL=<header>)
// carries that model's LDS carve-up and description as compile-time constants.
// A kernel instantiated with SL = 1 binds every view at a constant LDS address,
// so the ~80 views need no SGPRs (their spills to VGPR lanes and reloads
// disappear), LDS accesses carry their offsets as instruction immediates, and
// sizes / table offsets / options are constants (trip counts, immediates).
// The host attaches such an object to a model only after comparing the
// object's baked description and layout with the model's
// (mgs_model_attach_special).
#ifdef MGS_SPECIAL
#include MGS_SPECIAL
static_assert(MGS_SL_ABI == MGS_ABI_VERSION, "specialisation header of another ABI version: regenerate it");
static_assert(MGS_SL_DESC_BYTES == sizeof(mgs_model_desc), "specialisation header of another mgs_model_desc");
#else
#define MGS_SL_NV 0
constexpr int mgs_sl_words[L_COUNT + U_COUNT + 4] = {0};
constexpr mgs_model_desc mgs_sl_desc = {};
#endif
static_assert(sizeof(mgs_sl_words) == sizeof(int) * (L_COUNT + U_COUNT + 4), "specialised layout size");

template <int SL>
DEVI void bind(Dat& d, double* s, const Lay& l) {
#define LO(k) (SL ? mgs_sl_words[k] : l.o[k])
#define LU(k) (SL ? mgs_sl_words[L_COUNT + (k)] : l.u[k])
#define B(f) d.f = s + LO(L_##f)
  B(qpos); B(qvel); B(qacc_ws); B(ctrl); B(mocap_pos); B(mocap_quat); B(time); B(act); B(act_dot);
  B(xpos); B(xquat); B(xmat); B(subtree_com); B(cinert); B(cdof);
  B(M); B(Dv); B(Dinv); B(sD); B(isD); B(tmp); B(tmp2);
  B(qfrc_smooth); B(qacc_smooth); B(qfrc_constraint);
  B(act_force); B(act_moment); B(act_length); B(act_vel);
  B(con_pos); B(con_frame); B(con_dist); B(con_mu); B(con_blk);
  B(efc_R); B(efc_b); B(cert);
#undef B
  double* U = s + LO(L_U);
#define BU(f, k) d.f = U + LU(k)
  d.poly = (P2*)(U + LU(U_poly));
  BU(pdep, U_pdep); BU(geom_xpos, U_geom_xpos); BU(geom_xmat, U_geom_xmat); BU(xipos, U_xipos);
  BU(xanchor, U_xanchor); BU(xaxis, U_xaxis); BU(subtree_mass, U_subtree_mass); BU(comacc, U_comacc);
  BU(crb, U_crb); BU(cvel, U_cvel); BU(cacc, U_cacc); BU(cfrc, U_cfrc); BU(cdof_dot, U_cdof_dot);
  BU(qfrc_bias, U_qfrc_bias); BU(qfrc_passive, U_qfrc_passive); BU(qfrc_actuator, U_qfrc_actuator);
#ifdef MGS_G_GLOBAL
  // wide library (clutter piles): G = D^-1/2 L^-1 J' is too large for LDS at
  // nefc_max 256 x nv 58; it lives in this candidate's HBM slice (L2-cached).
  // Main-library objects with G in HBM (MGS_HBM_EXTRA) keep the separation
  // certificates, the contact frames and the contact blocks there too.
  {
    const int sl_nc = SL ? mgs_sl_words[L_COUNT + U_COUNT] : l.ncon_max;
    const int sl_ne = SL ? mgs_sl_words[L_COUNT + U_COUNT + 1] : l.nefc_max;
    const int sl_nv = SL ? mgs_sl_words[L_COUNT + U_COUNT + 2] : l.nv;
    d.G = l.gmem + (size_t)blockIdx.x * hbm_slice(sl_ne, sl_nv, sl_nc);
#if MGS_HBM_EXTRA
    double* x = d.G + (size_t)sl_ne * sl_nv;
    d.cert = x;
    x += K_CERT * CERT_W;
    d.con_frame = x;
    x += 9 * sl_nc;
    d.con_blk = x;
#endif
  }
#else
  BU(G, U_G);
#endif
  BU(efc_aref, U_aref); BU(efc_vel, U_vel); BU(efc_pos, U_pos); BU(efc_margin, U_margin);
  BU(nH, U_nH); BU(scratch, U_scratch); BU(efc_jar, U_jar); BU(efc_jv, U_jv); BU(efc_f, U_f);
  BU(efc_Dr, U_Dr); BU(efc_isR, U_isR); BU(nw, U_nw); BU(nw0, U_nw0); BU(ng, U_ng); BU(ndir, U_ndir);
  BU(qDeriv, U_qDeriv);
#undef BU
  d.con_hb = d.con_blk;   // Newton cone Hessians reuse the contact-block slots
  d.gs = (SL ? mgs_sl_words[L_COUNT + U_COUNT + 2] : l.nv) + MGS_GPAD;
  int* ib = (int*)(s + LO(L_ints));
  d.ints = ib;
  int ncmax = SL ? mgs_sl_words[L_COUNT + U_COUNT] : l.ncon_max;
  int nemax = SL ? mgs_sl_words[L_COUNT + U_COUNT + 1] : l.nefc_max;
  d.con_pair = ib + 16;
  d.con_g1 = d.con_pair + ncmax;
  d.con_g2 = d.con_g1 + ncmax;
  d.efc_type = d.con_g2 + ncmax;
  d.efc_dim = d.efc_type + nemax;
  d.efc_con = d.efc_dim + nemax;
  d.efc_state = d.efc_con + nemax;
#undef LO
#undef LU
}

// A_rr = G_r . G_r in the oracle's order (its efc_A)
DEVI double row_sqnorm(const Dat& d, int r, int nv) {
  const double* Gr = d.G + r * d.gs;
  double a = 0.0;
  for (int k = 0; k < nv; k++) a = a + Gr[k] * Gr[k];
  return a;
}

// first row of its block (contacts span dim rows with one efc_con)
DEVI int efc_lead(const Dat& d, int r) {
  return d.efc_type[r] != MGS_EFC_CONTACT || r == 0 || d.efc_type[r - 1] != MGS_EFC_CONTACT ||
         d.efc_con[r - 1] != d.efc_con[r];
}

// contact c's friction coefficients (see MGS_MU_MODEL)
DEVI const double* con_mu_of(const Mdl& md, const Dat& d, int c) {
#if MGS_MU_MODEL
  return DA(md, pair_friction) + 5 * d.con_pair[c];
#else
  (void)md;
  return d.con_mu + 5 * c;
#endif
}

// frictionloss of a FRICTION row (its efc_con is the dof), 0 otherwise
DEVI double row_floss(const Mdl& md, const Dat& d, int r) {
  return d.efc_type[r] == MGS_EFC_FRICTION ? DA(md, dof_frictionloss)[d.efc_con[r]] : 0.0;
}

// ---------------------------------------------------------------------------
// constraints
DEVI void jac_point(const Mdl& md, const Dat& d, int b, const double* pt, double* jacp, double* jacr) {
  int nv = md.m.nv;
  for (int k = 0; k < 3 * nv; k++) { jacp[k] = 0.0; jacr[k] = 0.0; }
  int dof = IA(md, body_lastdof)[b];
  const int32_t* dpar = IA(md, dof_parentid);
  const double* c = d.subtree_com + 3 * IA(md, body_rootid)[b];
  double off[3];
  sub3(off, pt, c);
  while (dof >= 0) {
    const double* cd = d.cdof + 6 * dof;
    double cr[3];
    cross3(cr, cd, off);
    for (int k = 0; k < 3; k++) {
      jacr[k * nv + dof] = cd[k];
      jacp[k * nv + dof] = cd[3 + k] + cr[k];
    }
    dof = dpar[dof];
  }
}

// column `col` of the point Jacobian of body b at pt (oracle jac_point(), one
// dof per lane): zero unless dof col moves the body (model body_dofmask).
DEVI void jac_col(const Mdl& md, const Dat& d, int b, const double* pt, int col, double* jp, double* jr) {
  if (dof_moves(md, b, col)) {
    const double* cd = d.cdof + 6 * col;
    const double* c = d.subtree_com + 3 * IA(md, body_rootid)[b];
    double off[3], cr[3];
    sub3(off, pt, c);
    cross3(cr, cd, off);
    for (int k = 0; k < 3; k++) {
      jr[k] = cd[k];
      jp[k] = cd[3 + k] + cr[k];
    }
  } else {
    for (int k = 0; k < 3; k++) { jr[k] = 0.0; jp[k] = 0.0; }
  }
}

DEVI double impedance(const double* si, double pos, double margin) {
  if (si[0] == si[1] || si[2] <= K_MINVAL) return 0.5 * (si[0] + si[1]);
  double x = (pos - margin) / si[2];
  if (x < 0.0) x = -x;
  if (x >= 1.0) return si[1];
  if (x <= 0.0) return si[0];
  int pw = (int)si[4];
  double mid = si[3], y;
  if (pw <= 1) y = x;
  else if (x <= mid) {
    double a = 1.0, xp = 1.0;
    for (int k = 0; k < pw - 1; k++) a = a * mid;
    a = 1.0 / a;
    for (int k = 0; k < pw; k++) xp = xp * x;
    y = a * xp;
  } else {
    double b = 1.0, xp = 1.0;
    for (int k = 0; k < pw - 1; k++) b = b * (1.0 - mid);
    b = 1.0 / b;
    for (int k = 0; k < pw; k++) xp = xp * (1.0 - x);
    y = 1.0 - b * xp;
  }
  return si[0] + y * (si[1] - si[0]);
}

// lane 0 only
DEVI int add_row(const Mdl& md, Dat& d, int type, double pos, double margin, int dim, int con) {
  if (d.NEFC >= md.m.nefc_max) { d.OVERFLOW |= 2; return -1; }
  int r = d.NEFC++;
  d.efc_type[r] = type; d.efc_pos[r] = pos; d.efc_margin[r] = margin;
  d.efc_dim[r] = dim; d.efc_con[r] = con;
  return r;
}

// lane 0 only; ipos: the violation the impedance is taken at (the row's own
// efc_pos, or an equality constraint's violation norm, eq_violation_norm)
DEVI void row_params(const Mdl& md, Dat& d, int r, int dim, const double* sr, const double* si,
                           const double* mu, int elliptic_contact, double ipos) {
  const double dt = md.m.timestep;
  double tc = sr[0], dr = sr[1];
  double imp = impedance(si, ipos, d.efc_margin[r]);
  double dmax = si[1];
  double B, Kc;
  if (tc > 0.0) {
    if (tc < 2.0 * dt) tc = 2.0 * dt;
    B = 2.0 / (dmax * tc);
    Kc = 1.0 / (((dmax * dmax) * (tc * tc)) * (dr * dr));
  } else {
    B = -dr / dmax;
    Kc = -tc / (dmax * dmax);
  }
  for (int j = 0; j < dim; j++) {
    int q = r + j;
    double p = (j == 0) ? (d.efc_pos[q] - d.efc_margin[q]) : 0.0;
    d.efc_aref[q] = -B * d.efc_vel[q] - (Kc * imp) * p;
  }
  double Rn = ((1.0 - imp) / imp) * d.scratch[r];
  if (Rn < K_MINVAL) Rn = K_MINVAL;
  d.efc_R[r] = Rn;
  if (elliptic_contact && dim > 1) {
    double R1 = Rn / md.m.impratio;
    d.efc_R[r + 1] = R1;
    for (int j = 1; j < dim - 1; j++) d.efc_R[r + j + 1] = (R1 * (mu[0] * mu[0])) / (mu[j] * mu[j]);
  } else {
    for (int j = 1; j < dim; j++) {
      double Rj = ((1.0 - imp) / imp) * d.scratch[r + j];
      d.efc_R[r + j] = Rj < K_MINVAL ? K_MINVAL : Rj;
    }
  }
}

// the norm of an equality constraint's violation over all of its rows (a
// connect's 3, a weld's 6, a joint equality's 1), summed in row order: the
// impedance of every row of the constraint is taken at it (oracle
// eq_violation_norm; round 5, the choice that reproduces MuJoCo's recorded
// Robotiq state_close)
DEVI double eq_violation_norm(const Dat& d, int r) {
  const int id = d.efc_con[r];
  int q = r;
  while (q > 0 && d.efc_type[q - 1] == MGS_EFC_EQUALITY && d.efc_con[q - 1] == id) q--;
  double s2 = 0.0;
  for (; d.efc_type[q] == MGS_EFC_EQUALITY && d.efc_con[q] == id; q++) {
    s2 = s2 + d.efc_pos[q] * d.efc_pos[q];
    if (q + 1 >= d.NEFC) break;
  }
  return sqrt(s2);
}

// MuJoCo mj_diagApprox from the qpos0 inverse weights (oracle diag_approx()); lane 0
DEVI void diag_approx_row(const Mdl& md, Dat& d, int r) {
  const double *biw = DA(md, body_invweight0), *diw = DA(md, dof_invweight0);
  const int32_t *et = IA(md, eq_type), *eo1 = IA(md, eq_obj1id), *eo2 = IA(md, eq_obj2id);
  const int32_t *jd = IA(md, jnt_dofadr), *gbody = IA(md, geom_bodyid);
  int t = d.efc_type[r], id = d.efc_con[r];
  int start = r;
  while (start > 0 && d.efc_type[start - 1] == t && d.efc_con[start - 1] == id) start--;
  int k = r - start;
  double v = 0.0;
  if (t == MGS_EFC_EQUALITY) {
    if (et[id] == MGS_EQ_CONNECT) v = biw[2 * eo1[id]] + biw[2 * eo2[id]];
    else if (et[id] == MGS_EQ_WELD) v = biw[2 * eo1[id] + (k > 2)] + biw[2 * eo2[id] + (k > 2)];
    else {
      v = diw[jd[eo1[id]]];
      if (eo2[id] >= 0) v = v + diw[jd[eo2[id]]];
    }
  } else if (t == MGS_EFC_FRICTION) {
    v = diw[id];
  } else if (t == MGS_EFC_LIMIT) {
    v = diw[jd[id]];
  } else {
    int b1 = gbody[d.con_g1[id]], b2 = gbody[d.con_g2[id]];
    v = (k < 3) ? biw[2 * b1] + biw[2 * b2] : biw[2 * b1 + 1] + biw[2 * b2 + 1];
  }
  d.scratch[r] = v;   // efc_diagApprox, consumed by row_params
}

// Build J rows (into the G slots), then per row: velocity, J.qacc_smooth,
// whitened row G = D^-1/2 L^-1 J^T in place, A = G.G; impedance; blocks.
template <int NV>
DEVI void make_constraints(const Mdl& md, Dat& d) {
  int nv = md.m.nv, lane = lane_id();
  int* ints = d.ints;
  double* J = d.G;
  if (lane == 0) { d.NEFC = 0; }
  wsync();
  const int32_t *et = IA(md, eq_type), *eo1 = IA(md, eq_obj1id), *eo2 = IA(md, eq_obj2id);
  const double* ed = DA(md, eq_data);
  if (md.m.neq <= WAVE) {
    // every equality at once.  Lane e: its rows' place (connect 3, weld 6,
    // joint 1, in equality order) and values; the kept set is the oracle's
    // (make_constraints): equalities before the first one whose rows do not
    // fit, which flags the overflow.  Then lanes over (equality, dof) fill the
    // J columns with the sequential expressions.
    const int neq = md.m.neq;
    const int32_t *jqa = IA(md, jnt_qposadr), *jda = IA(md, jnt_dofadr);
    int typ = -1, need = 0;
    if (lane < neq) {
      typ = et[lane];
      need = typ == MGS_EQ_CONNECT ? 3 : typ == MGS_EQ_WELD ? 6 : typ == MGS_EQ_JOINT ? 1 : 0;
    }
    int re = 0;
    for (int j = 0; j < neq; j++) {
      int nj = __builtin_amdgcn_readlane(need, j);
      if (j < lane) re += nj;
    }
    unsigned long long mbad = __ballot(need > 0 && re + need > md.m.nefc_max);
    int ebad = mbad ? __ffsll((long long)mbad) - 1 : neq;
    int nkeep = ebad;
    if (lane < nkeep && need > 0) {
      const double* data = ed + 11 * lane;
      if (typ == MGS_EQ_JOINT) {
        int j1 = eo1[lane], j2 = eo2[lane];
        double q1 = d.qpos[jqa[j1]] - data[5];
        double pos;
        if (j2 >= 0) {
          double x = d.qpos[jqa[j2]] - data[6];
          double poly = data[0] + x * (data[1] + x * (data[2] + x * (data[3] + x * data[4])));
          pos = q1 - poly;
        } else {
          pos = q1 - data[0];
        }
        d.efc_type[re] = MGS_EFC_EQUALITY; d.efc_pos[re] = pos; d.efc_margin[re] = 0.0;
        d.efc_dim[re] = 1; d.efc_con[re] = lane;
      } else {
        int b1 = eo1[lane], b2 = eo2[lane];
        double p1[3], p2[3], t[3];
        mulmv3(t, d.xmat + 9 * b1, data);
        add3(p1, d.xpos + 3 * b1, t);
        if (typ == MGS_EQ_CONNECT) {
          mulmv3(t, d.xmat + 9 * b2, data + 3);
          add3(p2, d.xpos + 3 * b2, t);
        } else {
          p2[0] = d.xpos[3 * b2]; p2[1] = d.xpos[3 * b2 + 1]; p2[2] = d.xpos[3 * b2 + 2];
        }
        for (int k = 0; k < 3; k++) {
          d.efc_type[re + k] = MGS_EFC_EQUALITY; d.efc_pos[re + k] = p1[k] - p2[k]; d.efc_margin[re + k] = 0.0;
          d.efc_dim[re + k] = 1; d.efc_con[re + k] = lane;
        }
        if (typ == MGS_EQ_WELD) {
          double q1r[4], q2c[4], qe[4];
          quatmul(q1r, d.xquat + 4 * b1, data + 3);
          q2c[0] = d.xquat[4 * b2]; q2c[1] = -d.xquat[4 * b2 + 1];
          q2c[2] = -d.xquat[4 * b2 + 2]; q2c[3] = -d.xquat[4 * b2 + 3];
          quatmul(qe, q2c, q1r);
          double ts = data[7];
          for (int k = 0; k < 3; k++) {
            d.efc_type[re + 3 + k] = MGS_EFC_EQUALITY; d.efc_pos[re + 3 + k] = qe[1 + k] * ts;
            d.efc_margin[re + 3 + k] = 0.0; d.efc_dim[re + 3 + k] = 1; d.efc_con[re + 3 + k] = lane;
          }
        }
      }
    }
    int last = nkeep > 0 ? nkeep - 1 : 0;
    int ne_eq = nkeep > 0 ? __builtin_amdgcn_readlane(re + need, last) : 0;
    for (int q0 = 0; q0 < nkeep * nv; q0 += WAVE) {
      int q = q0 + lane;
      int e = q / nv, col = q - e * nv;
      int es = e < nkeep ? e : nkeep - 1;
      int r = shfl(re, es), ty = shfl(typ, es);
      if (q < nkeep * nv && ty >= 0) {
        const double* data = ed + 11 * e;
        if (ty == MGS_EQ_JOINT) {
          int j1 = eo1[e], j2 = eo2[e];
          double v = (col == jda[j1]) ? 1.0 : 0.0;
          if (j2 >= 0 && col == jda[j2]) {
            double x = d.qpos[jqa[j2]] - data[6];
            double deriv = data[1] + x * (2.0 * data[2] + x * (3.0 * data[3] + x * (4.0 * data[4])));
            v = v - deriv;
          }
          J[r * d.gs + col] = v;
        } else if (ty == MGS_EQ_CONNECT || ty == MGS_EQ_WELD) {
          int b1 = eo1[e], b2 = eo2[e];
          double p1[3], p2[3], t[3];
          mulmv3(t, d.xmat + 9 * b1, data);
          add3(p1, d.xpos + 3 * b1, t);
          if (ty == MGS_EQ_CONNECT) {
            mulmv3(t, d.xmat + 9 * b2, data + 3);
            add3(p2, d.xpos + 3 * b2, t);
          } else {
            p2[0] = d.xpos[3 * b2]; p2[1] = d.xpos[3 * b2 + 1]; p2[2] = d.xpos[3 * b2 + 2];
          }
          double cjp1[3], cjr1[3], cjp2[3], cjr2[3];
          jac_col(md, d, b1, p1, col, cjp1, cjr1);
          jac_col(md, d, b2, p2, col, cjp2, cjr2);
          for (int k = 0; k < 3; k++) J[(r + k) * d.gs + col] = cjp1[k] - cjp2[k];
          if (ty == MGS_EQ_WELD) {
            double q1r[4], q2c[4];
            quatmul(q1r, d.xquat + 4 * b1, data + 3);
            q2c[0] = d.xquat[4 * b2]; q2c[1] = -d.xquat[4 * b2 + 1];
            q2c[2] = -d.xquat[4 * b2 + 2]; q2c[3] = -d.xquat[4 * b2 + 3];
            double ts = data[7];
            double ax[4] = {0.0, cjr1[0] - cjr2[0], cjr1[1] - cjr2[1], cjr1[2] - cjr2[2]};
            double t1q[4], t2q[4];
            quatmul(t1q, q2c, ax);
            quatmul(t2q, t1q, q1r);
            for (int k = 0; k < 3; k++) J[(r + 3 + k) * d.gs + col] = (0.5 * t2q[1 + k]) * ts;
          }
        }
      }
    }
    wsync();
    if (lane == 0) {
      d.NEFC = ne_eq;
      if (ebad < neq) d.OVERFLOW |= 2;
    }
    wsync();
  } else
  for (int e = 0; e < md.m.neq; e++) {
    const double* data = ed + 11 * e;
    if (et[e] == MGS_EQ_CONNECT || et[e] == MGS_EQ_WELD) {
      int b1 = eo1[e], b2 = eo2[e];
      double p1[3], p2[3], t[3];
      if (et[e] == MGS_EQ_CONNECT) {
        mulmv3(t, d.xmat + 9 * b1, data);
        add3(p1, d.xpos + 3 * b1, t);
        mulmv3(t, d.xmat + 9 * b2, data + 3);
        add3(p2, d.xpos + 3 * b2, t);
      } else {
        mulmv3(t, d.xmat + 9 * b1, data);
        add3(p1, d.xpos + 3 * b1, t);
        p2[0] = d.xpos[3 * b2]; p2[1] = d.xpos[3 * b2 + 1]; p2[2] = d.xpos[3 * b2 + 2];
      }
      // this equality's rows do not fit: flag and stop (the oracle's rule; a
      // flag left from an earlier step does not stop the loop)
      if (uni(d.NEFC) + (et[e] == MGS_EQ_WELD ? 6 : 3) > md.m.nefc_max) {
        if (lane == 0) d.OVERFLOW |= 2;
        break;
      }
      if (lane == 0)
        for (int k = 0; k < 3; k++) add_row(md, d, MGS_EFC_EQUALITY, p1[k] - p2[k], 0.0, 1, e);
      wsync();
      int r0 = d.NEFC - 3;
      double cjp1[MGS_DPL][3], cjr1[MGS_DPL][3], cjp2[MGS_DPL][3], cjr2[MGS_DPL][3];
#pragma unroll
      for (int h = 0; h < MGS_DPL; h++) {
        const int i = lane + h * WAVE;
        int col = i < nv ? i : 0;
        jac_col(md, d, b1, p1, col, cjp1[h], cjr1[h]);
        jac_col(md, d, b2, p2, col, cjp2[h], cjr2[h]);
        if (i < nv)
          for (int k = 0; k < 3; k++) J[(r0 + k) * d.gs + i] = cjp1[h][k] - cjp2[h][k];
      }
      if (et[e] == MGS_EQ_WELD) {
        double q1r[4], q2c[4], qe[4];
        quatmul(q1r, d.xquat + 4 * b1, data + 3);
        q2c[0] = d.xquat[4 * b2]; q2c[1] = -d.xquat[4 * b2 + 1];
        q2c[2] = -d.xquat[4 * b2 + 2]; q2c[3] = -d.xquat[4 * b2 + 3];
        quatmul(qe, q2c, q1r);
        double ts = data[7];
        wsync();
        if (lane == 0)
          for (int k = 0; k < 3; k++) add_row(md, d, MGS_EFC_EQUALITY, qe[1 + k] * ts, 0.0, 1, e);
        wsync();
        int rr = d.NEFC - 3;
#pragma unroll
        for (int h = 0; h < MGS_DPL; h++) {
          const int i = lane + h * WAVE;
          if (i < nv) {
            double ax[4] = {0.0, cjr1[h][0] - cjr2[h][0], cjr1[h][1] - cjr2[h][1], cjr1[h][2] - cjr2[h][2]};
            double t1q[4], t2q[4];
            quatmul(t1q, q2c, ax);
            quatmul(t2q, t1q, q1r);
            for (int k = 0; k < 3; k++) J[(rr + k) * d.gs + i] = (0.5 * t2q[1 + k]) * ts;
          }
        }
      }
      wsync();
    } else if (et[e] == MGS_EQ_JOINT) {
      int j1 = eo1[e], j2 = eo2[e];
      const int32_t *jq = IA(md, jnt_qposadr), *jd = IA(md, jnt_dofadr);
      double q1 = d.qpos[jq[j1]] - data[5];
      double pos, deriv = 0.0;
      if (j2 >= 0) {
        double x = d.qpos[jq[j2]] - data[6];
        double poly = data[0] + x * (data[1] + x * (data[2] + x * (data[3] + x * data[4])));
        deriv = data[1] + x * (2.0 * data[2] + x * (3.0 * data[3] + x * (4.0 * data[4])));
        pos = q1 - poly;
      } else {
        pos = q1 - data[0];
      }
      if (uni(d.NEFC) + 1 > md.m.nefc_max) {
        if (lane == 0) d.OVERFLOW |= 2;
        break;
      }
      if (lane == 0) add_row(md, d, MGS_EFC_EQUALITY, pos, 0.0, 1, e);
      wsync();
      int r = d.NEFC - 1;
      for (int c = lane; c < nv; c += WAVE) J[r * d.gs + c] = 0.0;
      wsync();
      if (lane == 0) {
        J[r * d.gs + jd[j1]] = 1.0;
        if (j2 >= 0) J[r * d.gs + jd[j2]] = J[r * d.gs + jd[j2]] - deriv;
      }
      wsync();
    }
  }
  PT(31);
  // dof friction-loss rows, then joint-limit rows (lower bound before upper),
  // in the oracle's order: lanes over dofs / joints, ballot prefixes place the
  // rows, rows past nefc_max are dropped with the overflow flag (add_row)
  {
    int ne0 = uni(d.NEFC);
    const double* floss = DA(md, dof_frictionloss);
    unsigned long long lt = (lane == 0) ? 0ull : (~0ull >> (WAVE - lane));
    // friction rows in dof order: slot h's rows follow the lower slots' rows
    int hasf[MGS_DPL], rf[MGS_DPL];
    int nf = 0;
#pragma unroll
    for (int h = 0; h < MGS_DPL; h++) {
      const int i = lane + h * WAVE;
      hasf[h] = (i < nv) && floss[i] > 0.0;
      unsigned long long mf = __ballot(hasf[h]);
      rf[h] = ne0 + nf + __popcll(mf & lt);
      nf += __popcll(mf);
      if (hasf[h] && rf[h] < md.m.nefc_max) {
        d.efc_type[rf[h]] = MGS_EFC_FRICTION; d.efc_pos[rf[h]] = 0.0; d.efc_margin[rf[h]] = 0.0;
        d.efc_dim[rf[h]] = 1; d.efc_con[rf[h]] = i;
      }
    }
    int ne1 = ne0 + nf;
    if (ne1 > md.m.nefc_max) ne1 = md.m.nefc_max;
    const int32_t *lim = IA(md, jnt_limited), *jq = IA(md, jnt_qposadr), *jd = IA(md, jnt_dofadr);
    const double *range = DA(md, jnt_range), *jmargin = DA(md, jnt_margin);
    int lo = 0, hi = 0;
    double dlo = 0.0, dhi = 0.0, jm = 0.0;
    if (lane < md.m.njnt && lim[lane]) {
      double q = d.qpos[jq[lane]];
      dlo = q - range[2 * lane];
      dhi = range[2 * lane + 1] - q;
      jm = jmargin[lane];
      lo = dlo < jm;
      hi = dhi < jm;
    }
    unsigned long long ml = __ballot(lo), mh = __ballot(hi);
    int nl = __popcll(ml) + __popcll(mh);
    int rl = ne1 + __popcll(ml & lt) + __popcll(mh & lt);
    int rh = rl + lo;
    if (lo && rl < md.m.nefc_max) {
      d.efc_type[rl] = MGS_EFC_LIMIT; d.efc_pos[rl] = dlo; d.efc_margin[rl] = jm; d.efc_dim[rl] = 1; d.efc_con[rl] = lane;
    }
    if (hi && rh < md.m.nefc_max) {
      d.efc_type[rh] = MGS_EFC_LIMIT; d.efc_pos[rh] = dhi; d.efc_margin[rh] = jm; d.efc_dim[rh] = 1; d.efc_con[rh] = lane;
    }
    int ne2 = ne1 + nl;
    int ovf = ne0 + nf > md.m.nefc_max || ne2 > md.m.nefc_max;
    if (ne2 > md.m.nefc_max) ne2 = md.m.nefc_max;
    // J rows [ne0, ne2): zeros, then the unit entries
    for (int e = lane; e < (ne2 - ne0) * GS; e += WAVE) J[ne0 * GS + e] = 0.0;
    wsync();
#pragma unroll
    for (int h = 0; h < MGS_DPL; h++)
      if (hasf[h] && rf[h] < md.m.nefc_max) J[rf[h] * GS + lane + h * WAVE] = 1.0;
    if (lo && rl < md.m.nefc_max) J[rl * GS + jd[lane]] = 1.0;
    if (hi && rh < md.m.nefc_max) J[rh * GS + jd[lane]] = -1.0;
    if (lane == 0) {
      ints[8] = ne0; ints[9] = ne0; ints[10] = ne1; ints[11] = ne1; ints[12] = ne2; ints[6] = ne2;
      d.NEFC = ne2;
      if (ovf) d.OVERFLOW |= 2;
    }
  }
  wsync();
  PT(32);
  const int32_t *gbody = IA(md, geom_bodyid), *pcd = IA(md, pair_condim);
  const double *pfr = DA(md, pair_friction), *pmar = DA(md, pair_margin);
  // contact rows, every contact at once: lane c places contact c's dim rows
  // after the rows of contacts 0..c-1 (the sequential order); contacts from
  // the first one that does not fit on are dropped with the overflow flag (the
  // sequential loop stops there).  Then lanes over (contact, dof) pairs fill
  // the J columns.
  int ncon = uni(d.NCON);
  if (ncon > WAVE) {
    // more contacts than lanes (wide capacities): one contact at a time
    for (int c = 0; c < ncon; c++) {
      int p = uni(d.con_pair[c]);
      int dim = pcd[p];
      if (d.NEFC + dim > md.m.nefc_max) {
        if (lane == 0) d.OVERFLOW |= 2;
        break;
      }
      int b1 = gbody[d.con_g1[c]], b2 = gbody[d.con_g2[c]];
      const double* pt = d.con_pos + 3 * c;
      const double* fr = d.con_frame + 9 * c;
      int r = d.NEFC;
      wsync();
      if (lane == 0) {
        for (int j = 0; j < dim; j++) add_row(md, d, MGS_EFC_CONTACT, j == 0 ? d.con_dist[c] : 0.0, pmar[p], dim, c);
        for (int j = 0; j < dim; j++)
          if (!MGS_MU_MODEL && (MGS_MAXDIM < 6 || j < 5)) d.con_mu[5 * c + j] = (j < dim - 1) ? pfr[5 * p + j] : 0.0;
      }
      wsync();
#pragma unroll
      for (int h = 0; h < MGS_DPL; h++) {
      const int i = lane + h * WAVE;
      int col = i < nv ? i : 0;
      double cjp1[3], cjr1[3], cjp2[3], cjr2[3];
      jac_col(md, d, b1, pt, col, cjp1, cjr1);
      jac_col(md, d, b2, pt, col, cjp2, cjr2);
      if (i < nv) {
        double dp[3] = {cjp2[0] - cjp1[0], cjp2[1] - cjp1[1], cjp2[2] - cjp1[2]};
        for (int j = 0; j < dim && j < 3; j++) J[(r + j) * d.gs + col] = dot3(fr + 3 * j, dp);
        if (dim >= 4) {
          double dr[3] = {cjr2[0] - cjr1[0], cjr2[1] - cjr1[1], cjr2[2] - cjr1[2]};
          J[(r + 3) * d.gs + col] = dot3(fr, dr);
#if MGS_MAXDIM > 4
          if (dim == 6) {
            J[(r + 4) * d.gs + col] = dot3(fr + 3, dr);
            J[(r + 5) * d.gs + col] = dot3(fr + 6, dr);
          }
#endif
        }
      }
      }
    }
  } else {
    const int ne0 = uni(d.NEFC);
    int cp = 0, cdim = 0;
    if (lane < ncon) {
      cp = d.con_pair[lane];
      cdim = pcd[cp];
    }
    int rc = ne0;
    for (int j = 0; j < ncon; j++) {
      int dj = __builtin_amdgcn_readlane(cdim, j);
      if (j < lane) rc += dj;
    }
    int bad = lane < ncon && rc + cdim > md.m.nefc_max;
    unsigned long long mb = __ballot(bad);
    int nkeep = mb ? (__ffsll((long long)mb) - 1) : ncon;
    if (lane < nkeep) {
      for (int j = 0; j < cdim; j++) {
        int r = rc + j;
        d.efc_type[r] = MGS_EFC_CONTACT; d.efc_pos[r] = j == 0 ? d.con_dist[lane] : 0.0;
        d.efc_margin[r] = pmar[cp]; d.efc_dim[r] = cdim; d.efc_con[r] = lane;
        // (5 friction coefficients per contact: a condim-6 block's sixth row has
        // no slot -- writing one would clobber the next contact's first)
        if (!MGS_MU_MODEL && (MGS_MAXDIM < 6 || j < 5))
          d.con_mu[5 * lane + j] = (j < cdim - 1) ? pfr[5 * cp + j] : 0.0;
      }
    }
    int last = nkeep > 0 ? nkeep - 1 : 0;
    int ne_end = nkeep > 0 ? __builtin_amdgcn_readlane(rc + cdim, last) : ne0;
    for (int q0 = 0; q0 < nkeep * nv; q0 += WAVE) {
      int q = q0 + lane;
      int c = q / nv, col = q - c * nv;
      int cs = c < nkeep ? c : nkeep - 1;
      int r = shfl(rc, cs), dim = shfl(cdim, cs);
      if (q < nkeep * nv) {
        int b1 = gbody[d.con_g1[c]], b2 = gbody[d.con_g2[c]];
        const double* pt = d.con_pos + 3 * c;
        const double* fr = d.con_frame + 9 * c;
        double cjp1[3], cjr1[3], cjp2[3], cjr2[3];
        jac_col(md, d, b1, pt, col, cjp1, cjr1);
        jac_col(md, d, b2, pt, col, cjp2, cjr2);
        double dp[3] = {cjp2[0] - cjp1[0], cjp2[1] - cjp1[1], cjp2[2] - cjp1[2]};
        for (int j = 0; j < dim && j < 3; j++) J[(r + j) * d.gs + col] = dot3(fr + 3 * j, dp);
        if (dim >= 4) {
          double dr[3] = {cjr2[0] - cjr1[0], cjr2[1] - cjr1[1], cjr2[2] - cjr1[2]};
          J[(r + 3) * d.gs + col] = dot3(fr, dr);
#if MGS_MAXDIM > 4
          if (dim == 6) {
            J[(r + 4) * d.gs + col] = dot3(fr + 3, dr);
            J[(r + 5) * d.gs + col] = dot3(fr + 6, dr);
          }
#endif
        }
      }
    }
    wsync();
    if (lane == 0) {
      d.NEFC = ne_end;
      if (nkeep < ncon) d.OVERFLOW |= 2;
    }
  }
  wsync();
  if (lane == 0) ints[7] = d.NEFC;
  wsync();
  PT(9);
  int ne = uni(d.NEFC);
  // per row (lanes over rows): vel, J.qacc_smooth, G in place, A
  // (the row lives in registers for the triangular solve)
  for (int r = lane; r < ne; r += WAVE) {
    double* Gr = d.G + r * GS;
    double g[NV];
#pragma unroll
    for (int k = 0; k < NV; k++) g[k] = Gr[k];
    double v = 0.0, bj = 0.0;
#pragma unroll
    for (int k = 0; k < NV; k++) v = v + g[k] * d.qvel[k];
#pragma unroll
    for (int k = 0; k < NV; k++) bj = bj + g[k] * d.qacc_smooth[k];
    d.efc_vel[r] = v;
    d.efc_b[r] = bj;
#pragma unroll
    for (int i = 0; i < NV; i++) {
      double s = g[i];
#pragma unroll
      for (int k = 0; k < i; k++) s = __builtin_fma(-d.M[TRI(i, k, NV)], g[k], s);
      g[i] = s;
    }
#pragma unroll
    for (int i = 0; i < NV; i++) Gr[i] = g[i] * d.isD[i];
  }
  wsync();
  PT(10);
  // diagApprox then impedance / reference acceleration, lanes over rows (blocks
  // by their leading row); each lane writes only its own rows
  for (int r = lane; r < ne; r += WAVE) diag_approx_row(md, d, r);
  wsync();
  for (int r = lane; r < ne; r += WAVE) {
    int t = d.efc_type[r], id = d.efc_con[r];
    if (t == MGS_EFC_EQUALITY) {
      row_params(md, d, r, 1, DA(md, eq_solref) + 2 * id, DA(md, eq_solimp) + 5 * id, nullptr, 0,
                 eq_violation_norm(d, r));
    } else if (t == MGS_EFC_FRICTION) {
      row_params(md, d, r, 1, DA(md, dof_solref) + 2 * id, DA(md, dof_solimp) + 5 * id, nullptr, 0, d.efc_pos[r]);
    } else if (t == MGS_EFC_LIMIT) {
      row_params(md, d, r, 1, DA(md, jnt_solref) + 2 * id, DA(md, jnt_solimp) + 5 * id, nullptr, 0, d.efc_pos[r]);
    } else if (efc_lead(d, r)) {
      int p = d.con_pair[id];
      row_params(md, d, r, d.efc_dim[r], DA(md, pair_solref) + 2 * p, DA(md, pair_solimp) + 5 * p,
                 con_mu_of(md, d, id), 1, d.efc_pos[r]);
    }
  }
  wsync();
  for (int r = lane; r < ne; r += WAVE) d.efc_b[r] = d.efc_b[r] - d.efc_aref[r];
  wsync();
  PT(11);
}

// contact blocks of A = G G^T for the (PGS / noslip) block updates, lanes over
// block entries; they share storage with the Newton cone Hessians
DEVI void contact_blocks(const Mdl& md, Dat& d) {
  int nv = md.m.nv, lane = lane_id();
  int* ints = d.ints;
  for (int r = uni(ints[6]); r < uni(ints[7]);) {
    int dim = uni(d.efc_dim[r]);
    double* blk = d.con_blk + BLKSTRIDE * uni(d.efc_con[r]);
    for (int e = lane; e < dim * dim; e += WAVE) {
      int i = e / dim, j = e % dim;
      const double* Gi = d.G + (r + i) * d.gs;
      const double* Gj = d.G + (r + j) * d.gs;
      double a = 0.0;
      for (int k = 0; k < nv; k++) a = a + Gi[k] * Gj[k];
      blk[i * dim + j] = a;
    }
    r += dim;
  }
  wsync();
}

// ---------------------------------------------------------------------------
// solver (all lanes execute the scalar logic with identical values)
DEVI void qcqp2(double A0, double A1, double A3, double bb0, double bb1, const double* mu, double r,
                                      double* x0, double* x1) {
  double a11 = (A0 * mu[0]) * mu[0], a12 = (A1 * mu[0]) * mu[1], a22 = (A3 * mu[1]) * mu[1];
  double b1 = bb0 * mu[0], b2 = bb1 * mu[1];
  double rr = r * r, la = 0.0, v1 = 0.0, v2 = 0.0;
  int sing = 0;
  for (int it = 0; it < 20; it++) {
    double m11 = a11 + la, m22 = a22 + la;
    double det = m11 * m22 - a12 * a12;
    if (det < 1e-10) { v1 = 0.0; v2 = 0.0; sing = 1; break; }
    double idet = 1.0 / det;
    double p11 = m22 * idet, p22 = m11 * idet, p12 = -a12 * idet;
    v1 = -(p11 * b1 + p12 * b2);
    v2 = -(p12 * b1 + p22 * b2);
    double val = (v1 * v1 + v2 * v2) - rr;
    if (val < 1e-10) break;
    double pv1 = p11 * v1 + p12 * v2, pv2 = p12 * v1 + p22 * v2;
    double deriv = -2.0 * (v1 * pv1 + v2 * pv2);
    double delta = -val / deriv;
    if (delta < 1e-10) break;
    la = la + delta;
    PCNT(45, 1);
  }
  double o0 = v1 * mu[0], o1 = v2 * mu[1];
  // active constraint: put the result on the ellipsoid (MuJoCo PGS / noslip)
  if (!sing && la != 0.0) {
    double s = (o0 * o0) / (mu[0] * mu[0]) + (o1 * o1) / (mu[1] * mu[1]);
    s = sqrt((r * r) / (s > K_MINVAL ? s : K_MINVAL));
    o0 = o0 * s;
    o1 = o1 * s;
  }
  *x0 = o0;
  *x1 = o1;
}

DEVI void qcqp3(const double* A, const double* b, const double* mu, double r, double* x) {
  double a00 = (A[0] * mu[0]) * mu[0], a01 = (A[1] * mu[0]) * mu[1], a02 = (A[2] * mu[0]) * mu[2];
  double a11 = (A[4] * mu[1]) * mu[1], a12 = (A[5] * mu[1]) * mu[2], a22 = (A[8] * mu[2]) * mu[2];
  double b0 = b[0] * mu[0], b1 = b[1] * mu[1], b2 = b[2] * mu[2];
  double rr = r * r, la = 0.0, v0 = 0.0, v1 = 0.0, v2 = 0.0;
  int sing = 0;
  for (int it = 0; it < 20; it++) {
    double m00 = a00 + la, m11 = a11 + la, m22 = a22 + la;
    double c00 = m11 * m22 - a12 * a12, c01 = a02 * a12 - a01 * m22, c02 = a01 * a12 - a02 * m11;
    double c11 = m00 * m22 - a02 * a02, c12 = a01 * a02 - m00 * a12, c22 = m00 * m11 - a01 * a01;
    double det = (m00 * c00 + a01 * c01) + a02 * c02;
    if (det < 1e-10) { v0 = 0.0; v1 = 0.0; v2 = 0.0; sing = 1; break; }
    double idet = 1.0 / det;
    double p00 = c00 * idet, p01 = c01 * idet, p02 = c02 * idet;
    double p11 = c11 * idet, p12 = c12 * idet, p22 = c22 * idet;
    v0 = -((p00 * b0 + p01 * b1) + p02 * b2);
    v1 = -((p01 * b0 + p11 * b1) + p12 * b2);
    v2 = -((p02 * b0 + p12 * b1) + p22 * b2);
    double val = ((v0 * v0 + v1 * v1) + v2 * v2) - rr;
    if (val < 1e-10) break;
    double pv0 = (p00 * v0 + p01 * v1) + p02 * v2;
    double pv1 = (p01 * v0 + p11 * v1) + p12 * v2;
    double pv2 = (p02 * v0 + p12 * v1) + p22 * v2;
    double deriv = -2.0 * ((v0 * pv0 + v1 * pv1) + v2 * pv2);
    double delta = -val / deriv;
    if (delta < 1e-10) break;
    la = la + delta;
  }
  x[0] = v0 * mu[0];
  x[1] = v1 * mu[1];
  x[2] = v2 * mu[2];
  if (!sing && la != 0.0) {
    double s = ((x[0] * x[0]) / (mu[0] * mu[0]) + (x[1] * x[1]) / (mu[1] * mu[1])) + (x[2] * x[2]) / (mu[2] * mu[2]);
    s = sqrt((r * r) / (s > K_MINVAL ? s : K_MINVAL));
    x[0] = x[0] * s;
    x[1] = x[1] * s;
    x[2] = x[2] * s;
  }
}

// n = 5 (condim-6 contacts: two sliding, one torsional, two rolling
// dimensions): MuJoCo's general mju_QCQP restated (oracle qcqpn): the same
// Newton iteration on the multiplier, with (A + la I) factored by Cholesky
// (a pivot below 1e-10 counts as singular: result 0) instead of the closed-form
// inverse.  Parity unpinned: MuJoCo's source is not here.
template <int N>
DEVI void qcqpn(const double* A, const double* b, const double* mu, double r, double* x) {
  double As[N * N], bs[N], v[N], L[N * N], t[N];
#pragma unroll
  for (int i = 0; i < N; i++) {
    bs[i] = b[i] * mu[i];
    v[i] = 0.0;
#pragma unroll
    for (int j = 0; j < N; j++) As[i * N + j] = (A[i * N + j] * mu[i]) * mu[j];
  }
  double rr = r * r, la = 0.0;
  int sing = 0;
  for (int it = 0; it < 20; it++) {
#pragma unroll
    for (int q = 0; q < N * N; q++) L[q] = As[q];
#pragma unroll
    for (int i = 0; i < N; i++) L[i * N + i] = L[i * N + i] + la;
#pragma unroll
    for (int j = 0; j < N; j++) {
      double p = L[j * N + j];
#pragma unroll
      for (int k = 0; k < j; k++) p = p - L[j * N + k] * L[j * N + k];
      if (p < 1e-10) sing = 1;
      p = sqrt(p < 1e-10 ? 1e-10 : p);
      L[j * N + j] = p;
#pragma unroll
      for (int i = j + 1; i < N; i++) {
        double s = L[i * N + j];
#pragma unroll
        for (int k = 0; k < j; k++) s = s - L[i * N + k] * L[j * N + k];
        L[i * N + j] = s / p;
      }
    }
    if (sing) {
#pragma unroll
      for (int i = 0; i < N; i++) v[i] = 0.0;
      break;
    }
    // v = -(L L')^-1 bs
#pragma unroll
    for (int i = 0; i < N; i++) {
      double s = bs[i];
#pragma unroll
      for (int k = 0; k < i; k++) s = s - L[i * N + k] * t[k];
      t[i] = s / L[i * N + i];
    }
#pragma unroll
    for (int i = N - 1; i >= 0; i--) {
      double s = t[i];
#pragma unroll
      for (int k = i + 1; k < N; k++) s = s - L[k * N + i] * v[k];
      v[i] = s / L[i * N + i];
    }
#pragma unroll
    for (int i = 0; i < N; i++) v[i] = -v[i];
    double val = -rr;
    {
      double vv = 0.0;
#pragma unroll
      for (int i = 0; i < N; i++) vv = vv + v[i] * v[i];
      val = vv - rr;
    }
    if (val < 1e-10) break;
    // deriv = -2 v' (A + la I)^-1 v
    double pv[N];
#pragma unroll
    for (int i = 0; i < N; i++) {
      double s = v[i];
#pragma unroll
      for (int k = 0; k < i; k++) s = s - L[i * N + k] * t[k];
      t[i] = s / L[i * N + i];
    }
#pragma unroll
    for (int i = N - 1; i >= 0; i--) {
      double s = t[i];
#pragma unroll
      for (int k = i + 1; k < N; k++) s = s - L[k * N + i] * pv[k];
      pv[i] = s / L[i * N + i];
    }
    double vp = 0.0;
#pragma unroll
    for (int i = 0; i < N; i++) vp = vp + v[i] * pv[i];
    double deriv = -2.0 * vp;
    double delta = -val / deriv;
    if (delta < 1e-10) break;
    la = la + delta;
  }
#pragma unroll
  for (int i = 0; i < N; i++) x[i] = v[i] * mu[i];
  if (!sing && la != 0.0) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < N; i++) s = s + (x[i] * x[i]) / (mu[i] * mu[i]);
    s = sqrt((r * r) / (s > K_MINVAL ? s : K_MINVAL));
#pragma unroll
    for (int i = 0; i < N; i++) x[i] = x[i] * s;
  }
}

// forces live in registers: lane l holds f[l + 64 h] in F.v[h], h < MGS_RPL
// (rows per lane: 2 in the main library, 4 in the wide one for clutter piles)
struct Frc {
  double v[MGS_RPL];
};
DEVI double getf(const Frc& F, int r) {
  double out = 0.0;
#pragma unroll
  for (int h = 0; h < MGS_RPL; h++)
    if ((r >> 6) == h) out = readlane_d(F.v[h], r & (WAVE - 1));
  return out;
}
DEVI void setf(Frc& F, int r, double v, int lane) {
#pragma unroll
  for (int h = 0; h < MGS_RPL; h++)
    if ((r >> 6) == h) F.v[h] = (lane == (r & (WAVE - 1))) ? v : F.v[h];
}
// registers <- efc_f (rows >= ne: 0)
DEVI void load_frc(Frc& F, const double* f, int ne, int lane) {
#pragma unroll
  for (int h = 0; h < MGS_RPL; h++) F.v[h] = (lane + h * WAVE < ne) ? f[lane + h * WAVE] : 0.0;
}

// MuJoCo's costChange (oracle cost_change1 / cost_change): dual-cost change of
// an update; one that raises the cost by more than 1e-10 is undone
DEVI double cost_change1(double A, double delta, double res) {
  return ((0.5 * delta) * delta) * A + delta * res;
}

template <int N, int LD>
DEVI double cost_change(const double* A, const double* delta, const double* res) {
  double vav = 0.0, dr = 0.0;
#pragma unroll
  for (int i = 0; i < N; i++) {
    double ad = 0.0;
#pragma unroll
    for (int j = 0; j < N; j++) ad = ad + A[i * LD + j] * delta[j];
    vav = vav + delta[i] * ad;
  }
#pragma unroll
  for (int i = 0; i < N; i++) dr = dr + delta[i] * res[i];
  return 0.5 * vav + dr;
}

// one PGS update of the contact block starting at row r with DIM rows
template <int DIM>
DEVI double pgs_contact(const Mdl& md, const Dat& d, int r, int nv, int P, int lane, DofV& u, Frc& F, int noslip,
                        const DofV* gpre = nullptr) {
  DofV g[DIM];
  double res[DIM], old[DIM], nw[DIM];
  const int c = uni(d.efc_con[r]);
  const double* blk = d.con_blk + BLKSTRIDE * c;
  const double* mu = con_mu_of(md, d, c);
#pragma unroll
  for (int i = 0; i < DIM; i++) {
    // gpre: the block's G rows loaded ahead by the caller (lanes over dofs)
    g[i] = gpre ? gpre[i] : dof_load(d.G + (r + i) * d.gs, nv, lane);
    old[i] = getf(F, r + i);
    // noslip never reads the normal row's residual: its reduction is skipped
    if (noslip && i == 0) { res[i] = 0.0; continue; }
    double jw = dof_tree(dof_mul(g[i], u), P);
    res[i] = noslip ? (jw + d.efc_b[r + i]) : ((jw + d.efc_R[r + i] * old[i]) + d.efc_b[r + i]);
  }
  PT(42);
  PCNT(46, 1);
  double Ab[DIM * DIM];
#pragma unroll
  for (int i = 0; i < DIM; i++) {
#pragma unroll
    for (int j = 0; j < DIM; j++) Ab[i * DIM + j] = blk[i * DIM + j];
    if (!noslip) Ab[i * DIM + i] = Ab[i * DIM + i] + d.efc_R[r + i];
  }
  double dc = 0.0;
  if (!noslip) {
    double fn = old[0] - res[0] * (1.0 / (blk[0] + d.efc_R[r]));
    if (fn < 0.0) fn = 0.0;
    double dn = fn - old[0];
    nw[0] = fn;
    if (fn < 1e-15) {
#pragma unroll
      for (int j = 1; j < DIM; j++) nw[j] = 0.0;
    } else {
      double bq[DIM - 1];
#pragma unroll
      for (int i = 0; i < DIM - 1; i++) {
        double v = res[1 + i] + Ab[(1 + i) * DIM] * dn;
        double s = v;
#pragma unroll
        for (int j = 0; j < DIM - 1; j++) s = s - Ab[(1 + i) * DIM + 1 + j] * old[1 + j];
        bq[i] = s;
      }
      if constexpr (DIM == 3) {
        qcqp2(Ab[4], Ab[5], Ab[8], bq[0], bq[1], mu, fn, &nw[1], &nw[2]);
      } else {
        double Ac[(DIM - 1) * (DIM - 1)];
#pragma unroll
        for (int i = 0; i < DIM - 1; i++)
#pragma unroll
          for (int j = 0; j < DIM - 1; j++) Ac[i * (DIM - 1) + j] = Ab[(1 + i) * DIM + 1 + j];
        if constexpr (DIM == 4) qcqp3(Ac, bq, mu, fn, nw + 1);
        else qcqpn<DIM - 1>(Ac, bq, mu, fn, nw + 1);
      }
    }
    double del[DIM];
#pragma unroll
    for (int i = 0; i < DIM; i++) del[i] = nw[i] - old[i];
    dc = cost_change<DIM, DIM>(Ab, del, res);
    if (dc > 1e-10) {
#pragma unroll
      for (int i = 0; i < DIM; i++) { nw[i] = old[i]; del[i] = 0.0; }
      dc = 0.0;
    }
#pragma unroll
    for (int h = 0; h < MGS_DPL; h++) {
      double s = u.v[h];
#pragma unroll
      for (int i = 0; i < DIM; i++) s = s + g[i].v[h] * del[i];
      if (lane + h * WAVE < nv) u.v[h] = s;
    }
#pragma unroll
    for (int i = 0; i < DIM; i++) setf(F, r + i, nw[i], lane);
  } else {
    // friction dims only, normal fixed, A without R
    const int NF = DIM - 1;
    double bq[NF];
#pragma unroll
    for (int i = 0; i < NF; i++) {
      double s = res[1 + i];
#pragma unroll
      for (int j = 0; j < NF; j++) s = s - Ab[(1 + i) * DIM + 1 + j] * old[1 + j];
      bq[i] = s;
    }
    double fnorm = old[0];
    if (!(fnorm < 1e-15)) {
      if constexpr (DIM == 3) {
        qcqp2(Ab[4], Ab[5], Ab[8], bq[0], bq[1], mu, fnorm, &nw[1], &nw[2]);
      } else {
        double Ac[(DIM - 1) * (DIM - 1)];
#pragma unroll
        for (int i = 0; i < DIM - 1; i++)
#pragma unroll
          for (int j = 0; j < DIM - 1; j++) Ac[i * (DIM - 1) + j] = Ab[(1 + i) * DIM + 1 + j];
        if constexpr (DIM == 4) qcqp3(Ac, bq, mu, fnorm, nw + 1);
        else qcqpn<DIM - 1>(Ac, bq, mu, fnorm, nw + 1);
      }
    } else {
#pragma unroll
      for (int i = 1; i < DIM; i++) nw[i] = 0.0;
    }
    PT(43);
    double del[NF];
#pragma unroll
    for (int i = 0; i < NF; i++) del[i] = nw[1 + i] - old[1 + i];
    dc = cost_change<NF, DIM>(Ab + DIM + 1, del, res + 1);
    if (dc > 1e-10) {
#pragma unroll
      for (int i = 0; i < NF; i++) { nw[1 + i] = old[1 + i]; del[i] = 0.0; }
      dc = 0.0;
    }
#pragma unroll
    for (int h = 0; h < MGS_DPL; h++) {
      double s = u.v[h];
#pragma unroll
      for (int i = 0; i < NF; i++) s = s + g[1 + i].v[h] * del[i];
      if (lane + h * WAVE < nv) u.v[h] = s;
    }
#pragma unroll
    for (int i = 0; i < NF; i++) setf(F, r + 1 + i, nw[1 + i], lane);
  }
  PT(44);
  return dc;
}

DEVI void project_scalar(int t, double floss, double* f) {
  if (t == MGS_EFC_FRICTION) {
    if (f[0] < -floss) f[0] = -floss;
    if (f[0] > floss) f[0] = floss;
  } else if (t == MGS_EFC_LIMIT || t == MGS_EFC_CONTACT) {
    if (f[0] < 0.0) f[0] = 0.0;
  }
}

DEVI void project_block_lds(const Mdl& md, const Dat& d, int r, double* f) {
  int t = d.efc_type[r];
  if (t == MGS_EFC_FRICTION) {
    double fl = row_floss(md, d, r);
    if (f[0] < -fl) f[0] = -fl;
    if (f[0] > fl) f[0] = fl;
  } else if (t == MGS_EFC_LIMIT) {
    if (f[0] < 0.0) f[0] = 0.0;
  } else if (t == MGS_EFC_CONTACT) {
    int dim = d.efc_dim[r];
    if (f[0] < 0.0) { for (int j = 0; j < dim; j++) f[j] = 0.0; return; }
    if (dim == 1) return;
    const double* mu = con_mu_of(md, d, d.efc_con[r]);
    double s = 0.0;
    for (int j = 1; j < dim; j++) { double q = f[j] / mu[j - 1]; s = s + q * q; }
    double nt = sqrt(s);
    if (nt > f[0]) {
      double sc = f[0] / nt;
      for (int j = 1; j < dim; j++) f[j] = f[j] * sc;
    }
  }
}

DEVI void solve_pgs(const Mdl& md, Dat& d, double scale, Frc& F, DofV& u) {
  int nv = md.m.nv, ne = uni(d.NEFC), lane = lane_id();
  int P = next_pow2(nv);
  // warmstart: hws = D^1/2 L^T qacc_ws (lane 0), f_r by lanes over rows, block projection
  if (lane == 0) {
    for (int i = 0; i < nv; i++) {
      double s = d.qacc_ws[i];
      for (int k = i + 1; k < nv; k++) s = s + d.M[TRI(k, i, nv)] * d.qacc_ws[k];
      d.tmp[i] = s * d.sD[i];
    }
  }
  wsync();
  double* fl = d.scratch;                 // f staging (ne)
  double* terms = d.scratch + md.m.nefc_max;
  for (int r = lane; r < ne; r += WAVE) {
    const double* Gr = d.G + r * d.gs;
    double jar = 0.0;
    for (int k = 0; k < nv; k++) jar = jar + Gr[k] * d.tmp[k];
    jar = jar - d.efc_aref[r];
    fl[r] = -jar / d.efc_R[r];
  }
  wsync();
  if (lane == 0) {
    for (int r = 0; r < ne;) {
      int dim = d.efc_type[r] == MGS_EFC_CONTACT ? d.efc_dim[r] : 1;
      if (d.efc_type[r] != MGS_EFC_EQUALITY) project_block_lds(md, d, r, fl + r);
      r += dim;
    }
  }
  wsync();
  // u = G^T f (lane k), then dual cost terms (lanes over rows), summed in row order
  u = dof_zero();
#pragma unroll
  for (int h = 0; h < MGS_DPL; h++) {
    const int i = lane + h * WAVE;
    if (i < nv) {
      double s = 0.0;
      for (int r = 0; r < ne; r++) s = s + d.G[r * d.gs + i] * fl[r];
      u.v[h] = s;
      d.tmp2[i] = s;
    }
  }
  wsync();
  for (int r = lane; r < ne; r += WAVE) {
    const double* Gr = d.G + r * d.gs;
    double jw = 0.0;
    for (int k = 0; k < nv; k++) jw = jw + Gr[k] * d.tmp2[k];
    terms[r] = fl[r] * ((0.5 * (jw + d.efc_R[r] * fl[r])) + d.efc_b[r]);
  }
  wsync();
  double cw = 0.0;
  for (int r = 0; r < ne; r++) cw = cw + terms[r];
  load_frc(F, fl, ne, lane);
  if (!(cw < 0.0)) {
#pragma unroll
    for (int h = 0; h < MGS_RPL; h++) F.v[h] = 0.0;
    u = dof_zero();
  }
  int it;
  for (it = 0; it < md.m.iterations && ne > 0; it++) {
    double improvement = 0.0;
    for (int r = 0; r < ne;) {
      int t = uni(d.efc_type[r]);
      int dim = uni(d.efc_dim[r]);
      if (t != MGS_EFC_CONTACT || dim == 1) {
        DofV g = dof_load(d.G + r * d.gs, nv, lane);
        double jw = dof_tree(dof_mul(g, u), P);
        double fo = getf(F, r);
        double res = (jw + d.efc_R[r] * fo) + d.efc_b[r];
        double AR = row_sqnorm(d, r, nv) + d.efc_R[r];
        double fnew[1] = {fo - res * (1.0 / AR)};
        if (t != MGS_EFC_EQUALITY) project_scalar(t, row_floss(md, d, r), fnew);
        double delta = fnew[0] - fo;
        double ch = cost_change1(AR, delta, res);
        if (ch > 1e-10) { delta = 0.0; ch = 0.0; }
        improvement = improvement - ch;
        if (delta != 0.0) {
          dof_axpy(u, g, delta, nv, lane);
          setf(F, r, fnew[0], lane);
        }
        r += 1;
      } else if (dim == 3) {
        improvement = improvement - pgs_contact<3>(md, d, r, nv, P, lane, u, F, 0);
        r += 3;
#if MGS_MAXDIM > 4
      } else if (dim == 6) {
        improvement = improvement - pgs_contact<6>(md, d, r, nv, P, lane, u, F, 0);
        r += 6;
#endif
      } else {
        improvement = improvement - pgs_contact<4>(md, d, r, nv, P, lane, u, F, 0);
        r += 4;
      }
    }
    if (improvement * scale < md.m.tolerance) { it++; break; }
  }
  if (lane == 0) d.ITERS += it;
}

// noslip post-pass (both solvers): friction dims only, unregularised, normals fixed.
// The sweep visits the rows the oracle's does work on -- friction rows and the
// first row of each contact block of dimension 3 or 4, in ascending order --
// from a row mask built once per call (lanes over rows), with each row's type
// and dimension held in registers: the rows a sweep only steps over (equality,
// limit, other contacts) cost nothing.  noslip_prefetch: per call, a friction row's A_rr (its
// row_sqnorm, the same ascending sum) and frictionloss are formed once on the
// row's lane instead of once per sweep, and each visited block's G rows are
// loaded while the previous block is processed (wide build: G is in HBM, a
// round trip per block otherwise).  Same values and order as the oracle.
template <int N>
DEVI int sel_i(const int (&a)[N], int r) {
  int out = 0;
#pragma unroll
  for (int h = 0; h < N; h++)
    if ((r >> 6) == h) out = __builtin_amdgcn_readlane(a[h], r & (WAVE - 1));
  return out;
}
template <int N>
DEVI double sel_d(const double (&a)[N], int r) {
  double out = 0.0;
#pragma unroll
  for (int h = 0; h < N; h++)
    if ((r >> 6) == h) out = readlane_d(a[h], r & (WAVE - 1));
  return out;
}
// the first visited row after r (r = -1: the first one), -1 if none
template <int N>
DEVI int next_visited(const unsigned long long (&vis)[N], int r) {
  const int s = r + 1;
  int out = -1;
#pragma unroll
  for (int h = N - 1; h >= 0; h--) {
    if (h < (s >> 6)) continue;
    unsigned long long m = vis[h];
    if (h == (s >> 6)) m &= ~0ull << (s & (WAVE - 1));
    if (m) out = h * WAVE + __ffsll((long long)m) - 1;
  }
  return out;
}
DEVI void load_block_rows(const Dat& d, int r, int dim, int nv, int lane, DofV (&g)[MGS_MAXDIM]) {
#pragma unroll
  for (int i = 0; i < MGS_MAXDIM; i++)
#pragma unroll
    for (int h = 0; h < MGS_DPL; h++)
      g[i].v[h] = (i < dim && lane + h * WAVE < nv) ? d.G[(r + i) * d.gs + lane + h * WAVE] : 0.0;
}

DEVI void noslip_prefetch(const Mdl& md, Dat& d, double scale, Frc& F, DofV& u) {
  int nv = md.m.nv, ne = uni(d.NEFC), lane = lane_id();
  int P = next_pow2(nv);
  if (md.m.noslip_iterations <= 0 || ne <= 0) return;
  int tk[MGS_RPL], dk[MGS_RPL];
  unsigned long long vis[MGS_RPL];
  double Ak[MGS_RPL], Fk[MGS_RPL];
#pragma unroll
  for (int h = 0; h < MGS_RPL; h++) {
    const int r = lane + h * WAVE;
    int t = -1, dim = 0, v = 0;
    if (r < ne) {
      t = d.efc_type[r];
      dim = d.efc_dim[r];
      v = t == MGS_EFC_FRICTION || (t == MGS_EFC_CONTACT && dim > 1 && efc_lead(d, r));
    }
    tk[h] = t;
    dk[h] = dim;
    vis[h] = __ballot(v);
    Ak[h] = 0.0;
    Fk[h] = 0.0;
    if (v && t == MGS_EFC_FRICTION) {
      Ak[h] = row_sqnorm(d, r, nv);
      Fk[h] = row_floss(md, d, r);
    }
  }
  for (int ns = 0; ns < md.m.noslip_iterations; ns++) {
    PCNT(38, 1);
    double improvement = 0.0;
    // the noslip cost drops the regulariser: count its removal at iteration 0
    // (row terms on their lanes, summed in row order)
    if (ns == 0) {
#pragma unroll
      for (int h = 0; h < MGS_RPL; h++) {
        const int r = lane + h * WAVE;
        const double f = F.v[h];
        const double term = r < ne ? ((0.5 * f) * f) * d.efc_R[r] : 0.0;
        const int nh = ne - h * WAVE < WAVE ? ne - h * WAVE : WAVE;
        for (int l = 0; l < nh; l++) improvement = improvement + readlane_d(term, l);
      }
    }
    int r = next_visited(vis, -1);
    int t = 0, dim = 0;
    DofV gc[MGS_MAXDIM];
    if (r >= 0) {
      t = sel_i(tk, r);
      dim = t == MGS_EFC_FRICTION ? 1 : sel_i(dk, r);
      load_block_rows(d, r, dim, nv, lane, gc);
    }
    while (r >= 0) {
      const int rn = next_visited(vis, r);
      int tn = 0, dimn = 0;
      DofV gn[MGS_MAXDIM];
#pragma unroll
      for (int i = 0; i < MGS_MAXDIM; i++) gn[i] = dof_zero();
      if (rn >= 0) {
        tn = sel_i(tk, rn);
        dimn = tn == MGS_EFC_FRICTION ? 1 : sel_i(dk, rn);
        load_block_rows(d, rn, dimn, nv, lane, gn);
      }
      if (t == MGS_EFC_FRICTION) {
        const DofV g = gc[0];
        double res = dof_tree(dof_mul(g, u), P) + d.efc_b[r];
        double fo = getf(F, r);
        double Arr = sel_d(Ak, r);
        double fnew[1] = {fo - res * (1.0 / Arr)};
        project_scalar(t, sel_d(Fk, r), fnew);
        double delta = fnew[0] - fo;
        double ch = cost_change1(Arr, delta, res);
        if (ch > 1e-10) { delta = 0.0; ch = 0.0; }
        improvement = improvement - ch;
        if (delta != 0.0) {
          dof_axpy(u, g, delta, nv, lane);
          setf(F, r, fnew[0], lane);
        }
      } else if (dim == 3) {
        improvement = improvement - pgs_contact<3>(md, d, r, nv, P, lane, u, F, 1, gc);
#if MGS_MAXDIM > 4
      } else if (dim == 6) {
        improvement = improvement - pgs_contact<6>(md, d, r, nv, P, lane, u, F, 1, gc);
#endif
      } else {
        improvement = improvement - pgs_contact<4>(md, d, r, nv, P, lane, u, F, 1, gc);
      }
      r = rn;
      t = tn;
      dim = dimn;
#pragma unroll
      for (int i = 0; i < MGS_MAXDIM; i++) gc[i] = gn[i];
    }
    if (improvement * scale < md.m.noslip_tolerance) break;
  }
}

// G in LDS (main build): rows are a few LDS loads away, the sweep reads them
// in place; G in HBM (wide build): noslip_prefetch (C5 pile rollout 2148 ->
// 2058 ms, profiles/r04m_noslip_ab.txt; the main build measured 1 % slower
// with it)
DEVI void noslip_inplace(const Mdl& md, Dat& d, double scale, Frc& F, DofV& u) {
  int nv = md.m.nv, ne = uni(d.NEFC), lane = lane_id();
  int P = next_pow2(nv);
  if (md.m.noslip_iterations <= 0 || ne <= 0) return;
  int tk[MGS_RPL], dk[MGS_RPL];
  unsigned long long vis[MGS_RPL];
#pragma unroll
  for (int h = 0; h < MGS_RPL; h++) {
    const int r = lane + h * WAVE;
    int t = -1, dim = 0, v = 0;
    if (r < ne) {
      t = d.efc_type[r];
      dim = d.efc_dim[r];
      v = t == MGS_EFC_FRICTION || (t == MGS_EFC_CONTACT && dim > 1 && efc_lead(d, r));
    }
    tk[h] = t;
    dk[h] = dim;
    vis[h] = __ballot(v);
  }
  for (int ns = 0; ns < md.m.noslip_iterations; ns++) {
    PCNT(38, 1);
    double improvement = 0.0;
    // the noslip cost drops the regulariser: count its removal at iteration 0
    // (row terms on their lanes, summed in row order)
    if (ns == 0) {
#pragma unroll
      for (int h = 0; h < MGS_RPL; h++) {
        const int r = lane + h * WAVE;
        const double f = F.v[h];
        const double term = r < ne ? ((0.5 * f) * f) * d.efc_R[r] : 0.0;
        const int nh = ne - h * WAVE < WAVE ? ne - h * WAVE : WAVE;
        for (int l = 0; l < nh; l++) improvement = improvement + readlane_d(term, l);
      }
    }
#pragma unroll
    for (int h = 0; h < MGS_RPL; h++) {
      unsigned long long m = vis[h];
      while (m) {
        const int l = __ffsll((long long)m) - 1;
        m &= m - 1ull;
        const int r = l + h * WAVE;
        const int t = __builtin_amdgcn_readlane(tk[h], l), dim = __builtin_amdgcn_readlane(dk[h], l);
        if (t == MGS_EFC_FRICTION) {
          DofV g = dof_load(d.G + r * d.gs, nv, lane);
          double res = dof_tree(dof_mul(g, u), P) + d.efc_b[r];
          double fo = getf(F, r);
          double Arr = row_sqnorm(d, r, nv);
          double fnew[1] = {fo - res * (1.0 / Arr)};
          project_scalar(t, row_floss(md, d, r), fnew);
          double delta = fnew[0] - fo;
          double ch = cost_change1(Arr, delta, res);
          if (ch > 1e-10) { delta = 0.0; ch = 0.0; }
          improvement = improvement - ch;
          if (delta != 0.0) {
            dof_axpy(u, g, delta, nv, lane);
            setf(F, r, fnew[0], lane);
          }
        } else if (dim == 3) {
          improvement = improvement - pgs_contact<3>(md, d, r, nv, P, lane, u, F, 1);
#if MGS_MAXDIM > 4
        } else if (dim == 6) {
          improvement = improvement - pgs_contact<6>(md, d, r, nv, P, lane, u, F, 1);
#endif
        } else {
          improvement = improvement - pgs_contact<4>(md, d, r, nv, P, lane, u, F, 1);
        }
      }
    }
    if (improvement * scale < md.m.noslip_tolerance) break;
  }
}

DEVI void noslip(const Mdl& md, Dat& d, double scale, Frc& F, DofV& u) {
#ifdef MGS_G_GLOBAL
  noslip_prefetch(md, d, scale, F, u);
#else
  noslip_inplace(md, d, scale, F, u);
#endif
}

// qacc = qacc_smooth + L^-T D^-1/2 u ; qfrc_constraint = L D^1/2 u, lane i owns
// dof i: backward substitution column by column (k descending, as the oracle),
// the L-multiply row by row (k ascending), broadcasts by v_readlane.
// u_main: the main solver's u (MuJoCo saves qacc_warmstart before noslip;
// qacc feeds only the warmstart, implicitfast integrates qfrc_constraint)
template <int NV>
DEVI void finalize_solution(const Mdl& md, Dat& d, const DofV& u_main, const DofV& u) {
  int lane = lane_id();
#define FS_ROW(h) (lane + (h) * WAVE < NV ? lane + (h) * WAVE : 0)
#if MGS_REG_ROWS
  static_assert(MGS_DPL == 1, "register rows hold one dof per lane");
  int li = FS_ROW(0);
  double Lr[NV], Lc[NV];
#pragma unroll
  for (int k = 0; k < NV; k++) { Lr[k] = d.M[TRI(li, k, NV)]; Lc[k] = d.M[TRI(k, li, NV)]; }
#define FS_LR(h, k) Lr[k]
#define FS_LC(h, k) Lc[k]
#else
#define FS_LR(h, k) d.M[TRI(FS_ROW(h), (k), NV)]
#define FS_LC(h, k) d.M[TRI((k), FS_ROW(h), NV)]
#endif
  DofV z;
#pragma unroll
  for (int h = 0; h < MGS_DPL; h++) z.v[h] = u_main.v[h] * d.isD[FS_ROW(h)];
#pragma unroll
  for (int k = NV - 1; k >= 0; k--) {
    double zk = dof_readlane(z, k);
#pragma unroll
    for (int h = 0; h < MGS_DPL; h++)
      if (lane + h * WAVE < k) z.v[h] = __builtin_fma(-FS_LC(h, k), zk, z.v[h]);
  }
  DofV t, q;
#pragma unroll
  for (int h = 0; h < MGS_DPL; h++) {
    t.v[h] = u.v[h] * d.sD[FS_ROW(h)];
    q.v[h] = t.v[h];
  }
#pragma unroll
  for (int k = 0; k < NV; k++) {
    double tk = dof_readlane(t, k);
#pragma unroll
    for (int h = 0; h < MGS_DPL; h++)
      if (lane + h * WAVE > k) q.v[h] = __builtin_fma(FS_LR(h, k), tk, q.v[h]);
  }
#undef FS_LR
#undef FS_LC
#undef FS_ROW
#pragma unroll
  for (int h = 0; h < MGS_DPL; h++) {
    const int i = lane + h * WAVE;
    if (i < NV) {
      d.qfrc_constraint[i] = q.v[h];
      d.qacc_ws[i] = d.qacc_smooth[i] + z.v[h];   // qacc, kept as next step's warmstart
    }
  }
  wsync();
}

// ---------------------------------------------------------------------------
// Newton solver on the primal (MuJoCo mj_solNewton restated; oracle
// solve_newton() is the arithmetic contract).  Whitened coordinates
// w = D^1/2 L^T qacc; Gauss cost 1/2|w - w0|^2; row violations jar = G w - aref.
// Lanes over rows for violations / row costs (block leaders evaluate a whole
// contact block), lanes over dofs for gradients, lanes over (i, j) for the
// Hessian, columns of the LDL in parallel; scalar line search replicated.
#define ST_OFF 0
#define ST_QUAD 1
#define ST_CONE 2
#define ST_SAT 3

// evaluate the block led by row r at violations jr[] (registers, dim <= 4):
// forces f[], zone, cone Hessian hb[a*4+b] (if want_hb); returns cost
DEVI double row_eval(const Mdl& md, const Dat& d, int r, int t, int dim, const double* jr, double* f, int& st,
                     double* hb, bool want_hb, double mup, double k1, double* cq = nullptr) {
  if (t == MGS_EFC_EQUALITY) {
    double Dr = d.efc_Dr[r];
    f[0] = -jr[0] * Dr;
    st = ST_QUAD;
    return ((0.5 * Dr) * jr[0]) * jr[0];
  }
  if (t == MGS_EFC_LIMIT || (t == MGS_EFC_CONTACT && dim == 1)) {
    double Dr = d.efc_Dr[r];
    if (jr[0] < 0.0) {
      f[0] = -jr[0] * Dr;
      st = ST_QUAD;
      return ((0.5 * Dr) * jr[0]) * jr[0];
    }
    f[0] = 0.0;
    st = ST_OFF;
    return 0.0;
  }
  if (t == MGS_EFC_FRICTION) {
    double isr = d.efc_isR[r];
    double z = -jr[0] * isr;
    double lim = row_floss(md, d, r) * sqrt(d.efc_R[r]);
    double y = z;
    st = ST_QUAD;
    if (z > lim) { y = lim; st = ST_SAT; }
    else if (z < -lim) { y = -lim; st = ST_SAT; }
    f[0] = y * isr;
    return y * z - 0.5 * (y * y);
  }
  // mup = mu0 / sqrt(impratio), k1 = 1 / (1 + mup^2): per-block constants of the
  // solve (oracle efc_mup, efc_k1), held in registers by the caller
  double z[MGS_MAXDIM], y[MGS_MAXDIM], isr[MGS_MAXDIM];
#pragma unroll
  for (int a = 0; a < MGS_MAXDIM; a++) {
    isr[a] = (a < dim) ? d.efc_isR[r + a] : 0.0;
    z[a] = (a < dim) ? -jr[a] * isr[a] : 0.0;
  }
  double t2 = 0.0;
#pragma unroll
  for (int a = 1; a < MGS_MAXDIM; a++)
    if (a < dim) t2 = t2 + z[a] * z[a];
  double tn = sqrt(t2);
  double yn = 0.0, itn = 0.0, sc = 0.0;
  if (tn <= mup * z[0]) {
    st = ST_QUAD;
#pragma unroll
    for (int a = 0; a < MGS_MAXDIM; a++) y[a] = z[a];
  } else if (mup * tn <= -z[0]) {
    st = ST_OFF;
#pragma unroll
    for (int a = 0; a < MGS_MAXDIM; a++) y[a] = 0.0;
  } else {
    st = ST_CONE;
    yn = (z[0] + mup * tn) * k1;
    itn = 1.0 / tn;
    sc = (mup * yn) * itn;
    y[0] = yn;
#pragma unroll
    for (int a = 1; a < MGS_MAXDIM; a++) y[a] = sc * z[a];
  }
  double c = 0.0;
#pragma unroll
  for (int a = 0; a < MGS_MAXDIM; a++) {
    if (a < dim) {
      f[a] = y[a] * isr[a];
      c = c + y[a] * y[a];
    }
  }
  if (cq && st == ST_CONE) {
    cq[0] = k1;
    cq[1] = sc;
#pragma unroll
    for (int a = 1; a < MGS_MAXDIM; a++) cq[1 + a] = z[a] * itn;
  }
  if (want_hb && st == ST_CONE) {
    double k2 = sc;
    double v[MGS_MAXDIM], e[MGS_MAXDIM];
    v[0] = 1.0;
    e[0] = 0.0;
#pragma unroll
    for (int a = 1; a < MGS_MAXDIM; a++) { e[a] = z[a] * itn; v[a] = mup * e[a]; }
#pragma unroll
    for (int a = 0; a < MGS_MAXDIM; a++)
#pragma unroll
      for (int b = 0; b < MGS_MAXDIM; b++) {
        double Pm = (k1 * v[a]) * v[b];
        if (a >= 1 && b >= 1) Pm = Pm + k2 * ((a == b ? 1.0 : 0.0) - e[a] * e[b]);
        hb[a * MGS_MAXDIM + b] = (isr[a] * isr[b]) * Pm;
      }
  }
  return 0.5 * c;
}

// sum over rows in the oracle's tree_rows order: leaf l = ((v[l] + v[l + 64]) +
// v[l + 128]) + v[l + 192], rows past ne left out
DEVI double tree_rows(const double (&v)[MGS_RPL], int ne) {
  int n = ne < WAVE ? ne : WAVE;
  if (n <= 0) return 0.0;
  int lane = lane_id();
  double leaf = v[0];
#pragma unroll
  for (int h = 1; h < MGS_RPL; h++)
    if (lane + h * WAVE < ne) leaf = leaf + v[h];
  if (lane >= n) leaf = 0.0;
  return tree_sum(leaf, next_pow2(n));
}

// jar = G w - aref; forces, zones, cone Hessians into LDS; returns total cost
template <int NV>
DEVI double newton_eval(const Mdl& md, Dat& d, const double* w, int P, const double* mupR, const double* k1R) {
  int ne = uni(d.NEFC), lane = lane_id();
  PCNT(37, 1);
  DofV q;
#pragma unroll
  for (int h = 0; h < MGS_DPL; h++) q.v[h] = (lane + h * WAVE < NV) ? w[lane + h * WAVE] - d.nw0[lane + h * WAVE] : 0.0;
  double gauss = 0.5 * dof_tree(dof_mul(q, q), P);
#if MGS_REG_ROWS
  double wr[NV];
#pragma unroll
  for (int k = 0; k < NV; k++) wr[k] = w[k];
#else
  const double* wr = w;
#endif
  for (int r = lane; r < ne; r += WAVE) {
    const double* Gr = d.G + r * GS;
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < NV; k++) s = __builtin_fma(Gr[k], wr[k], s);
    d.efc_jar[r] = s - d.efc_aref[r];
  }
  wsync();
  double cr[MGS_RPL];
#pragma unroll
  for (int h = 0; h < MGS_RPL; h++) {
    cr[h] = 0.0;
    int r = lane + h * WAVE;
    if (r < ne && efc_lead(d, r)) {
      int t = d.efc_type[r];
      int dim = (t == MGS_EFC_CONTACT) ? d.efc_dim[r] : 1;
      double jr[MGS_MAXDIM], f[MGS_MAXDIM], hb[BLKSTRIDE];
      int st = ST_OFF;
#pragma unroll
      for (int a = 0; a < MGS_MAXDIM; a++) jr[a] = (a < dim) ? d.efc_jar[r + a] : 0.0;
      cr[h] = row_eval(md, d, r, t, dim, jr, f, st, hb, true, mupR[h], k1R[h]);
#pragma unroll
      for (int a = 0; a < MGS_MAXDIM; a++)
        if (a < dim) { d.efc_f[r + a] = f[a]; d.efc_state[r + a] = st; }
      if (st == ST_CONE) {
        double* o = d.con_hb + BLKSTRIDE * d.efc_con[r];
#pragma unroll
        for (int a = 0; a < MGS_MAXDIM; a++)
#pragma unroll
          for (int b = 0; b < MGS_MAXDIM; b++)
            if (a < dim && b < dim) o[a * dim + b] = hb[a * MGS_MAXDIM + b];
      }
    }
  }
  double tot = gauss + tree_rows(cr, ne);
  wsync();
  return tot;
}

// newton_eval at two points in one pass over the rows: c0 at wa (cost only:
// its violations go to the idle scratch slot, nothing else is stored), c1 at
// wb with every side effect of newton_eval(wb).  Same arithmetic per cost as
// two newton_eval calls; the row loads and the latency chains are shared.
template <int NV>
DEVI void newton_eval_pair(const Mdl& md, Dat& d, const double* wa, const double* wb, int P, const double* mupR,
                           const double* k1R, double& c0, double& c1) {
  int ne = uni(d.NEFC), lane = lane_id();
  PCNT(37, 2);
  DofV qa, qb;
#pragma unroll
  for (int h = 0; h < MGS_DPL; h++) {
    const int i = lane + h * WAVE;
    qa.v[h] = (i < NV) ? wa[i] - d.nw0[i] : 0.0;
    qb.v[h] = (i < NV) ? wb[i] - d.nw0[i] : 0.0;
  }
  double gauss0 = 0.5 * dof_tree(dof_mul(qa, qa), P);
  double gauss1 = 0.5 * dof_tree(dof_mul(qb, qb), P);
  double* jar0 = d.scratch;   // idle until the first Newton Hessian
#if MGS_REG_ROWS
  double ra[NV], rb[NV];
#pragma unroll
  for (int k = 0; k < NV; k++) { ra[k] = wa[k]; rb[k] = wb[k]; }
#else
  const double *ra = wa, *rb = wb;
#endif
  for (int r = lane; r < ne; r += WAVE) {
    const double* Gr = d.G + r * GS;
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int k = 0; k < NV; k++) {
      double g = Gr[k];
      s0 = __builtin_fma(g, ra[k], s0);
      s1 = __builtin_fma(g, rb[k], s1);
    }
    jar0[r] = s0 - d.efc_aref[r];
    d.efc_jar[r] = s1 - d.efc_aref[r];
  }
  wsync();
  double cr0[MGS_RPL], cr1[MGS_RPL];
#pragma unroll
  for (int h = 0; h < MGS_RPL; h++) {
    cr0[h] = 0.0;
    cr1[h] = 0.0;
    int r = lane + h * WAVE;
    if (r < ne && efc_lead(d, r)) {
      int t = d.efc_type[r];
      int dim = (t == MGS_EFC_CONTACT) ? d.efc_dim[r] : 1;
      double jr[MGS_MAXDIM], f[MGS_MAXDIM], hb[BLKSTRIDE];
      int st = ST_OFF;
#pragma unroll
      for (int a = 0; a < MGS_MAXDIM; a++) jr[a] = (a < dim) ? jar0[r + a] : 0.0;
      cr0[h] = row_eval(md, d, r, t, dim, jr, f, st, hb, true, mupR[h], k1R[h]);
      st = ST_OFF;
#pragma unroll
      for (int a = 0; a < MGS_MAXDIM; a++) jr[a] = (a < dim) ? d.efc_jar[r + a] : 0.0;
      cr1[h] = row_eval(md, d, r, t, dim, jr, f, st, hb, true, mupR[h], k1R[h]);
#pragma unroll
      for (int a = 0; a < MGS_MAXDIM; a++)
        if (a < dim) { d.efc_f[r + a] = f[a]; d.efc_state[r + a] = st; }
      if (st == ST_CONE) {
        double* o = d.con_hb + BLKSTRIDE * d.efc_con[r];
#pragma unroll
        for (int a = 0; a < MGS_MAXDIM; a++)
#pragma unroll
          for (int b = 0; b < MGS_MAXDIM; b++)
            if (a < dim && b < dim) o[a * dim + b] = hb[a * MGS_MAXDIM + b];
      }
    }
  }
  c0 = gauss0 + tree_rows(cr0, ne);
  c1 = gauss1 + tree_rows(cr1, ne);
  wsync();
}

// g = (w - w0) - G^T f   (lanes over dofs, rows summed in order)
template <int NV>
DEVI void newton_grad(const Mdl& md, Dat& d, const double* w) {
  int ne = uni(d.NEFC), lane = lane_id();
#pragma unroll
  for (int h = 0; h < MGS_DPL; h++) {
    const int i = lane + h * WAVE;   // this slot's dof
    if (i >= NV) continue;
    double s = 0.0;
    int r = 0;
#ifdef MGS_G_GLOBAL
    // G in HBM: sixteen rows' loads in flight per step (one memory latency per
    // sixteen terms), same ascending FMA chain
    for (; r + 16 <= ne; r += 16) {
      double g[16], f[16];
#pragma unroll
      for (int q = 0; q < 16; q++) { g[q] = d.G[(r + q) * GS + i]; f[q] = d.efc_f[r + q]; }
#pragma unroll
      for (int q = 0; q < 16; q++) s = __builtin_fma(g[q], f[q], s);
    }
#endif
    // rows in order, four loads in flight per step
    for (; r + 4 <= ne; r += 4) {
      double g0 = d.G[r * GS + i], g1 = d.G[(r + 1) * GS + i], g2 = d.G[(r + 2) * GS + i],
             g3 = d.G[(r + 3) * GS + i];
      double f0 = d.efc_f[r], f1 = d.efc_f[r + 1], f2 = d.efc_f[r + 2], f3 = d.efc_f[r + 3];
      s = __builtin_fma(g0, f0, s);
      s = __builtin_fma(g1, f1, s);
      s = __builtin_fma(g2, f2, s);
      s = __builtin_fma(g3, f3, s);
    }
    for (; r < ne; r++) s = __builtin_fma(d.G[r * GS + i], d.efc_f[r], s);
    d.ng[i] = (w[i] - d.nw0[i]) - s;
  }
  wsync();
}

// cost derivatives along the search direction at step alpha
DEVI void ls_eval(const Mdl& md, const Dat& d, int ne, double alpha, double A1, double A2, double* d1, double* d2,
                  const double* mupR, const double* k1R) {
  int lane = lane_id();
  PCNT(36, 1);
  double c1[MGS_RPL], c2[MGS_RPL];
#pragma unroll
  for (int h = 0; h < MGS_RPL; h++) {
    c1[h] = 0.0;
    c2[h] = 0.0;
    int r = lane + h * WAVE;
    if (r < ne && efc_lead(d, r)) {
      int t = d.efc_type[r];
      int dim = (t == MGS_EFC_CONTACT) ? d.efc_dim[r] : 1;
      double jr[MGS_MAXDIM], jv[MGS_MAXDIM], f[MGS_MAXDIM], hb[BLKSTRIDE], cq[MGS_MAXDIM + 1];
      int st = ST_OFF;
#pragma unroll
      for (int a = 0; a < MGS_MAXDIM; a++) {
        jv[a] = (a < dim) ? d.efc_jv[r + a] : 0.0;
        jr[a] = (a < dim) ? d.efc_jar[r + a] + alpha * jv[a] : 0.0;
      }
      row_eval(md, d, r, t, dim, jr, f, st, hb, false, mupR[h], k1R[h], cq);
      double s1 = 0.0, s2 = 0.0;
      if (dim == 1) {
        s1 = -f[0] * jv[0];
        if (st == ST_QUAD) s2 = (jv[0] * d.efc_Dr[r]) * jv[0];
      } else {
#pragma unroll
        for (int a = 0; a < MGS_MAXDIM; a++)
          if (a < dim) s1 = s1 - f[a] * jv[a];
        if (st == ST_QUAD) {
#pragma unroll
          for (int a = 0; a < MGS_MAXDIM; a++)
            if (a < dim) s2 = s2 + (jv[a] * d.efc_Dr[r + a]) * jv[a];
        } else if (st == ST_CONE) {
          // jv' hb jv in closed form (oracle ls_eval)
          double mup = mupR[h];
          double u[MGS_MAXDIM];
#pragma unroll
          for (int a = 0; a < MGS_MAXDIM; a++) u[a] = (a < dim) ? jv[a] * d.efc_isR[r + a] : 0.0;
          double vu = u[0], eu = 0.0, uu = 0.0;
#pragma unroll
          for (int a = 1; a < MGS_MAXDIM; a++) {
            if (a < dim) {
              vu = vu + (mup * cq[1 + a]) * u[a];
              eu = eu + cq[1 + a] * u[a];
              uu = uu + u[a] * u[a];
            }
          }
          s2 = (cq[0] * vu) * vu + cq[1] * (uu - eu * eu);
        }
      }
      c1[h] = s1;
      c2[h] = s2;
    }
  }
  *d1 = (A1 + alpha * A2) + tree_rows(c1, ne);
  *d2 = A2 + tree_rows(c2, ne);
}

typedef double v4d __attribute__((ext_vector_type(4)));

// Newton Hessian (see solve_newton): per-row weights into the (idle) nH
// region, then the lower tiles of G' X by v_mfma_f64_16x16x4, written to nH
// as full rows of H = I + G' W G (upper entries left unwritten).
template <int NV>
DEVI void hessian_mfma(const Mdl& md, Dat& d, int ne) {
  constexpr int NT = (NV + 15) / 16;
  int lane = lane_id();
  // weight table: wt[M r .. M r + M - 1] = w_a (M = MGS_MAXDIM), wi[r] = lead * 8 + nd (exact in f64)
  double* wt = d.nH;
  double* wi = d.nH + MGS_MAXDIM * md.m.nefc_max;
  for (int r = lane; r < ne; r += WAVE) {
    int t = d.efc_type[r];
    int st = d.efc_state[r];
    double wv[MGS_MAXDIM];
#pragma unroll
    for (int a = 0; a < MGS_MAXDIM; a++) wv[a] = 0.0;
    int lead = r, nd = 0;
    if (st == ST_QUAD) {
      wv[0] = d.efc_Dr[r];
      nd = 1;
    } else if (st == ST_CONE && t == MGS_EFC_CONTACT) {
      int c = d.efc_con[r], dim = d.efc_dim[r];
      int bp = 0;
      for (int q = 1; q < MGS_MAXDIM; q++)
        if (r - q >= 0 && bp == q - 1 && d.efc_type[r - q] == MGS_EFC_CONTACT && d.efc_con[r - q] == c) bp = q;
      const double* hb = d.con_hb + BLKSTRIDE * c + bp;
      lead = r - bp;
      nd = dim;
      wv[0] = hb[0];
#pragma unroll
      for (int a = 1; a < MGS_MAXDIM; a++) wv[a] = (dim > a) ? hb[a * dim] : 0.0;
    }
#pragma unroll
    for (int a = 0; a < MGS_MAXDIM; a++) wt[MGS_MAXDIM * r + a] = wv[a];
    wi[r] = (double)(lead * 8 + nd);
  }
  wsync();
  int cl = lane & 15, rg = lane >> 4;
  v4d acc[NT * (NT + 1) / 2];
#pragma unroll
  for (int q = 0; q < NT * (NT + 1) / 2; q++) acc[q] = (v4d){0.0, 0.0, 0.0, 0.0};
  int ks = (ne + 3) >> 2;
  for (int s = 0; s < ks; s++) {
    int r = 4 * s + rg;
    bool valid = r < ne;
    int rr = valid ? r : 0;
    double gv[NT], x[NT];
    const double* Gr = d.G + rr * GS;
#pragma unroll
    for (int t = 0; t < NT; t++) {
      int c = cl + 16 * t;
      double v = Gr[c < NV ? c : 0];
      gv[t] = (valid && c < NV) ? v : 0.0;
    }
    const double* wr = wt + MGS_MAXDIM * rr;
    double w[MGS_MAXDIM];
#pragma unroll
    for (int a = 0; a < MGS_MAXDIM; a++) w[a] = wr[a];
    int info = (int)wi[rr];
    int lead = info >> 3, nd = valid ? (info & 7) : 0;
    bool multi = __ballot(nd > 1) != 0ull;
    if (!multi) {
#pragma unroll
      for (int t = 0; t < NT; t++) x[t] = (nd == 1) ? 0.0 + gv[t] * w[0] : 0.0;
    } else {
#pragma unroll
      for (int t = 0; t < NT; t++) {
        int c = cl + 16 * t;
        int cc = c < NV ? c : 0;
        double xs = 0.0;
#pragma unroll
        for (int a = 0; a < MGS_MAXDIM; a++) {
          int aa = a < nd ? a : 0;
          double tv = xs + d.G[(lead + aa) * GS + cc] * w[a];
          xs = (a < nd) ? tv : xs;
        }
        x[t] = (c < NV) ? xs : 0.0;
      }
    }
    // tile (tj, ti), tj <= ti: D[j][i] += G_rj X_ri
    int q = 0;
#pragma unroll
    for (int ti = 0; ti < NT; ti++)
#pragma unroll
      for (int tj = 0; tj <= ti; tj++) {
        acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(gv[tj], x[ti], acc[q], 0, 0, 0);
        q++;
      }
  }
  wsync();   // the weight table is dead; H overwrites the region
  int q = 0;
#pragma unroll
  for (int ti = 0; ti < NT; ti++)
#pragma unroll
    for (int tj = 0; tj <= ti; tj++) {
      int i = cl + 16 * ti;
#pragma unroll
      for (int g = 0; g < 4; g++) {
        int j = rg + 4 * g + 16 * tj;
        if (i < NV && j <= i) d.nH[TRI(i, j, NV)] = (i == j ? 1.0 : 0.0) + acc[q][g];
      }
      q++;
    }
  wsync();
}

// Line-search rows in registers: lane r holds block-leader row r (rows >= 64
// take the LDS path of ls_eval).  Loaded once per Newton iteration, so each
// evaluation along the direction is register arithmetic plus two reductions;
// the expressions are row_eval()'s and ls_eval()'s (oracle ls_eval), per kind.
struct LsRow {
  int kind, dim;   // kind: 0 none, 1 equality, 2 limit / frictionless contact, 3 friction, 4 cone block
  double jar[MGS_MAXDIM], jv[MGS_MAXDIM], isr[MGS_MAXDIM], Dr[MGS_MAXDIM];
  double mup, k1, lim;
};
DEVI void ls_row_load(const Mdl& md, const Dat& d, int r, int ne, double mup, double k1, LsRow& L) {
  L.kind = 0;
  L.dim = 1;
  L.mup = mup;
  L.k1 = k1;
  L.lim = 0.0;
#pragma unroll
  for (int a = 0; a < MGS_MAXDIM; a++) { L.jar[a] = 0.0; L.jv[a] = 0.0; L.isr[a] = 0.0; L.Dr[a] = 0.0; }
  if (r < ne && efc_lead(d, r)) {
    int t = d.efc_type[r];
    int dim = (t == MGS_EFC_CONTACT) ? d.efc_dim[r] : 1;
    L.dim = dim;
    L.kind = (t == MGS_EFC_EQUALITY) ? 1 : (t == MGS_EFC_FRICTION) ? 3 : (dim == 1) ? 2 : 4;
#pragma unroll
    for (int a = 0; a < MGS_MAXDIM; a++) {
      if (a < dim) {
        L.jar[a] = d.efc_jar[r + a];
        L.jv[a] = d.efc_jv[r + a];
        L.isr[a] = d.efc_isR[r + a];
        L.Dr[a] = d.efc_Dr[r + a];
      }
    }
    if (L.kind == 3) L.lim = row_floss(md, d, r) * sqrt(d.efc_R[r]);
  }
}
DEVI void ls_row(const LsRow& L, double alpha, double& s1o, double& s2o) {
  double s1 = 0.0, s2 = 0.0;
  double jr0 = L.jar[0] + alpha * L.jv[0];
  if (L.kind == 1 || L.kind == 2) {
    double f0 = 0.0;
    bool quad = (L.kind == 1) || (jr0 < 0.0);
    if (quad) f0 = -jr0 * L.Dr[0];
    s1 = -f0 * L.jv[0];
    if (quad) s2 = (L.jv[0] * L.Dr[0]) * L.jv[0];
  } else if (L.kind == 3) {
    double z = -jr0 * L.isr[0];
    double y = z;
    bool quad = true;
    if (z > L.lim) { y = L.lim; quad = false; }
    else if (z < -L.lim) { y = -L.lim; quad = false; }
    double f0 = y * L.isr[0];
    s1 = -f0 * L.jv[0];
    if (quad) s2 = (L.jv[0] * L.Dr[0]) * L.jv[0];
  } else if (L.kind == 4) {
    int dim = L.dim;
    double mup = L.mup;
    double z[MGS_MAXDIM], y[MGS_MAXDIM];
#pragma unroll
    for (int a = 0; a < MGS_MAXDIM; a++) {
      double jr = (a < dim) ? L.jar[a] + alpha * L.jv[a] : 0.0;
      z[a] = (a < dim) ? -jr * L.isr[a] : 0.0;
    }
    double t2 = 0.0;
#pragma unroll
    for (int a = 1; a < MGS_MAXDIM; a++)
      if (a < dim) t2 = t2 + z[a] * z[a];
    double tn = sqrt(t2);
    int st;
    double yn = 0.0, itn = 0.0, sc = 0.0;
    if (tn <= mup * z[0]) {
      st = ST_QUAD;
#pragma unroll
      for (int a = 0; a < MGS_MAXDIM; a++) y[a] = z[a];
    } else if (mup * tn <= -z[0]) {
      st = ST_OFF;
#pragma unroll
      for (int a = 0; a < MGS_MAXDIM; a++) y[a] = 0.0;
    } else {
      st = ST_CONE;
      yn = (z[0] + mup * tn) * L.k1;
      itn = 1.0 / tn;
      sc = (mup * yn) * itn;
      y[0] = yn;
#pragma unroll
      for (int a = 1; a < MGS_MAXDIM; a++) y[a] = sc * z[a];
    }
#pragma unroll
    for (int a = 0; a < MGS_MAXDIM; a++)
      if (a < dim) s1 = s1 - (y[a] * L.isr[a]) * L.jv[a];
    if (st == ST_QUAD) {
#pragma unroll
      for (int a = 0; a < MGS_MAXDIM; a++)
        if (a < dim) s2 = s2 + (L.jv[a] * L.Dr[a]) * L.jv[a];
    } else if (st == ST_CONE) {
      double u[MGS_MAXDIM];
#pragma unroll
      for (int a = 0; a < MGS_MAXDIM; a++) u[a] = (a < dim) ? L.jv[a] * L.isr[a] : 0.0;
      double vu = u[0], eu = 0.0, uu = 0.0;
#pragma unroll
      for (int a = 1; a < MGS_MAXDIM; a++) {
        if (a < dim) {
          double e = z[a] * itn;
          vu = vu + (mup * e) * u[a];
          eu = eu + e * u[a];
          uu = uu + u[a] * u[a];
        }
      }
      s2 = (L.k1 * vu) * vu + sc * (uu - eu * eu);
    }
  }
  s1o = s1;
  s2o = s2;
}
// ls_eval with the first 64 rows from registers
DEVI void ls_eval_fast(const Mdl& md, const Dat& d, int ne, const LsRow& L, double alpha, double A1, double A2,
                       double* d1, double* d2, const double* mupR, const double* k1R) {
  PCNT(36, 1);
  double c1[MGS_RPL], c2[MGS_RPL];
#pragma unroll
  for (int h = 0; h < MGS_RPL; h++) { c1[h] = 0.0; c2[h] = 0.0; }
  ls_row(L, alpha, c1[0], c2[0]);
#pragma unroll
  for (int h = 1; h < MGS_RPL; h++) {
    if (ne > h * WAVE) {
      LsRow L1;
      ls_row_load(md, d, lane_id() + h * WAVE, ne, mupR[h], k1R[h], L1);
      ls_row(L1, alpha, c1[h], c2[h]);
    }
  }
  *d1 = (A1 + alpha * A2) + tree_rows(c1, ne);
  *d2 = A2 + tree_rows(c2, ne);
}

template <int NV>
DEVI void solve_newton(const Mdl& md, Dat& d, double scale, Frc& F, DofV& u) {
  int nv = md.m.nv, ne = uni(d.NEFC), lane = lane_id();
  int P = next_pow2(nv);
  for (int r = lane; r < ne; r += WAVE) {
    double sq = sqrt(d.efc_R[r]);
    d.efc_isR[r] = 1.0 / sq;
    d.efc_Dr[r] = 1.0 / d.efc_R[r];
  }
  // per-block cone constants of this solve, rows lane and lane + 64
  double mupR[MGS_RPL], k1R[MGS_RPL];
#pragma unroll
  for (int h = 0; h < MGS_RPL; h++) {
    mupR[h] = 0.0;
    k1R[h] = 0.0;
    int r = lane + h * WAVE;
    if (r < ne && d.efc_type[r] == MGS_EFC_CONTACT && d.efc_dim[r] > 1) {
      double mup = con_mu_of(md, d, d.efc_con[r])[0] / sqrt(md.m.impratio);
      mupR[h] = mup;
      k1R[h] = 1.0 / (1.0 + mup * mup);
    }
  }
  // w0 = W(qacc_smooth), w = W(qacc_ws)   (lane i: s_i = a_i + sum_{k>i} L_ki a_k)
#pragma unroll
  for (int h = 0; h < MGS_DPL; h++) {
    const int i = lane + h * WAVE;
    int li = i < NV ? i : 0;
    double s = d.qacc_smooth[li], s2 = d.qacc_ws[li];
#pragma unroll
    for (int k = 1; k < NV; k++) {
      double l = d.M[TRI(k, li, NV)];
      if (k > i) {
        s = __builtin_fma(l, d.qacc_smooth[k], s);
        s2 = __builtin_fma(l, d.qacc_ws[k], s2);
      }
    }
    if (i < NV) {
      d.nw0[i] = s * d.sD[i];
      d.nw[i] = s2 * d.sD[i];
    }
  }
  wsync();
  double C = 0.0;
  if (ne > 0) {
    // (oracle: evaluate warmstart, smooth, keep the cheaper; evaluating the
    // smooth point first leaves the warmstart's rows current in the common case)
    double c0, cws;
    newton_eval_pair<NV>(md, d, d.nw0, d.nw, P, mupR, k1R, c0, cws);
    if (cws < c0) {
      C = cws;
    } else {
      DOF_SLOTS(k, nv) d.nw[k] = d.nw0[k];
      wsync();
      C = newton_eval<NV>(md, d, d.nw, P, mupR, k1R);
    }
  } else {
    DOF_SLOTS(k, nv) d.nw[k] = d.nw0[k];
    wsync();
  }
  newton_grad<NV>(md, d, d.nw);
  PT(12);
  int npair = (nv * (nv + 1)) / 2;
  int it;
  for (it = 0; it < md.m.iterations && ne > 0; it++) {
    {
      // Hessian I + G' W G on the matrix cores.  W is block diagonal (Dr on quad
      // rows, the cone Hessian on cone blocks, 0 on inactive rows); X = W G row
      // by row (x = 0.0 + sum_a G_{lead+a,i} w_a), then H_ij = (i == j) +
      // sum_r G_rj X_ri as v_mfma_f64_16x16x4 k-steps over 4 rows at a time: an
      // fma chain over the rows in ascending order, which the oracle restates.
      // Lane l takes row 4s + (l >> 4) of k-step s and column (l & 15) + 16 t.
      hessian_mfma<NV>(md, d, ne);
      PT(23);
      PT(24);
      ldl_factor<NV>(d.nH, d.tmp, d.tmp2);
      PT(25);
    }
    PT(13);
    ldl_solve<NV>(d.nH, d.tmp2, d.ng, d.ndir);
    DOF_SLOTS(k, nv) d.ndir[k] = -d.ndir[k];
    wsync();
    {
#if MGS_REG_ROWS
      double dr[NV];
#pragma unroll
      for (int k = 0; k < NV; k++) dr[k] = d.ndir[k];
#else
      const double* dr = d.ndir;
#endif
      for (int r = lane; r < ne; r += WAVE) {
        const double* Gr = d.G + r * GS;
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < NV; k++) s = __builtin_fma(Gr[k], dr[k], s);
        d.efc_jv[r] = s;
      }
    }
    wsync();
    PT(14);
    DofV dl = dof_load(d.ndir, nv, lane), q;
#pragma unroll
    for (int h = 0; h < MGS_DPL; h++)
      q.v[h] = (lane + h * WAVE < nv) ? d.nw[lane + h * WAVE] - d.nw0[lane + h * WAVE] : 0.0;
    double A1 = dof_tree(dof_mul(q, dl), P);
    double A2 = dof_tree(dof_mul(dl, dl), P);
    double p0, q0, alpha = 0.0;
    LsRow LR;
    ls_row_load(md, d, lane, ne, mupR[0], k1R[0], LR);
    ls_eval_fast(md, d, ne, LR, 0.0, A1, A2, &p0, &q0, mupR, k1R);
    if (p0 < 0.0) {
      double lo = 0.0, hi = 0.0;
      int hi_ok = 0;
      alpha = -p0 / q0;
      for (int ls = 0; ls < md.m.ls_iterations; ls++) {
        double pp, qq;
        ls_eval_fast(md, d, ne, LR, alpha, A1, A2, &pp, &qq, mupR, k1R);
        if (fabs(pp) < md.m.ls_tolerance * (-p0)) break;
        if (pp < 0.0) lo = alpha;
        else { hi = alpha; hi_ok = 1; }
        double an = alpha - pp / qq;
        if (!(an > lo) || (hi_ok && !(an < hi))) an = hi_ok ? 0.5 * (lo + hi) : 2.0 * alpha;
        alpha = an;
      }
    }
    PT(15);
    if (!(alpha > 0.0)) { it++; break; }
#pragma unroll
    for (int h = 0; h < MGS_DPL; h++)
      if (lane + h * WAVE < nv) d.nw[lane + h * WAVE] = d.nw[lane + h * WAVE] + alpha * dl.v[h];
    wsync();
    double Cn = newton_eval<NV>(md, d, d.nw, P, mupR, k1R);
    newton_grad<NV>(md, d, d.nw);
    double improvement = scale * (C - Cn);
    C = Cn;
    DofV gl = dof_load(d.ng, nv, lane);
    double gn = scale * sqrt(dof_tree(dof_mul(gl, gl), P));
    PT(16);
    if (improvement < md.m.tolerance || gn < md.m.tolerance) { it++; break; }
  }
  if (lane == 0) d.ITERS += it;
  // forces to registers, u = G^T f
  load_frc(F, d.efc_f, ne, lane);
  u = dof_zero();
#pragma unroll
  for (int h = 0; h < MGS_DPL; h++) {
    const int i = lane + h * WAVE;
    if (i >= NV) continue;
    double s = 0.0;
    int r = 0;
    for (; r + 4 <= ne; r += 4) {
      double g0 = d.G[r * GS + i], g1 = d.G[(r + 1) * GS + i], g2 = d.G[(r + 2) * GS + i],
             g3 = d.G[(r + 3) * GS + i];
      double f0 = d.efc_f[r], f1 = d.efc_f[r + 1], f2 = d.efc_f[r + 2], f3 = d.efc_f[r + 3];
      s = __builtin_fma(g0, f0, s);
      s = __builtin_fma(g1, f1, s);
      s = __builtin_fma(g2, f2, s);
      s = __builtin_fma(g3, f3, s);
    }
    for (; r < ne; r++) s = __builtin_fma(d.G[r * GS + i], d.efc_f[r], s);
    u.v[h] = s;
  }
}

template <int NV>
DEVI void solve(const Mdl& md, Dat& d) {
  int nv = md.m.nv;
  // MuJoCo: scale = 1 / (m->stat.meaninertia * max(1, nv)), meaninertia being the
  // mean diagonal of M at qpos0 (mj_setConst), a model constant
  double scale = 1.0 / (md.m.meaninertia * (double)(nv > 1 ? nv : 1));
  Frc F;
  DofV u;
  if (md.m.solver == 0) {
    contact_blocks(md, d);
    solve_pgs(md, d, scale, F, u);
  } else {
    solve_newton<NV>(md, d, scale, F, u);
    if (md.m.noslip_iterations > 0) contact_blocks(md, d);   // overwrites the cone Hessians
  }
  PT(16);
  const DofV u_main = u;
  noslip(md, d, scale, F, u);
  PT(17);
  finalize_solution<NV>(md, d, u_main, u);
  PT(18);
}

// ---------------------------------------------------------------------------
// M survives the step in the unused tail of the G rows (rows >= nefc are never
// read), so integrate need not recompute it: the copy sits in the last nv*nv
// doubles of the G slot, clear of the dynamics-stage views that share U with G,
// and is valid while the step's rows stay below it.  The wide build (G in HBM)
// recomputes.
template <int NV>
DEVI double* m_copy_slot(const Mdl& md, const Dat& d) {
#ifdef MGS_G_GLOBAL
  return nullptr;
#else
  const int nv = md.m.nv;
  const int tail0 = md.m.nefc_max * GS - TRI_SIZE(NV);
  const int dyn_end = 6 * (3 * md.m.nbody + nv) + 3 * nv;
  return tail0 >= dyn_end ? d.G + tail0 : nullptr;
#endif
}
template <int NV>
DEVI void save_M(const Mdl& md, Dat& d) {
  double* mc = m_copy_slot<NV>(md, d);
  if (!mc) return;
  for (int k = lane_id(); k < TRI_SIZE(NV); k += WAVE) mc[k] = d.M[k];
  wsync();
}

// mj_forward up to the constraint rows (everything before the solver): a
// candidate whose contacts / rows overflow here still holds the state entering
// the step (qpos, qvel, qacc_warmstart, time change only in solve / integrate)
template <int NV>
DEVI void forward_rows(const Mdl& md, Dat& d) {
  int nv = md.m.nv, lane = lane_id();
  kinematics(md, d);
  com_pos(md, d);
  collision(md, d);
  crb(md, d);
  save_M<NV>(md, d);
  ldl_factor<NV>(d.M, d.Dv, d.Dinv);
  for (int k = lane; k < nv; k += WAVE) {
    double sd = sqrt(d.Dv[k]);
    d.sD[k] = sd;
    d.isD[k] = 1.0 / sd;
  }
  actuation(md, d);
  passive(md, d);
  rne(md, d);
#pragma unroll
  for (int h = 0; h < MGS_DPL; h++) {
    const int i = lane + h * WAVE;
    if (i < nv) d.qfrc_smooth[i] = (d.qfrc_passive[i] - d.qfrc_bias[i]) + d.qfrc_actuator[i];
  }
  wsync();
  ldl_solve<NV>(d.M, d.Dinv, d.qfrc_smooth, d.qacc_smooth);
  make_constraints<NV>(md, d);
}

template <int NV>
DEVI void forward(const Mdl& md, Dat& d, int full) {
  if (!full) {
    kinematics(md, d);
    com_pos(md, d);
    collision(md, d, 0);
    return;
  }
  forward_rows<NV>(md, d);
  solve<NV>(md, d);
}

template <int NV>
DEVI void integrate(const Mdl& md, Dat& d) {
  int nv = md.m.nv, lane = lane_id();
  double dt = md.m.timestep;
  // M (factored in place by forward): from its copy in the G tail when the
  // step's rows left it intact, else recomputed; then MI = M - dt*qDeriv
  {
    const double* mc = m_copy_slot<NV>(md, d);
    if (mc && uni(d.NEFC) * GS <= (int)(mc - d.G)) {
      for (int k = lane; k < TRI_SIZE(NV); k += WAVE) d.M[k] = mc[k];
      wsync();
    } else {
      crb(md, d);
    }
  }
  PT(19);
  // M - dt * qDeriv, lane i forms row i of qDeriv (-damping on the diagonal,
  // then each active affine actuator's mom_i (mom_j dv) in actuator order) and
  // applies it straight to M (the oracle's element expressions); with two
  // dofs per lane, row lane then row lane + 64
#pragma unroll
  for (int h = 0; h < MGS_DPL; h++) {
    const int i = lane + h * WAVE;   // this slot's row
    if (i >= nv) continue;
    const double* damp = DA(md, dof_damping);
    const int32_t *gtype = IA(md, actuator_gaintype), *btype = IA(md, actuator_biastype);
    const int32_t* flim = IA(md, actuator_forcelimited);
    const double *gain = DA(md, actuator_gainprm), *bias = DA(md, actuator_biasprm);
    const double* frange = DA(md, actuator_forcerange);
    double q[NV];
#pragma unroll
    for (int j = 0; j < NV; j++) q[j] = (j == i) ? -damp[i] : 0.0;
    for (int u = 0; u < md.m.nu; u++) {
      double f = d.act_force[u];
      if (flim[u] && (f <= frange[2 * u] || f >= frange[2 * u + 1])) continue;
      double dv = 0.0;
      if (btype[u] == MGS_BIAS_AFFINE) dv = dv + bias[3 * u + 2];
      if (gtype[u] == MGS_GAIN_AFFINE) dv = dv + gain[3 * u + 2] * d.ctrl[u];
      if (dv == 0.0) continue;
#if MGS_PACKED
      const double* mom = DA(md, actuator_moment) + u * nv;
#else
      const double* mom = d.act_moment + u * nv;
#endif
      double mi = mom[i];
      if (mi == 0.0) continue;
#pragma unroll
      for (int j = 0; j < NV; j++) q[j] = q[j] + mi * (mom[j] * dv);
    }
#pragma unroll
    for (int j = 0; j < NV; j++)
      if (!MGS_PACKED || j <= i) d.M[TRI(i, j, NV)] = d.M[TRI(i, j, NV)] - dt * q[j];
  }
  wsync();
  PT(20);
  ldl_factor<NV>(d.M, d.Dv, d.Dinv);
  double* qa = d.scratch;
  for (int k = lane; k < nv; k += WAVE) qa[k] = d.qfrc_smooth[k] + d.qfrc_constraint[k];
  wsync();
  ldl_solve<NV>(d.M, d.Dinv, qa, qa);
  // qvel per dof, then qpos per joint (lanes over joints: their qpos ranges
  // are disjoint, each lane runs the oracle's per-joint expressions)
  for (int k = lane; k < nv; k += WAVE) d.qvel[k] = d.qvel[k] + dt * qa[k];
  wsync();
  {
    const int32_t *jtype = IA(md, jnt_type), *jq = IA(md, jnt_qposadr), *jd = IA(md, jnt_dofadr);
    for (int j = lane; j < md.m.njnt; j += WAVE) {
      int a = jq[j], v = jd[j];
      if (jtype[j] == MGS_JNT_FREE) {
        d.qpos[a] = d.qpos[a] + dt * d.qvel[v];
        d.qpos[a + 1] = d.qpos[a + 1] + dt * d.qvel[v + 1];
        d.qpos[a + 2] = d.qpos[a + 2] + dt * d.qvel[v + 2];
        double ax[3] = {d.qvel[v + 3], d.qvel[v + 4], d.qvel[v + 5]};
        double nrm = normalize3(ax);
        double qr[4], qn[4];
        axisangle2quat(qr, ax, dt * nrm);
        quatmul(qn, d.qpos + a + 3, qr);
        normalize4(qn);
        d.qpos[a + 3] = qn[0]; d.qpos[a + 4] = qn[1]; d.qpos[a + 5] = qn[2]; d.qpos[a + 6] = qn[3];
      } else {
        d.qpos[a] = d.qpos[a] + dt * d.qvel[v];
      }
    }
    if (lane == 0) d.time[0] = d.time[0] + dt;
  }
  // actuator state (mj_advance: act += dt act_dot; a mujoco.pid integral then
  // clamped to |ki integral| <= imax), lanes over actuators
  if (md.m.nact > 0) {
    const int32_t *gtype = IA(md, actuator_gaintype), *aadr = IA(md, actuator_actadr);
    const double* pid = DA(md, actuator_pidprm);
    for (int u = lane; u < md.m.nu; u += WAVE) {
      if (gtype[u] != MGS_GAIN_PID) continue;
      const double* pp = pid + 5 * u;
      int k = aadr[u];
      if (pp[4] >= 0.0) {
        d.act[k] = d.act[k] + dt * d.act_dot[k];
        k++;
      }
      if (pp[1] != 0.0) {
        double v = d.act[k] + dt * d.act_dot[k];
        if (pp[3] >= 0.0) {
          const double lim = pp[3] / fabs(pp[1]);
          if (v < -lim) v = -lim;
          if (v > lim) v = lim;
        }
        d.act[k] = v;
      }
    }
  }
  wsync();
}

DEVI int obj_contact(const Mdl& md, const Dat& d) {
  const int32_t* side = IA(md, geom_side);
  int ncon = uni(d.NCON);
  for (int c = 0; c < ncon; c++) {
    int s1 = side[d.con_g1[c]], s2 = side[d.con_g2[c]];
    if ((s1 < 0 && s2 > 0) || (s1 > 0 && s2 < 0)) return 1;
  }
  return 0;
}

// clutter collision predicate: a gripper geom against the table or any geom past it
DEVI int obj_contact_incl(const Mdl& md, const Dat& d) {
  const int32_t* side = IA(md, geom_side);
  int ncon = uni(d.NCON);
  for (int c = 0; c < ncon; c++) {
    int s1 = side[d.con_g1[c]], s2 = side[d.con_g2[c]];
    if ((s1 < 0 && s2 >= 0) || (s1 >= 0 && s2 < 0)) return 1;
  }
  return 0;
}

DEVI void reset(const Mdl& md, Dat& d, const double* qpos_init, const double* mpos, const double* mquat,
                const double* vstate = nullptr) {
  int lane = lane_id();
  int nv = md.m.nv;
  const double* v0 = vstate ? vstate : DA(md, qvel0);
  const double* w0 = vstate ? vstate + nv : DA(md, qacc_ws0);
  for (int k = lane; k < md.m.nq; k += WAVE) d.qpos[k] = qpos_init[k];
  for (int k = lane; k < nv; k += WAVE) { d.qvel[k] = v0[k]; d.qacc_ws[k] = w0[k]; }
  for (int k = lane; k < md.m.nact; k += WAVE) {
    d.act[k] = vstate ? vstate[2 * nv + k] : DA(md, act0)[k];
    d.act_dot[k] = 0.0;
  }
  if (lane == 0) {
    for (int u = 0; u < (md.m.nu > 0 ? md.m.nu : 1); u++) d.ctrl[u] = 0.0;
    for (int k = 0; k < 3; k++) d.mocap_pos[k] = mpos ? mpos[k] : 0.0;
    for (int k = 0; k < 4; k++) d.mocap_quat[k] = mquat[k];
    d.time[0] = 0.0;
    for (int k = 0; k < 16; k++) d.ints[k] = 0;
  }
  if (lane < K_CERT) d.cert[CERT_W * lane] = -1.0;
  wsync();
}

// ---------------------------------------------------------------------------
// kernels: one 64-lane workgroup per candidate
// kernel bodies (mgs_collision_kernel / mgs_rollout_kernel below and the
// specialised entry points of mgs_special.hip)
template <int NV, int SL>
DEVI void collision_entry(double* smem, const Mdl& mdarg, const int32_t* __restrict__ mI,
                          const double* __restrict__ mD, const Lay& lay, int n, const double* __restrict__ qpos_init,
                          const double* __restrict__ mocap_pos, const double* __restrict__ mocap_quat,
                          int predicate, uint8_t* __restrict__ out) {
  Mdl md = mdarg;
  if constexpr (SL != 0) md.m = mgs_sl_desc;
  md.I = mI;
  md.D = mD;
  int i = blockIdx.x;
  if (i >= n) return;
  Dat d;
  bind<SL>(d, smem, lay);
  reset(md, d, qpos_init + (size_t)i * md.m.nq, mocap_pos + 3 * i, mocap_quat + 4 * i);
  forward<NV>(md, d, 0);
  if (lane_id() == 0) {
    int hit = (predicate == MGS_PRED_ANY_CONTACT) ? (d.NCON != 0)
              : (predicate == MGS_PRED_PARTITION_INCL) ? obj_contact_incl(md, d) : obj_contact(md, d);
    out[i] = (uint8_t)(hit ? 0 : 1);
  }
}

template <int NV, int SL = 0>
__global__ void __launch_bounds__(64)
mgs_collision_kernel(Mdl mdarg, const int32_t* __restrict__ mI, const double* __restrict__ mD, Lay lay, int n,
                     const double* __restrict__ qpos_init,
                     const double* __restrict__ mocap_pos, const double* __restrict__ mocap_quat, int predicate,
                     uint8_t* __restrict__ out) {
  extern __shared__ double smem[];
  collision_entry<NV, SL>(smem, mdarg, mI, mD, lay, n, qpos_init, mocap_pos, mocap_quat, predicate, out);
}

// a candidate's resume record: the state entering step (p, t) -- qpos, qvel,
// qacc_warmstart, time -- the schedule position and the partial stats
// (mgs_rollout_out.resume)
DEVI void save_record(const Mdl& md, Dat& d, double* rec, int p, int t, int gstep, int maxcon, int maxefc,
                      int sumcon, int sumefc) {
  const int lane = lane_id(), nq = md.m.nq, nvr = md.m.nv;
  for (int k = lane; k < nq; k += WAVE) rec[k] = d.qpos[k];
  for (int k = lane; k < nvr; k += WAVE) { rec[nq + k] = d.qvel[k]; rec[nq + nvr + k] = d.qacc_ws[k]; }
  for (int k = lane; k < md.m.nact; k += WAVE) rec[nq + 2 * nvr + k] = d.act[k];
  if (lane == 0) {
    double* tail = rec + nq + 2 * nvr + md.m.nact;
    tail[0] = d.time[0];
    tail[1] = p; tail[2] = t; tail[3] = gstep;
    tail[4] = maxcon; tail[5] = maxefc; tail[6] = sumcon; tail[7] = sumefc;
    tail[8] = d.ITERS;
    tail[9] = d.OVERFLOW;
  }
}

// ---------------------------------------------------------------------------
// In-launch rotation (ABI 19).  A work-queue launch whose schedule sets
// yield_every keeps, next to its candidate counter, a ring of yielded
// candidates: every yield_every steps a candidate checks whether anyone is
// waiting (a candidate not started yet, or one in the ring); if so it writes
// its resume record, appends itself to the ring and its workgroup takes the
// next un-started candidate, else the ring's oldest.  So a launch with more
// rollouts than slots runs them round robin and ends about one slice after
// the last one finishes, instead of one whole rollout after the last one
// started.  No workgroup ever waits for another's candidate: the only waits
// are for a ring slot between a producer's two atomics (tail, then the slot),
// a few instructions of a running wave.  Queue header (MGS_QHDR words): [0]
// next candidate, [1] exits, [2] ring head, [3] ring tail, [4..5] the ring's
// address (set by the host when it allocates the rings; MGS_QRING_F(n) words,
// candidate + 1, 0 = empty), [6] yields and [7] expired spins, both
// cumulative over the batch's launches (mgs_queue_stats).  An expired spin
// -- a protocol error, never seen -- keeps the candidate on its workgroup
// (push side) or loses the slot's candidate (pop side).  A lost candidate is
// never silent (ABI 20): a yielding candidate marks its outputs with the
// MGS_FAIL_YIELDED sentinel before it joins the ring (its continuation
// overwrites them), and the host entries compare word 7 after every launch
// and fail with MGS_EQUEUE when it grew.  The ring holds MGS_QRING_F(n)
// words for the launch's n (the host sizes the rings for the largest n it
// launched, so a ring slot index never leaves its allocation).  [8..9] /
// [10..11]: the launch's start / end on the 100 MHz real-time counter (the
// workgroup that takes candidate 0 / the last one to leave; mgs_queue_spans).
#define MGS_QHDR 12
#define MGS_QRING_F(n) (2u * (uint32_t)(n))
#ifndef MGS_SPIN_MAX
#define MGS_SPIN_MAX (1u << 22)
#endif

DEVI uint32_t* ring_of(const uint32_t* q) { return (uint32_t*)((const uint64_t*)q)[2]; }

// is any candidate waiting for a slot (un-started, or yielded to the ring)?
DEVI int queue_waiting(const uint32_t* q, int n) {
  uint32_t w = 0;
  if (lane_id() == 0) {
    uint32_t nx = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t h = __hip_atomic_load(q + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t t = __hip_atomic_load(q + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    w = (nx < (uint32_t)n) || (h < t);
  }
  return (int)__builtin_amdgcn_readfirstlane(w);
}

// append candidate i (its record already written by the whole wave) to the
// ring; 0 if the slot never emptied (then the caller keeps the candidate)
DEVI int ring_push(uint32_t* q, int n, int i) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");   // every lane's record stores
  wsync();
  uint32_t ok = 0;
  if (lane_id() == 0) {
    const uint32_t F = MGS_QRING_F(n);
    uint32_t t = __hip_atomic_fetch_add(q + 3, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t* slot = ring_of(q) + (t % F);
    for (uint32_t it = 0; it < MGS_SPIN_MAX; it++) {
      uint32_t z = 0;
      if (__hip_atomic_compare_exchange_strong(slot, &z, (uint32_t)i + 1u, __ATOMIC_RELEASE, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_AGENT)) {
        ok = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(4);
    }
    if (ok) __hip_atomic_fetch_add(q + 6, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else __hip_atomic_fetch_add(q + 7, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  return (int)__builtin_amdgcn_readfirstlane(ok);
}

// the ring's oldest candidate, or -1 if the ring is empty
DEVI int ring_pop(uint32_t* q, int n) {
  int c = -1;
  if (lane_id() == 0) {
    const uint32_t F = MGS_QRING_F(n);
    for (;;) {
      uint32_t h = __hip_atomic_load(q + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      uint32_t t = __hip_atomic_load(q + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (h >= t) break;
      if (!__hip_atomic_compare_exchange_strong(q + 2, &h, h + 1u, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT))
        continue;
      uint32_t* slot = ring_of(q) + (h % F);
      for (uint32_t it = 0; it < MGS_SPIN_MAX; it++) {
        uint32_t v = __hip_atomic_exchange(slot, 0u, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
        if (v) { c = (int)(v - 1u); break; }
        __builtin_amdgcn_s_sleep(4);
      }
#ifdef MGS_TEST_DROP_POP
      c = -1;     // fault injection (tests only): every pop expires and loses its candidate
#endif
      if (c < 0) __hip_atomic_fetch_add(q + 7, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
  }
  c = (int)__builtin_amdgcn_readfirstlane(c);
  if (c >= 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // the record, for every lane
  return c;
}

// one candidate's rollout (the body of mgs_rollout_kernel)
template <int NV, int SL>
DEVI void rollout_one(const Mdl& md, double* smem, const Lay& lay, const mgs_schedule& sc, int i,
                      const double* __restrict__ qpos_init, const double* __restrict__ mocap_quat,
                      const double* __restrict__ phase_start, const double* __restrict__ phase_target,
                      const uint8_t* __restrict__ active, uint8_t* __restrict__ label,
                      int32_t* __restrict__ fail_step, double* __restrict__ obj_qpos, int32_t* __restrict__ stats,
                      const double* __restrict__ vstate_init, double* __restrict__ state_out,
                      double* resume_out, const double* resume_in, const double* __restrict__ mask_mpos,
                      int mask_pred, uint8_t* __restrict__ mask_out, int32_t* ovf_count, int32_t* ovf_list,
                      uint32_t* yq = nullptr, int n = 0, int from_ring = 0) {
  int lane = lane_id();
  if (from_ring) {
    // a candidate that yielded earlier in this launch: accepted, and its
    // record (in resume_out) holds the state to continue from
    active = nullptr;
    mask_out = nullptr;
    resume_in = resume_out;
  }
  int reject = active && !active[i];
  if (mask_out) {
    // fused collision mask (mgs_mask_rollout_device): collision_entry's
    // computation for this candidate, then the rollout of the collision-free
    // ones in the same workgroup -- no separate mask launch to wait for
    Dat d0;
    bind<SL>(d0, smem, lay);
    reset(md, d0, qpos_init + (size_t)i * md.m.nq, mask_mpos + 3 * i, mocap_quat + 4 * i);
    forward<NV>(md, d0, 0);
    int hit = (mask_pred == MGS_PRED_ANY_CONTACT) ? (uni(d0.NCON) != 0)
              : (mask_pred == MGS_PRED_PARTITION_INCL) ? obj_contact_incl(md, d0) : obj_contact(md, d0);
    if (lane == 0) mask_out[i] = (uint8_t)(hit ? 0 : 1);
    wsync();
    reject = hit;
  }
  if (reject) {
    // collision-mask reject: not simulated (filter_to_stable.py:39-44)
    if (lane == 0) {
      label[i] = 0;
      if (fail_step) fail_step[i] = -2;
      if (stats)
        for (int k = 0; k < MGS_NSTATS; k++) stats[MGS_NSTATS * i + k] = 0;
    }
    // no object joint reported (obj_qposadr < 0): zeros, as the oracle's output
    if (obj_qpos && lane < 7)
      obj_qpos[7 * i + lane] = sc.obj_qposadr >= 0 ? qpos_init[(size_t)i * md.m.nq + sc.obj_qposadr + lane] : 0.0;
    return;
  }
  Dat d;
  bind<SL>(d, smem, lay);
  int np = sc.nphase;
  const double* ps = phase_start + (size_t)i * np * 3;
  const double* pt = phase_target + (size_t)i * np * 3;
  reset(md, d, qpos_init + (size_t)i * md.m.nq, ps, mocap_quat + 4 * i,
        vstate_init ? vstate_init + (size_t)i * (2 * md.m.nv + md.m.nact) : nullptr);
  int ok = 1, gstep = 0, fstep = -1, maxcon = 0, maxefc = 0, sumcon = 0, sumefc = 0;
  const int nq = md.m.nq, nvr = md.m.nv, RS = nq + 2 * nvr + md.m.nact + MGS_RESUME_EXTRA;
  int p0 = 0, t0 = 0;
  if (resume_in) {
    // continue a capacity-capped run from its last step before the overflow
    // (the capped run and a wider one are identical up to that step)
    const double* rec = resume_in + (size_t)i * RS;
    for (int k = lane; k < nq; k += WAVE) d.qpos[k] = rec[k];
    for (int k = lane; k < nvr; k += WAVE) { d.qvel[k] = rec[nq + k]; d.qacc_ws[k] = rec[nq + nvr + k]; }
    for (int k = lane; k < md.m.nact; k += WAVE) d.act[k] = rec[nq + 2 * nvr + k];
    const double* tail = rec + nq + 2 * nvr + md.m.nact;
    if (lane == 0) {
      d.time[0] = tail[0];
      d.ITERS = (int)tail[8];
      // a yielded candidate keeps its flags, a paused one (time slice by
      // relaunch) keeps them without the pause (a capacity flag of a capped
      // run that paused stays, as in one launch); a capacity escalation starts
      // the continued run's flags afresh (the wider run is not capped there)
      const int fl = (int)tail[9];
      if (from_ring) d.OVERFLOW = fl;
      else if (fl & MGS_FLAG_PAUSED) d.OVERFLOW = fl & ~MGS_FLAG_PAUSED;
    }
    p0 = (int)tail[1]; t0 = (int)tail[2]; gstep = (int)tail[3];
    maxcon = (int)tail[4]; maxefc = (int)tail[5]; sumcon = (int)tail[6]; sumefc = (int)tail[7];
    wsync();
  }
  PROF_DECL
  int since = 0;     // steps run since this candidate (re)started in this launch
  for (int p = p0; p < np && ok; p++) {
    if (lane == 0)
      for (int u = 0; u < md.m.nu; u++) d.ctrl[u] = sc.ctrl[p * 32 + u];
    int ns = sc.nsteps[p];
    for (int t = (p == p0 ? t0 : 0); t < ns && ok; t++) {
      if (yq && since >= sc.yield_every) {
        // in-launch rotation (ABI 19): the state entering this step goes to the
        // record and the candidate to the ring if anyone waits for a slot
        since = 0;
        if (queue_waiting(yq, n)) {
          save_record(md, d, resume_out + (size_t)i * RS, p, t, gstep, maxcon, maxefc, sumcon, sumefc);
          // the sentinel a lost candidate would keep (its continuation, ordered
          // after the push's release, overwrites it)
          if (lane == 0) {
            label[i] = 0;
            if (fail_step) fail_step[i] = MGS_FAIL_YIELDED;
          }
          if (ring_push(yq, n, i)) {
            ok = 0;
            fstep = -5;
            break;
          }
        }
      }
      since++;
      if (sc.pause_step > 0 && gstep >= sc.pause_step && resume_out) {
        // time slice (ABI 18): the state entering this step, the schedule
        // position and the partial stats go to the resume record, exactly as
        // for a capacity stop, and a later launch continues from there
        // (the record carries the pause flag: its relaunch keeps the flags)
        if (lane == 0) d.OVERFLOW |= MGS_FLAG_PAUSED;
        wsync();
        save_record(md, d, resume_out + (size_t)i * RS, p, t, gstep, maxcon, maxefc, sumcon, sumefc);
        ok = 0;
        fstep = -4;
        break;
      }
      double frac = (double)t / (double)ns;
      if (lane == 0)
        for (int k = 0; k < 3; k++) d.mocap_pos[k] = ps[3 * p + k] + (pt[3 * p + k] - ps[3 * p + k]) * frac;
      wsync();
#ifdef MGS_PROFILE
      PT(0);
      kinematics(md, d);
      wsync(); PT(1);
      com_pos(md, d);
      wsync(); PT(2);
      collision(md, d); PT(5);
      crb(md, d); PT(6);
      save_M<NV>(md, d);
      ldl_factor<NV>(d.M, d.Dv, d.Dinv);
      for (int k = lane; k < md.m.nv; k += WAVE) { double sd = sqrt(d.Dv[k]); d.sD[k] = sd; d.isD[k] = 1.0 / sd; }
      wsync(); PT(7);
      actuation(md, d);
      wsync(); PT(33);
      passive(md, d);
      wsync(); PT(34);
      rne(md, d);
      PT(35);
#pragma unroll
      for (int h = 0; h < MGS_DPL; h++) {
        const int i = lane + h * WAVE;
        if (i < md.m.nv) d.qfrc_smooth[i] = (d.qfrc_passive[i] - d.qfrc_bias[i]) + d.qfrc_actuator[i];
      }
      wsync();
      ldl_solve<NV>(d.M, d.Dinv, d.qfrc_smooth, d.qacc_smooth);
      PT(8);
      make_constraints<NV>(md, d);
#else
      forward_rows<NV>(md, d);
#endif
      if (resume_out && !sc.capped_continue && (uni(d.OVERFLOW) & MGS_FLAG_CAPACITY)) {
        // capacity exceeded in this step (contacts in collision, rows in
        // make_constraints, both before anything of the state moved): the
        // state entering the step, the schedule position and the partial stats
        // go to the candidate's resume record and the candidate stops (the
        // escalation continues it from here with more capacity)
        save_record(md, d, resume_out + (size_t)i * RS, p, t, gstep, maxcon, maxefc, sumcon, sumefc);
        ok = 0;
        fstep = -3;
        break;
      }
      solve<NV>(md, d);
      integrate<NV>(md, d);
#ifdef MGS_PROFILE
      PT(21);
#endif
      if (uni(d.NCON) > maxcon) maxcon = uni(d.NCON);
      if (uni(d.NEFC) > maxefc) maxefc = uni(d.NEFC);
      sumcon += uni(d.NCON);
      sumefc += uni(d.NEFC);
      // divergence guard (MuJoCo's mj_checkPos / mj_checkVel / mj_checkAcc flag a
      // NaN or |x| > mjMAXVAL and reset the data): the candidate stops here,
      // label 0, flagged in stats[2]
      {
        int bad = 0;
        for (int k = lane; k < md.m.nq; k += WAVE) bad |= !(fabs(d.qpos[k]) <= MGS_MAXVAL);
        for (int k = lane; k < md.m.nv; k += WAVE)
          bad |= !(fabs(d.qvel[k]) <= MGS_MAXVAL) || !(fabs(d.qacc_ws[k]) <= MGS_MAXVAL);
        if (__ballot(bad)) {
          ok = 0;
          fstep = gstep;
          if (lane == 0) d.OVERFLOW |= MGS_FLAG_DIVERGED;
          wsync();
          break;
        }
      }
      int ce = sc.check_every[p];
      if (sc.vclip > 0.0) {
        for (int k = lane; k < md.m.nv; k += WAVE) {
          double v = d.qvel[k];
          if (v > sc.vclip) v = sc.vclip;
          if (v < -sc.vclip) v = -sc.vclip;
          d.qvel[k] = v;
        }
        wsync();
      }
      int tc = t + sc.check_offset[p];
      if (ce > 0 && tc > 0 && (tc % ce) == 0 && !obj_contact(md, d)) { ok = 0; fstep = gstep; }
      gstep++;
    }
    if (ok && sc.check_at_end[p] && !obj_contact(md, d)) { ok = 0; fstep = gstep - 1; }
    if (fstep <= -3) break;
  }
  if (fstep == -5) {   // yielded: another workgroup of this launch continues it
    PROF_FLUSH
    return;
  }
  if (lane == 0) {
    label[i] = (uint8_t)ok;
    if (fail_step) fail_step[i] = fstep;
    if (stats) {
      int32_t* st = stats + MGS_NSTATS * i;
      st[0] = maxcon; st[1] = maxefc; st[2] = d.OVERFLOW; st[3] = d.ITERS; st[4] = sumcon; st[5] = sumefc;
    }
    // the launch's overflow list (ABI 17): a capacity-capped candidate appends
    // itself, so the escalation re-run needs no list kernel (nor a fill of its
    // count) between this launch and the next one on the stream
    if (ovf_list && (d.OVERFLOW & MGS_FLAG_CAPACITY)) ovf_list[atomicAdd(ovf_count, 1)] = i;
  }
  if (obj_qpos && lane < 7) obj_qpos[7 * i + lane] = sc.obj_qposadr >= 0 ? d.qpos[sc.obj_qposadr + lane] : 0.0;
  if (state_out) {
    int nq = md.m.nq, nv = md.m.nv;
    double* so = state_out + (size_t)i * (nq + 2 * nv + md.m.nact);
    for (int k = lane; k < nq; k += WAVE) so[k] = d.qpos[k];
    for (int k = lane; k < nv; k += WAVE) { so[nq + k] = d.qvel[k]; so[nq + nv + k] = d.qacc_ws[k]; }
    for (int k = lane; k < md.m.nact; k += WAVE) so[nq + 2 * nv + k] = d.act[k];
  }
  PROF_FLUSH
}

// One workgroup (one wave) per candidate: candidate blockIdx.x, or -- list mode
// (list != nullptr) -- candidates list[s] for s = blockIdx.x, blockIdx.x +
// gridDim.x, ... < *list_count: a small grid re-runs a device-built subset
// (capacity escalation) without launching a workgroup per batch entry.
#ifdef MGS_WAVES_PER_EU
#define MGS_ROLL_ATTR __attribute__((amdgpu_waves_per_eu(MGS_WAVES_PER_EU)))
#else
#define MGS_ROLL_ATTR
#endif
template <int NV, int SL>
DEVI void rollout_entry(double* smem, const Mdl& mdarg, const int32_t* __restrict__ mI,
                        const double* __restrict__ mD, const Lay& lay, const mgs_schedule& sc, int n,
                        const double* __restrict__ qpos_init, const double* __restrict__ mocap_quat,
                        const double* __restrict__ phase_start, const double* __restrict__ phase_target,
                        const uint8_t* __restrict__ active, uint8_t* __restrict__ label,
                        int32_t* __restrict__ fail_step, double* __restrict__ obj_qpos, int32_t* __restrict__ stats,
                        const double* __restrict__ vstate_init, double* __restrict__ state_out,
                        const int32_t* __restrict__ list, int32_t* list_count,
                        double* resume_out, const double* resume_in, const double* __restrict__ mask_mpos,
                        int mask_pred, uint8_t* __restrict__ mask_out, uint32_t* queue, int32_t* ovf_count,
                        int32_t* ovf_list) {
  Mdl md = mdarg;
  // SL: the model description is the baked one too, so sizes, table offsets and
  // options are compile-time constants (trip counts, immediate offsets)
  if constexpr (SL != 0) md.m = mgs_sl_desc;
  md.I = mI;
  md.D = mD;
  if (queue) {
    // work queue (queue != nullptr): the grid is the device's resident capacity
    // and each workgroup takes the next candidate index when its previous one
    // ends, so short (rejected, early-failing) and long rollouts pack the slots
    // regardless of which XCD a workgroup landed on; the launch has a single
    // tail.  queue[0] is the next index, queue[1] counts the workgroups that
    // have made their one failing pop: the last of them returns both words to
    // zero (every pop of this launch is behind it), so each launch on this slot
    // starts from zero with no fill kernel and no host-tracked base (ABI 17)
    // rotation (sc.yield_every > 0 with resume records): un-started candidates
    // first, then the ring of yielded ones; a workgroup leaves when both are
    // empty (a candidate pushed later is taken by its pusher's own next pop)
    uint32_t* yq = (sc.yield_every > 0 && resume_out && ring_of(queue)) ? queue : nullptr;
    int fresh = 1;
    for (;;) {
      int s = -1, ring = 0;
      if (fresh) {
        uint32_t t = 0;
        if (lane_id() == 0) t = __hip_atomic_fetch_add(queue, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t u = __builtin_amdgcn_readfirstlane(t);
        if (u < (uint32_t)n) s = (int)u;
        else fresh = 0;
        if (u == 0 && lane_id() == 0)
          __hip_atomic_store((unsigned long long*)(queue + 8), (unsigned long long)__builtin_amdgcn_s_memrealtime(),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (s < 0 && yq) {
        s = ring_pop(yq, n);
        ring = 1;
      }
      if (s < 0) break;
      rollout_one<NV, SL>(md, smem, lay, sc, s, qpos_init, mocap_quat, phase_start, phase_target, active, label,
                          fail_step, obj_qpos, stats, vstate_init, state_out, resume_out, resume_in, mask_mpos,
                          mask_pred, mask_out, ovf_count, ovf_list, yq, n, ring);
    }
    if (lane_id() == 0 &&
        __hip_atomic_fetch_add(queue + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1) {
      __hip_atomic_store((unsigned long long*)(queue + 10), (unsigned long long)__builtin_amdgcn_s_memrealtime(),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(queue, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(queue + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(queue + 3, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(queue + 1, 0u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  const int end = list ? list_count[0] : (blockIdx.x < (unsigned)n ? (int)blockIdx.x + 1 : 0);
  const int stride = list ? (int)gridDim.x : 1;
  for (int s = blockIdx.x; s < end; s += stride) {
    int i = list ? list[s] : s;
    if (i < 0 || i >= n) continue;
    rollout_one<NV, SL>(md, smem, lay, sc, i, qpos_init, mocap_quat, phase_start, phase_target, active, label,
                    fail_step, obj_qpos, stats, vstate_init, state_out, resume_out, resume_in, mask_mpos,
                    mask_pred, mask_out, ovf_count, ovf_list);
  }
  if (list && lane_id() == 0 &&
      __hip_atomic_fetch_add(list_count + 1, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == (int)gridDim.x - 1) {
    // list header (MGS_LIST_HEADER words: count, exits, consumed): the last
    // workgroup out records the count it ran and leaves the header zeroed for
    // the next launch that appends to it
    __hip_atomic_store(list_count + 2, list_count[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(list_count, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(list_count + 1, 0, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// resume_out / resume_in may be the same buffer (mgs_rollout_resume continues a
// capped run's records in place): not __restrict__; each candidate's record is
// read into LDS before its own record is rewritten
template <int NV, int SL = 0>
__global__ void __launch_bounds__(64) MGS_ROLL_ATTR
mgs_rollout_kernel(Mdl mdarg, const int32_t* __restrict__ mI, const double* __restrict__ mD, Lay lay,
                   mgs_schedule sc, int n, const double* __restrict__ qpos_init,
                   const double* __restrict__ mocap_quat, const double* __restrict__ phase_start,
                   const double* __restrict__ phase_target, const uint8_t* __restrict__ active,
                   uint8_t* __restrict__ label, int32_t* __restrict__ fail_step, double* __restrict__ obj_qpos,
                   int32_t* __restrict__ stats, const double* __restrict__ vstate_init,
                   double* __restrict__ state_out, const int32_t* __restrict__ list,
                   int32_t* list_count, double* resume_out, const double* resume_in,
                   const double* __restrict__ mask_mpos, int mask_pred, uint8_t* __restrict__ mask_out,
                   uint32_t* queue, int32_t* ovf_count, int32_t* ovf_list) {
  extern __shared__ double smem[];
  rollout_entry<NV, SL>(smem, mdarg, mI, mD, lay, sc, n, qpos_init, mocap_quat, phase_start, phase_target, active,
                        label, fail_step, obj_qpos, stats, vstate_init, state_out, list, list_count, resume_out,
                        resume_in, mask_mpos, mask_pred, mask_out, queue, ovf_count, ovf_list);
}

// the library's non-template kernels live in the C-ABI translation unit only
// (the per-dof-count units and specialised code objects define MGS_TEMPLATES_ONLY)
#ifndef MGS_TEMPLATES_ONLY
// capacity-escalation list: indices of the candidates whose stats flags meet
// mask (order of arrival; each re-run is independent of the order)
__global__ void __launch_bounds__(256)
mgs_overflow_list_kernel(const int32_t* __restrict__ stats, int n, int mask, int32_t* __restrict__ count,
                         int32_t* __restrict__ list) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && (stats[MGS_NSTATS * i + 2] & mask)) list[atomicAdd(count, 1)] = i;
}

// device-side arithmetic probe (tests): sqrt, division, sincos against the oracle
extern "C" __global__ void mgs_arith_probe_kernel(const double* x, const double* y, int n, double* out) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double s, c;
  k_sincos(x[i], &s, &c);
  out[4 * i] = sqrt(fabs(x[i]));
  out[4 * i + 1] = x[i] / y[i];
  out[4 * i + 2] = s;
  out[4 * i + 3] = c;
}

// tree-reduction probe (tests): out[b] = tree_sum over lanes of a[b*64+l]*c[b*64+l] with P = nextpow2(n)
extern "C" __global__ void __launch_bounds__(64) mgs_tree_probe_kernel(const double* a, const double* c, int n,
                                                                         double* out) {
  int l = lane_id();
  int b = blockIdx.x;
  double leaf = (l < n) ? a[b * 64 + l] * c[b * 64 + l] : 0.0;
  double s = tree_sum(leaf, next_pow2(n));
  if (l == 0) out[b] = s;
}
#endif  // MGS_TEMPLATES_ONLY
