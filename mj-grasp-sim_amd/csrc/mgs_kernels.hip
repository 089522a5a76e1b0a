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
#define K_MPR_MAXIT 64
#define K_FEAT_EPS 1e-5
#define WAVE 64

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

// per-candidate working set in LDS
struct Dat {
  double *qpos, *qvel, *qacc_ws, *ctrl, *mocap_pos, *mocap_quat, *time;
  double *xpos, *xquat, *xmat, *xipos, *ximat, *xanchor, *xaxis;
  double *subtree_com, *subtree_mass, *cinert, *crb, *cdof, *cdof_dot, *cvel, *cacc, *cfrc;
  double *geom_xpos, *geom_xmat;
  double *M, *L, *Dv, *Dinv, *qDeriv;
  double *qfrc_bias, *qfrc_passive, *qfrc_actuator, *qfrc_smooth, *qacc_smooth, *qfrc_constraint, *qacc;
  double *act_force, *act_moment, *act_length, *act_vel;
  double *con_pos, *con_frame, *con_dist;
  double *J, *K, *efc_pos, *efc_margin, *efc_vel, *efc_aref, *efc_R, *efc_A, *efc_b, *efc_f, *efc_mu, *efc_blk,
      *efc_floss;
  double *w, *jac, *scratch;
  int *con_pair, *con_g1, *con_g2, *efc_type, *efc_dim, *efc_con, *ints;
  P2* poly;   // 3 * K_MAXPOLY
};
// ints[]: 0 ncon, 1 nefc, 2 overflow, 3 iters, 4 maxcon, 5 maxefc, 6 cr0, 7 cr1, 8 neq rows, 9 fr0, 10 fr1,
//         11 lr0, 12 lr1
#define NCON ints[0]
#define NEFC ints[1]
#define OVERFLOW ints[2]
#define ITERS ints[3]

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }
__device__ __forceinline__ void wsync() { __syncthreads(); }

// ---------------------------------------------------------------------------
// math primitives: identical expressions to the oracle
__device__ void k_sincos(double x, double* s, double* c) {
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

__device__ __forceinline__ double dot3(const double* a, const double* b) {
  return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2];
}
__device__ __forceinline__ void cross3(double* r, const double* a, const double* b) {
  double r0 = a[1] * b[2] - a[2] * b[1];
  double r1 = a[2] * b[0] - a[0] * b[2];
  double r2 = a[0] * b[1] - a[1] * b[0];
  r[0] = r0; r[1] = r1; r[2] = r2;
}
__device__ __forceinline__ void sub3(double* r, const double* a, const double* b) {
  r[0] = a[0] - b[0]; r[1] = a[1] - b[1]; r[2] = a[2] - b[2];
}
__device__ __forceinline__ void add3(double* r, const double* a, const double* b) {
  r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2];
}
__device__ __forceinline__ void mulmv3(double* r, const double* m, const double* v) {
  double r0 = (m[0] * v[0] + m[1] * v[1]) + m[2] * v[2];
  double r1 = (m[3] * v[0] + m[4] * v[1]) + m[5] * v[2];
  double r2 = (m[6] * v[0] + m[7] * v[1]) + m[8] * v[2];
  r[0] = r0; r[1] = r1; r[2] = r2;
}
__device__ __forceinline__ void mulmtv3(double* r, const double* m, const double* v) {
  double r0 = (m[0] * v[0] + m[3] * v[1]) + m[6] * v[2];
  double r1 = (m[1] * v[0] + m[4] * v[1]) + m[7] * v[2];
  double r2 = (m[2] * v[0] + m[5] * v[1]) + m[8] * v[2];
  r[0] = r0; r[1] = r1; r[2] = r2;
}
__device__ __forceinline__ void quatmul(double* r, const double* a, const double* b) {
  double r0 = ((a[0] * b[0] - a[1] * b[1]) - a[2] * b[2]) - a[3] * b[3];
  double r1 = ((a[0] * b[1] + a[1] * b[0]) + a[2] * b[3]) - a[3] * b[2];
  double r2 = ((a[0] * b[2] - a[1] * b[3]) + a[2] * b[0]) + a[3] * b[1];
  double r3 = ((a[0] * b[3] + a[1] * b[2]) - a[2] * b[1]) + a[3] * b[0];
  r[0] = r0; r[1] = r1; r[2] = r2; r[3] = r3;
}
__device__ __forceinline__ void quat2mat(double* m, const double* q) {
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
__device__ __forceinline__ void normalize4(double* q) {
  double n = sqrt(((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3]);
  if (n < K_MINVAL) { q[0] = 1.0; q[1] = q[2] = q[3] = 0.0; return; }
  double inv = 1.0 / n;
  q[0] = q[0] * inv; q[1] = q[1] * inv; q[2] = q[2] * inv; q[3] = q[3] * inv;
}
__device__ __forceinline__ double normalize3(double* v) {
  double n = sqrt(dot3(v, v));
  if (n < K_MINVAL) { v[0] = 1.0; v[1] = v[2] = 0.0; return 0.0; }
  double inv = 1.0 / n;
  v[0] = v[0] * inv; v[1] = v[1] * inv; v[2] = v[2] * inv;
  return n;
}
__device__ __forceinline__ void axisangle2quat(double* q, const double* axis, double angle) {
  double s, c;
  k_sincos(0.5 * angle, &s, &c);
  q[0] = c; q[1] = axis[0] * s; q[2] = axis[1] * s; q[3] = axis[2] * s;
}
__device__ __forceinline__ void mul_inert_vec(double* r, const double* i, const double* v) {
  double r0 = ((i[0] * v[0] + i[3] * v[1]) + i[4] * v[2]) - i[8] * v[4] + i[7] * v[5];
  double r1 = ((i[3] * v[0] + i[1] * v[1]) + i[5] * v[2]) + i[8] * v[3] - i[6] * v[5];
  double r2 = ((i[4] * v[0] + i[5] * v[1]) + i[2] * v[2]) - i[7] * v[3] + i[6] * v[4];
  double r3 = (i[8] * v[1] - i[7] * v[2]) + i[9] * v[3];
  double r4 = (i[6] * v[2] - i[8] * v[0]) + i[9] * v[4];
  double r5 = (i[7] * v[0] - i[6] * v[1]) + i[9] * v[5];
  r[0] = r0; r[1] = r1; r[2] = r2; r[3] = r3; r[4] = r4; r[5] = r5;
}
__device__ __forceinline__ double dot6(const double* a, const double* b) {
  return ((((a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]) + a[3] * b[3]) + a[4] * b[4]) + a[5] * b[5];
}
__device__ __forceinline__ void cross_motion(double* r, const double* v, const double* u) {
  double r0 = v[1] * u[2] - v[2] * u[1];
  double r1 = v[2] * u[0] - v[0] * u[2];
  double r2 = v[0] * u[1] - v[1] * u[0];
  double r3 = (v[1] * u[5] - v[2] * u[4]) + (v[4] * u[2] - v[5] * u[1]);
  double r4 = (v[2] * u[3] - v[0] * u[5]) + (v[5] * u[0] - v[3] * u[2]);
  double r5 = (v[0] * u[4] - v[1] * u[3]) + (v[3] * u[1] - v[4] * u[0]);
  r[0] = r0; r[1] = r1; r[2] = r2; r[3] = r3; r[4] = r4; r[5] = r5;
}
__device__ __forceinline__ void cross_force(double* r, const double* v, const double* f) {
  double r0 = (v[1] * f[2] - v[2] * f[1]) + (v[4] * f[5] - v[5] * f[4]);
  double r1 = (v[2] * f[0] - v[0] * f[2]) + (v[5] * f[3] - v[3] * f[5]);
  double r2 = (v[0] * f[1] - v[1] * f[0]) + (v[3] * f[4] - v[4] * f[3]);
  double r3 = v[1] * f[5] - v[2] * f[4];
  double r4 = v[2] * f[3] - v[0] * f[5];
  double r5 = v[0] * f[4] - v[1] * f[3];
  r[0] = r0; r[1] = r1; r[2] = r2; r[3] = r3; r[4] = r4; r[5] = r5;
}

// pairwise tree reduction of lane products: leaf[k] = a[k]*b[k] (k < n),
// level s: leaf[k] = leaf[k] + leaf[k^s] for s < P = nextpow2(n).
__device__ __forceinline__ double tree_sum(double leaf, int P) {
  for (int s = 1; s < P; s <<= 1) leaf = leaf + __shfl_xor(leaf, s);
  return leaf;
}
__device__ __forceinline__ int next_pow2(int n) {
  int P = 1;
  while (P < n) P <<= 1;
  return P;
}

// ---------------------------------------------------------------------------
// LDS layout
struct Lay {
  int o[64];
  int ncon_max;
  int nefc_max;
  int total_doubles;
};
enum {
  L_qpos, L_qvel, L_qacc_ws, L_ctrl, L_mocap_pos, L_mocap_quat, L_time, L_xpos, L_xquat, L_xmat, L_xipos,
  L_ximat, L_xanchor, L_xaxis, L_subtree_com, L_subtree_mass, L_cinert, L_crb, L_cdof, L_cdof_dot, L_cvel,
  L_cacc, L_cfrc, L_geom_xpos, L_geom_xmat, L_M, L_L, L_Dv, L_Dinv, L_qDeriv, L_qfrc_bias, L_qfrc_passive,
  L_qfrc_actuator, L_qfrc_smooth, L_qacc_smooth, L_qfrc_constraint, L_qacc, L_act_force, L_act_moment,
  L_act_length, L_act_vel, L_con_pos, L_con_frame, L_con_dist, L_J, L_K, L_efc_pos, L_efc_margin,
  L_efc_vel, L_efc_aref, L_efc_R, L_efc_A, L_efc_b, L_efc_f, L_efc_mu, L_efc_blk, L_efc_floss, L_w, L_jac,
  L_scratch, L_poly, L_ints, L_COUNT
};

__device__ void bind(Dat& d, double* s, const Lay& l) {
  d.qpos = s + l.o[L_qpos]; d.qvel = s + l.o[L_qvel]; d.qacc_ws = s + l.o[L_qacc_ws]; d.ctrl = s + l.o[L_ctrl];
  d.mocap_pos = s + l.o[L_mocap_pos]; d.mocap_quat = s + l.o[L_mocap_quat]; d.time = s + l.o[L_time];
  d.xpos = s + l.o[L_xpos]; d.xquat = s + l.o[L_xquat]; d.xmat = s + l.o[L_xmat]; d.xipos = s + l.o[L_xipos];
  d.ximat = s + l.o[L_ximat]; d.xanchor = s + l.o[L_xanchor]; d.xaxis = s + l.o[L_xaxis];
  d.subtree_com = s + l.o[L_subtree_com]; d.subtree_mass = s + l.o[L_subtree_mass];
  d.cinert = s + l.o[L_cinert]; d.crb = s + l.o[L_crb]; d.cdof = s + l.o[L_cdof];
  d.cdof_dot = s + l.o[L_cdof_dot]; d.cvel = s + l.o[L_cvel]; d.cacc = s + l.o[L_cacc]; d.cfrc = s + l.o[L_cfrc];
  d.geom_xpos = s + l.o[L_geom_xpos]; d.geom_xmat = s + l.o[L_geom_xmat];
  d.M = s + l.o[L_M]; d.L = s + l.o[L_L]; d.Dv = s + l.o[L_Dv]; d.Dinv = s + l.o[L_Dinv];
  d.qDeriv = s + l.o[L_qDeriv];
  d.qfrc_bias = s + l.o[L_qfrc_bias]; d.qfrc_passive = s + l.o[L_qfrc_passive];
  d.qfrc_actuator = s + l.o[L_qfrc_actuator]; d.qfrc_smooth = s + l.o[L_qfrc_smooth];
  d.qacc_smooth = s + l.o[L_qacc_smooth]; d.qfrc_constraint = s + l.o[L_qfrc_constraint];
  d.qacc = s + l.o[L_qacc];
  d.act_force = s + l.o[L_act_force]; d.act_moment = s + l.o[L_act_moment];
  d.act_length = s + l.o[L_act_length]; d.act_vel = s + l.o[L_act_vel];
  d.con_pos = s + l.o[L_con_pos]; d.con_frame = s + l.o[L_con_frame]; d.con_dist = s + l.o[L_con_dist];
  d.J = s + l.o[L_J]; d.K = s + l.o[L_K]; d.efc_pos = s + l.o[L_efc_pos]; d.efc_margin = s + l.o[L_efc_margin];
  d.efc_vel = s + l.o[L_efc_vel]; d.efc_aref = s + l.o[L_efc_aref]; d.efc_R = s + l.o[L_efc_R];
  d.efc_A = s + l.o[L_efc_A]; d.efc_b = s + l.o[L_efc_b]; d.efc_f = s + l.o[L_efc_f];
  d.efc_mu = s + l.o[L_efc_mu]; d.efc_blk = s + l.o[L_efc_blk]; d.efc_floss = s + l.o[L_efc_floss];
  d.w = s + l.o[L_w]; d.jac = s + l.o[L_jac]; d.scratch = s + l.o[L_scratch];
  d.poly = (P2*)(s + l.o[L_poly]);
  int* ib = (int*)(s + l.o[L_ints]);
  d.ints = ib;
  // int arrays follow the 16 counters
  int ncmax = l.ncon_max, nemax = l.nefc_max;
  d.con_pair = ib + 16;
  d.con_g1 = d.con_pair + ncmax;
  d.con_g2 = d.con_g1 + ncmax;
  d.efc_type = d.con_g2 + ncmax;
  d.efc_dim = d.efc_type + nemax;
  d.efc_con = d.efc_dim + nemax;
}

// ---------------------------------------------------------------------------
// kinematics (lane 0)
__device__ void kinematics(const Mdl& md, Dat& d) {
  const int32_t *parent = IA(md, body_parentid), *mocapid = IA(md, body_mocapid);
  const int32_t *jntnum = IA(md, body_jntnum), *jntadr = IA(md, body_jntadr);
  const int32_t *jtype = IA(md, jnt_type), *qadr = IA(md, jnt_qposadr);
  const double *bpos = DA(md, body_pos), *bquat = DA(md, body_quat);
  const double *ipos = DA(md, body_ipos), *iquat = DA(md, body_iquat);
  const double *jpos = DA(md, jnt_pos), *jaxis = DA(md, jnt_axis), *qpos0 = DA(md, qpos0);
  d.xpos[0] = d.xpos[1] = d.xpos[2] = 0.0;
  d.xquat[0] = 1.0; d.xquat[1] = d.xquat[2] = d.xquat[3] = 0.0;
  quat2mat(d.xmat, d.xquat);
  for (int b = 1; b < md.m.nbody; b++) {
    double pos[3], quat[4], mat[9];
    if (mocapid[b] >= 0) {
      const double* mp = d.mocap_pos + 3 * mocapid[b];
      const double* mq = d.mocap_quat + 4 * mocapid[b];
      pos[0] = mp[0]; pos[1] = mp[1]; pos[2] = mp[2];
      quat[0] = mq[0]; quat[1] = mq[1]; quat[2] = mq[2]; quat[3] = mq[3];
      normalize4(quat);
    } else {
      int p = parent[b];
      double t[3];
      mulmv3(t, d.xmat + 9 * p, bpos + 3 * b);
      add3(pos, d.xpos + 3 * p, t);
      quatmul(quat, d.xquat + 4 * p, bquat + 4 * b);
      for (int k = 0; k < jntnum[b]; k++) {
        int j = jntadr[b] + k;
        int a = qadr[j];
        if (jtype[j] == MGS_JNT_FREE) {
          pos[0] = d.qpos[a]; pos[1] = d.qpos[a + 1]; pos[2] = d.qpos[a + 2];
          quat[0] = d.qpos[a + 3]; quat[1] = d.qpos[a + 4]; quat[2] = d.qpos[a + 5]; quat[3] = d.qpos[a + 6];
          normalize4(quat);
          d.xanchor[3 * j] = pos[0]; d.xanchor[3 * j + 1] = pos[1]; d.xanchor[3 * j + 2] = pos[2];
          d.xaxis[3 * j] = 0.0; d.xaxis[3 * j + 1] = 0.0; d.xaxis[3 * j + 2] = 1.0;
        } else {
          quat2mat(mat, quat);
          mulmv3(d.xaxis + 3 * j, mat, jaxis + 3 * j);
          mulmv3(t, mat, jpos + 3 * j);
          add3(d.xanchor + 3 * j, t, pos);
          if (jtype[j] == MGS_JNT_HINGE) {
            double ql[4], qn[4];
            axisangle2quat(ql, jaxis + 3 * j, d.qpos[a] - qpos0[a]);
            quatmul(qn, quat, ql);
            quat[0] = qn[0]; quat[1] = qn[1]; quat[2] = qn[2]; quat[3] = qn[3];
            quat2mat(mat, quat);
            mulmv3(t, mat, jpos + 3 * j);
            sub3(pos, d.xanchor + 3 * j, t);
          } else {
            double dq = d.qpos[a] - qpos0[a];
            pos[0] = pos[0] + d.xaxis[3 * j] * dq;
            pos[1] = pos[1] + d.xaxis[3 * j + 1] * dq;
            pos[2] = pos[2] + d.xaxis[3 * j + 2] * dq;
          }
        }
      }
      normalize4(quat);
    }
    d.xpos[3 * b] = pos[0]; d.xpos[3 * b + 1] = pos[1]; d.xpos[3 * b + 2] = pos[2];
    d.xquat[4 * b] = quat[0]; d.xquat[4 * b + 1] = quat[1]; d.xquat[4 * b + 2] = quat[2]; d.xquat[4 * b + 3] = quat[3];
    quat2mat(d.xmat + 9 * b, quat);
    double t[3], qi[4];
    mulmv3(t, d.xmat + 9 * b, ipos + 3 * b);
    add3(d.xipos + 3 * b, d.xpos + 3 * b, t);
    quatmul(qi, quat, iquat + 4 * b);
    quat2mat(d.ximat + 9 * b, qi);
  }
  const int32_t* gbody = IA(md, geom_bodyid);
  const double *gpos = DA(md, geom_pos), *gquat = DA(md, geom_quat);
  for (int g = 0; g < md.m.ngeom; g++) {
    int b = gbody[g];
    double t[3], q[4];
    mulmv3(t, d.xmat + 9 * b, gpos + 3 * g);
    add3(d.geom_xpos + 3 * g, d.xpos + 3 * b, t);
    quatmul(q, d.xquat + 4 * b, gquat + 4 * g);
    quat2mat(d.geom_xmat + 9 * g, q);
  }
}

// mj_comPos (lane 0)
__device__ void com_pos(const Mdl& md, Dat& d) {
  const int32_t *parent = IA(md, body_parentid), *rootid = IA(md, body_rootid);
  const int32_t *jntnum = IA(md, body_jntnum), *jntadr = IA(md, body_jntadr);
  const int32_t *jtype = IA(md, jnt_type), *dadr = IA(md, jnt_dofadr);
  const double *mass = DA(md, body_mass), *inertia = DA(md, body_inertia);
  int nb = md.m.nbody;
  for (int b = 0; b < nb; b++) {
    d.subtree_mass[b] = mass[b];
    d.subtree_com[3 * b] = mass[b] * d.xipos[3 * b];
    d.subtree_com[3 * b + 1] = mass[b] * d.xipos[3 * b + 1];
    d.subtree_com[3 * b + 2] = mass[b] * d.xipos[3 * b + 2];
  }
  for (int b = nb - 1; b > 0; b--) {
    int p = parent[b];
    d.subtree_mass[p] = d.subtree_mass[p] + d.subtree_mass[b];
    d.subtree_com[3 * p] = d.subtree_com[3 * p] + d.subtree_com[3 * b];
    d.subtree_com[3 * p + 1] = d.subtree_com[3 * p + 1] + d.subtree_com[3 * b + 1];
    d.subtree_com[3 * p + 2] = d.subtree_com[3 * p + 2] + d.subtree_com[3 * b + 2];
  }
  for (int b = 0; b < nb; b++) {
    if (d.subtree_mass[b] < K_MINVAL) {
      d.subtree_com[3 * b] = d.xipos[3 * b];
      d.subtree_com[3 * b + 1] = d.xipos[3 * b + 1];
      d.subtree_com[3 * b + 2] = d.xipos[3 * b + 2];
    } else {
      double inv = 1.0 / d.subtree_mass[b];
      d.subtree_com[3 * b] = d.subtree_com[3 * b] * inv;
      d.subtree_com[3 * b + 1] = d.subtree_com[3 * b + 1] * inv;
      d.subtree_com[3 * b + 2] = d.subtree_com[3 * b + 2] * inv;
    }
  }
  for (int b = 0; b < nb; b++) {
    double* ci = d.cinert + 10 * b;
    const double* R = d.ximat + 9 * b;
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
  }
  for (int b = 1; b < nb; b++) {
    const double* c = d.subtree_com + 3 * rootid[b];
    for (int k = 0; k < jntnum[b]; k++) {
      int j = jntadr[b] + k;
      int da = dadr[j];
      double off[3];
      sub3(off, c, d.xanchor + 3 * j);
      if (jtype[j] == MGS_JNT_FREE) {
        for (int i = 0; i < 3; i++) {
          double* cd = d.cdof + 6 * (da + i);
          cd[0] = cd[1] = cd[2] = 0.0;
          cd[3] = (i == 0) ? 1.0 : 0.0; cd[4] = (i == 1) ? 1.0 : 0.0; cd[5] = (i == 2) ? 1.0 : 0.0;
        }
        const double* R = d.xmat + 9 * b;
        for (int i = 0; i < 3; i++) {
          double* cd = d.cdof + 6 * (da + 3 + i);
          double ax[3] = {R[i], R[3 + i], R[6 + i]};
          cd[0] = ax[0]; cd[1] = ax[1]; cd[2] = ax[2];
          cross3(cd + 3, ax, off);
        }
      } else if (jtype[j] == MGS_JNT_HINGE) {
        double* cd = d.cdof + 6 * da;
        const double* ax = d.xaxis + 3 * j;
        cd[0] = ax[0]; cd[1] = ax[1]; cd[2] = ax[2];
        cross3(cd + 3, ax, off);
      } else {
        double* cd = d.cdof + 6 * da;
        const double* ax = d.xaxis + 3 * j;
        cd[0] = cd[1] = cd[2] = 0.0;
        cd[3] = ax[0]; cd[4] = ax[1]; cd[5] = ax[2];
      }
    }
  }
}

// composite rigid bodies (lane 0) + mass matrix (lanes over dofs)
__device__ void crb(const Mdl& md, Dat& d) {
  int nb = md.m.nbody, nv = md.m.nv, lane = lane_id();
  const int32_t *parent = IA(md, body_parentid), *dbody = IA(md, dof_bodyid), *dpar = IA(md, dof_parentid);
  const double* arm = DA(md, dof_armature);
  if (lane == 0) {
    for (int k = 0; k < 10 * nb; k++) d.crb[k] = d.cinert[k];
    for (int b = nb - 1; b > 0; b--) {
      int p = parent[b];
      if (p > 0)
        for (int k = 0; k < 10; k++) d.crb[10 * p + k] = d.crb[10 * p + k] + d.crb[10 * b + k];
    }
  }
  for (int k = lane; k < nv * nv; k += WAVE) d.M[k] = 0.0;
  wsync();
  for (int i = lane; i < nv; i += WAVE) {
    double buf[6];
    mul_inert_vec(buf, d.crb + 10 * dbody[i], d.cdof + 6 * i);
    d.M[i * nv + i] = dot6(d.cdof + 6 * i, buf) + arm[i];
    int j = dpar[i];
    while (j >= 0) {
      double v = dot6(d.cdof + 6 * j, buf);
      d.M[i * nv + j] = v;
      d.M[j * nv + i] = v;
      j = dpar[j];
    }
  }
  wsync();
}

// dense LDL^T, columns sequential, rows across lanes (same products as oracle)
__device__ void ldl_factor(int n, const double* A, double* L, double* Dv, double* Dinv) {
  int lane = lane_id();
  for (int j = 0; j < n; j++) {
    double dj = A[j * n + j];
    for (int k = 0; k < j; k++) dj = dj - (L[j * n + k] * Dv[k]) * L[j * n + k];
    double inv = 1.0 / dj;
    for (int i = j + 1 + lane; i < n; i += WAVE) {
      double s = A[i * n + j];
      for (int k = 0; k < j; k++) s = s - L[i * n + k] * (L[j * n + k] * Dv[k]);
      L[i * n + j] = s * inv;
    }
    if (lane == 0) { Dv[j] = dj; Dinv[j] = inv; }
    wsync();
  }
}
// single-lane solve
__device__ void ldl_solve(int n, const double* L, const double* Dinv, const double* b, double* x) {
  double y[64];
  for (int i = 0; i < n; i++) {
    double s = b[i];
    for (int k = 0; k < i; k++) s = s - L[i * n + k] * y[k];
    y[i] = s;
  }
  for (int i = n - 1; i >= 0; i--) {
    double s = y[i] * Dinv[i];
    for (int k = i + 1; k < n; k++) s = s - L[k * n + i] * x[k];
    x[i] = s;
  }
}

// actuation (lane 0)
__device__ void actuation(const Mdl& md, Dat& d) {
  int nv = md.m.nv;
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
  for (int k = 0; k < nv; k++) d.qfrc_actuator[k] = 0.0;
  for (int u = 0; u < md.m.nu; u++) {
    double* mom = d.act_moment + u * nv;
    for (int k = 0; k < nv; k++) mom[k] = 0.0;
    double len;
    if (trntype[u] == MGS_TRN_JOINT) {
      int j = trnid[u];
      len = d.qpos[jq[j]] * gear[u];
      mom[jd[j]] = gear[u];
    } else {
      int t = trnid[u];
      double tl = 0.0;
      for (int w = tadr[t]; w < tadr[t] + tnum[t]; w++) {
        tl = tl + wcoef[w] * d.qpos[wq[w]];
        mom[wdof[w]] = mom[wdof[w]] + wcoef[w] * gear[u];
      }
      len = tl * gear[u];
    }
    double vel = 0.0;
    for (int k = 0; k < nv; k++) vel = vel + mom[k] * d.qvel[k];
    d.act_length[u] = len;
    d.act_vel[u] = vel;
    double c = d.ctrl[u];
    if (clim[u]) {
      if (c < crange[2 * u]) c = crange[2 * u];
      if (c > crange[2 * u + 1]) c = crange[2 * u + 1];
    }
    double g = gain[3 * u];
    if (gtype[u] == MGS_GAIN_AFFINE) g = (gain[3 * u] + gain[3 * u + 1] * len) + gain[3 * u + 2] * vel;
    double f = g * c;
    if (btype[u] == MGS_BIAS_AFFINE) f = f + ((bias[3 * u] + bias[3 * u + 1] * len) + bias[3 * u + 2] * vel);
    if (flim[u]) {
      if (f < frange[2 * u]) f = frange[2 * u];
      if (f > frange[2 * u + 1]) f = frange[2 * u + 1];
    }
    d.act_force[u] = f;
    for (int k = 0; k < nv; k++) d.qfrc_actuator[k] = d.qfrc_actuator[k] + mom[k] * f;
  }
}

__device__ void passive(const Mdl& md, Dat& d) {
  const int32_t *jtype = IA(md, jnt_type), *jq = IA(md, jnt_qposadr), *jd = IA(md, jnt_dofadr);
  const double *stiff = DA(md, jnt_stiffness), *qspring = DA(md, qpos_spring), *damp = DA(md, dof_damping);
  for (int k = 0; k < md.m.nv; k++) d.qfrc_passive[k] = 0.0;
  for (int j = 0; j < md.m.njnt; j++) {
    if (stiff[j] == 0.0) continue;
    if (jtype[j] == MGS_JNT_HINGE || jtype[j] == MGS_JNT_SLIDE)
      d.qfrc_passive[jd[j]] = -stiff[j] * (d.qpos[jq[j]] - qspring[jq[j]]);
  }
  for (int k = 0; k < md.m.nv; k++) d.qfrc_passive[k] = d.qfrc_passive[k] - damp[k] * d.qvel[k];
}

__device__ void rne(const Mdl& md, Dat& d) {
  int nb = md.m.nbody;
  const int32_t *parent = IA(md, body_parentid), *dnum = IA(md, body_dofnum), *dadr = IA(md, body_dofadr);
  const int32_t* dbody = IA(md, dof_bodyid);
  for (int k = 0; k < 6; k++) { d.cvel[k] = 0.0; d.cacc[k] = 0.0; }
  d.cacc[3] = -md.m.gravity[0]; d.cacc[4] = -md.m.gravity[1]; d.cacc[5] = -md.m.gravity[2];
  for (int b = 1; b < nb; b++) {
    int p = parent[b];
    double* cv = d.cvel + 6 * b;
    double* ca = d.cacc + 6 * b;
    for (int k = 0; k < 6; k++) { cv[k] = d.cvel[6 * p + k]; ca[k] = d.cacc[6 * p + k]; }
    for (int i = 0; i < dnum[b]; i++) {
      int dd = dadr[b] + i;
      cross_motion(d.cdof_dot + 6 * dd, cv, d.cdof + 6 * dd);
      for (int k = 0; k < 6; k++) cv[k] = cv[k] + d.cdof[6 * dd + k] * d.qvel[dd];
    }
    for (int i = 0; i < dnum[b]; i++) {
      int dd = dadr[b] + i;
      for (int k = 0; k < 6; k++) ca[k] = ca[k] + d.cdof_dot[6 * dd + k] * d.qvel[dd];
    }
    double f1[6], f2[6], f3[6];
    mul_inert_vec(f1, d.cinert + 10 * b, ca);
    mul_inert_vec(f2, d.cinert + 10 * b, cv);
    cross_force(f3, cv, f2);
    for (int k = 0; k < 6; k++) d.cfrc[6 * b + k] = f1[k] + f3[k];
  }
  for (int b = nb - 1; b > 0; b--) {
    int p = parent[b];
    if (p > 0)
      for (int k = 0; k < 6; k++) d.cfrc[6 * p + k] = d.cfrc[6 * p + k] + d.cfrc[6 * b + k];
  }
  for (int i = 0; i < md.m.nv; i++) d.qfrc_bias[i] = dot6(d.cdof + 6 * i, d.cfrc + 6 * dbody[i]);
}

// ---------------------------------------------------------------------------
// collision
struct SupPt { double v[3], a[3], b[3]; };

// wave-parallel support mapping: all lanes pass the same dir, all lanes get the result
__device__ int support_geom(const Mdl& md, const Dat& d, int g, const double* dir, double* out) {
  int lane = lane_id();
  int h = IA(md, geom_hullid)[g];
  int adr = IA(md, hull_vertadr)[h], num = IA(md, hull_vertnum)[h];
  const double* V = DA(md, hull_vert) + 3 * adr;
  const double* R = d.geom_xmat + 9 * g;
  double dl[3];
  mulmtv3(dl, R, dir);
  double best = -INFINITY;
  int bi = 0x7fffffff;
  for (int i = lane; i < num; i += WAVE) {
    double s = (V[3 * i] * dl[0] + V[3 * i + 1] * dl[1]) + V[3 * i + 2] * dl[2];
    if (s > best) { best = s; bi = i; }
  }
  for (int s = 32; s >= 1; s >>= 1) {
    double ob = __shfl_xor(best, s);
    int oi = __shfl_xor(bi, s);
    if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
  if (bi == 0x7fffffff) bi = 0;
  double t[3];
  mulmv3(t, R, V + 3 * bi);
  add3(out, d.geom_xpos + 3 * g, t);
  return bi;
}

__device__ void mink_support(const Mdl& md, const Dat& d, int g1, int g2, const double* dir, SupPt* p) {
  double nd[3] = {-dir[0], -dir[1], -dir[2]};
  support_geom(md, d, g1, dir, p->a);
  support_geom(md, d, g2, nd, p->b);
  sub3(p->v, p->a, p->b);
}

__device__ void portal_normal(double* n, const SupPt* p1, const SupPt* p2, const SupPt* p3) {
  double e1[3], e2[3];
  sub3(e1, p2->v, p1->v);
  sub3(e2, p3->v, p1->v);
  cross3(n, e1, e2);
  normalize3(n);
}
__device__ int portal_reach_tol(const SupPt* p1, const SupPt* p2, const SupPt* p3, const SupPt* p4,
                                const double* n, double tol) {
  double dv4 = dot3(p4->v, n);
  double t1 = dv4 - dot3(p1->v, n);
  double t2 = dv4 - dot3(p2->v, n);
  double t3 = dv4 - dot3(p3->v, n);
  double mn = t1 < t2 ? t1 : t2;
  mn = mn < t3 ? mn : t3;
  return mn <= tol;
}
__device__ void portal_expand(SupPt* p0, SupPt* p1, SupPt* p2, SupPt* p3, const SupPt* p4) {
  double c[3];
  cross3(c, p4->v, p0->v);
  if (dot3(p1->v, c) > 0.0) {
    if (dot3(p2->v, c) > 0.0) *p1 = *p4; else *p3 = *p4;
  } else {
    if (dot3(p3->v, c) > 0.0) *p2 = *p4; else *p1 = *p4;
  }
}

__device__ int mpr_penetration(const Mdl& md, const Dat& d, int g1, int g2, double* n, double* depth, double* pos) {
  const double tol = md.m.mpr_tolerance;
  const int32_t* ghull = IA(md, geom_hullid);
  const double* HC = DA(md, hull_center);
  SupPt p0, p1, p2, p3, p4;
  double t[3], dir[3];
  mulmv3(t, d.geom_xmat + 9 * g1, HC + 3 * ghull[g1]);
  add3(p0.a, d.geom_xpos + 3 * g1, t);
  mulmv3(t, d.geom_xmat + 9 * g2, HC + 3 * ghull[g2]);
  add3(p0.b, d.geom_xpos + 3 * g2, t);
  sub3(p0.v, p0.a, p0.b);
  if (p0.v[0] == 0.0 && p0.v[1] == 0.0 && p0.v[2] == 0.0) p0.v[0] = 1e-9;
  dir[0] = -p0.v[0]; dir[1] = -p0.v[1]; dir[2] = -p0.v[2];
  normalize3(dir);
  mink_support(md, d, g1, g2, dir, &p1);
  if (dot3(p1.v, dir) <= 0.0) return 0;
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
  mink_support(md, d, g1, g2, dir, &p2);
  if (dot3(p2.v, dir) <= 0.0) return 0;
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
    mink_support(md, d, g1, g2, dir, &p3);
    if (dot3(p3.v, dir) <= 0.0) return 0;
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
    mink_support(md, d, g1, g2, dir, &p4);
    if (dot3(p4.v, dir) < 0.0) return 0;
    if (portal_reach_tol(&p1, &p2, &p3, &p4, dir, tol)) return 0;
    portal_expand(&p0, &p1, &p2, &p3, &p4);
  }
  if (it == K_MPR_MAXIT) return 0;
  for (it = 0;; it++) {
    portal_normal(dir, &p1, &p2, &p3);
    mink_support(md, d, g1, g2, dir, &p4);
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
      for (int k = 0; k < 3; k++) {
        double pa = (u1 * p1.a[k] + u2 * p2.a[k]) + u3 * p3.a[k];
        double pb = (u1 * p1.b[k] + u2 * p2.b[k]) + u3 * p3.b[k];
        pos[k] = 0.5 * (pa + pb);
      }
      return 1;
    }
    portal_expand(&p0, &p1, &p2, &p3, &p4);
  }
}

__device__ void make_frame(const double* n, double* t1, double* t2) {
  double a[3];
  if (fabs(n[0]) < 0.6) { a[0] = 1.0; a[1] = 0.0; a[2] = 0.0; }
  else { a[0] = 0.0; a[1] = 1.0; a[2] = 0.0; }
  double an = dot3(a, n);
  t1[0] = a[0] - n[0] * an; t1[1] = a[1] - n[1] * an; t1[2] = a[2] - n[2] * an;
  normalize3(t1);
  cross3(t2, n, t1);
}

// feature extraction: wave max over heights, then ballot compaction in vertex
// order of the vertices within tol of the extreme; out[] written to LDS.
__device__ int feature(const Mdl& md, const Dat& d, int g, const double* n, const double* t1, const double* t2,
                       int sign, double tol, P2* out, double* ext) {
  int lane = lane_id();
  int h = IA(md, geom_hullid)[g];
  int adr = IA(md, hull_vertadr)[h], num = IA(md, hull_vertnum)[h];
  const double* V = DA(md, hull_vert) + 3 * adr;
  const double* R = d.geom_xmat + 9 * g;
  const double* x = d.geom_xpos + 3 * g;
  double nl[3];
  mulmtv3(nl, R, n);
  double base = dot3(x, n);
  double best = (sign > 0) ? -INFINITY : INFINITY;
  for (int i = lane; i < num; i += WAVE) {
    double s = base + ((V[3 * i] * nl[0] + V[3 * i + 1] * nl[1]) + V[3 * i + 2] * nl[2]);
    if (sign > 0 ? (s > best) : (s < best)) best = s;
  }
  for (int s = 32; s >= 1; s >>= 1) {
    double ob = __shfl_xor(best, s);
    if (sign > 0 ? (ob > best) : (ob < best)) best = ob;
  }
  *ext = best;
  double lim = (sign > 0) ? best - tol : best + tol;
  int cnt = 0;
  for (int c0 = 0; c0 < num && cnt < K_MAXF; c0 += WAVE) {
    int i = c0 + lane;
    double s = 0.0;
    int pred = 0;
    if (i < num) {
      s = base + ((V[3 * i] * nl[0] + V[3 * i + 1] * nl[1]) + V[3 * i + 2] * nl[2]);
      pred = sign > 0 ? (s >= lim) : (s <= lim);
    }
    unsigned long long mask = __ballot(pred);
    int before = __popcll(mask & ((1ull << lane) - 1ull));
    int pos = cnt + before;
    if (pred && pos < K_MAXF) {
      double t[3], P[3];
      mulmv3(t, R, V + 3 * i);
      add3(P, x, t);
      out[pos].x = dot3(P, t1);
      out[pos].y = dot3(P, t2);
      out[pos].h = s;
    }
    cnt += __popcll(mask);
  }
  wsync();
  return cnt < K_MAXF ? cnt : K_MAXF;
}

__device__ __forceinline__ double cross2(const P2* o, const P2* a, const P2* b) {
  return (a->x - o->x) * (b->y - o->y) - (a->y - o->y) * (b->x - o->x);
}

__device__ int hull2d(P2* pts, int n, P2* out) {
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
  n = m;
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

__device__ __forceinline__ P2 lerp2(const P2* a, const P2* b, double t) {
  P2 r;
  r.x = a->x + t * (b->x - a->x);
  r.y = a->y + t * (b->y - a->y);
  r.h = a->h + t * (b->h - a->h);
  return r;
}

__device__ int clip_poly(const P2* P, int np, P2* Q, int nq, P2* buf) {
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

__device__ __forceinline__ double dist2d(const P2* a, const P2* b) {
  double dx = a->x - b->x, dy = a->y - b->y;
  return dx * dx + dy * dy;
}

__device__ void add_contact(Dat& d, int ncon_max, int pair, int g1, int g2, const double* pos, const double* n,
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

// narrowphase of one admissible pair, all lanes participate
__device__ void collide_pair(const Mdl& md, Dat& d, int pair) {
  int lane = lane_id();
  int g1 = IA(md, pair_geom1)[pair], g2 = IA(md, pair_geom2)[pair];
  double n[3], depth, mpos[3];
  if (!mpr_penetration(md, d, g1, g2, n, &depth, mpos)) return;
  double t1[3], t2[3];
  make_frame(n, t1, t2);
  P2* fa = d.poly;                 // K_MAXPOLY each
  P2* fb = d.poly + K_MAXPOLY;
  P2* buf = d.poly + 2 * K_MAXPOLY;
  double s1, s2;
  int na = feature(md, d, g1, n, t1, t2, +1, 0.0, fa, &s1);
  int nb = feature(md, d, g2, n, t1, t2, -1, 0.0, fb, &s2);
  double dn = s1 - s2;
  if (!(dn > 0.0)) return;
  double tol = dn + K_FEAT_EPS;
  na = feature(md, d, g1, n, t1, t2, +1, tol, fa, &s1);
  nb = feature(md, d, g2, n, t1, t2, -1, tol, fb, &s2);
  if (lane == 0) {
    int refB = (nb >= na);
    P2 refpoly[K_MAXPOLY], inc[K_MAXPOLY];
    int nr = refB ? hull2d(fb, nb, refpoly) : hull2d(fa, na, refpoly);
    int ni = refB ? hull2d(fa, na, inc) : hull2d(fb, nb, inc);
    P2 pts[K_MAXPOLY];
    double dep[K_MAXPOLY];
    int np = 0;
    if (nr >= 3) {
      int nc = clip_poly(refpoly, nr, inc, ni, buf);
      for (int i = 0; i < nc; i++) {
        double dd = refB ? (inc[i].h - s2) : (s1 - inc[i].h);
        if (dd > 0.0) { pts[np] = inc[i]; dep[np] = dd; np++; }
      }
    }
    int ncmax = md.m.ncon_max;
    if (np == 0) {
      add_contact(d, ncmax, pair, g1, g2, mpos, n, t1, t2, -dn);
    } else {
      int sel[4];
      int ns;
      if (np <= 4) {
        for (int i = 0; i < np; i++) sel[i] = i;
        ns = np;
      } else {
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
        ns = 4;
      }
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
}

// broadphase over all admissible pairs (lanes over pairs), then narrowphase in pair order
__device__ void collision(const Mdl& md, Dat& d) {
  int lane = lane_id();
  const int32_t *p1 = IA(md, pair_geom1), *p2 = IA(md, pair_geom2);
  const double *aabb = DA(md, geom_aabb), *pm = DA(md, pair_margin);
  if (lane == 0) d.NCON = 0;
  wsync();
  int npair = md.m.npair;
  for (int c0 = 0; c0 < npair; c0 += WAVE) {
    int p = c0 + lane;
    int ov = 0;
    if (p < npair) {
      int g[2] = {p1[p], p2[p]};
      double c[2][3], hw[2][3];
      for (int s = 0; s < 2; s++) {
        const double* R = d.geom_xmat + 9 * g[s];
        const double* lc = aabb + 6 * g[s];
        const double* lh = lc + 3;
        double t[3];
        mulmv3(t, R, lc);
        add3(c[s], d.geom_xpos + 3 * g[s], t);
        for (int k = 0; k < 3; k++)
          hw[s][k] = (fabs(R[3 * k]) * lh[0] + fabs(R[3 * k + 1]) * lh[1]) + fabs(R[3 * k + 2]) * lh[2];
      }
      ov = 1;
      for (int k = 0; k < 3; k++)
        if (fabs(c[0][k] - c[1][k]) > (hw[0][k] + hw[1][k]) + pm[p]) ov = 0;
    }
    unsigned long long mask = __ballot(ov);
    while (mask) {
      int b = __ffsll((long long)mask) - 1;
      mask &= mask - 1ull;
      collide_pair(md, d, c0 + b);
    }
  }
}

// ---------------------------------------------------------------------------
// constraints
__device__ void jac_point(const Mdl& md, const Dat& d, int b, const double* pt, double* jacp, double* jacr) {
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

__device__ double impedance(const double* si, double pos, double margin) {
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
__device__ int add_row(const Mdl& md, Dat& d, int type, double pos, double margin, int dim, int con) {
  if (d.NEFC >= md.m.nefc_max) { d.OVERFLOW |= 2; return -1; }
  int r = d.NEFC++;
  d.efc_type[r] = type; d.efc_pos[r] = pos; d.efc_margin[r] = margin;
  d.efc_dim[r] = dim; d.efc_con[r] = con;
  return r;
}

__device__ void row_params(const Mdl& md, Dat& d, int r, int dim, const double* sr, const double* si,
                           const double* mu, int elliptic_contact) {
  const double dt = md.m.timestep;
  double tc = sr[0], dr = sr[1];
  double imp = impedance(si, d.efc_pos[r], d.efc_margin[r]);
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
  double Rn = ((1.0 - imp) / imp) * d.efc_A[r];
  if (Rn < K_MINVAL) Rn = K_MINVAL;
  d.efc_R[r] = Rn;
  if (elliptic_contact && dim > 1) {
    double R1 = Rn / md.m.impratio;
    d.efc_R[r + 1] = R1;
    for (int j = 1; j < dim - 1; j++) d.efc_R[r + j + 1] = (R1 * (mu[0] * mu[0])) / (mu[j] * mu[j]);
  } else {
    for (int j = 1; j < dim; j++) {
      double Rj = ((1.0 - imp) / imp) * d.efc_A[r + j];
      d.efc_R[r + j] = Rj < K_MINVAL ? K_MINVAL : Rj;
    }
  }
}

// fill J rows r..r+nr-1 from jacobian scratch according to kind (lanes over columns)
__device__ void make_constraints(const Mdl& md, Dat& d) {
  int nv = md.m.nv, lane = lane_id();
  double* jp1 = d.jac;
  double* jr1 = d.jac + 3 * nv;
  double* jp2 = d.jac + 6 * nv;
  double* jr2 = d.jac + 9 * nv;
  int* ints = d.ints;
  if (lane == 0) { d.NEFC = 0; }
  wsync();
  const int32_t *et = IA(md, eq_type), *eo1 = IA(md, eq_obj1id), *eo2 = IA(md, eq_obj2id);
  const double* ed = DA(md, eq_data);
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
      if (lane == 0) {
        jac_point(md, d, b1, p1, jp1, jr1);
        jac_point(md, d, b2, p2, jp2, jr2);
        if (d.NEFC + (et[e] == MGS_EQ_WELD ? 6 : 3) > md.m.nefc_max) d.OVERFLOW |= 2;
        else for (int k = 0; k < 3; k++) add_row(md, d, MGS_EFC_EQUALITY, p1[k] - p2[k], 0.0, 1, e);
      }
      wsync();
      if (d.OVERFLOW & 2) break;
      int r0 = d.NEFC - 3;
      for (int c = lane; c < nv; c += WAVE)
        for (int k = 0; k < 3; k++) d.J[(r0 + k) * nv + c] = jp1[k * nv + c] - jp2[k * nv + c];
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
        for (int c = lane; c < nv; c += WAVE) {
          double ax[4] = {0.0, jr1[c] - jr2[c], jr1[nv + c] - jr2[nv + c], jr1[2 * nv + c] - jr2[2 * nv + c]};
          double t1q[4], t2q[4];
          quatmul(t1q, q2c, ax);
          quatmul(t2q, t1q, q1r);
          for (int k = 0; k < 3; k++) d.J[(rr + k) * nv + c] = (0.5 * t2q[1 + k]) * ts;
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
      if (lane == 0) {
        if (d.NEFC + 1 > md.m.nefc_max) d.OVERFLOW |= 2;
        else add_row(md, d, MGS_EFC_EQUALITY, pos, 0.0, 1, e);
      }
      wsync();
      if (d.OVERFLOW & 2) break;
      int r = d.NEFC - 1;
      for (int c = lane; c < nv; c += WAVE) d.J[r * nv + c] = 0.0;
      wsync();
      if (lane == 0) {
        d.J[r * nv + jd[j1]] = 1.0;
        if (j2 >= 0) d.J[r * nv + jd[j2]] = d.J[r * nv + jd[j2]] - deriv;
      }
      wsync();
    }
  }
  if (lane == 0) ints[8] = d.NEFC;
  // dof friction loss
  const double* floss = DA(md, dof_frictionloss);
  if (lane == 0) {
    ints[9] = d.NEFC;
    for (int k = 0; k < nv; k++) {
      if (floss[k] > 0.0) {
        int r = add_row(md, d, MGS_EFC_FRICTION, 0.0, 0.0, 1, k);
        if (r < 0) break;
        for (int c = 0; c < nv; c++) d.J[r * nv + c] = 0.0;
        d.J[r * nv + k] = 1.0;
        d.efc_floss[r] = floss[k];
      }
    }
    ints[10] = d.NEFC;
    // joint limits
    const int32_t *lim = IA(md, jnt_limited), *jq = IA(md, jnt_qposadr), *jd = IA(md, jnt_dofadr);
    const double *range = DA(md, jnt_range), *jmargin = DA(md, jnt_margin);
    ints[11] = d.NEFC;
    for (int j = 0; j < md.m.njnt; j++) {
      if (!lim[j]) continue;
      double q = d.qpos[jq[j]];
      double dlo = q - range[2 * j], dhi = range[2 * j + 1] - q;
      if (dlo < jmargin[j]) {
        int r = add_row(md, d, MGS_EFC_LIMIT, dlo, jmargin[j], 1, j);
        if (r >= 0) { for (int c = 0; c < nv; c++) d.J[r * nv + c] = 0.0; d.J[r * nv + jd[j]] = 1.0; }
      }
      if (dhi < jmargin[j]) {
        int r = add_row(md, d, MGS_EFC_LIMIT, dhi, jmargin[j], 1, j);
        if (r >= 0) { for (int c = 0; c < nv; c++) d.J[r * nv + c] = 0.0; d.J[r * nv + jd[j]] = -1.0; }
      }
    }
    ints[12] = d.NEFC;
    ints[6] = d.NEFC;
  }
  wsync();
  // contacts
  const int32_t *gbody = IA(md, geom_bodyid), *pcd = IA(md, pair_condim);
  const double *pfr = DA(md, pair_friction), *pmar = DA(md, pair_margin);
  int ncon = d.NCON;
  for (int c = 0; c < ncon; c++) {
    int p = d.con_pair[c];
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
      jac_point(md, d, b1, pt, jp1, jr1);
      jac_point(md, d, b2, pt, jp2, jr2);
      for (int j = 0; j < dim; j++) add_row(md, d, MGS_EFC_CONTACT, j == 0 ? d.con_dist[c] : 0.0, pmar[p], dim, c);
      for (int j = 0; j < dim; j++) d.efc_mu[5 * r + j] = (j < dim - 1) ? pfr[5 * p + j] : 0.0;
    }
    wsync();
    for (int col = lane; col < nv; col += WAVE) {
      double dp[3] = {jp2[col] - jp1[col], jp2[nv + col] - jp1[nv + col], jp2[2 * nv + col] - jp1[2 * nv + col]};
      for (int j = 0; j < dim && j < 3; j++) d.J[(r + j) * nv + col] = dot3(fr + 3 * j, dp);
      if (dim >= 4) {
        double dr[3] = {jr2[col] - jr1[col], jr2[nv + col] - jr1[nv + col], jr2[2 * nv + col] - jr1[2 * nv + col]};
        d.J[(r + 3) * nv + col] = dot3(fr, dr);
        if (dim == 6) {
          d.J[(r + 4) * nv + col] = dot3(fr + 3, dr);
          d.J[(r + 5) * nv + col] = dot3(fr + 6, dr);
        }
      }
    }
  }
  wsync();
  if (lane == 0) ints[7] = d.NEFC;
  wsync();
  int ne = d.NEFC;
  // velocities, K = M^-1 J^T, diagonal of A (lanes over rows)
  for (int r = lane; r < ne; r += WAVE) {
    const double* Jr = d.J + r * nv;
    double v = 0.0;
    for (int k = 0; k < nv; k++) v = v + Jr[k] * d.qvel[k];
    d.efc_vel[r] = v;
    ldl_solve(nv, d.L, d.Dinv, Jr, d.K + r * nv);
    double a = 0.0;
    for (int k = 0; k < nv; k++) a = a + Jr[k] * d.K[r * nv + k];
    d.efc_A[r] = a;
  }
  wsync();
  if (lane == 0) {
    const double *eqsr = DA(md, eq_solref), *eqsi = DA(md, eq_solimp);
    for (int r = 0; r < ints[8]; r++) {
      int e = d.efc_con[r];
      row_params(md, d, r, 1, eqsr + 2 * e, eqsi + 5 * e, nullptr, 0);
    }
    const double *dsr = DA(md, dof_solref), *dsi = DA(md, dof_solimp);
    for (int r = ints[9]; r < ints[10]; r++) {
      int k = d.efc_con[r];
      row_params(md, d, r, 1, dsr + 2 * k, dsi + 5 * k, nullptr, 0);
    }
    const double *jsr = DA(md, jnt_solref), *jsi = DA(md, jnt_solimp);
    for (int r = ints[11]; r < ints[12]; r++) {
      int j = d.efc_con[r];
      row_params(md, d, r, 1, jsr + 2 * j, jsi + 5 * j, nullptr, 0);
    }
    const double *psr = DA(md, pair_solref), *psi = DA(md, pair_solimp);
    for (int r = ints[6]; r < ints[7];) {
      int c = d.efc_con[r];
      int p = d.con_pair[c];
      int dim = d.efc_dim[r];
      row_params(md, d, r, dim, psr + 2 * p, psi + 5 * p, d.efc_mu + 5 * r, 1);
      r += dim;
    }
  }
  wsync();
  for (int r = lane; r < ne; r += WAVE) {
    const double* Jr = d.J + r * nv;
    double v = 0.0;
    for (int k = 0; k < nv; k++) v = v + Jr[k] * d.qacc_smooth[k];
    d.efc_b[r] = v - d.efc_aref[r];
  }
  // contact blocks of A (lanes over block entries)
  for (int r = ints[6]; r < ints[7];) {
    int dim = d.efc_dim[r];
    double* blk = d.efc_blk + 36 * r;
    for (int e = lane; e < dim * dim; e += WAVE) {
      int i = e / dim, j = e % dim;
      const double* Ji = d.J + (r + i) * nv;
      const double* Kj = d.K + (r + j) * nv;
      double a = 0.0;
      for (int k = 0; k < nv; k++) a = a + Ji[k] * Kj[k];
      blk[i * dim + j] = a;
    }
    r += dim;
  }
  wsync();
}

// ---------------------------------------------------------------------------
// solver
__device__ void qcqp(int n, const double* A, const double* b, const double* mu, double r, double* x) {
  double As[25], bs[5], y[5], P[25];
  for (int i = 0; i < n; i++) {
    bs[i] = b[i] * mu[i];
    for (int j = 0; j < n; j++) As[i * n + j] = (A[i * n + j] * mu[i]) * mu[j];
  }
  double la = 0.0;
  double rr = r * r;
  for (int i = 0; i < n; i++) y[i] = 0.0;
  for (int it = 0; it < 20; it++) {
    double T[25];
    for (int i = 0; i < n * n; i++) T[i] = As[i];
    for (int i = 0; i < n; i++) T[i * n + i] = T[i * n + i] + la;
    for (int i = 0; i < n * n; i++) P[i] = 0.0;
    for (int i = 0; i < n; i++) P[i * n + i] = 1.0;
    int bad = 0;
    for (int c = 0; c < n; c++) {
      double piv = T[c * n + c];
      if (piv < 1e-15) { bad = 1; break; }
      double ip = 1.0 / piv;
      for (int j = 0; j < n; j++) { T[c * n + j] = T[c * n + j] * ip; P[c * n + j] = P[c * n + j] * ip; }
      for (int i = 0; i < n; i++) {
        if (i == c) continue;
        double f = T[i * n + c];
        if (f == 0.0) continue;
        for (int j = 0; j < n; j++) {
          T[i * n + j] = T[i * n + j] - f * T[c * n + j];
          P[i * n + j] = P[i * n + j] - f * P[c * n + j];
        }
      }
    }
    if (bad) { for (int i = 0; i < n; i++) y[i] = 0.0; break; }
    for (int i = 0; i < n; i++) {
      double s = 0.0;
      for (int j = 0; j < n; j++) s = s - P[i * n + j] * bs[j];
      y[i] = s;
    }
    double val = 0.0;
    for (int i = 0; i < n; i++) val = val + y[i] * y[i];
    val = val - rr;
    if (val < 1e-10) break;
    double pv[5];
    for (int i = 0; i < n; i++) {
      double s = 0.0;
      for (int j = 0; j < n; j++) s = s + P[i * n + j] * y[j];
      pv[i] = s;
    }
    double deriv = 0.0;
    for (int i = 0; i < n; i++) deriv = deriv + y[i] * pv[i];
    deriv = -2.0 * deriv;
    double delta = -val / deriv;
    if (delta < 1e-10) break;
    la = la + delta;
  }
  for (int i = 0; i < n; i++) x[i] = y[i] * mu[i];
}

__device__ void project_block(const Dat& d, int r, double* f) {
  int t = d.efc_type[r];
  if (t == MGS_EFC_FRICTION) {
    double fl = d.efc_floss[r];
    if (f[0] < -fl) f[0] = -fl;
    if (f[0] > fl) f[0] = fl;
  } else if (t == MGS_EFC_LIMIT) {
    if (f[0] < 0.0) f[0] = 0.0;
  } else if (t == MGS_EFC_CONTACT) {
    int dim = d.efc_dim[r];
    if (f[0] < 0.0) { for (int j = 0; j < dim; j++) f[j] = 0.0; return; }
    if (dim == 1) return;
    const double* mu = d.efc_mu + 5 * r;
    double s = 0.0;
    for (int j = 1; j < dim; j++) { double q = f[j] / mu[j - 1]; s = s + q * q; }
    double nt = sqrt(s);
    if (nt > f[0]) {
      double sc = f[0] / nt;
      for (int j = 1; j < dim; j++) f[j] = f[j] * sc;
    }
  }
}

__device__ void solve_pgs(const Mdl& md, Dat& d) {
  int nv = md.m.nv, ne = d.NEFC, lane = lane_id();
  int P = next_pow2(nv);
  double meaninertia = 0.0;
  for (int k = 0; k < nv; k++) meaninertia = meaninertia + d.M[k * nv + k];
  meaninertia = meaninertia / (double)nv;
  double scale = 1.0 / (meaninertia * (double)(nv > 1 ? nv : 1));
  // warmstart
  for (int r = lane; r < ne; r += WAVE) {
    const double* Jr = d.J + r * nv;
    double jar = 0.0;
    for (int k = 0; k < nv; k++) jar = jar + Jr[k] * d.qacc_ws[k];
    jar = jar - d.efc_aref[r];
    d.efc_f[r] = -jar / d.efc_R[r];
  }
  wsync();
  if (lane == 0) {
    for (int r = 0; r < ne;) {
      int dim = d.efc_type[r] == MGS_EFC_CONTACT ? d.efc_dim[r] : 1;
      if (d.efc_type[r] != MGS_EFC_EQUALITY) project_block(d, r, d.efc_f + r);
      r += dim;
    }
  }
  wsync();
  for (int k = lane; k < nv; k += WAVE) {
    double s = 0.0;
    for (int r = 0; r < ne; r++) s = s + d.K[r * nv + k] * d.efc_f[r];
    d.w[k] = s;
  }
  wsync();
  // dual cost: per-row terms by lanes, summed in row order by lane 0
  for (int r = lane; r < ne; r += WAVE) {
    const double* Jr = d.J + r * nv;
    double jw = 0.0;
    for (int k = 0; k < nv; k++) jw = jw + Jr[k] * d.w[k];
    d.scratch[r] = d.efc_f[r] * ((0.5 * (jw + d.efc_R[r] * d.efc_f[r])) + d.efc_b[r]);
  }
  wsync();
  double cw = 0.0;
  for (int r = 0; r < ne; r++) cw = cw + d.scratch[r];
  if (!(cw < 0.0)) {
    for (int r = lane; r < ne; r += WAVE) d.efc_f[r] = 0.0;
    for (int k = lane; k < nv; k += WAVE) d.w[k] = 0.0;
  }
  wsync();
  int it;
  for (it = 0; it < md.m.iterations && ne > 0; it++) {
    double improvement = 0.0;
    for (int r = 0; r < ne;) {
      int t = d.efc_type[r];
      if (t != MGS_EFC_CONTACT || d.efc_dim[r] == 1) {
        const double* Jr = d.J + r * nv;
        double leaf = (lane < nv) ? Jr[lane] * d.w[lane] : 0.0;
        double jw = tree_sum(leaf, P);
        double res = (jw + d.efc_R[r] * d.efc_f[r]) + d.efc_b[r];
        double AR = d.efc_A[r] + d.efc_R[r];
        double fo = d.efc_f[r];
        double fnew[1] = {fo - res / AR};
        if (t != MGS_EFC_EQUALITY) project_block(d, r, fnew);
        double delta = fnew[0] - fo;
        improvement = improvement - delta * (0.5 * AR * delta + res);
        if (delta != 0.0) {
          const double* Kr = d.K + r * nv;
          if (lane < nv) d.w[lane] = d.w[lane] + Kr[lane] * delta;
          wsync();
          if (lane == 0) d.efc_f[r] = fnew[0];
          wsync();
        }
        r += 1;
      } else {
        int dim = d.efc_dim[r];
        double res[6], old[6], nw[6], Ab[36];
        const double* blk = d.efc_blk + 36 * r;
        for (int i = 0; i < dim; i++) {
          const double* Ji = d.J + (r + i) * nv;
          double leaf = (lane < nv) ? Ji[lane] * d.w[lane] : 0.0;
          double jw = tree_sum(leaf, P);
          res[i] = (jw + d.efc_R[r + i] * d.efc_f[r + i]) + d.efc_b[r + i];
          old[i] = d.efc_f[r + i];
          for (int j = 0; j < dim; j++) Ab[i * dim + j] = blk[i * dim + j];
          Ab[i * dim + i] = Ab[i * dim + i] + d.efc_R[r + i];
        }
        double fn = old[0] - res[0] / Ab[0];
        if (fn < 0.0) fn = 0.0;
        double dn = fn - old[0];
        nw[0] = fn;
        if (fn == 0.0) {
          for (int j = 1; j < dim; j++) nw[j] = 0.0;
        } else {
          int nf = dim - 1;
          double Ac[25], bq[5];
          for (int i = 0; i < nf; i++) {
            double v = res[1 + i] + Ab[(1 + i) * dim] * dn;
            double s = v;
            for (int j = 0; j < nf; j++) {
              Ac[i * nf + j] = Ab[(1 + i) * dim + 1 + j];
              s = s - Ac[i * nf + j] * old[1 + j];
            }
            bq[i] = s;
          }
          qcqp(nf, Ac, bq, d.efc_mu + 5 * r, fn, nw + 1);
        }
        double del[6];
        for (int i = 0; i < dim; i++) del[i] = nw[i] - old[i];
        double dc = 0.0;
        for (int i = 0; i < dim; i++) {
          double ad = 0.0;
          for (int j = 0; j < dim; j++) ad = ad + Ab[i * dim + j] * del[j];
          dc = dc + del[i] * (0.5 * ad + res[i]);
        }
        improvement = improvement - dc;
        if (lane < nv) {
          double s = d.w[lane];
          for (int i = 0; i < dim; i++) s = s + d.K[(r + i) * nv + lane] * del[i];
          d.w[lane] = s;
        }
        wsync();
        if (lane == 0)
          for (int i = 0; i < dim; i++) d.efc_f[r + i] = nw[i];
        wsync();
        r += dim;
      }
    }
    if (improvement * scale < md.m.tolerance) { it++; break; }
  }
  if (lane == 0) d.ITERS += it;
  // noslip
  for (int ns = 0; ns < md.m.noslip_iterations && ne > 0; ns++) {
    double improvement = 0.0;
    for (int r = 0; r < ne;) {
      int t = d.efc_type[r];
      if (t == MGS_EFC_FRICTION) {
        const double* Jr = d.J + r * nv;
        double leaf = (lane < nv) ? Jr[lane] * d.w[lane] : 0.0;
        double res = tree_sum(leaf, P) + d.efc_b[r];
        double fo = d.efc_f[r];
        double fnew[1] = {fo - res / d.efc_A[r]};
        project_block(d, r, fnew);
        double delta = fnew[0] - fo;
        improvement = improvement - delta * (0.5 * d.efc_A[r] * delta + res);
        if (delta != 0.0) {
          const double* Kr = d.K + r * nv;
          if (lane < nv) d.w[lane] = d.w[lane] + Kr[lane] * delta;
          wsync();
          if (lane == 0) d.efc_f[r] = fnew[0];
          wsync();
        }
        r += 1;
      } else if (t == MGS_EFC_CONTACT && d.efc_dim[r] > 1) {
        int dim = d.efc_dim[r];
        int nf = dim - 1;
        const double* blk = d.efc_blk + 36 * r;
        double res[5], old[5], Ac[25], bq[5], nw[5], del[5];
        for (int i = 0; i < nf; i++) {
          const double* Ji = d.J + (r + 1 + i) * nv;
          double leaf = (lane < nv) ? Ji[lane] * d.w[lane] : 0.0;
          res[i] = tree_sum(leaf, P) + d.efc_b[r + 1 + i];
          old[i] = d.efc_f[r + 1 + i];
        }
        for (int i = 0; i < nf; i++) {
          double s = res[i];
          for (int j = 0; j < nf; j++) {
            Ac[i * nf + j] = blk[(1 + i) * dim + 1 + j];
            s = s - Ac[i * nf + j] * old[j];
          }
          bq[i] = s;
        }
        if (d.efc_f[r] > 0.0) qcqp(nf, Ac, bq, d.efc_mu + 5 * r, d.efc_f[r], nw);
        else for (int i = 0; i < nf; i++) nw[i] = 0.0;
        for (int i = 0; i < nf; i++) del[i] = nw[i] - old[i];
        double dc = 0.0;
        for (int i = 0; i < nf; i++) {
          double ad = 0.0;
          for (int j = 0; j < nf; j++) ad = ad + Ac[i * nf + j] * del[j];
          dc = dc + del[i] * (0.5 * ad + res[i]);
        }
        improvement = improvement - dc;
        if (lane < nv) {
          double s = d.w[lane];
          for (int i = 0; i < nf; i++) s = s + d.K[(r + 1 + i) * nv + lane] * del[i];
          d.w[lane] = s;
        }
        wsync();
        if (lane == 0)
          for (int i = 0; i < nf; i++) d.efc_f[r + 1 + i] = nw[i];
        wsync();
        r += dim;
      } else {
        r += (t == MGS_EFC_CONTACT) ? d.efc_dim[r] : 1;
      }
    }
    if (improvement * scale < md.m.noslip_tolerance) break;
  }
  wsync();
  for (int k = lane; k < nv; k += WAVE) {
    double s = 0.0;
    for (int r = 0; r < ne; r++) s = s + d.J[r * nv + k] * d.efc_f[r];
    d.qfrc_constraint[k] = s;
    d.qacc[k] = d.qacc_smooth[k] + d.w[k];
  }
  wsync();
}

// ---------------------------------------------------------------------------
__device__ void forward(const Mdl& md, Dat& d, int full) {
  int nv = md.m.nv, lane = lane_id();
  if (lane == 0) {
    kinematics(md, d);
    com_pos(md, d);
  }
  wsync();
  collision(md, d);
  if (!full) return;
  crb(md, d);
  ldl_factor(nv, d.M, d.L, d.Dv, d.Dinv);
  if (lane == 0) {
    actuation(md, d);
    passive(md, d);
    rne(md, d);
    for (int k = 0; k < nv; k++) d.qfrc_smooth[k] = (d.qfrc_passive[k] - d.qfrc_bias[k]) + d.qfrc_actuator[k];
    ldl_solve(nv, d.L, d.Dinv, d.qfrc_smooth, d.qacc_smooth);
  }
  wsync();
  make_constraints(md, d);
  solve_pgs(md, d);
}

__device__ void integrate(const Mdl& md, Dat& d) {
  int nv = md.m.nv, lane = lane_id();
  double dt = md.m.timestep;
  if (lane == 0) {
    for (int i = 0; i < nv * nv; i++) d.qDeriv[i] = 0.0;
    const double* damp = DA(md, dof_damping);
    for (int k = 0; k < nv; k++) d.qDeriv[k * nv + k] = -damp[k];
    const int32_t *gtype = IA(md, actuator_gaintype), *btype = IA(md, actuator_biastype);
    const int32_t* flim = IA(md, actuator_forcelimited);
    const double *gain = DA(md, actuator_gainprm), *bias = DA(md, actuator_biasprm);
    const double* frange = DA(md, actuator_forcerange);
    for (int u = 0; u < md.m.nu; u++) {
      double f = d.act_force[u];
      if (flim[u] && (f <= frange[2 * u] || f >= frange[2 * u + 1])) continue;
      double dv = 0.0;
      if (btype[u] == MGS_BIAS_AFFINE) dv = dv + bias[3 * u + 2];
      if (gtype[u] == MGS_GAIN_AFFINE) dv = dv + gain[3 * u + 2] * d.ctrl[u];
      if (dv == 0.0) continue;
      const double* mom = d.act_moment + u * nv;
      for (int i = 0; i < nv; i++) {
        if (mom[i] == 0.0) continue;
        for (int j = 0; j < nv; j++) d.qDeriv[i * nv + j] = d.qDeriv[i * nv + j] + mom[i] * (mom[j] * dv);
      }
    }
  }
  wsync();
  // MI = M - dt*qDeriv (in place into M; M no longer needed this step)
  for (int i = lane; i < nv * nv; i += WAVE) d.M[i] = d.M[i] - dt * d.qDeriv[i];
  wsync();
  ldl_factor(nv, d.M, d.L, d.Dv, d.Dinv);
  if (lane == 0) {
    double rhs[64], qa[64];
    for (int k = 0; k < nv; k++) rhs[k] = d.qfrc_smooth[k] + d.qfrc_constraint[k];
    ldl_solve(nv, d.L, d.Dinv, rhs, qa);
    for (int k = 0; k < nv; k++) d.qvel[k] = d.qvel[k] + dt * qa[k];
    const int32_t *jtype = IA(md, jnt_type), *jq = IA(md, jnt_qposadr), *jd = IA(md, jnt_dofadr);
    for (int j = 0; j < md.m.njnt; j++) {
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
    for (int k = 0; k < nv; k++) d.qacc_ws[k] = d.qacc[k];
    d.time[0] = d.time[0] + dt;
  }
  wsync();
}

__device__ int obj_contact(const Mdl& md, const Dat& d) {
  const int32_t* side = IA(md, geom_side);
  int ncon = d.NCON;
  for (int c = 0; c < ncon; c++) {
    int s1 = side[d.con_g1[c]], s2 = side[d.con_g2[c]];
    if ((s1 < 0 && s2 > 0) || (s1 > 0 && s2 < 0)) return 1;
  }
  return 0;
}

__device__ void reset(const Mdl& md, Dat& d, const double* qpos_init, const double* mpos, const double* mquat) {
  int lane = lane_id();
  for (int k = lane; k < md.m.nq; k += WAVE) d.qpos[k] = qpos_init[k];
  for (int k = lane; k < md.m.nv; k += WAVE) { d.qvel[k] = 0.0; d.qacc_ws[k] = 0.0; }
  if (lane == 0) {
    for (int u = 0; u < (md.m.nu > 0 ? md.m.nu : 1); u++) d.ctrl[u] = 0.0;
    for (int k = 0; k < 3; k++) d.mocap_pos[k] = mpos ? mpos[k] : 0.0;
    for (int k = 0; k < 4; k++) d.mocap_quat[k] = mquat[k];
    d.time[0] = 0.0;
    for (int k = 0; k < 16; k++) d.ints[k] = 0;
  }
  wsync();
}

// ---------------------------------------------------------------------------
// kernels
extern "C" __global__ void __launch_bounds__(64)
mgs_collision_kernel(Mdl md, Lay lay, int n, const double* __restrict__ qpos_init,
                     const double* __restrict__ mocap_pos, const double* __restrict__ mocap_quat, int predicate,
                     uint8_t* __restrict__ out) {
  extern __shared__ double smem[];
  int i = blockIdx.x;
  if (i >= n) return;
  Dat d;
  bind(d, smem, lay);
  reset(md, d, qpos_init + (size_t)i * md.m.nq, mocap_pos + 3 * i, mocap_quat + 4 * i);
  forward(md, d, 0);
  if (lane_id() == 0) {
    int hit = (predicate == MGS_PRED_ANY_CONTACT) ? (d.NCON != 0) : obj_contact(md, d);
    out[i] = (uint8_t)(hit ? 0 : 1);
  }
}

extern "C" __global__ void __launch_bounds__(64)
mgs_rollout_kernel(Mdl md, Lay lay, mgs_schedule sc, int n, const double* __restrict__ qpos_init,
                   const double* __restrict__ mocap_quat, const double* __restrict__ phase_start,
                   const double* __restrict__ phase_target, uint8_t* __restrict__ label,
                   int32_t* __restrict__ fail_step, double* __restrict__ obj_qpos, int32_t* __restrict__ stats) {
  extern __shared__ double smem[];
  int i = blockIdx.x;
  if (i >= n) return;
  int lane = lane_id();
  Dat d;
  bind(d, smem, lay);
  int np = sc.nphase;
  const double* ps = phase_start + (size_t)i * np * 3;
  const double* pt = phase_target + (size_t)i * np * 3;
  reset(md, d, qpos_init + (size_t)i * md.m.nq, ps, mocap_quat + 4 * i);
  int ok = 1, gstep = 0, fstep = -1, maxcon = 0, maxefc = 0;
  for (int p = 0; p < np && ok; p++) {
    if (lane == 0)
      for (int u = 0; u < md.m.nu; u++) d.ctrl[u] = sc.ctrl[p * 32 + u];
    int ns = sc.nsteps[p];
    for (int t = 0; t < ns && ok; t++) {
      double frac = (double)t / (double)ns;
      if (lane == 0)
        for (int k = 0; k < 3; k++) d.mocap_pos[k] = ps[3 * p + k] + (pt[3 * p + k] - ps[3 * p + k]) * frac;
      wsync();
      forward(md, d, 1);
      integrate(md, d);
      if (d.NCON > maxcon) maxcon = d.NCON;
      if (d.NEFC > maxefc) maxefc = d.NEFC;
      int ce = sc.check_every[p];
      if (ce > 0 && t > 0 && (t % ce) == 0 && !obj_contact(md, d)) { ok = 0; fstep = gstep; }
      gstep++;
    }
    if (ok && sc.check_at_end[p] && !obj_contact(md, d)) { ok = 0; fstep = gstep - 1; }
  }
  if (lane == 0) {
    label[i] = (uint8_t)ok;
    if (fail_step) fail_step[i] = fstep;
    if (stats) {
      stats[4 * i] = maxcon; stats[4 * i + 1] = maxefc; stats[4 * i + 2] = d.OVERFLOW; stats[4 * i + 3] = d.ITERS;
    }
  }
  if (obj_qpos && sc.obj_qposadr >= 0 && lane < 7) obj_qpos[7 * i + lane] = d.qpos[sc.obj_qposadr + lane];
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
