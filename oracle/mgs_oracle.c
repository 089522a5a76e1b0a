/*
 * mgs_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this library.  The product path (mj-grasp-sim_amd/, libmgs_gpu.so) never
 * links or calls it.
 *
 * What it restates.  The reference's hot path is
 *   mgs/env/gravityless_object_grasping.py:90-125   grasp_collision_mask
 *   mgs/env/gravityless_object_grasping.py:127-295  grasp_stability_evaluation_from_joints
 *   mgs/gripper/robotiq2f85.py:240-244             close_gripper_at (ctrl 255, mj_step)
 *   mgs/env/gravityless_object_grasping.py:306-320 check_contact / check_contact_with_object
 * and every physics step is `mujoco.mj_step` of MuJoCo 3.2.2 (requirements.txt:1),
 * a third-party C library that is NOT vendored in the reference and not
 * installed here or on the GPU box.  This file restates MuJoCo's documented
 * pipeline for the option set the reference uses (implicitfast, elliptic cones,
 * impratio, noslip, tolerance; gravityless_object_grasping.py:36-42):
 *   mj_kinematics -> mj_comPos -> mj_crb/LDL -> tendon/actuator/passive -> RNE
 *   -> collision (AABB broadphase, MPR narrowphase as in libccd, multi-contact)
 *   -> constraint assembly with solref/solimp impedance -> PGS dual solver with
 *   elliptic cones (QCQP friction blocks) -> noslip -> implicitfast integration.
 * PARITY vs MuJoCo IS UNPINNED (no MuJoCo anywhere, reference has no tests;
 * SURVEY.md §8c).  The harness logic (schedule, checks, labels) is pinned by
 * golden traces of the reference harness (tests/golden/).
 *
 * Numerical contract with the HIP kernel (csrc/mgs_kernels.hip): both are
 * compiled with -ffp-contract=off and evaluate every expression in the order
 * written here; the only cross-lane reduction the kernel uses is tree_dot()
 * below (pairwise tree over the next power of two >= n).  sin/cos come from the
 * polynomial o_sincos() (no libm transcendental), sqrt and division are IEEE.
 * Under this contract the kernel's fp64 results are bit-identical.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/mgs_gpu.h"

#define O_MINVAL 1e-15
#define O_MAXF 16          /* max vertices in a contact feature */
#define O_MAXPOLY 40
#define O_MPR_MAXIT 64
#define O_FEAT_EPS 1e-5
#ifndef BB_MERGE
#define BB_MERGE 1e-6       /* box-box: merge distance of manifold points, x face half size */
#endif
/* separation certificates (kernel cert_*): slots, doubles per slot, least
 * margin kept, validity safety margin */
#define O_CERT 8
#define O_CERT_W 17
#define O_CERT_STORE 1e-6
#define O_CERT_EPS 1e-10

/* ------------------------------------------------------------------------ */
typedef struct {
  const mgs_model_desc* m;
  const int32_t* I;
  const double* D;
} Mdl;

#define IA(md, f) ((md)->I + (md)->m->i_##f)
#define DA(md, f) ((md)->D + (md)->m->d_##f)

typedef struct {
  int nq, nv, nb, ng, nu, ncon_max, nefc_max;
  /* state */
  double *qpos, *qvel, *qacc_ws, *ctrl, *mocap_pos, *mocap_quat;
  double *act, *act_dot;   /* actuator state (mujoco.pid) and its rate */
  double time;
  /* kinematics */
  double *xpos, *xquat, *xmat, *xipos, *ximat, *xanchor, *xaxis;
  double *subtree_com, *subtree_mass, *cinert, *crb, *cdof, *cdof_dot, *cvel, *cacc, *cfrc;
  double *geom_xpos, *geom_xmat;
  /* dynamics */
  double *M, *L, *Dinv, *MI, *LI, *DIinv, *qDeriv;
  double *qfrc_bias, *qfrc_passive, *qfrc_actuator, *qfrc_smooth, *qacc_smooth;
  double *qfrc_constraint, *qacc, *act_force, *act_moment, *act_length, *act_vel;
  /* contacts */
  int ncon;
  double *con_pos, *con_frame, *con_dist;
  int *con_pair, *con_g1, *con_g2;
  /* constraints */
  int nefc;
  double *J, *K, *efc_pos, *efc_margin, *efc_vel, *efc_aref, *efc_R, *efc_A, *efc_b, *efc_f;
  double *efc_mu, *efc_blk, *efc_hb, *efc_dA, *efc_floss, *efc_AR, *efc_ARinv, *efc_Ainv;
  double *efc_Dr, *efc_sqR, *efc_isR, *efc_mup, *efc_k1, *efc_jar, *efc_jv, *hX;
  int* efc_state;
  double *Dv, *sD, *isD;
  int *efc_type, *efc_dim, *efc_con;
  double *w;
  double* cert;      /* O_CERT separation certificate slots */
  int overflow;
  int iters;
  int mask_only;     /* collision without multiccd (oracle_collision_free) */
} Dat;

/* ------------------------------------------------------------------------ */
/* math primitives (ORDER matters: left-to-right as written) */
static void o_sincos(double x, double* s, double* c) {
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

static inline double dot3(const double* a, const double* b) {
  return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2];
}
static inline void cross3(double* r, const double* a, const double* b) {
  double r0 = a[1] * b[2] - a[2] * b[1];
  double r1 = a[2] * b[0] - a[0] * b[2];
  double r2 = a[0] * b[1] - a[1] * b[0];
  r[0] = r0; r[1] = r1; r[2] = r2;
}
static inline void sub3(double* r, const double* a, const double* b) {
  r[0] = a[0] - b[0]; r[1] = a[1] - b[1]; r[2] = a[2] - b[2];
}
static inline void add3(double* r, const double* a, const double* b) {
  r[0] = a[0] + b[0]; r[1] = a[1] + b[1]; r[2] = a[2] + b[2];
}
/* r = m*v, m row-major 3x3 */
static inline void mulmv3(double* r, const double* m, const double* v) {
  double r0 = (m[0] * v[0] + m[1] * v[1]) + m[2] * v[2];
  double r1 = (m[3] * v[0] + m[4] * v[1]) + m[5] * v[2];
  double r2 = (m[6] * v[0] + m[7] * v[1]) + m[8] * v[2];
  r[0] = r0; r[1] = r1; r[2] = r2;
}
/* r = m^T*v */
static inline void mulmtv3(double* r, const double* m, const double* v) {
  double r0 = (m[0] * v[0] + m[3] * v[1]) + m[6] * v[2];
  double r1 = (m[1] * v[0] + m[4] * v[1]) + m[7] * v[2];
  double r2 = (m[2] * v[0] + m[5] * v[1]) + m[8] * v[2];
  r[0] = r0; r[1] = r1; r[2] = r2;
}
static inline void quatmul(double* r, const double* a, const double* b) {
  double r0 = ((a[0] * b[0] - a[1] * b[1]) - a[2] * b[2]) - a[3] * b[3];
  double r1 = ((a[0] * b[1] + a[1] * b[0]) + a[2] * b[3]) - a[3] * b[2];
  double r2 = ((a[0] * b[2] - a[1] * b[3]) + a[2] * b[0]) + a[3] * b[1];
  double r3 = ((a[0] * b[3] + a[1] * b[2]) - a[2] * b[1]) + a[3] * b[0];
  r[0] = r0; r[1] = r1; r[2] = r2; r[3] = r3;
}
static inline void quat2mat(double* m, const double* q) {
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
static inline void normalize4(double* q) {
  double n = sqrt(((q[0] * q[0] + q[1] * q[1]) + q[2] * q[2]) + q[3] * q[3]);
  if (n < O_MINVAL) { q[0] = 1.0; q[1] = q[2] = q[3] = 0.0; return; }
  double inv = 1.0 / n;
  q[0] = q[0] * inv; q[1] = q[1] * inv; q[2] = q[2] * inv; q[3] = q[3] * inv;
}
static inline double normalize3(double* v) {
  double n = sqrt(dot3(v, v));
  if (n < O_MINVAL) { v[0] = 1.0; v[1] = v[2] = 0.0; return 0.0; }
  double inv = 1.0 / n;
  v[0] = v[0] * inv; v[1] = v[1] * inv; v[2] = v[2] * inv;
  return n;
}
static inline void axisangle2quat(double* q, const double* axis, double angle) {
  double s, c;
  o_sincos(0.5 * angle, &s, &c);
  q[0] = c; q[1] = axis[0] * s; q[2] = axis[1] * s; q[3] = axis[2] * s;
}
/* spatial inertia (10) times motion vector (6), MuJoCo layout */
static inline void mul_inert_vec(double* r, const double* i, const double* v) {
  double r0 = ((i[0] * v[0] + i[3] * v[1]) + i[4] * v[2]) - i[8] * v[4] + i[7] * v[5];
  double r1 = ((i[3] * v[0] + i[1] * v[1]) + i[5] * v[2]) + i[8] * v[3] - i[6] * v[5];
  double r2 = ((i[4] * v[0] + i[5] * v[1]) + i[2] * v[2]) - i[7] * v[3] + i[6] * v[4];
  double r3 = (i[8] * v[1] - i[7] * v[2]) + i[9] * v[3];
  double r4 = (i[6] * v[2] - i[8] * v[0]) + i[9] * v[4];
  double r5 = (i[7] * v[0] - i[6] * v[1]) + i[9] * v[5];
  r[0] = r0; r[1] = r1; r[2] = r2; r[3] = r3; r[4] = r4; r[5] = r5;
}
static inline double dot6(const double* a, const double* b) {
  return ((((a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]) + a[3] * b[3]) + a[4] * b[4]) + a[5] * b[5];
}
/* motion cross product v x u (spatial) */
static inline void cross_motion(double* r, const double* v, const double* u) {
  double r0 = v[1] * u[2] - v[2] * u[1];
  double r1 = v[2] * u[0] - v[0] * u[2];
  double r2 = v[0] * u[1] - v[1] * u[0];
  double r3 = (v[1] * u[5] - v[2] * u[4]) + (v[4] * u[2] - v[5] * u[1]);
  double r4 = (v[2] * u[3] - v[0] * u[5]) + (v[5] * u[0] - v[3] * u[2]);
  double r5 = (v[0] * u[4] - v[1] * u[3]) + (v[3] * u[1] - v[4] * u[0]);
  r[0] = r0; r[1] = r1; r[2] = r2; r[3] = r3; r[4] = r4; r[5] = r5;
}
/* force cross product v x* f (spatial) */
static inline void cross_force(double* r, const double* v, const double* f) {
  double r0 = (v[1] * f[2] - v[2] * f[1]) + (v[4] * f[5] - v[5] * f[4]);
  double r1 = (v[2] * f[0] - v[0] * f[2]) + (v[5] * f[3] - v[3] * f[5]);
  double r2 = (v[0] * f[1] - v[1] * f[0]) + (v[3] * f[4] - v[4] * f[3]);
  double r3 = v[1] * f[5] - v[2] * f[4];
  double r4 = v[2] * f[3] - v[0] * f[5];
  double r5 = v[0] * f[4] - v[1] * f[3];
  r[0] = r0; r[1] = r1; r[2] = r2; r[3] = r3; r[4] = r4; r[5] = r5;
}

/* Pairwise tree sum of a[k]*b[k], k < n, over P leaves (P = next pow2 >= n,
 * zero leaves beyond n): level s = 1,2,4,...: leaf[k] = leaf[k] + leaf[k^s].
 * This is the kernel's wave reduction over lanes (DPP butterfly). */
static double tree_dot(const double* a, const double* b, int n) {
  double leaf[128];
  int P = 1;
  while (P < n) P <<= 1;
  for (int k = 0; k < P; k++) leaf[k] = (k < n) ? a[k] * b[k] : 0.0;
  for (int s = 1; s < P; s <<= 1) {
    double nxt[128];
    for (int k = 0; k < P; k++) nxt[k] = leaf[k] + leaf[k ^ s];
    memcpy(leaf, nxt, sizeof(double) * P);
  }
  return leaf[0];
}

/* ------------------------------------------------------------------------ */
/* allocation */
static Dat* dat_alloc(const Mdl* md) {
  const mgs_model_desc* m = md->m;
  Dat* d = (Dat*)calloc(1, sizeof(Dat));
  d->nq = m->nq; d->nv = m->nv; d->nb = m->nbody; d->ng = m->ngeom; d->nu = m->nu;
  d->ncon_max = m->ncon_max; d->nefc_max = m->nefc_max;
  int nq = m->nq, nv = m->nv, nb = m->nbody, ng = m->ngeom, nu = m->nu > 0 ? m->nu : 1;
  int nc = m->ncon_max, ne = m->nefc_max, nj = m->njnt > 0 ? m->njnt : 1;
  /* pass 0 counts, pass 1 assigns: one list of fields, no separate size table */
  double* base = NULL;
  for (int pass = 0; pass < 2; pass++) {
  double* p = base;
  size_t tot = 0;
#define TAKE(ptr, n) do { d->ptr = p; if (p) p += (n); tot += (size_t)(n); } while (0)
  TAKE(qpos, nq); TAKE(qvel, nv); TAKE(qacc_ws, nv); TAKE(ctrl, nu);
  TAKE(act, m->nact > 0 ? m->nact : 1); TAKE(act_dot, m->nact > 0 ? m->nact : 1);
  TAKE(mocap_pos, 3 * m->nmocap + 3); TAKE(mocap_quat, 4 * m->nmocap + 4);
  TAKE(xpos, 3 * nb); TAKE(xquat, 4 * nb); TAKE(xmat, 9 * nb); TAKE(xipos, 3 * nb); TAKE(ximat, 9 * nb);
  TAKE(xanchor, 3 * nj); TAKE(xaxis, 3 * nj);
  TAKE(subtree_com, 3 * nb); TAKE(subtree_mass, nb); TAKE(cinert, 10 * nb); TAKE(crb, 10 * nb);
  TAKE(cdof, 6 * nv); TAKE(cdof_dot, 6 * nv); TAKE(cvel, 6 * nb); TAKE(cacc, 6 * nb); TAKE(cfrc, 6 * nb);
  TAKE(geom_xpos, 3 * ng); TAKE(geom_xmat, 9 * ng);
  TAKE(M, nv * nv); TAKE(L, nv * nv); TAKE(Dinv, nv); TAKE(MI, nv * nv); TAKE(LI, nv * nv);
  TAKE(DIinv, nv); TAKE(qDeriv, nv * nv);
  TAKE(qfrc_bias, nv); TAKE(qfrc_passive, nv); TAKE(qfrc_actuator, nv); TAKE(qfrc_smooth, nv);
  TAKE(qacc_smooth, nv); TAKE(qfrc_constraint, nv); TAKE(qacc, nv);
  TAKE(act_force, nu); TAKE(act_moment, nu * nv); TAKE(act_length, nu); TAKE(act_vel, nu);
  TAKE(con_pos, 3 * nc); TAKE(con_frame, 9 * nc); TAKE(con_dist, nc);
  TAKE(J, ne * nv); TAKE(K, ne * nv); TAKE(efc_pos, ne); TAKE(efc_margin, ne); TAKE(efc_vel, ne);
  TAKE(efc_aref, ne); TAKE(efc_R, ne); TAKE(efc_A, ne); TAKE(efc_b, ne); TAKE(efc_f, ne);
  TAKE(efc_mu, 5 * ne); TAKE(efc_blk, 36 * ne); TAKE(efc_hb, 36 * ne); TAKE(efc_dA, ne); TAKE(efc_floss, ne); TAKE(w, nv);
  TAKE(efc_AR, ne); TAKE(efc_ARinv, ne); TAKE(efc_Ainv, ne); TAKE(Dv, nv); TAKE(sD, nv); TAKE(isD, nv);
  TAKE(efc_Dr, ne); TAKE(efc_sqR, ne); TAKE(efc_isR, ne); TAKE(efc_mup, ne); TAKE(efc_k1, ne); TAKE(efc_jar, ne); TAKE(efc_jv, ne); TAKE(hX, ne * nv);
  TAKE(cert, O_CERT * O_CERT_W);
#undef TAKE
  if (pass == 0) base = (double*)calloc(tot, sizeof(double));
  }
  d->con_pair = (int*)calloc((size_t)nc, sizeof(int));
  d->con_g1 = (int*)calloc((size_t)nc, sizeof(int));
  d->con_g2 = (int*)calloc((size_t)nc, sizeof(int));
  d->efc_type = (int*)calloc((size_t)ne, sizeof(int));
  d->efc_dim = (int*)calloc((size_t)ne, sizeof(int));
  d->efc_con = (int*)calloc((size_t)ne, sizeof(int));
  d->efc_state = (int*)calloc((size_t)ne, sizeof(int));
  return d;
}

static void dat_free(Dat* d) {
  if (!d) return;
  free(d->qpos);
  free(d->con_pair); free(d->con_g1); free(d->con_g2);
  free(d->efc_type); free(d->efc_dim); free(d->efc_con); free(d->efc_state);
  free(d);
}

/* ------------------------------------------------------------------------ */
/* mj_kinematics */
static void kinematics(const Mdl* md, Dat* d) {
  const mgs_model_desc* m = md->m;
  const int32_t *parent = IA(md, body_parentid), *mocapid = IA(md, body_mocapid);
  const int32_t *jntnum = IA(md, body_jntnum), *jntadr = IA(md, body_jntadr);
  const int32_t *jtype = IA(md, jnt_type), *qadr = IA(md, jnt_qposadr);
  const double *bpos = DA(md, body_pos), *bquat = DA(md, body_quat);
  const double *ipos = DA(md, body_ipos), *iquat = DA(md, body_iquat);
  const double *jpos = DA(md, jnt_pos), *jaxis = DA(md, jnt_axis), *qpos0 = DA(md, qpos0);
  d->xpos[0] = d->xpos[1] = d->xpos[2] = 0.0;
  d->xquat[0] = 1.0; d->xquat[1] = d->xquat[2] = d->xquat[3] = 0.0;
  quat2mat(d->xmat, d->xquat);
  for (int b = 1; b < m->nbody; b++) {
    double pos[3], quat[4], mat[9];
    if (mocapid[b] >= 0) {
      const double* mp = d->mocap_pos + 3 * mocapid[b];
      const double* mq = d->mocap_quat + 4 * mocapid[b];
      pos[0] = mp[0]; pos[1] = mp[1]; pos[2] = mp[2];
      quat[0] = mq[0]; quat[1] = mq[1]; quat[2] = mq[2]; quat[3] = mq[3];
      normalize4(quat);
    } else {
      int p = parent[b];
      double t[3];
      mulmv3(t, d->xmat + 9 * p, bpos + 3 * b);
      add3(pos, d->xpos + 3 * p, t);
      quatmul(quat, d->xquat + 4 * p, bquat + 4 * b);
      for (int k = 0; k < jntnum[b]; k++) {
        int j = jntadr[b] + k;
        int a = qadr[j];
        if (jtype[j] == MGS_JNT_FREE) {
          pos[0] = d->qpos[a]; pos[1] = d->qpos[a + 1]; pos[2] = d->qpos[a + 2];
          quat[0] = d->qpos[a + 3]; quat[1] = d->qpos[a + 4]; quat[2] = d->qpos[a + 5]; quat[3] = d->qpos[a + 6];
          normalize4(quat);
          d->xanchor[3 * j] = pos[0]; d->xanchor[3 * j + 1] = pos[1]; d->xanchor[3 * j + 2] = pos[2];
          d->xaxis[3 * j] = 0.0; d->xaxis[3 * j + 1] = 0.0; d->xaxis[3 * j + 2] = 1.0;
        } else {
          quat2mat(mat, quat);
          mulmv3(d->xaxis + 3 * j, mat, jaxis + 3 * j);
          mulmv3(t, mat, jpos + 3 * j);
          add3(d->xanchor + 3 * j, t, pos);
          if (jtype[j] == MGS_JNT_HINGE) {
            double ql[4], qn[4];
            axisangle2quat(ql, jaxis + 3 * j, d->qpos[a] - qpos0[a]);
            quatmul(qn, quat, ql);
            quat[0] = qn[0]; quat[1] = qn[1]; quat[2] = qn[2]; quat[3] = qn[3];
            quat2mat(mat, quat);
            mulmv3(t, mat, jpos + 3 * j);
            sub3(pos, d->xanchor + 3 * j, t);
          } else { /* slide */
            double dq = d->qpos[a] - qpos0[a];
            pos[0] = pos[0] + d->xaxis[3 * j] * dq;
            pos[1] = pos[1] + d->xaxis[3 * j + 1] * dq;
            pos[2] = pos[2] + d->xaxis[3 * j + 2] * dq;
          }
        }
      }
      normalize4(quat);
    }
    d->xpos[3 * b] = pos[0]; d->xpos[3 * b + 1] = pos[1]; d->xpos[3 * b + 2] = pos[2];
    d->xquat[4 * b] = quat[0]; d->xquat[4 * b + 1] = quat[1]; d->xquat[4 * b + 2] = quat[2]; d->xquat[4 * b + 3] = quat[3];
    quat2mat(d->xmat + 9 * b, quat);
    double t[3], qi[4];
    mulmv3(t, d->xmat + 9 * b, ipos + 3 * b);
    add3(d->xipos + 3 * b, d->xpos + 3 * b, t);
    quatmul(qi, quat, iquat + 4 * b);
    quat2mat(d->ximat + 9 * b, qi);
  }
  /* geoms */
  const int32_t* gbody = IA(md, geom_bodyid);
  const double *gpos = DA(md, geom_pos), *gquat = DA(md, geom_quat);
  for (int g = 0; g < m->ngeom; g++) {
    int b = gbody[g];
    double t[3], q[4];
    mulmv3(t, d->xmat + 9 * b, gpos + 3 * g);
    add3(d->geom_xpos + 3 * g, d->xpos + 3 * b, t);
    quatmul(q, d->xquat + 4 * b, gquat + 4 * g);
    quat2mat(d->geom_xmat + 9 * g, q);
  }
}

/* mj_comPos: subtree com, cinert, cdof */
static void com_pos(const Mdl* md, Dat* d) {
  const mgs_model_desc* m = md->m;
  const int32_t *parent = IA(md, body_parentid), *rootid = IA(md, body_rootid);
  const int32_t *jntnum = IA(md, body_jntnum), *jntadr = IA(md, body_jntadr);
  const int32_t *jtype = IA(md, jnt_type), *dadr = IA(md, jnt_dofadr);
  const double *mass = DA(md, body_mass), *inertia = DA(md, body_inertia);
  int nb = m->nbody;
  for (int b = 0; b < nb; b++) {
    d->subtree_mass[b] = mass[b];
    d->subtree_com[3 * b] = mass[b] * d->xipos[3 * b];
    d->subtree_com[3 * b + 1] = mass[b] * d->xipos[3 * b + 1];
    d->subtree_com[3 * b + 2] = mass[b] * d->xipos[3 * b + 2];
  }
  for (int b = nb - 1; b > 0; b--) {
    int p = parent[b];
    d->subtree_mass[p] = d->subtree_mass[p] + d->subtree_mass[b];
    d->subtree_com[3 * p] = d->subtree_com[3 * p] + d->subtree_com[3 * b];
    d->subtree_com[3 * p + 1] = d->subtree_com[3 * p + 1] + d->subtree_com[3 * b + 1];
    d->subtree_com[3 * p + 2] = d->subtree_com[3 * p + 2] + d->subtree_com[3 * b + 2];
  }
  for (int b = 0; b < nb; b++) {
    if (d->subtree_mass[b] < O_MINVAL) {
      d->subtree_com[3 * b] = d->xipos[3 * b];
      d->subtree_com[3 * b + 1] = d->xipos[3 * b + 1];
      d->subtree_com[3 * b + 2] = d->xipos[3 * b + 2];
    } else {
      double inv = 1.0 / d->subtree_mass[b];
      d->subtree_com[3 * b] = d->subtree_com[3 * b] * inv;
      d->subtree_com[3 * b + 1] = d->subtree_com[3 * b + 1] * inv;
      d->subtree_com[3 * b + 2] = d->subtree_com[3 * b + 2] * inv;
    }
  }
  for (int b = 0; b < nb; b++) {
    double* ci = d->cinert + 10 * b;
    const double* R = d->ximat + 9 * b;
    const double* in = inertia + 3 * b;
    double mm = mass[b];
    double off[3];
    sub3(off, d->xipos + 3 * b, d->subtree_com + 3 * rootid[b]);
    /* tmp = R diag(in) R^T */
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
    const double* c = d->subtree_com + 3 * rootid[b];
    for (int k = 0; k < jntnum[b]; k++) {
      int j = jntadr[b] + k;
      int da = dadr[j];
      double off[3];
      sub3(off, c, d->xanchor + 3 * j);
      if (jtype[j] == MGS_JNT_FREE) {
        for (int i = 0; i < 3; i++) {
          double* cd = d->cdof + 6 * (da + i);
          cd[0] = cd[1] = cd[2] = 0.0;
          cd[3] = (i == 0) ? 1.0 : 0.0; cd[4] = (i == 1) ? 1.0 : 0.0; cd[5] = (i == 2) ? 1.0 : 0.0;
        }
        const double* R = d->xmat + 9 * b;
        for (int i = 0; i < 3; i++) {
          double* cd = d->cdof + 6 * (da + 3 + i);
          double ax[3] = {R[i], R[3 + i], R[6 + i]};
          cd[0] = ax[0]; cd[1] = ax[1]; cd[2] = ax[2];
          cross3(cd + 3, ax, off);
        }
      } else if (jtype[j] == MGS_JNT_HINGE) {
        double* cd = d->cdof + 6 * da;
        const double* ax = d->xaxis + 3 * j;
        cd[0] = ax[0]; cd[1] = ax[1]; cd[2] = ax[2];
        cross3(cd + 3, ax, off);
      } else { /* slide */
        double* cd = d->cdof + 6 * da;
        const double* ax = d->xaxis + 3 * j;
        cd[0] = cd[1] = cd[2] = 0.0;
        cd[3] = ax[0]; cd[4] = ax[1]; cd[5] = ax[2];
      }
    }
  }
}

/* mj_crb + armature -> M (dense) */
static void crb(const Mdl* md, Dat* d) {
  const mgs_model_desc* m = md->m;
  int nb = m->nbody, nv = m->nv;
  const int32_t *parent = IA(md, body_parentid), *dbody = IA(md, dof_bodyid), *dpar = IA(md, dof_parentid);
  const double* arm = DA(md, dof_armature);
  memcpy(d->crb, d->cinert, sizeof(double) * 10 * nb);
  for (int b = nb - 1; b > 0; b--) {
    int p = parent[b];
    if (p > 0)
      for (int k = 0; k < 10; k++) d->crb[10 * p + k] = d->crb[10 * p + k] + d->crb[10 * b + k];
  }
  memset(d->M, 0, sizeof(double) * nv * nv);
  for (int i = 0; i < nv; i++) {
    double buf[6];
    mul_inert_vec(buf, d->crb + 10 * dbody[i], d->cdof + 6 * i);
    d->M[i * nv + i] = dot6(d->cdof + 6 * i, buf) + arm[i];
    int j = dpar[i];
    while (j >= 0) {
      double v = dot6(d->cdof + 6 * j, buf);
      d->M[i * nv + j] = v;
      d->M[j * nv + i] = v;
      j = dpar[j];
    }
  }
}

/* dense LDL^T: A = L D L^T, L unit lower (stored strictly lower), Dinv = 1/D */
static void ldl_factor(int n, const double* A, double* L, double* Dinv, double* Dv) {
  double W[128];
  for (int j = 0; j < n; j++) {
    for (int k = 0; k < j; k++) W[k] = L[j * n + k] * Dv[k];
    double dj = A[j * n + j];
    for (int k = 0; k < j; k++) dj = fma(-W[k], L[j * n + k], dj);
    Dv[j] = dj;
    Dinv[j] = 1.0 / dj;
    for (int i = j + 1; i < n; i++) {
      double s = A[i * n + j];
      for (int k = 0; k < j; k++) s = fma(-L[i * n + k], W[k], s);
      L[i * n + j] = s * Dinv[j];
    }
  }
}
static void ldl_solve(int n, const double* L, const double* Dinv, const double* b, double* x) {
  double y[128];
  for (int i = 0; i < n; i++) {
    double s = b[i];
    for (int k = 0; k < i; k++) s = fma(-L[i * n + k], y[k], s);
    y[i] = s;
  }
  /* backward substitution, k descending (the kernel's column order) */
  for (int i = n - 1; i >= 0; i--) {
    double s = y[i] * Dinv[i];
    for (int k = n - 1; k > i; k--) s = fma(-L[k * n + i], x[k], s);
    x[i] = s;
  }
}

/* MuJoCo's mujoco.pid actuator plugin, restated from its documented
 * semantics (parity unpinned: the plugin's source is not in the reference or
 * this image).  pidprm = kp, ki, kd, imax, slewmax (imax / slewmax < 0: not
 * set).  Setpoint: the clamped ctrl, held within slewmax dt of the previous
 * setpoint (act entry 0 when slewmax is set); error = setpoint - length;
 * force = kp error + kd (setpoint rate - velocity) + ki integral (the next act
 * entry when ki != 0).  act_dot: the setpoint rate and the error, advanced by
 * integrate() (mj_advance) with the integral clamped to |ki integral| <= imax. */
static double pid_force(const Mdl* md, Dat* d, int u, double c, double len, double vel) {
  const double* pp = DA(md, actuator_pidprm) + 5 * u;
  const double dt = md->m->timestep;
  int k = IA(md, actuator_actadr)[u];
  double cdot = 0.0;
  if (pp[4] >= 0.0) {
    const double prev = d->act[k];
    const double lo = prev - pp[4] * dt, hi = prev + pp[4] * dt;
    if (c < lo) c = lo;
    if (c > hi) c = hi;
    cdot = (c - prev) / dt;
    d->act_dot[k] = cdot;
    k++;
  }
  const double err = c - len;
  double f = pp[0] * err + pp[2] * (cdot - vel);
  if (pp[1] != 0.0) {
    f = f + pp[1] * d->act[k];
    d->act_dot[k] = err;
  }
  return f;
}

/* tendon length/moment, actuator length/moment/velocity/force, qfrc_actuator */
static void actuation(const Mdl* md, Dat* d) {
  const mgs_model_desc* m = md->m;
  int nv = m->nv;
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
  for (int k = 0; k < nv; k++) d->qfrc_actuator[k] = 0.0;
  for (int u = 0; u < m->nu; u++) {
    double* mom = d->act_moment + u * nv;
    for (int k = 0; k < nv; k++) mom[k] = 0.0;
    double len;
    if (trntype[u] == MGS_TRN_JOINT) {
      int j = trnid[u];
      len = d->qpos[jq[j]] * gear[u];
      mom[jd[j]] = gear[u];
    } else {
      int t = trnid[u];
      double tl = 0.0;
      for (int w = tadr[t]; w < tadr[t] + tnum[t]; w++) {
        tl = tl + wcoef[w] * d->qpos[wq[w]];
        mom[wdof[w]] = mom[wdof[w]] + wcoef[w] * gear[u];
      }
      len = tl * gear[u];
    }
    double vel = 0.0;
    for (int k = 0; k < nv; k++) vel = vel + mom[k] * d->qvel[k];
    d->act_length[u] = len;
    d->act_vel[u] = vel;
    double c = d->ctrl[u];
    if (clim[u]) {
      if (c < crange[2 * u]) c = crange[2 * u];
      if (c > crange[2 * u + 1]) c = crange[2 * u + 1];
    }
    double f;
    if (gtype[u] == MGS_GAIN_PID) {
      f = pid_force(md, d, u, c, len, vel);
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
    d->act_force[u] = f;
    for (int k = 0; k < nv; k++) d->qfrc_actuator[k] = d->qfrc_actuator[k] + mom[k] * f;
  }
}

/* joint springs and dof damping */
static void passive(const Mdl* md, Dat* d) {
  const mgs_model_desc* m = md->m;
  const int32_t *jtype = IA(md, jnt_type), *jq = IA(md, jnt_qposadr), *jd = IA(md, jnt_dofadr);
  const double *stiff = DA(md, jnt_stiffness), *qspring = DA(md, qpos_spring), *damp = DA(md, dof_damping);
  for (int k = 0; k < m->nv; k++) d->qfrc_passive[k] = 0.0;
  for (int j = 0; j < m->njnt; j++) {
    if (stiff[j] == 0.0) continue;
    if (jtype[j] == MGS_JNT_HINGE || jtype[j] == MGS_JNT_SLIDE)
      d->qfrc_passive[jd[j]] = -stiff[j] * (d->qpos[jq[j]] - qspring[jq[j]]);
  }
  for (int k = 0; k < m->nv; k++) d->qfrc_passive[k] = d->qfrc_passive[k] - damp[k] * d->qvel[k];
  /* gravity compensation (MuJoCo mj_gravcomp: mj_applyFT of -gravity mass
   * gravcomp at xipos, added to qfrc_passive; parity unpinned -- only the
   * dexee's bodies carry gravcomp and no reference vector covers it).  With h
   * = mass (xipos - subtree_com) = cinert[6..8], a dof's Jacobian column
   * dotted with the force is -gravcomp ((g . cdof_lin) mass + g . (cdof_ang x h)),
   * summed over bodies in order. */
  const double* g = m->gravity;
  if (g[0] != 0.0 || g[1] != 0.0 || g[2] != 0.0) {
    const double* gc = DA(md, body_gravcomp);
    const int32_t *last = IA(md, body_lastdof), *dpar = IA(md, dof_parentid);
    double acc[128] = {0};
    int any[128] = {0};
    for (int b = 1; b < m->nbody; b++) {
      if (gc[b] == 0.0) continue;
      const double* ci = d->cinert + 10 * b;
      for (int k = last[b]; k >= 0; k = dpar[k]) {
        const double* cd = d->cdof + 6 * k;
        double cr[3];
        cross3(cr, cd, ci + 6);
        double t = ((g[0] * cd[3] + g[1] * cd[4]) + g[2] * cd[5]) * ci[9] + ((g[0] * cr[0] + g[1] * cr[1]) + g[2] * cr[2]);
        acc[k] = acc[k] + (-gc[b]) * t;
        any[k] = 1;
      }
    }
    for (int k = 0; k < m->nv; k++)
      if (any[k]) d->qfrc_passive[k] = d->qfrc_passive[k] + acc[k];
  }
}

/* mj_comVel + mj_rne (no acceleration term) -> qfrc_bias */
static void rne(const Mdl* md, Dat* d) {
  const mgs_model_desc* m = md->m;
  int nb = m->nbody;
  const int32_t *parent = IA(md, body_parentid), *dnum = IA(md, body_dofnum), *dadr = IA(md, body_dofadr);
  const int32_t* dbody = IA(md, dof_bodyid);
  for (int k = 0; k < 6; k++) { d->cvel[k] = 0.0; d->cacc[k] = 0.0; }
  d->cacc[3] = -m->gravity[0]; d->cacc[4] = -m->gravity[1]; d->cacc[5] = -m->gravity[2];
  for (int b = 1; b < nb; b++) {
    int p = parent[b];
    double* cv = d->cvel + 6 * b;
    double* ca = d->cacc + 6 * b;
    for (int k = 0; k < 6; k++) { cv[k] = d->cvel[6 * p + k]; ca[k] = d->cacc[6 * p + k]; }
    for (int i = 0; i < dnum[b]; i++) {
      int dd = dadr[b] + i;
      cross_motion(d->cdof_dot + 6 * dd, cv, d->cdof + 6 * dd);
      for (int k = 0; k < 6; k++) cv[k] = cv[k] + d->cdof[6 * dd + k] * d->qvel[dd];
    }
    for (int i = 0; i < dnum[b]; i++) {
      int dd = dadr[b] + i;
      for (int k = 0; k < 6; k++) ca[k] = ca[k] + d->cdof_dot[6 * dd + k] * d->qvel[dd];
    }
    double f1[6], f2[6], f3[6];
    mul_inert_vec(f1, d->cinert + 10 * b, ca);
    mul_inert_vec(f2, d->cinert + 10 * b, cv);
    cross_force(f3, cv, f2);
    for (int k = 0; k < 6; k++) d->cfrc[6 * b + k] = f1[k] + f3[k];
  }
  for (int b = nb - 1; b > 0; b--) {
    int p = parent[b];
    if (p > 0)
      for (int k = 0; k < 6; k++) d->cfrc[6 * p + k] = d->cfrc[6 * p + k] + d->cfrc[6 * b + k];
  }
  for (int i = 0; i < m->nv; i++) d->qfrc_bias[i] = dot6(d->cdof + 6 * i, d->cfrc + 6 * dbody[i]);
}

/* ------------------------------------------------------------------------ */
/* collision */
typedef struct { double v[3], a[3], b[3]; } SupPt;

/* support point of geom g along world direction dir; returns vertex index */
static long g_sup_calls;   /* diagnostics: support calls (single-threaded use) */
int g_sep_log; long g_sep_n; double g_sep_val[200000]; int g_sep_pair[200000];
double* oracle_sep_vals(void) { return g_sep_val; }
int* oracle_sep_pairs(void) { return g_sep_pair; }
long oracle_sep_count(void) { return g_sep_n; }
void oracle_sep_enable(int on) { g_sep_log = on; g_sep_n = 0; }
/* exact cylinder support in the geom frame (MuJoCo's ccd support of
 * mjGEOM_CYLINDER, engine_collision_convex.c): the rim point along the radial
 * part of dl, on the cap dl points to; (0, 0, +-h) when dl is along the axis */
static void cyl_support(double* v, const double* cy, const double* dl) {
  // MuJoCo's operation order (dir / length * size) and mju_sign (0 at 0)
  double rho = sqrt(dl[0] * dl[0] + dl[1] * dl[1]);
  if (rho > O_MINVAL) {
    v[0] = dl[0] / rho * cy[0];
    v[1] = dl[1] / rho * cy[0];
  } else {
    v[0] = 0.0;
    v[1] = 0.0;
  }
  v[2] = dl[2] > 0.0 ? cy[1] : (dl[2] < 0.0 ? -cy[1] : 0.0);
}

/* support of geom g posed at (R, x) along the unit world direction dir */
static int support_pose(const Mdl* md, int g, const double* R, const double* x, const double* dir, double* out) {
  int h = IA(md, geom_hullid)[g];
  int adr = IA(md, hull_vertadr)[h], num = IA(md, hull_vertnum)[h];
  const double* V = DA(md, hull_vert) + 3 * adr;
  double dl[3];
  mulmtv3(dl, R, dir);
  double best = -INFINITY;
  int bi = 0;
  for (int i = 0; i < num; i++) {
    double s = (V[i] * dl[0] + V[num + i] * dl[1]) + V[2 * num + i] * dl[2];
    if (s > best) { best = s; bi = i; }
  }
  double t[3], vb[3] = {V[bi], V[num + bi], V[2 * num + bi]};
  const double* cy = DA(md, geom_cyl) + 2 * g;
  if (cy[0] > 0.0) cyl_support(vb, cy, dl);
  mulmv3(t, R, vb);
  add3(out, x, t);
  /* rounded geoms (sphere, capsule): hull (+) ball; dir is a unit vector */
  double r = DA(md, geom_radius)[g];
  if (r > 0.0) { out[0] = out[0] + r * dir[0]; out[1] = out[1] + r * dir[1]; out[2] = out[2] + r * dir[2]; }
  return bi;
}

static int support_geom(const Mdl* md, const Dat* d, int g, const double* dir, double* out) {
  return support_pose(md, g, d->geom_xmat + 9 * g, d->geom_xpos + 3 * g, dir, out);
}

static void mink_support(const Mdl* md, const Dat* d, int g1, int g2, const double* dir, SupPt* p) {
  g_sup_calls++;
  double nd[3] = {-dir[0], -dir[1], -dir[2]};
  support_geom(md, d, g1, dir, p->a);
  support_geom(md, d, g2, nd, p->b);
  sub3(p->v, p->a, p->b);
}

static void portal_normal(double* n, const SupPt* p1, const SupPt* p2, const SupPt* p3) {
  double e1[3], e2[3];
  sub3(e1, p2->v, p1->v);
  sub3(e2, p3->v, p1->v);
  cross3(n, e1, e2);
  normalize3(n);
}

static int portal_reach_tol(const SupPt* p1, const SupPt* p2, const SupPt* p3, const SupPt* p4,
                            const double* n, double tol) {
  double dv4 = dot3(p4->v, n);
  double t1 = dv4 - dot3(p1->v, n);
  double t2 = dv4 - dot3(p2->v, n);
  double t3 = dv4 - dot3(p3->v, n);
  double mn = t1 < t2 ? t1 : t2;
  mn = mn < t3 ? mn : t3;
  return mn <= tol;
}

static void portal_expand(SupPt* p0, SupPt* p1, SupPt* p2, SupPt* p3, const SupPt* p4) {
  double c[3];
  cross3(c, p4->v, p0->v);
  if (dot3(p1->v, c) > 0.0) {
    if (dot3(p2->v, c) > 0.0) *p1 = *p4; else *p3 = *p4;
  } else {
    if (dot3(p3->v, c) > 0.0) *p2 = *p4; else *p1 = *p4;
  }
}

/* Minkowski Portal Refinement (penetration variant, as in libccd, which
 * MuJoCo 3.2.x uses for convex mesh collisions).  Returns 1 on penetration
 * with unit normal n (from geom g1 towards g2), depth > 0 and point pos. */
/* On a miss certified by a separating direction (support of the Minkowski
 * difference along dir <= 0): *cm = -h(dir) >= 0, cd = dir; else *cm = -1. */
#define MPR_CERT(P) do { *cm = -dot3((P).v, dir); cd[0] = dir[0]; cd[1] = dir[1]; cd[2] = dir[2]; } while (0)
static int mpr_penetration(const Mdl* md, const Dat* d, int g1, int g2, double* n, double* depth,
                           double* pos, double* cd, double* cm) {
  *cm = -1.0;
  const double tol = md->m->mpr_tolerance;
  const int32_t* ghull = IA(md, geom_hullid);
  const double* HC = DA(md, hull_center);
  SupPt p0, p1, p2, p3, p4;
  double t[3], dir[3];
  mulmv3(t, d->geom_xmat + 9 * g1, HC + 3 * ghull[g1]);
  add3(p0.a, d->geom_xpos + 3 * g1, t);
  mulmv3(t, d->geom_xmat + 9 * g2, HC + 3 * ghull[g2]);
  add3(p0.b, d->geom_xpos + 3 * g2, t);
  sub3(p0.v, p0.a, p0.b);
  if (p0.v[0] == 0.0 && p0.v[1] == 0.0 && p0.v[2] == 0.0) p0.v[0] = 1e-9;
  dir[0] = -p0.v[0]; dir[1] = -p0.v[1]; dir[2] = -p0.v[2];
  normalize3(dir);
  mink_support(md, d, g1, g2, dir, &p1);
  if (g_sep_log && g_sep_n < 200000) { g_sep_val[g_sep_n] = dot3(p1.v, dir); g_sep_pair[g_sep_n] = g1 * 64 + g2; g_sep_n++; }
  if (dot3(p1.v, dir) <= 0.0) { MPR_CERT(p1); return 0; }
  cross3(dir, p0.v, p1.v);
  if (dot3(dir, dir) < 1e-30) {
    /* origin on segment v0-v1 */
    double nn = sqrt(dot3(p1.v, p1.v));
    if (nn < O_MINVAL) return 0;
    n[0] = p1.v[0] / nn; n[1] = p1.v[1] / nn; n[2] = p1.v[2] / nn;
    *depth = nn;
    pos[0] = 0.5 * (p1.a[0] + p1.b[0]); pos[1] = 0.5 * (p1.a[1] + p1.b[1]); pos[2] = 0.5 * (p1.a[2] + p1.b[2]);
    return 1;
  }
  normalize3(dir);
  mink_support(md, d, g1, g2, dir, &p2);
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
  for (it = 0; it < O_MPR_MAXIT; it++) {
    mink_support(md, d, g1, g2, dir, &p3);
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
  if (it == O_MPR_MAXIT) return 0;
  /* refine until the portal encloses the origin */
  for (it = 0; it < O_MPR_MAXIT; it++) {
    portal_normal(dir, &p1, &p2, &p3);
    if (dot3(dir, p1.v) >= 0.0) break;
    mink_support(md, d, g1, g2, dir, &p4);
    if (dot3(p4.v, dir) < 0.0) { MPR_CERT(p4); return 0; }
    if (portal_reach_tol(&p1, &p2, &p3, &p4, dir, tol)) return 0;
    portal_expand(&p0, &p1, &p2, &p3, &p4);
  }
  if (it == O_MPR_MAXIT) return 0;
  /* penetration */
  for (it = 0;; it++) {
    portal_normal(dir, &p1, &p2, &p3);
    mink_support(md, d, g1, g2, dir, &p4);
    if (it >= O_MPR_MAXIT || portal_reach_tol(&p1, &p2, &p3, &p4, dir, tol)) {
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

#undef MPR_CERT

static void make_frame(const double* n, double* t1, double* t2) {
  double a[3];
  /* mju_makeFrame: tangent seed (0,1,0) unless |n_y| >= 0.5, then (0,0,1) */
  if (n[1] < 0.5 && n[1] > -0.5) { a[0] = 0.0; a[1] = 1.0; a[2] = 0.0; }
  else { a[0] = 0.0; a[1] = 0.0; a[2] = 1.0; }
  double an = dot3(a, n);
  t1[0] = a[0] - n[0] * an; t1[1] = a[1] - n[1] * an; t1[2] = a[2] - n[2] * an;
  normalize3(t1);
  cross3(t2, n, t1);
}

typedef struct { double x, y, h; } P2;

/* collect the vertices of geom g whose height along n is within tol of the
 * extreme (sign=+1: max, sign=-1: min); returns count (<= O_MAXF) and extreme */
static int feature(const Mdl* md, const Dat* d, int g, const double* n, const double* t1, const double* t2,
                   int sign, double tol, P2* out, double* ext) {
  int h = IA(md, geom_hullid)[g];
  int adr = IA(md, hull_vertadr)[h], num = IA(md, hull_vertnum)[h];
  const double* V = DA(md, hull_vert) + 3 * adr;
  const double* R = d->geom_xmat + 9 * g;
  const double* x = d->geom_xpos + 3 * g;
  double nl[3];
  mulmtv3(nl, R, n);
  double base = dot3(x, n);
  double r = DA(md, geom_radius)[g];
  if (r > 0.0) base = (sign > 0) ? base + r : base - r;   /* rounded: surface = hull (+) ball */
  /* exact cylinder: its rim polygons turned about the axis so that vertex 0
   * of each cap is the true rim extreme along n (the generator through the
   * surface's extreme); n along the axis keeps the prism (a cap face) */
  double c0 = 1.0, s0 = 0.0;
  const double* cy = DA(md, geom_cyl) + 2 * g;
  if (cy[0] > 0.0) {
    double rho = sqrt(nl[0] * nl[0] + nl[1] * nl[1]);
    if (rho > O_MINVAL) {
      double sg = (sign > 0) ? 1.0 : -1.0;
      c0 = sg * (nl[0] / rho);
      s0 = sg * (nl[1] / rho);
    }
  }
  double best = (sign > 0) ? -INFINITY : INFINITY;
  for (int i = 0; i < num; i++) {
    double vx = V[i], vy = V[num + i];
    if (cy[0] > 0.0) { double tx = c0 * vx - s0 * vy; vy = s0 * vx + c0 * vy; vx = tx; }
    double s = base + ((vx * nl[0] + vy * nl[1]) + V[2 * num + i] * nl[2]);
    if (sign > 0 ? (s > best) : (s < best)) best = s;
  }
  *ext = best;
  int cnt = 0;
  double lim = (sign > 0) ? best - tol : best + tol;
  for (int i = 0; i < num && cnt < O_MAXF; i++) {
    double vx = V[i], vy = V[num + i];
    if (cy[0] > 0.0) { double tx = c0 * vx - s0 * vy; vy = s0 * vx + c0 * vy; vx = tx; }
    double s = base + ((vx * nl[0] + vy * nl[1]) + V[2 * num + i] * nl[2]);
    if (sign > 0 ? (s >= lim) : (s <= lim)) {
      double t[3], P[3], vi[3] = {vx, vy, V[2 * num + i]};
      mulmv3(t, R, vi);
      add3(P, x, t);
      out[cnt].x = dot3(P, t1);
      out[cnt].y = dot3(P, t2);
      out[cnt].h = s;
      cnt++;
    }
  }
  return cnt;
}

static inline double cross2(const P2* o, const P2* a, const P2* b) {
  return (a->x - o->x) * (b->y - o->y) - (a->y - o->y) * (b->x - o->x);
}

/* 2D convex hull (Andrew monotone chain), CCW, collinear points removed */
static int hull2d(P2* pts, int n, P2* out) {
  /* insertion sort by (x, y) */
  for (int i = 1; i < n; i++) {
    P2 key = pts[i];
    int j = i - 1;
    while (j >= 0 && (pts[j].x > key.x || (pts[j].x == key.x && pts[j].y > key.y))) {
      pts[j + 1] = pts[j];
      j--;
    }
    pts[j + 1] = key;
  }
  /* drop exact duplicates */
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

static inline P2 lerp2(const P2* a, const P2* b, double t) {
  P2 r;
  r.x = a->x + t * (b->x - a->x);
  r.y = a->y + t * (b->y - a->y);
  r.h = a->h + t * (b->h - a->h);
  return r;
}

/* clip polygon/segment/point Q (nq) against CCW convex polygon P (np >= 3) */
static int clip_poly(const P2* P, int np, P2* Q, int nq) {
  P2 buf[O_MAXPOLY];
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
        if (dp < 0.0 && no < O_MAXPOLY) buf[no++] = lerp2(prv, cur, dp / (dp - dc));
        if (no < O_MAXPOLY) buf[no++] = *cur;
      } else if (dp >= 0.0) {
        if (no < O_MAXPOLY) buf[no++] = lerp2(prv, cur, dp / (dp - dc));
      }
    }
    for (int i = 0; i < no; i++) Q[i] = buf[i];
    nq = no;
  }
  return nq;
}

static inline double dist2d(const P2* a, const P2* b) {
  double dx = a->x - b->x, dy = a->y - b->y;
  return dx * dx + dy * dy;
}

/* keep <= 4 of np manifold points: the deepest, the farthest from it, the one
 * spanning the largest triangle with those, the one farthest from all three */
static void select4(const P2* pts, const double* dep, int np, int* sel, int* ns) {
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

static void add_contact(const Mdl* md, Dat* d, int pair, int g1, int g2, const double* pos,
                        const double* n, const double* t1, const double* t2, double dist) {
  if (d->ncon >= d->ncon_max) { d->overflow |= 1; return; }
  int c = d->ncon++;
  (void)md;
  d->con_pos[3 * c] = pos[0]; d->con_pos[3 * c + 1] = pos[1]; d->con_pos[3 * c + 2] = pos[2];
  double* f = d->con_frame + 9 * c;
  f[0] = n[0]; f[1] = n[1]; f[2] = n[2];
  f[3] = t1[0]; f[4] = t1[1]; f[5] = t1[2];
  f[6] = t2[0]; f[7] = t2[1]; f[8] = t2[2];
  d->con_dist[c] = dist;
  d->con_pair[c] = pair;
  d->con_g1[c] = g1;
  d->con_g2[c] = g2;
}

/* ------------------------------------------------------------------------ */
/* Separation certificates (kernel cert_check / cert_update).  A convex pair
 * whose MPR missed with separating direction d (the Minkowski difference
 * g1 - g2 has support -m < 0 along d) stays separated while the motion of g1
 * relative to g2 cannot close the margin: in g2's frame the supports of g2 are
 * fixed and those of g1 along d_B grow by at most d_B . dp + ||dR||_F rho_1.
 * Certified pairs skip the narrowphase (MPR would miss them again).  Slot:
 * pair, m, d_B (3), g1's origin (3) and rotation (9) in g2's frame at the
 * certifying step; pair -1 = free.  oracle_set_cull(0) turns the skipping off
 * (tests: the contacts are the same either way). */
static int g_nocull = 0;
void oracle_set_cull(int on) { g_nocull = on ? 0 : 1; }
static void rel_pose(const Dat* d, int g1, int g2, double* p, double* R) {
  const double *R1 = d->geom_xmat + 9 * g1, *R2 = d->geom_xmat + 9 * g2;
  double dx[3];
  sub3(dx, d->geom_xpos + 3 * g1, d->geom_xpos + 3 * g2);
  mulmtv3(p, R2, dx);
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) R[3 * i + j] = (R2[i] * R1[j] + R2[3 + i] * R1[3 + j]) + R2[6 + i] * R1[6 + j];
}

static int cert_ok(const Mdl* md, const Dat* d, const double* c) {
  int pair = (int)c[0];
  int g1 = IA(md, pair_geom1)[pair], g2 = IA(md, pair_geom2)[pair];
  double p[3], R[9], dp[3];
  rel_pose(d, g1, g2, p, R);
  sub3(dp, p, c + 5);
  double f = 0.0;
  for (int k = 0; k < 9; k++) {
    double e = R[k] - c[8 + k];
    f = f + e * e;
  }
  double grow = dot3(c + 2, dp) + sqrt(f) * DA(md, geom_rbound)[g1];
  return c[1] - grow > O_CERT_EPS;
}

/* slots of the pairs [c0, c0 + 64): freed if the pair left the broadphase set
 * (ov bits), else tested; returns the bits of the certified pairs */
static unsigned long long cert_check(const Mdl* md, Dat* d, int c0, unsigned long long ov) {
  unsigned long long skip = 0ull;
  for (int k = 0; k < O_CERT; k++) {
    double* c = d->cert + O_CERT_W * k;
    int pr = (int)c[0];
    if (pr < c0 || pr >= c0 + 64) continue;
    int bit = pr - c0;
    if (!((ov >> bit) & 1ull)) c[0] = -1.0;
    else if (cert_ok(md, d, c)) skip |= 1ull << bit;
  }
  return g_nocull ? 0ull : skip;
}

static void cert_update(const Mdl* md, Dat* d, int pair, int g1, int g2, int hit, const double* cd, double cm) {
  int mine = -1, fr = -1;
  for (int k = 0; k < O_CERT; k++) {
    int pr = (int)d->cert[O_CERT_W * k];
    if (pr == pair && mine < 0) mine = k;
    if (pr < 0 && fr < 0) fr = k;
  }
  int keep = !hit && cm > O_CERT_STORE;
  int sl = mine >= 0 ? mine : ((keep && fr >= 0) ? fr : -1);
  if (sl < 0) return;
  double* c = d->cert + O_CERT_W * sl;
  if (!keep) { c[0] = -1.0; return; }
  double p[3], R[9], db[3];
  rel_pose(d, g1, g2, p, R);
  mulmtv3(db, d->geom_xmat + 9 * g2, cd);
  c[0] = (double)pair;
  c[1] = cm;
  c[2] = db[0]; c[3] = db[1]; c[4] = db[2];
  c[5] = p[0]; c[6] = p[1]; c[7] = p[2];
  for (int k = 0; k < 9; k++) c[8 + k] = R[k];
}

/* convex-convex narrowphase with multi-contact manifold (<= 4 points) */
static void collide_pair(const Mdl* md, Dat* d, int pair) {
  int g1 = IA(md, pair_geom1)[pair], g2 = IA(md, pair_geom2)[pair];
  double n[3], depth, mpos[3], cd[3] = {0.0, 0.0, 0.0}, cm;
  int hit = mpr_penetration(md, d, g1, g2, n, &depth, mpos, cd, &cm);
  cert_update(md, d, pair, g1, g2, hit, cd, cm);
  if (!hit) return;
  double t1[3], t2[3];
  make_frame(n, t1, t2);
  P2 fa[O_MAXF], fb[O_MAXF];
  double s1, s2;
  /* extremes first (tolerance uses the support depth along n) */
  int na = feature(md, d, g1, n, t1, t2, +1, 0.0, fa, &s1);
  int nb = feature(md, d, g2, n, t1, t2, -1, 0.0, fb, &s2);
  double dn = s1 - s2;
  if (!(dn > 0.0)) return;
  double tol = dn + O_FEAT_EPS;
  na = feature(md, d, g1, n, t1, t2, +1, tol, fa, &s1);
  nb = feature(md, d, g2, n, t1, t2, -1, tol, fb, &s2);
  int refB = (nb >= na);
  P2 refpoly[O_MAXPOLY], inc[O_MAXPOLY];
  int nr = refB ? hull2d(fb, nb, refpoly) : hull2d(fa, na, refpoly);
  int ni = refB ? hull2d(fa, na, inc) : hull2d(fb, nb, inc);
  P2 pts[O_MAXPOLY];
  double dep[O_MAXPOLY];
  int np = 0;
  if (nr >= 3) {
    int nc = clip_poly(refpoly, nr, inc, ni);
    for (int i = 0; i < nc; i++) {
      double dd = refB ? (inc[i].h - s2) : (s1 - inc[i].h);
      if (dd > 0.0) { pts[np] = inc[i]; dep[np] = dd; np++; }
    }
  }
  if (np == 0) {
    double dist = -dn;
    add_contact(md, d, pair, g1, g2, mpos, n, t1, t2, dist);
    return;
  }
  int sel[4], ns;
  select4(pts, dep, np, sel, &ns);
  double sref = refB ? s2 : s1;
  for (int k = 0; k < ns; k++) {
    const P2* p = &pts[sel[k]];
    double hm = 0.5 * (p->h + sref);
    double pos[3];
    for (int c = 0; c < 3; c++) pos[c] = (p->x * t1[c] + p->y * t2[c]) + hm * n[c];
    add_contact(md, d, pair, g1, g2, pos, n, t1, t2, -dep[sel[k]]);
  }
}

/* ------------------------------------------------------------------------ */
/* Box-box: the dedicated collider MuJoCo dispatches box pairs to (mjc_BoxBox,
 * engine_collision_box.c) instead of the general convex path.  Separating-axis
 * test over the 3 + 3 face normals and the 9 edge-edge cross products; the axis
 * of least penetration wins, ties going to box 1's faces, then box 2's, and an
 * edge-edge axis only when it is shallower than the best face axis by more than
 * 5 % of the depth (faces are the stable choice for resting boxes).  The face
 * choice is a deterministic function of the poses, so a symmetric wedge (two
 * gripper pads closed on each other) keeps one normal instead of flipping
 * between the two faces as MPR's portal does.
 * Face axis: the incident face of the other box (the face most anti-parallel
 * to the normal) is clipped against the reference face rectangle; every clipped
 * vertex below the reference plane is a contact at the midpoint between the
 * two surfaces (<= 8; the 4 spanning ones are kept as in collide_pair).
 * Edge axis: one contact at the closest points of the two edges. */
static int bb_clip(P2* Q, int nq, int axis, double lim, double sgn) {
  /* keep sgn * coord <= lim, coord = x (axis 0) or y (axis 1) */
  P2 buf[16];
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

/* Which points a face contact of the box-box collider emits.  0 = the
 * contract (the kernels' collide_boxbox): the penetrating clipped vertices of
 * the incident face, reduced to <= 4 by select4, except that an edge on a face
 * (exactly two penetrating vertices) gives one contact at the deeper vertex --
 * the set that reproduces MuJoCo's recorded Robotiq state_close (round 5,
 * tests/test_oracle.py::test_state_close_contact_set_study).
 * Study variants (never the product's): 1 = the round-4 contract (both edge
 * vertices kept), 2 = every clipped vertex of the incident face at its own
 * signed distance (the face-overlap corners, non-penetrating ones included),
 * 3 = the single deepest vertex always, 4 = one contact at the centroid of
 * the penetrating vertices at the deepest depth. */
static int g_bbmode = 0;
void oracle_set_bbmode(int mode) { g_bbmode = mode; }

static void collide_boxbox(const Mdl* md, Dat* d, int pair) {
  int g1 = IA(md, pair_geom1)[pair], g2 = IA(md, pair_geom2)[pair];
  const double *R1 = d->geom_xmat + 9 * g1, *R2 = d->geom_xmat + 9 * g2;
  const double *x1 = d->geom_xpos + 3 * g1, *x2 = d->geom_xpos + 3 * g2;
  const double *h1 = DA(md, geom_aabb) + 6 * g1 + 3, *h2 = DA(md, geom_aabb) + 6 * g2 + 3;
  const double margin = DA(md, pair_margin)[pair];
  double A1[9], A2[9], D[3];
  for (int k = 0; k < 3; k++)
    for (int i = 0; i < 3; i++) { A1[3 * k + i] = R1[3 * i + k]; A2[3 * k + i] = R2[3 * i + k]; }
  sub3(D, x2, x1);
  double best = -INFINITY;
  int code = -1;
  for (int k = 0; k < 3; k++) {
    const double* L = A1 + 3 * k;
    double r2 = (h2[0] * fabs(dot3(A2, L)) + h2[1] * fabs(dot3(A2 + 3, L))) + h2[2] * fabs(dot3(A2 + 6, L));
    double s = fabs(dot3(D, L)) - (h1[k] + r2);
    if (s > margin) return;
    if (s > best) { best = s; code = k; }
  }
  for (int k = 0; k < 3; k++) {
    const double* L = A2 + 3 * k;
    double r1 = (h1[0] * fabs(dot3(A1, L)) + h1[1] * fabs(dot3(A1 + 3, L))) + h1[2] * fabs(dot3(A1 + 6, L));
    double s = fabs(dot3(D, L)) - (h2[k] + r1);
    if (s > margin) return;
    if (s > best) { best = s; code = 3 + k; }
  }
  double ebest = -INFINITY, eL[3] = {0.0, 0.0, 0.0};
  int ecode = -1;
  for (int a = 0; a < 3; a++)
    for (int b = 0; b < 3; b++) {
      double L[3];
      cross3(L, A1 + 3 * a, A2 + 3 * b);
      double ll = sqrt(dot3(L, L));
      if (ll < 1e-6) continue;      /* (nearly) parallel edges: covered by the face axes */
      L[0] = L[0] / ll; L[1] = L[1] / ll; L[2] = L[2] / ll;
      double r1 = (h1[0] * fabs(dot3(A1, L)) + h1[1] * fabs(dot3(A1 + 3, L))) + h1[2] * fabs(dot3(A1 + 6, L));
      double r2 = (h2[0] * fabs(dot3(A2, L)) + h2[1] * fabs(dot3(A2 + 3, L))) + h2[2] * fabs(dot3(A2 + 6, L));
      double s = fabs(dot3(D, L)) - (r1 + r2);
      if (s > margin) return;
      if (s > ebest) { ebest = s; ecode = 3 * a + b; eL[0] = L[0]; eL[1] = L[1]; eL[2] = L[2]; }
    }
  double t1[3], t2[3];
  if (ecode >= 0 && 1.05 * ebest > best) {
    /* edge-edge: n from box 1 towards box 2 */
    int a = ecode / 3, b = ecode % 3;
    double n[3] = {eL[0], eL[1], eL[2]};
    if (dot3(n, D) < 0.0) { n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2]; }
    double e1[3] = {x1[0], x1[1], x1[2]}, e2[3] = {x2[0], x2[1], x2[2]};
    for (int k = 0; k < 3; k++) {
      if (k != a) {
        double s = dot3(A1 + 3 * k, n) >= 0.0 ? h1[k] : -h1[k];
        for (int i = 0; i < 3; i++) e1[i] = e1[i] + s * A1[3 * k + i];
      }
      if (k != b) {
        double s = dot3(A2 + 3 * k, n) >= 0.0 ? -h2[k] : h2[k];
        for (int i = 0; i < 3; i++) e2[i] = e2[i] + s * A2[3 * k + i];
      }
    }
    const double *U = A1 + 3 * a, *V = A2 + 3 * b;
    double w[3];
    sub3(w, e1, e2);
    double bu = dot3(U, V), du = dot3(U, w), ev = dot3(V, w);
    double den = 1.0 - bu * bu;
    double s = (bu * ev - du) / den, t = (ev - bu * du) / den;
    if (s < -h1[a]) s = -h1[a];
    if (s > h1[a]) s = h1[a];
    if (t < -h2[b]) t = -h2[b];
    if (t > h2[b]) t = h2[b];
    double pos[3];
    for (int i = 0; i < 3; i++) pos[i] = 0.5 * ((e1[i] + s * U[i]) + (e2[i] + t * V[i]));
    make_frame(n, t1, t2);
    add_contact(md, d, pair, g1, g2, pos, n, t1, t2, ebest);
    return;
  }
  /* face: reference box A (code < 3: box 1), incident box B */
  int ref1 = code < 3, k = code % 3;
  const double *RA = ref1 ? A1 : A2, *RB = ref1 ? A2 : A1, *hA = ref1 ? h1 : h2, *hB = ref1 ? h2 : h1;
  const double *xA = ref1 ? x1 : x2, *xB = ref1 ? x2 : x1;
  double DAB[3];
  sub3(DAB, xB, xA);
  double nr[3] = {RA[3 * k], RA[3 * k + 1], RA[3 * k + 2]};
  if (dot3(DAB, nr) < 0.0) { nr[0] = -nr[0]; nr[1] = -nr[1]; nr[2] = -nr[2]; }
  double n[3] = {nr[0], nr[1], nr[2]};
  if (!ref1) { n[0] = -n[0]; n[1] = -n[1]; n[2] = -n[2]; }
  int ku = (k + 1) % 3, kv = (k + 2) % 3;
  const double *u = RA + 3 * ku, *v = RA + 3 * kv;
  double cA[3];
  for (int i = 0; i < 3; i++) cA[i] = xA[i] + hA[k] * nr[i];
  int j = 0;
  double bj = fabs(dot3(RB, nr));
  for (int q = 1; q < 3; q++) { double c = fabs(dot3(RB + 3 * q, nr)); if (c > bj) { bj = c; j = q; } }
  double sB = dot3(RB + 3 * j, nr) > 0.0 ? -hB[j] : hB[j];
  int jp = (j + 1) % 3, jq = (j + 2) % 3;
  static const double cs[4][2] = {{1.0, 1.0}, {-1.0, 1.0}, {-1.0, -1.0}, {1.0, -1.0}};
  P2 poly[16];
  double deep = INFINITY, deep_c[3] = {0.0, 0.0, 0.0};
  for (int c = 0; c < 4; c++) {
    double P[3], rel[3];
    for (int i = 0; i < 3; i++)
      P[i] = ((xB[i] + sB * RB[3 * j + i]) + (cs[c][0] * hB[jp]) * RB[3 * jp + i]) + (cs[c][1] * hB[jq]) * RB[3 * jq + i];
    sub3(rel, P, cA);
    poly[c].x = dot3(rel, u);
    poly[c].y = dot3(rel, v);
    poly[c].h = dot3(rel, nr);
    if (poly[c].h < deep) { deep = poly[c].h; deep_c[0] = P[0]; deep_c[1] = P[1]; deep_c[2] = P[2]; }
  }
  int nq = 4;
  nq = bb_clip(poly, nq, 0, hA[ku], 1.0);
  if (nq) nq = bb_clip(poly, nq, 0, hA[ku], -1.0);
  if (nq) nq = bb_clip(poly, nq, 1, hA[kv], 1.0);
  if (nq) nq = bb_clip(poly, nq, 1, hA[kv], -1.0);
  P2 pts[16];
  double dep[16];
  int np = 0;
  /* clipped vertices closer than BB_MERGE x the face size to a kept one are the
   * same point (equal-size faces: a corner on the rectangle's edge) */
  double mtol = BB_MERGE * (hA[ku] > hA[kv] ? hA[ku] : hA[kv]);
  mtol = mtol * mtol;
  for (int i = 0; i < nq; i++) {
    if (!(poly[i].h < margin) && g_bbmode != 2) continue;
    int dup = 0;
    for (int q = 0; q < np; q++) if (dist2d(&pts[q], &poly[i]) < mtol) dup = 1;
    if (!dup) { pts[np] = poly[i]; dep[np] = -poly[i].h; np++; }
  }
  make_frame(n, t1, t2);
  if (np == 0) {
    /* no incident-face point over the reference face: the deepest corner */
    double pos[3];
    for (int i = 0; i < 3; i++) pos[i] = deep_c[i] - (0.5 * deep) * nr[i];
    add_contact(md, d, pair, g1, g2, pos, n, t1, t2, deep);
    return;
  }
  int sel[16], ns;
  if (g_bbmode == 0 && np == 2) {
    ns = 1;
    sel[0] = dep[1] > dep[0] ? 1 : 0;
  } else if (g_bbmode == 2) {
    ns = np;
    for (int q = 0; q < np; q++) sel[q] = q;
  } else if (g_bbmode == 3) {
    ns = 1;
    sel[0] = 0;
    for (int q = 1; q < np; q++) if (dep[q] > dep[sel[0]]) sel[0] = q;
  } else if (g_bbmode == 4) {
    /* one contact at the centroid of the penetrating vertices, deepest depth */
    P2 c = pts[0];
    double dm = dep[0];
    for (int q = 1; q < np; q++) { c.x = c.x + pts[q].x; c.y = c.y + pts[q].y; if (dep[q] > dm) dm = dep[q]; }
    c.x = c.x / np; c.y = c.y / np; c.h = -dm;
    pts[0] = c;
    ns = 1;
    sel[0] = 0;
  } else {
    select4(pts, dep, np, sel, &ns);
  }
  for (int q = 0; q < ns; q++) {
    const P2* p = &pts[sel[q]];
    double pos[3];
    for (int i = 0; i < 3; i++) pos[i] = ((cA[i] + p->x * u[i]) + p->y * v[i]) + (0.5 * p->h) * nr[i];
    add_contact(md, d, pair, g1, g2, pos, n, t1, t2, p->h);
  }
}

/* ------------------------------------------------------------------------ */
/* MuJoCo 3.2.2's collision table restated (ccd_mode 1 / 2, ABI 23; the kernels'
 * collide_convex_mj / collide_prim).  PARITY UNPINNED: MuJoCo's source is not
 * vendored in the reference or installed here, and no reference fixture holds
 * a contact; the rules below restate the published algorithms (libccd 2.x's
 * mpr.c, which MuJoCo 3.2.2 links for mjc_Convex; engine_collision_convex.c's
 * multiccd; engine_collision_primitive.c) as documented in DESIGN.md §2.
 *
 * Convex pairs (mjc_Convex): libccd's ccdMPRPenetration -- portal discovery,
 * refinement, penetration -- with libccd's tolerance tests (ccdIsZero / ccdEq at
 * CCD_EPS = DBL_EPSILON), the depth as the distance from the origin to the final
 * portal triangle (ccdVec3PointTriDist2) along its witness direction, and the
 * position as the tetrahedron barycentre of the origin (findPos).  With the
 * multiccd flag (both envs: gravityless_object_grasping.py:40,
 * clutter_table.py:48) and no sphere in the pair, four more MPR runs with the
 * geoms turned about the first contact's point (mjc_rotateFrame) -- geom 1 by
 * -+1e-3 rad and geom 2 by the opposite angle about each tangent of the first
 * contact's frame -- add every contact farther than 1e-3 x the smaller
 * bounding radius from the pair's contacts so far (<= 5 per pair).  A point or
 * edge contact stays put under such a turn (its repeats are not distinct); a
 * face contact tips onto the overlap's edges.  Box pairs keep collide_boxbox. */
#define CCD_EPS 2.2204460492503131e-16   /* libccd CCD_EPS, double build (DBL_EPSILON) */
#define MCCD_ANGLE 1e-3                  /* multiccd perturbation angle */
#define MCCD_RELTOL 1e-3                 /* multiccd distinct-contact tolerance, x min rbound */
/* half-angle sine / cosine of the perturbation (literals: the kernels use the same doubles) */
#define MCCD_C 0.9999998750000026       /* cos(5e-4) */
#define MCCD_S 4.999999791666669e-04    /* sin(5e-4) */
#define CCD_MAXLOOP 64                   /* safety cap of libccd's unbounded discovery / refinement loops */
static inline int ccd_iszero(double x) { return fabs(x) < CCD_EPS; }
static inline int ccd_eq(double a, double b) {
  double ab = fabs(a - b);
  if (ab < CCD_EPS) return 1;
  double fa = fabs(a), fb = fabs(b);
  return fb > fa ? (ab < CCD_EPS * fb) : (ab < CCD_EPS * fa);
}
static inline int ccd_vzero(const double* a) { return ccd_eq(a[0], 0.0) && ccd_eq(a[1], 0.0) && ccd_eq(a[2], 0.0); }
/* ccdVec3Normalize: scale by 1 / sqrt(|v|^2) */
static inline void ccd_normalize(double* v) {
  double k = 1.0 / sqrt(dot3(v, v));
  v[0] = v[0] * k; v[1] = v[1] * k; v[2] = v[2] * k;
}
static inline void mulmm3(double* r, const double* a, const double* b) {
  double t[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) t[3 * i + j] = (a[3 * i] * b[j] + a[3 * i + 1] * b[3 + j]) + a[3 * i + 2] * b[6 + j];
  for (int k = 0; k < 9; k++) r[k] = t[k];
}

typedef struct { int g; const double* R; const double* x; } CObj;
static void ccd_support(const Mdl* md, const CObj* o1, const CObj* o2, const double* dir, SupPt* p) {
  g_sup_calls++;
  double nd[3] = {-dir[0], -dir[1], -dir[2]};
  support_pose(md, o1->g, o1->R, o1->x, dir, p->a);
  support_pose(md, o2->g, o2->R, o2->x, nd, p->b);
  sub3(p->v, p->a, p->b);
}
/* portalReachTolerance with ccdEq */
static int ccd_reach_tol(const SupPt* p1, const SupPt* p2, const SupPt* p3, const SupPt* p4, const double* n,
                         double tol) {
  double dv4 = dot3(p4->v, n);
  double t1 = dv4 - dot3(p1->v, n);
  double t2 = dv4 - dot3(p2->v, n);
  double t3 = dv4 - dot3(p3->v, n);
  double mn = t1 < t2 ? t1 : t2;
  mn = mn < t3 ? mn : t3;
  return ccd_eq(mn, tol) || mn < tol;
}
static void ccd_portal_dir(double* n, const SupPt* p1, const SupPt* p2, const SupPt* p3) {
  double e1[3], e2[3];
  sub3(e1, p2->v, p1->v);
  sub3(e2, p3->v, p1->v);
  cross3(n, e1, e2);
  ccd_normalize(n);
}
/* __ccdVec3PointSegmentDist2 (P = origin) */
static double ccd_seg_dist2(const double* x0, const double* b, double* w) {
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
/* ccdVec3PointTriDist2 (P = origin) with its witness point */
static double ccd_tri_dist2(const double* x0, const double* B, const double* C, double* w) {
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
/* findPos: the origin's barycentric coordinates in the tetrahedron (v0..v3),
 * or in the portal triangle when they degenerate; pos = mean of the two
 * objects' weighted support points */
static void ccd_find_pos(const SupPt* p0, const SupPt* p1, const SupPt* p2, const SupPt* p3, double* pos) {
  double dir[3], c[3], b[4];
  ccd_portal_dir(dir, p1, p2, p3);
  cross3(c, p1->v, p2->v); b[0] = dot3(c, p3->v);
  cross3(c, p3->v, p2->v); b[1] = dot3(c, p0->v);
  cross3(c, p0->v, p1->v); b[2] = dot3(c, p3->v);
  cross3(c, p2->v, p1->v); b[3] = dot3(c, p0->v);
  double sum = ((b[0] + b[1]) + b[2]) + b[3];
  if (ccd_iszero(sum) || sum < 0.0) {
    b[0] = 0.0;
    cross3(c, p2->v, p3->v); b[1] = dot3(c, dir);
    cross3(c, p3->v, p1->v); b[2] = dot3(c, dir);
    cross3(c, p1->v, p2->v); b[3] = dot3(c, dir);
    sum = (b[1] + b[2]) + b[3];
  }
  double inv = 1.0 / sum;
  const SupPt* P[4] = {p0, p1, p2, p3};
  double a1[3] = {0.0, 0.0, 0.0}, a2[3] = {0.0, 0.0, 0.0};
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 3; k++) {
      a1[k] = a1[k] + P[i]->a[k] * b[i];
      a2[k] = a2[k] + P[i]->b[k] * b[i];
    }
  for (int k = 0; k < 3; k++) pos[k] = (a1[k] * inv + a2[k] * inv) * 0.5;
}

#define CCD_CERT(P) do { *cm = -dot3((P).v, dir); cd[0] = dir[0]; cd[1] = dir[1]; cd[2] = dir[2]; } while (0)
/* ccdMPRPenetration: 1 with the unit normal n (geom 1 -> geom 2), depth > 0 and
 * position; 0 without penetration, or when libccd's normal is undefined
 * (touching, depth 0: mjc_CCDIteration then makes no contact).  cd / cm: the
 * separating direction of a certified miss (as mpr_penetration). */
static int ccd_mpr(const Mdl* md, const CObj* o1, const CObj* o2, double* n, double* depth, double* pos,
                   double* cd, double* cm) {
  *cm = -1.0;
  const double tol = md->m->mpr_tolerance;
  const int maxit = md->m->ccd_iterations;
  SupPt p0, p1, p2, p3, p4;
  double dir[3], dt;
  /* findOrigin: the geom centres (mjccd_center: geom_xpos) */
  for (int k = 0; k < 3; k++) { p0.a[k] = o1->x[k]; p0.b[k] = o2->x[k]; }
  sub3(p0.v, p0.a, p0.b);
  if (ccd_vzero(p0.v)) p0.v[0] = p0.v[0] + CCD_EPS * 10.0;
  dir[0] = -p0.v[0]; dir[1] = -p0.v[1]; dir[2] = -p0.v[2];
  ccd_normalize(dir);
  ccd_support(md, o1, o2, dir, &p1);
  dt = dot3(p1.v, dir);
  if (ccd_iszero(dt) || dt < 0.0) { CCD_CERT(p1); return 0; }
  cross3(dir, p0.v, p1.v);
  if (ccd_iszero(dot3(dir, dir))) {
    if (ccd_vzero(p1.v)) return 0;           /* touching at v1: normal undefined */
    /* findPenetrSegment: the origin on the segment v0-v1 */
    for (int k = 0; k < 3; k++) { n[k] = p1.v[k]; pos[k] = (p1.a[k] + p1.b[k]) * 0.5; }
    *depth = sqrt(dot3(n, n));
    ccd_normalize(n);
    return 1;
  }
  ccd_normalize(dir);
  ccd_support(md, o1, o2, dir, &p2);
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
    ccd_support(md, o1, o2, dir, &p3);
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
  /* refinePortal */
  for (it = 0; it < CCD_MAXLOOP; it++) {
    ccd_portal_dir(dir, &p1, &p2, &p3);
    dt = dot3(dir, p1.v);
    if (ccd_iszero(dt) || dt > 0.0) break;
    ccd_support(md, o1, o2, dir, &p4);
    dt = dot3(p4.v, dir);
    if (!(ccd_iszero(dt) || dt > 0.0)) { CCD_CERT(p4); return 0; }
    if (ccd_reach_tol(&p1, &p2, &p3, &p4, dir, tol)) return 0;
    portal_expand(&p0, &p1, &p2, &p3, &p4);
  }
  if (it == CCD_MAXLOOP) return 0;
  /* findPenetr */
  for (it = 0;; it++) {
    ccd_portal_dir(dir, &p1, &p2, &p3);
    ccd_support(md, o1, o2, dir, &p4);
    if (ccd_reach_tol(&p1, &p2, &p3, &p4, dir, tol) || it > maxit) {
      double w[3];
      double dep = sqrt(ccd_tri_dist2(p1.v, p2.v, p3.v, w));
      if (ccd_iszero(dep)) return 0;         /* touching: normal undefined */
      n[0] = w[0]; n[1] = w[1]; n[2] = w[2];
      ccd_normalize(n);
      *depth = dep;
      ccd_find_pos(&p0, &p1, &p2, &p3, pos);
      return 1;
    }
    portal_expand(&p0, &p1, &p2, &p3, &p4);
  }
}
#undef CCD_CERT

static inline double mccd_rbound(const Mdl* md, int g) {
  return DA(md, geom_rbound)[g] + DA(md, geom_radius)[g];    /* MuJoCo geom_rbound */
}
/* mjc_Convex with multiccd (multi = 1) or one contact (multi = 0) */
static void collide_convex_mj(const Mdl* md, Dat* d, int pair, int multi) {
  int g1 = IA(md, pair_geom1)[pair], g2 = IA(md, pair_geom2)[pair];
  const double *R1 = d->geom_xmat + 9 * g1, *R2 = d->geom_xmat + 9 * g2;
  const double *x1 = d->geom_xpos + 3 * g1, *x2 = d->geom_xpos + 3 * g2;
  CObj o1 = {g1, R1, x1}, o2 = {g2, R2, x2};
  double n[3], depth, pos[3], cd[3] = {0.0, 0.0, 0.0}, cm;
  int hit = ccd_mpr(md, &o1, &o2, n, &depth, pos, cd, &cm);
  cert_update(md, d, pair, g1, g2, hit, cd, cm);
  if (!hit) return;
  double t1[3], t2[3];
  make_frame(n, t1, t2);
  add_contact(md, d, pair, g1, g2, pos, n, t1, t2, -depth);
  if (!multi) return;
  double cp[5][3];
  cp[0][0] = pos[0]; cp[0][1] = pos[1]; cp[0][2] = pos[2];
  int nc = 1;
  double rb1 = mccd_rbound(md, g1), rb2 = mccd_rbound(md, g2);
  double tolr = MCCD_RELTOL * (rb1 < rb2 ? rb1 : rb2);
  for (int ax = 0; ax < 2; ax++) {
    const double* axis = ax ? t2 : t1;
    for (int sg = 0; sg < 2; sg++) {
      /* geom 1 turned by -angle then +angle about the axis, geom 2 the opposite way */
      double s = sg ? MCCD_S : -MCCD_S;
      double q1[4] = {MCCD_C, axis[0] * s, axis[1] * s, axis[2] * s};
      double q2[4] = {MCCD_C, -(axis[0] * s), -(axis[1] * s), -(axis[2] * s)};
      double M1[9], M2[9], R1p[9], R2p[9], x1p[3], x2p[3], r[3], t[3];
      quat2mat(M1, q1);
      quat2mat(M2, q2);
      /* mjc_rotateFrame: x' = p + M (x - p), R' = M R about the first contact p */
      mulmm3(R1p, M1, R1);
      sub3(r, x1, pos);
      mulmv3(t, M1, r);
      add3(x1p, t, pos);
      mulmm3(R2p, M2, R2);
      sub3(r, x2, pos);
      mulmv3(t, M2, r);
      add3(x2p, t, pos);
      CObj p1o = {g1, R1p, x1p}, p2o = {g2, R2p, x2p};
      double nn[3], dd, pp[3], cdx[3], cmx;
      if (!ccd_mpr(md, &p1o, &p2o, nn, &dd, pp, cdx, &cmx)) continue;
      int isnew = 1;
      for (int k = 0; k < nc; k++) {
        double dx[3];
        sub3(dx, pp, cp[k]);
        if (sqrt(dot3(dx, dx)) < tolr) isnew = 0;
      }
      if (!isnew) continue;
      cp[nc][0] = pp[0]; cp[nc][1] = pp[1]; cp[nc][2] = pp[2];
      nc++;
      double u1[3], u2[3];
      make_frame(nn, u1, u2);
      add_contact(md, d, pair, g1, g2, pp, nn, u1, u2, -dd);
    }
  }
}

/* Analytic primitive colliders (engine_collision_primitive.c restated; the
 * normal points from geom 1 to geom 2, the position is midway between the two
 * surfaces, dist < 0 in penetration; a pair makes contacts with dist <= margin). */
static inline double dist3(const double* a, const double* b) {
  double dx[3];
  sub3(dx, a, b);
  return sqrt(dot3(dx, dx));
}
/* mjraw_SphereSphere: spheres (p1, r1) and (p2, r2); z1 / z2 the geoms' z axes
 * (the normal of concentric spheres: their cross product, else x) */
static int raw_sphere_sphere(const double* p1, const double* z1, double r1, const double* p2, const double* z2,
                             double r2, double margin, double* pos, double* n, double* dist) {
  double dd = (dist3(p1, p2) - r1) - r2;
  if (dd > margin) return 0;
  sub3(n, p2, p1);
  if (normalize3(n) < O_MINVAL) {
    cross3(n, z1, z2);
    normalize3(n);
  }
  double s = r1 + 0.5 * dd;
  for (int k = 0; k < 3; k++) pos[k] = p1[k] + n[k] * s;
  *dist = dd;
  return 1;
}
/* sphere (centre c, radius r) against the box (x, R, half sizes s): the box
 * point nearest the centre; a centre inside the box leaves through the face of
 * least depth (first on ties) */
static int raw_sphere_box(const double* c, double r, const double* x, const double* R, const double* s, double margin,
                          double* pos, double* n, double* dist) {
  double t[3], cl[3], q[3], df[3], nl[3], pl[3];
  sub3(t, c, x);
  mulmtv3(cl, R, t);
  for (int k = 0; k < 3; k++) q[k] = cl[k] < -s[k] ? -s[k] : (cl[k] > s[k] ? s[k] : cl[k]);
  sub3(df, q, cl);
  double dc = sqrt(dot3(df, df));
  if (dc - r > margin) return 0;
  double dd;
  if (dc > O_MINVAL) {
    for (int k = 0; k < 3; k++) nl[k] = df[k] / dc;
    dd = dc - r;
  } else {
    int kk = 0;
    double a = s[0] - fabs(cl[0]);
    for (int k = 1; k < 3; k++) {
      double ak = s[k] - fabs(cl[k]);
      if (ak < a) { a = ak; kk = k; }
    }
    nl[0] = nl[1] = nl[2] = 0.0;
    nl[kk] = cl[kk] >= 0.0 ? -1.0 : 1.0;
    dd = -(a + r);
  }
  double h = r + 0.5 * dd;
  for (int k = 0; k < 3; k++) pl[k] = cl[k] + nl[k] * h;
  mulmv3(n, R, nl);
  mulmv3(t, R, pl);
  add3(pos, x, t);
  *dist = dd;
  return 1;
}
/* signed distance of a box-frame point to the box (negative inside) */
static double box_phi(const double* p, const double* s) {
  double o0 = fabs(p[0]) - s[0], o1 = fabs(p[1]) - s[1], o2 = fabs(p[2]) - s[2];
  if (o0 > 0.0 || o1 > 0.0 || o2 > 0.0) {
    double a = o0 > 0.0 ? o0 : 0.0, b = o1 > 0.0 ? o1 : 0.0, c = o2 > 0.0 ? o2 : 0.0;
    return sqrt((a * a + b * b) + c * c);
  }
  double m = o0 > o1 ? o0 : o1;
  return m > o2 ? m : o2;
}
/* capsule segment parameter of candidate k (0..MGS_CB_NCAND-1) in the box frame
 * (centre c, half axis a): the stationary points of the segment's signed
 * distance to the box, which is convex along the segment -- the ends, the slab
 * crossings, the minimisers of each outside active set, the equal-depth points
 * of two face planes.  Returns 0 for a candidate that does not exist. */
#define MGS_CB_NCAND 49
static int capbox_cand(int k, const double* c, const double* a, const double* s, double* tout) {
  double t;
  if (k < 2) { *tout = k ? 1.0 : -1.0; return 1; }
  if (k < 8) {
    int i = (k - 2) >> 1;
    double sg = ((k - 2) & 1) ? 1.0 : -1.0;
    if (fabs(a[i]) < O_MINVAL) return 0;
    t = (sg * s[i] - c[i]) / a[i];
  } else if (k < 34) {
    int code = k - 8 + 1;      /* 1..26: base-3 digits = per-axis side (0 in, 1 below, 2 above) */
    double num = 0.0, den = 0.0;
    for (int i = 0; i < 3; i++) {
      int dgt = code % 3;
      code /= 3;
      if (dgt == 0) continue;
      double sg = dgt == 1 ? -1.0 : 1.0;
      num = num + (c[i] - sg * s[i]) * a[i];
      den = den + a[i] * a[i];
    }
    if (den < O_MINVAL) return 0;
    t = -num / den;
    t = t < -1.0 ? -1.0 : (t > 1.0 ? 1.0 : t);
    *tout = t;
    return 1;
  } else {
    /* face lines l = 2 i + side: side(c_i + t a_i) - s_i; pairs in lexicographic order */
    int q = k - 34, l1 = 0, l2 = 1;
    for (int x = 0; x < 6; x++)
      for (int y = x + 1; y < 6; y++) {
        if (q == 0) { l1 = x; l2 = y; }
        q--;
      }
    int i = l1 >> 1, j = l2 >> 1;
    double si = (l1 & 1) ? 1.0 : -1.0, sj = (l2 & 1) ? 1.0 : -1.0;
    double coef = si * a[i] - sj * a[j];
    if (fabs(coef) < O_MINVAL) return 0;
    t = ((s[i] - s[j]) - (si * c[i] - sj * c[j])) / coef;
  }
  if (!(t >= -1.0 && t <= 1.0)) return 0;
  *tout = t;
  return 1;
}
static void collide_prim(const Mdl* md, Dat* d, int pair, int kind) {
  int g1 = IA(md, pair_geom1)[pair], g2 = IA(md, pair_geom2)[pair];
  const double *R1 = d->geom_xmat + 9 * g1, *R2 = d->geom_xmat + 9 * g2;
  const double *x1 = d->geom_xpos + 3 * g1, *x2 = d->geom_xpos + 3 * g2;
  const double *s1 = DA(md, geom_size) + 3 * g1, *s2 = DA(md, geom_size) + 3 * g2;
  const double margin = DA(md, pair_margin)[pair];
  double z1[3] = {R1[2], R1[5], R1[8]}, z2[3] = {R2[2], R2[5], R2[8]};
  double pos[2][3], n[2][3], dist[2];
  int nc = 0;
  if (kind == MGS_PAIR_SPHERE_SPHERE) {
    nc = raw_sphere_sphere(x1, z1, s1[0], x2, z2, s2[0], margin, pos[0], n[0], dist);
  } else if (kind == MGS_PAIR_SPHERE_CAPSULE) {
    /* the capsule axis point nearest the sphere centre, then sphere-sphere */
    double v[3], q[3];
    sub3(v, x1, x2);
    double xx = dot3(z2, v);
    xx = xx < -s2[1] ? -s2[1] : (xx > s2[1] ? s2[1] : xx);
    for (int k = 0; k < 3; k++) q[k] = x2[k] + z2[k] * xx;
    nc = raw_sphere_sphere(x1, z1, s1[0], q, z2, s2[0], margin, pos[0], n[0], dist);
  } else if (kind == MGS_PAIR_CAPSULE_CAPSULE) {
    double a1[3], a2[3], df[3];
    for (int k = 0; k < 3; k++) { a1[k] = z1[k] * s1[1]; a2[k] = z2[k] * s2[1]; }
    sub3(df, x1, x2);
    double ma = dot3(a1, a1), mb = -dot3(a1, a2), mc = dot3(a2, a2);
    double u = -dot3(a1, df), v = dot3(a2, df);
    double det = ma * mc - mb * mb;
    double v1[3], v2[3];
    if (fabs(det) >= O_MINVAL) {
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
      for (int k = 0; k < 3; k++) { v1[k] = x1[k] + a1[k] * xa; v2[k] = x2[k] + a2[k] * xb; }
      nc = raw_sphere_sphere(v1, z1, s1[0], v2, z2, s2[0], margin, pos[0], n[0], dist);
    } else {
      /* parallel axes: the ends of each against the other segment, <= 2 contacts */
      for (int e = 0; e < 4 && nc < 2; e++) {
        double sg = (e & 1) ? -1.0 : 1.0, xx;
        if (e < 2) {
          xx = (sg > 0.0 ? (v - mb) : (v + mb)) / mc;
          xx = xx < -1.0 ? -1.0 : (xx > 1.0 ? 1.0 : xx);
          for (int k = 0; k < 3; k++) { v1[k] = x1[k] + sg * a1[k]; v2[k] = x2[k] + a2[k] * xx; }
        } else {
          xx = (sg > 0.0 ? (u - mb) : (u + mb)) / ma;
          xx = xx < -1.0 ? -1.0 : (xx > 1.0 ? 1.0 : xx);
          for (int k = 0; k < 3; k++) { v2[k] = x2[k] + sg * a2[k]; v1[k] = x1[k] + a1[k] * xx; }
        }
        nc += raw_sphere_sphere(v1, z1, s1[0], v2, z2, s2[0], margin, pos[nc], n[nc], dist + nc);
      }
    }
  } else if (kind == MGS_PAIR_SPHERE_BOX) {
    nc = raw_sphere_box(x1, s1[0], x2, R2, s2, margin, pos[0], n[0], dist);
  } else if (kind == MGS_PAIR_CAPSULE_BOX) {
    /* the segment point deepest in / nearest to the box, then sphere-box; a
     * capsule whose two ends both touch the same face makes one contact at
     * each end */
    double t[3], c[3], a[3], hz[3];
    sub3(t, x1, x2);
    mulmtv3(c, R2, t);
    for (int k = 0; k < 3; k++) hz[k] = z1[k] * s1[1];
    mulmtv3(a, R2, hz);
    double best = INFINITY, tb = -1.0;
    for (int k = 0; k < MGS_CB_NCAND; k++) {
      double tk, p[3];
      if (!capbox_cand(k, c, a, s2, &tk)) continue;
      for (int i = 0; i < 3; i++) p[i] = c[i] + a[i] * tk;
      double ph = box_phi(p, s2);
      if (ph < best) { best = ph; tb = tk; }
    }
    double ctr[3], pe[2][3], ne[2][3], de[2];
    for (int k = 0; k < 3; k++) ctr[k] = x1[k] + hz[k] * tb;
    nc = raw_sphere_box(ctr, s1[0], x2, R2, s2, margin, pos[0], n[0], dist);
    if (nc) {
      int ok = 1;
      for (int e = 0; e < 2 && ok; e++) {
        double sg = e ? 1.0 : -1.0, ce[3];
        for (int k = 0; k < 3; k++) ce[k] = x1[k] + hz[k] * sg;
        ok = raw_sphere_box(ce, s1[0], x2, R2, s2, margin, pe[e], ne[e], de + e) &&
             ne[e][0] == n[0][0] && ne[e][1] == n[0][1] && ne[e][2] == n[0][2];
      }
      if (ok) {
        for (int e = 0; e < 2; e++) {
          for (int k = 0; k < 3; k++) { pos[e][k] = pe[e][k]; n[e][k] = ne[e][k]; }
          dist[e] = de[e];
        }
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
      if (dc > O_MINVAL) {
        for (int k = 0; k < 3; k++) nl[k] = df[k] / dc;
        dd = dc - r;
      } else {
        double side = cr - rho, cap = ch - fabs(cl[2]), a;
        if (side < cap && rho > O_MINVAL) {
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
      for (int k = 0; k < 3; k++) pl[k] = cl[k] + nl[k] * h;
      mulmv3(n[0], R2, nl);
      mulmv3(t, R2, pl);
      add3(pos[0], x2, t);
      dist[0] = dd;
      nc = 1;
    }
  }
  for (int c = 0; c < nc; c++) {
    double t1[3], t2[3];
    make_frame(n[c], t1, t2);
    add_contact(md, d, pair, g1, g2, pos[c], n[c], t1, t2, dist[c]);
  }
}

#define OBB_FN static
/* Second broadphase stage: separating-axis test between the geoms' oriented
 * bounding boxes (their local AABBs posed in the world; 15 axes).  Each convex
 * hull lies inside its box, so separated boxes cannot produce a contact and the
 * narrowphase is skipped (MuJoCo would run MPR and find nothing; on the round-1
 * benchmark this removes ~55% of narrowphase calls).  Returns 1 if separated. */
OBB_FN int obb_separated(const double* R1, const double* x1, const double* b1, const double* R2,
                         const double* x2, const double* b2, double margin) {
  double c1[3], c2[3], t[3], D[3];
  mulmv3(t, R1, b1);
  add3(c1, x1, t);
  mulmv3(t, R2, b2);
  add3(c2, x2, t);
  sub3(D, c2, c1);
  const double *h1 = b1 + 3, *h2 = b2 + 3;
  double A1[9], A2[9];  /* box axes as rows: A[k] = column k of R */
  for (int k = 0; k < 3; k++)
    for (int i = 0; i < 3; i++) { A1[3 * k + i] = R1[3 * i + k]; A2[3 * k + i] = R2[3 * i + k]; }
  for (int q = 0; q < 15; q++) {
    double L[3];
    if (q < 3) { L[0] = A1[3 * q]; L[1] = A1[3 * q + 1]; L[2] = A1[3 * q + 2]; }
    else if (q < 6) { L[0] = A2[3 * (q - 3)]; L[1] = A2[3 * (q - 3) + 1]; L[2] = A2[3 * (q - 3) + 2]; }
    else { int a = (q - 6) / 3, b = (q - 6) % 3; cross3(L, A1 + 3 * a, A2 + 3 * b); }
    double ll = dot3(L, L);
    if (ll < 1e-20) continue;
    double r1 = (h1[0] * fabs(dot3(A1, L)) + h1[1] * fabs(dot3(A1 + 3, L))) + h1[2] * fabs(dot3(A1 + 6, L));
    double r2 = (h2[0] * fabs(dot3(A2, L)) + h2[1] * fabs(dot3(A2 + 3, L))) + h2[2] * fabs(dot3(A2 + 6, L));
    if (fabs(dot3(D, L)) > (r1 + r2) + (margin + 1e-12) * sqrt(ll)) return 1;
  }
  return 0;
}

/* diagnostics (single-threaded use only): broadphase passes / hits per pair */
static long g_pair_bp[256], g_pair_hit[256], g_pair_sup[256];
long* oracle_pair_counters(void) { static long buf[768]; for (int i = 0; i < 256; i++) { buf[i] = g_pair_bp[i]; buf[256 + i] = g_pair_hit[i]; buf[512 + i] = g_pair_sup[i]; g_pair_bp[i] = g_pair_hit[i] = g_pair_sup[i] = 0; } return buf; }
static void collision(const Mdl* md, Dat* d) {
  const mgs_model_desc* m = md->m;
  const int32_t *p1 = IA(md, pair_geom1), *p2 = IA(md, pair_geom2);
  const double *aabb = DA(md, geom_aabb), *pm = DA(md, pair_margin);
  d->ncon = 0;
  /* pairs in chunks of 64, as the kernel's lanes: broadphase of the chunk, the
   * certificates of its pairs, then the narrowphase in pair order */
  for (int c0 = 0; c0 < m->npair; c0 += 64) {
  int cend = c0 + 64 < m->npair ? c0 + 64 : m->npair;
  unsigned long long ovm = 0ull;
  for (int p = c0; p < cend; p++) {
    int g[2] = {p1[p], p2[p]};
    double c[2][3], hw[2][3];
    for (int s = 0; s < 2; s++) {
      const double* R = d->geom_xmat + 9 * g[s];
      const double* lc = aabb + 6 * g[s];
      const double* lh = lc + 3;
      double t[3];
      mulmv3(t, R, lc);
      add3(c[s], d->geom_xpos + 3 * g[s], t);
      for (int k = 0; k < 3; k++)
        hw[s][k] = (fabs(R[3 * k]) * lh[0] + fabs(R[3 * k + 1]) * lh[1]) + fabs(R[3 * k + 2]) * lh[2];
    }
    int ov = 1;
    for (int k = 0; k < 3; k++)
      if (fabs(c[0][k] - c[1][k]) > (hw[0][k] + hw[1][k]) + pm[p]) ov = 0;
    if (ov && obb_separated(d->geom_xmat + 9 * g[0], d->geom_xpos + 3 * g[0], aabb + 6 * g[0],
                            d->geom_xmat + 9 * g[1], d->geom_xpos + 3 * g[1], aabb + 6 * g[1], pm[p]))
      ov = 0;
    if (ov) ovm |= 1ull << (p - c0);
  }
  unsigned long long skip = cert_check(md, d, c0, ovm);
  for (int p = c0; p < cend; p++) {
    if (((ovm & ~skip) >> (p - c0)) & 1ull) {
      if (p < 256) g_pair_bp[p]++;
      int n0 = d->ncon;
      long s0 = g_sup_calls;
      int kind = IA(md, pair_kind)[p];
      if (kind == MGS_PAIR_BOXBOX) collide_boxbox(md, d, p);
      else if (m->ccd_mode == MGS_CCD_R5) collide_pair(md, d, p);
      else if (kind == MGS_PAIR_CONVEX || kind == MGS_PAIR_CONVEX_SMOOTH)
        collide_convex_mj(md, d, p, kind == MGS_PAIR_CONVEX && m->ccd_mode == MGS_CCD_MULTI && !d->mask_only);
      else collide_prim(md, d, p, kind);
      if (p < 256) g_pair_sup[p] += g_sup_calls - s0;
      if (p < 256 && d->ncon > n0) g_pair_hit[p]++;
    }
  }
  }
}

/* ------------------------------------------------------------------------ */
/* Jacobians of a point on body b: jacp, jacr (3 x nv, row-major) */
static void jac_point(const Mdl* md, const Dat* d, int b, const double* pt, double* jacp, double* jacr) {
  int nv = md->m->nv;
  memset(jacp, 0, sizeof(double) * 3 * nv);
  memset(jacr, 0, sizeof(double) * 3 * nv);
  int dof = IA(md, body_lastdof)[b];
  const int32_t* dpar = IA(md, dof_parentid);
  const double* c = d->subtree_com + 3 * IA(md, body_rootid)[b];
  double off[3];
  sub3(off, pt, c);
  while (dof >= 0) {
    const double* cd = d->cdof + 6 * dof;
    double cr[3];
    cross3(cr, cd, off);
    for (int k = 0; k < 3; k++) {
      jacr[k * nv + dof] = cd[k];
      jacp[k * nv + dof] = cd[3 + k] + cr[k];
    }
    dof = dpar[dof];
  }
}

/* impedance from solimp at violation x (MuJoCo getimpedance, integer power) */
static double impedance(const double* si, double pos, double margin) {
  if (si[0] == si[1] || si[2] <= O_MINVAL) return 0.5 * (si[0] + si[1]);
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

static int add_row(Dat* d, int type, double pos, double margin, int dim, int con) {
  if (d->nefc >= d->nefc_max) { d->overflow |= 2; return -1; }
  int r = d->nefc++;
  d->efc_type[r] = type; d->efc_pos[r] = pos; d->efc_margin[r] = margin;
  d->efc_dim[r] = dim; d->efc_con[r] = con;
  memset(d->J + (size_t)r * d->nv, 0, sizeof(double) * d->nv);
  return r;
}

/* reference acceleration and regularizer for rows r..r+dim-1 sharing solref/solimp */
/* The violation an equality row's impedance is taken at.  0 = the contract
 * (the kernels' eq_violation_norm): the norm of its constraint's violation over
 * all of the constraint's rows (a connect's 3, a weld's 6, a joint equality's
 * 1), summed in row order -- with the box-box edge rule above, the choice that
 * reproduces MuJoCo's recorded Robotiq state_close (round 5).  1 = the round-4
 * contract, each row's own violation (study variant). */
static int g_eqimp = 0;
void oracle_set_eqimp(int mode) { g_eqimp = mode; }

static double eq_violation_norm(const Dat* d, int r, int neqrows) {
  int e = d->efc_con[r];
  double s2 = 0.0;
  for (int q = 0; q < neqrows; q++)
    if (d->efc_con[q] == e) s2 = s2 + d->efc_pos[q] * d->efc_pos[q];
  return sqrt(s2);
}

/* ipos: the violation the impedance is taken at */
static void row_params(const Mdl* md, Dat* d, int r, int dim, const double* sr, const double* si,
                       const double* mu, int elliptic_contact, double ipos) {
  const double dt = md->m->timestep;
  double tc = sr[0], dr = sr[1];
  double imp = impedance(si, ipos, d->efc_margin[r]);
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
    double p = (j == 0) ? (d->efc_pos[q] - d->efc_margin[q]) : 0.0;
    d->efc_aref[q] = -B * d->efc_vel[q] - (Kc * imp) * p;
  }
  double Rn = ((1.0 - imp) / imp) * d->efc_dA[r];
  if (Rn < O_MINVAL) Rn = O_MINVAL;
  d->efc_R[r] = Rn;
  if (elliptic_contact && dim > 1) {
    double R1 = Rn / md->m->impratio;
    d->efc_R[r + 1] = R1;
    for (int j = 1; j < dim - 1; j++)
      d->efc_R[r + j + 1] = (R1 * (mu[0] * mu[0])) / (mu[j] * mu[j]);
  } else {
    for (int j = 1; j < dim; j++) {
      double Rj = ((1.0 - imp) / imp) * d->efc_dA[r + j];
      d->efc_R[r + j] = Rj < O_MINVAL ? O_MINVAL : Rj;
    }
  }
}

/* MuJoCo mj_diagApprox (engine_core_constraint.c): the approximate diagonal of
 * A used for R, from the qpos0 inverse weights (body_invweight0: translation,
 * rotation; dof_invweight0).  Connect rows: translation of both bodies; weld
 * rows 0-2 translation, 3-5 rotation; joint equality: dof weights of both
 * joints; dof friction / joint limits: the dof weight; contacts: translation of
 * both geom bodies for the normal and tangent rows, rotation beyond row 2. */
static void diag_approx(const Mdl* md, Dat* d) {
  const double *biw = DA(md, body_invweight0), *diw = DA(md, dof_invweight0);
  const int32_t *et = IA(md, eq_type), *eo1 = IA(md, eq_obj1id), *eo2 = IA(md, eq_obj2id);
  const int32_t *jd = IA(md, jnt_dofadr), *gbody = IA(md, geom_bodyid);
  int start = 0;
  for (int r = 0; r < d->nefc; r++) {
    int t = d->efc_type[r], id = d->efc_con[r];
    if (r == 0 || d->efc_type[r - 1] != t || d->efc_con[r - 1] != id) start = r;
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
      int b1 = gbody[d->con_g1[id]], b2 = gbody[d->con_g2[id]];
      v = (k < 3) ? biw[2 * b1] + biw[2 * b2] : biw[2 * b1 + 1] + biw[2 * b2 + 1];
    }
    d->efc_dA[r] = v;
  }
}

static void make_constraints(const Mdl* md, Dat* d) {
  const mgs_model_desc* m = md->m;
  int nv = m->nv;
  d->nefc = 0;
  double jp1[3 * 128], jr1[3 * 128], jp2[3 * 128], jr2[3 * 128];
  /* --- equality */
  const int32_t *et = IA(md, eq_type), *eo1 = IA(md, eq_obj1id), *eo2 = IA(md, eq_obj2id);
  const double* ed = DA(md, eq_data);
  for (int e = 0; e < m->neq; e++) {
    const double* data = ed + 11 * e;
    if (et[e] == MGS_EQ_CONNECT || et[e] == MGS_EQ_WELD) {
      int b1 = eo1[e], b2 = eo2[e];
      double p1[3], p2[3], t[3];
      if (et[e] == MGS_EQ_CONNECT) {
        mulmv3(t, d->xmat + 9 * b1, data);
        add3(p1, d->xpos + 3 * b1, t);
        mulmv3(t, d->xmat + 9 * b2, data + 3);
        add3(p2, d->xpos + 3 * b2, t);
      } else {
        mulmv3(t, d->xmat + 9 * b1, data);
        add3(p1, d->xpos + 3 * b1, t);
        p2[0] = d->xpos[3 * b2]; p2[1] = d->xpos[3 * b2 + 1]; p2[2] = d->xpos[3 * b2 + 2];
      }
      jac_point(md, d, b1, p1, jp1, jr1);
      jac_point(md, d, b2, p2, jp2, jr2);
      if (d->nefc + (et[e] == MGS_EQ_WELD ? 6 : 3) > d->nefc_max) { d->overflow |= 2; break; }
      for (int k = 0; k < 3; k++) {
        int r = add_row(d, MGS_EFC_EQUALITY, p1[k] - p2[k], 0.0, 1, e);
        for (int c = 0; c < nv; c++) d->J[r * nv + c] = jp1[k * nv + c] - jp2[k * nv + c];
      }
      if (et[e] == MGS_EQ_WELD) {
        double q1r[4], q2c[4], qe[4];
        quatmul(q1r, d->xquat + 4 * b1, data + 3);
        q2c[0] = d->xquat[4 * b2]; q2c[1] = -d->xquat[4 * b2 + 1];
        q2c[2] = -d->xquat[4 * b2 + 2]; q2c[3] = -d->xquat[4 * b2 + 3];
        quatmul(qe, q2c, q1r);
        double ts = data[7];
        int rr[3];
        for (int k = 0; k < 3; k++) rr[k] = add_row(d, MGS_EFC_EQUALITY, qe[1 + k] * ts, 0.0, 1, e);
        for (int c = 0; c < nv; c++) {
          double ax[4] = {0.0, jr1[c] - jr2[c], jr1[nv + c] - jr2[nv + c], jr1[2 * nv + c] - jr2[2 * nv + c]};
          double t1q[4], t2q[4];
          quatmul(t1q, q2c, ax);
          quatmul(t2q, t1q, q1r);
          for (int k = 0; k < 3; k++) d->J[rr[k] * nv + c] = (0.5 * t2q[1 + k]) * ts;
        }
      }
    } else if (et[e] == MGS_EQ_JOINT) {
      int j1 = eo1[e], j2 = eo2[e];
      const int32_t *jq = IA(md, jnt_qposadr), *jd = IA(md, jnt_dofadr);
      double q1 = d->qpos[jq[j1]] - data[5];
      double pos, deriv = 0.0;
      if (j2 >= 0) {
        double x = d->qpos[jq[j2]] - data[6];
        double poly = data[0] + x * (data[1] + x * (data[2] + x * (data[3] + x * data[4])));
        deriv = data[1] + x * (2.0 * data[2] + x * (3.0 * data[3] + x * (4.0 * data[4])));
        pos = q1 - poly;
      } else {
        pos = q1 - data[0];
      }
      if (d->nefc + 1 > d->nefc_max) { d->overflow |= 2; break; }
      int r = add_row(d, MGS_EFC_EQUALITY, pos, 0.0, 1, e);
      d->J[r * nv + jd[j1]] = 1.0;
      if (j2 >= 0) d->J[r * nv + jd[j2]] = d->J[r * nv + jd[j2]] - deriv;
    }
  }
  int neqrows = d->nefc;
  /* --- dof friction loss */
  const double* floss = DA(md, dof_frictionloss);
  int fr0 = d->nefc;
  for (int k = 0; k < nv; k++) {
    if (floss[k] > 0.0) {
      int r = add_row(d, MGS_EFC_FRICTION, 0.0, 0.0, 1, k);
      if (r < 0) break;
      d->J[r * nv + k] = 1.0;
      d->efc_floss[r] = floss[k];
    }
  }
  int fr1 = d->nefc;
  /* --- joint limits */
  const int32_t *lim = IA(md, jnt_limited), *jq = IA(md, jnt_qposadr), *jd = IA(md, jnt_dofadr);
  const double *range = DA(md, jnt_range), *jmargin = DA(md, jnt_margin);
  int lr0 = d->nefc;
  for (int j = 0; j < m->njnt; j++) {
    if (!lim[j]) continue;
    double q = d->qpos[jq[j]];
    double dlo = q - range[2 * j], dhi = range[2 * j + 1] - q;
    if (dlo < jmargin[j]) {
      int r = add_row(d, MGS_EFC_LIMIT, dlo, jmargin[j], 1, j);
      if (r >= 0) d->J[r * nv + jd[j]] = 1.0;
    }
    if (dhi < jmargin[j]) {
      int r = add_row(d, MGS_EFC_LIMIT, dhi, jmargin[j], 1, j);
      if (r >= 0) d->J[r * nv + jd[j]] = -1.0;
    }
  }
  int lr1 = d->nefc;
  /* --- contacts */
  const int32_t *gbody = IA(md, geom_bodyid), *pcd = IA(md, pair_condim);
  const double *pfr = DA(md, pair_friction), *pmar = DA(md, pair_margin);
  int cr0 = d->nefc;
  for (int c = 0; c < d->ncon; c++) {
    int p = d->con_pair[c];
    int dim = pcd[p];
    if (d->nefc + dim > d->nefc_max) { d->overflow |= 2; break; }
    int b1 = gbody[d->con_g1[c]], b2 = gbody[d->con_g2[c]];
    const double* pt = d->con_pos + 3 * c;
    const double* fr = d->con_frame + 9 * c;
    jac_point(md, d, b1, pt, jp1, jr1);
    jac_point(md, d, b2, pt, jp2, jr2);
    int r = d->nefc;
    for (int j = 0; j < dim; j++) add_row(d, MGS_EFC_CONTACT, j == 0 ? d->con_dist[c] : 0.0, pmar[p], dim, c);
    for (int col = 0; col < nv; col++) {
      double dp[3] = {jp2[col] - jp1[col], jp2[nv + col] - jp1[nv + col], jp2[2 * nv + col] - jp1[2 * nv + col]};
      for (int j = 0; j < dim && j < 3; j++) d->J[(r + j) * nv + col] = dot3(fr + 3 * j, dp);
      if (dim >= 4) {
        double dr[3] = {jr2[col] - jr1[col], jr2[nv + col] - jr1[nv + col], jr2[2 * nv + col] - jr1[2 * nv + col]};
        d->J[(r + 3) * nv + col] = dot3(fr, dr);
        if (dim == 6) {
          d->J[(r + 4) * nv + col] = dot3(fr + 3, dr);
          d->J[(r + 5) * nv + col] = dot3(fr + 6, dr);
        }
      }
    }
    for (int j = 0; j < dim; j++) d->efc_mu[5 * r + j] = (j < dim - 1) ? pfr[5 * p + j] : 0.0;
  }
  int cr1 = d->nefc;
  /* --- per row: velocity, J.qacc_smooth, whitened row G = D^-1/2 L^-1 J^T
   * (stored in K), diagonal A = G.G */
  int ne = d->nefc;
  for (int r = 0; r < ne; r++) {
    const double* Jr = d->J + (size_t)r * nv;
    double* Gr = d->K + (size_t)r * nv;
    double v = 0.0, bj = 0.0;
    for (int k = 0; k < nv; k++) v = v + Jr[k] * d->qvel[k];
    for (int k = 0; k < nv; k++) bj = bj + Jr[k] * d->qacc_smooth[k];
    d->efc_vel[r] = v;
    d->efc_b[r] = bj;
    for (int i = 0; i < nv; i++) {
      double s = Jr[i];
      for (int k = 0; k < i; k++) s = fma(-d->L[i * nv + k], Gr[k], s);
      Gr[i] = s;
    }
    for (int i = 0; i < nv; i++) Gr[i] = Gr[i] * d->isD[i];
    double a = 0.0;
    for (int k = 0; k < nv; k++) a = a + Gr[k] * Gr[k];
    d->efc_A[r] = a;
  }
  diag_approx(md, d);
  const double *eqsr = DA(md, eq_solref), *eqsi = DA(md, eq_solimp);
  for (int r = 0; r < neqrows; r++) {
    int e = d->efc_con[r];
    row_params(md, d, r, 1, eqsr + 2 * e, eqsi + 5 * e, NULL, 0,
               g_eqimp == 1 ? d->efc_pos[r] : eq_violation_norm(d, r, neqrows));
  }
  const double *dsr = DA(md, dof_solref), *dsi = DA(md, dof_solimp);
  for (int r = fr0; r < fr1; r++) {
    int k = d->efc_con[r];
    row_params(md, d, r, 1, dsr + 2 * k, dsi + 5 * k, NULL, 0, d->efc_pos[r]);
  }
  const double *jsr = DA(md, jnt_solref), *jsi = DA(md, jnt_solimp);
  for (int r = lr0; r < lr1; r++) {
    int j = d->efc_con[r];
    row_params(md, d, r, 1, jsr + 2 * j, jsi + 5 * j, NULL, 0, d->efc_pos[r]);
  }
  const double *psr = DA(md, pair_solref), *psi = DA(md, pair_solimp);
  for (int r = cr0; r < cr1;) {
    int c = d->efc_con[r];
    int p = d->con_pair[c];
    int dim = d->efc_dim[r];
    row_params(md, d, r, dim, psr + 2 * p, psi + 5 * p, d->efc_mu + 5 * r, 1, d->efc_pos[r]);
    r += dim;
  }
  for (int r = 0; r < ne; r++) {
    d->efc_b[r] = d->efc_b[r] - d->efc_aref[r];
    double ar = d->efc_A[r] + d->efc_R[r];
    d->efc_AR[r] = ar;
    d->efc_ARinv[r] = 1.0 / ar;
    d->efc_Ainv[r] = 1.0 / d->efc_A[r];
  }
  /* contact blocks of A = G G^T */
  for (int r = cr0; r < cr1;) {
    int dim = d->efc_dim[r];
    double* blk = d->efc_blk + 36 * r;
    for (int i = 0; i < dim; i++)
      for (int j = 0; j < dim; j++) {
        const double* Gi = d->K + (size_t)(r + i) * nv;
        const double* Gj = d->K + (size_t)(r + j) * nv;
        double a = 0.0;
        for (int k = 0; k < nv; k++) a = a + Gi[k] * Gj[k];
        blk[i * dim + j] = a;
      }
    r += dim;
  }
}

/* ------------------------------------------------------------------------ */
/* QCQP: minimize 0.5 x'Ax + x'b  s.t.  sum (x_j/mu_j)^2 <= r^2 (n = 2, 3),
 * Newton on the Lagrange multiplier with closed-form inverses (cf. MuJoCo's
 * mju_QCQP2 / mju_QCQP3). */
static void qcqp2(const double* A, const double* b, const double* mu, double r, double* x) {
  double a11 = (A[0] * mu[0]) * mu[0], a12 = (A[1] * mu[0]) * mu[1], a22 = (A[3] * mu[1]) * mu[1];
  double b1 = b[0] * mu[0], b2 = b[1] * mu[1];
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
  }
  x[0] = v1 * mu[0];
  x[1] = v2 * mu[1];
  /* active constraint: put the result on the ellipsoid (MuJoCo PGS / noslip) */
  if (!sing && la != 0.0) {
    double s = (x[0] * x[0]) / (mu[0] * mu[0]) + (x[1] * x[1]) / (mu[1] * mu[1]);
    s = sqrt((r * r) / (s > O_MINVAL ? s : O_MINVAL));
    x[0] = x[0] * s;
    x[1] = x[1] * s;
  }
}

static void qcqp3(const double* A, const double* b, const double* mu, double r, double* x) {
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
    s = sqrt((r * r) / (s > O_MINVAL ? s : O_MINVAL));
    x[0] = x[0] * s;
    x[1] = x[1] * s;
    x[2] = x[2] * s;
  }
}

/* n = 5 (condim-6 contacts): MuJoCo's general mju_QCQP restated (parity
 * unpinned: its source is not here).  The same Newton iteration on the
 * multiplier with (A + la I) factored by Cholesky; a pivot below 1e-10 counts
 * as singular (result 0).  The kernel's qcqpn<N> has this arithmetic. */
static void qcqpn(int n, const double* A, const double* b, const double* mu, double r, double* x) {
  double As[25], bs[5], v[5], L[25], t[5], pv[5];
  for (int i = 0; i < n; i++) {
    bs[i] = b[i] * mu[i];
    v[i] = 0.0;
    for (int j = 0; j < n; j++) As[i * n + j] = (A[i * n + j] * mu[i]) * mu[j];
  }
  double rr = r * r, la = 0.0;
  int sing = 0;
  for (int it = 0; it < 20; it++) {
    for (int q = 0; q < n * n; q++) L[q] = As[q];
    for (int i = 0; i < n; i++) L[i * n + i] = L[i * n + i] + la;
    for (int j = 0; j < n; j++) {
      double p = L[j * n + j];
      for (int k = 0; k < j; k++) p = p - L[j * n + k] * L[j * n + k];
      if (p < 1e-10) sing = 1;
      p = sqrt(p < 1e-10 ? 1e-10 : p);
      L[j * n + j] = p;
      for (int i = j + 1; i < n; i++) {
        double s = L[i * n + j];
        for (int k = 0; k < j; k++) s = s - L[i * n + k] * L[j * n + k];
        L[i * n + j] = s / p;
      }
    }
    if (sing) {
      for (int i = 0; i < n; i++) v[i] = 0.0;
      break;
    }
    for (int i = 0; i < n; i++) {
      double s = bs[i];
      for (int k = 0; k < i; k++) s = s - L[i * n + k] * t[k];
      t[i] = s / L[i * n + i];
    }
    for (int i = n - 1; i >= 0; i--) {
      double s = t[i];
      for (int k = i + 1; k < n; k++) s = s - L[k * n + i] * v[k];
      v[i] = s / L[i * n + i];
    }
    for (int i = 0; i < n; i++) v[i] = -v[i];
    double vv = 0.0;
    for (int i = 0; i < n; i++) vv = vv + v[i] * v[i];
    double val = vv - rr;
    if (val < 1e-10) break;
    for (int i = 0; i < n; i++) {
      double s = v[i];
      for (int k = 0; k < i; k++) s = s - L[i * n + k] * t[k];
      t[i] = s / L[i * n + i];
    }
    for (int i = n - 1; i >= 0; i--) {
      double s = t[i];
      for (int k = i + 1; k < n; k++) s = s - L[k * n + i] * pv[k];
      pv[i] = s / L[i * n + i];
    }
    double vp = 0.0;
    for (int i = 0; i < n; i++) vp = vp + v[i] * pv[i];
    double deriv = -2.0 * vp;
    double delta = -val / deriv;
    if (delta < 1e-10) break;
    la = la + delta;
  }
  for (int i = 0; i < n; i++) x[i] = v[i] * mu[i];
  if (!sing && la != 0.0) {
    double s = 0.0;
    for (int i = 0; i < n; i++) s = s + (x[i] * x[i]) / (mu[i] * mu[i]);
    s = sqrt((r * r) / (s > O_MINVAL ? s : O_MINVAL));
    for (int i = 0; i < n; i++) x[i] = x[i] * s;
  }
}

static void qcqp(int n, const double* A, const double* b, const double* mu, double r, double* x) {
  if (n == 2) qcqp2(A, b, mu, r, x);
  else if (n == 3) qcqp3(A, b, mu, r, x);
  else qcqpn(n, A, b, mu, r, x);
}

/* MuJoCo's costChange (engine_solver.c): the change of the dual cost
 * 0.5 d'Ad + d'res of a block update; an update that raises the cost by more
 * than 1e-10 is undone (force restored, change 0).  PGS and noslip apply it
 * to every scalar row and every contact block. */
static double cost_change1(double A, double delta, double res) {
  return ((0.5 * delta) * delta) * A + delta * res;
}

static double cost_change(int n, const double* A, const double* delta, const double* res) {
  double vav = 0.0, dr = 0.0;
  for (int i = 0; i < n; i++) {
    double ad = 0.0;
    for (int j = 0; j < n; j++) ad = ad + A[i * n + j] * delta[j];
    vav = vav + delta[i] * ad;
  }
  for (int i = 0; i < n; i++) dr = dr + delta[i] * res[i];
  return 0.5 * vav + dr;
}

static void project_block(const Dat* d, int r, double* f) {
  int t = d->efc_type[r];
  if (t == MGS_EFC_FRICTION) {
    double fl = d->efc_floss[r];
    if (f[0] < -fl) f[0] = -fl;
    if (f[0] > fl) f[0] = fl;
  } else if (t == MGS_EFC_LIMIT) {
    if (f[0] < 0.0) f[0] = 0.0;
  } else if (t == MGS_EFC_CONTACT) {
    int dim = d->efc_dim[r];
    if (f[0] < 0.0) { for (int j = 0; j < dim; j++) f[j] = 0.0; return; }
    if (dim == 1) return;
    const double* mu = d->efc_mu + 5 * r;
    double s = 0.0;
    for (int j = 1; j < dim; j++) { double q = f[j] / mu[j - 1]; s = s + q * q; }
    double nt = sqrt(s);
    if (nt > f[0]) {
      double sc = f[0] / nt;
      for (int j = 1; j < dim; j++) f[j] = f[j] * sc;
    }
  }
}

/* PGS on the dual with elliptic cones (MuJoCo mj_solPGS restated) in the
 * whitened form A = G G^T, u = G^T f, followed by noslip. */
static void solve_pgs_main(const Mdl* md, Dat* d) {
  const mgs_model_desc* m = md->m;
  int nv = m->nv, ne = d->nefc;
  /* MuJoCo engine_solver.c: scale = 1 / (m->stat.meaninertia * mjMAX(1, nv)) with
   * stat.meaninertia the mean diagonal of M at qpos0 (mj_setConst) */
  double scale = 1.0 / (m->meaninertia * (double)(nv > 1 ? nv : 1));
  /* warmstart: f from qacc_warmstart through the primal map, projected;
   * J_r . qacc_ws = G_r . (D^1/2 L^T qacc_ws) */
  double hws[128];
  for (int i = 0; i < nv; i++) {
    double s = d->qacc_ws[i];
    for (int k = i + 1; k < nv; k++) s = s + d->L[k * nv + i] * d->qacc_ws[k];
    hws[i] = s * d->sD[i];
  }
  for (int r = 0; r < ne; r++) {
    const double* Gr = d->K + (size_t)r * nv;
    double jar = 0.0;
    for (int k = 0; k < nv; k++) jar = jar + Gr[k] * hws[k];
    jar = jar - d->efc_aref[r];
    d->efc_f[r] = -jar / d->efc_R[r];
  }
  for (int r = 0; r < ne;) {
    int dim = d->efc_type[r] == MGS_EFC_CONTACT ? d->efc_dim[r] : 1;
    if (d->efc_type[r] != MGS_EFC_EQUALITY) project_block(d, r, d->efc_f + r);
    r += dim;
  }
  for (int k = 0; k < nv; k++) {
    double s = 0.0;
    for (int r = 0; r < ne; r++) s = s + d->K[(size_t)r * nv + k] * d->efc_f[r];
    d->w[k] = s;
  }
  double cw = 0.0;
  for (int r = 0; r < ne; r++) {
    const double* Gr = d->K + (size_t)r * nv;
    double jw = 0.0;
    for (int k = 0; k < nv; k++) jw = jw + Gr[k] * d->w[k];
    cw = cw + d->efc_f[r] * ((0.5 * (jw + d->efc_R[r] * d->efc_f[r])) + d->efc_b[r]);
  }
  if (!(cw < 0.0)) {
    for (int r = 0; r < ne; r++) d->efc_f[r] = 0.0;
    for (int k = 0; k < nv; k++) d->w[k] = 0.0;
  }
  int it;
  for (it = 0; it < m->iterations && ne > 0; it++) {
    double improvement = 0.0;
    for (int r = 0; r < ne;) {
      int t = d->efc_type[r];
      if (t != MGS_EFC_CONTACT || d->efc_dim[r] == 1) {
        const double* Gr = d->K + (size_t)r * nv;
        double res = (tree_dot(Gr, d->w, nv) + d->efc_R[r] * d->efc_f[r]) + d->efc_b[r];
        double AR = d->efc_AR[r];
        double fo = d->efc_f[r];
        double fnew[1] = {fo - res * d->efc_ARinv[r]};
        if (t != MGS_EFC_EQUALITY) project_block(d, r, fnew);
        double delta = fnew[0] - fo;
        double ch = cost_change1(AR, delta, res);
        if (ch > 1e-10) { delta = 0.0; ch = 0.0; }
        improvement = improvement - ch;
        if (delta != 0.0) {
          d->efc_f[r] = fnew[0];
          for (int k = 0; k < nv; k++) d->w[k] = d->w[k] + Gr[k] * delta;
        }
        r += 1;
      } else {
        int dim = d->efc_dim[r];
        double res[6], old[6], nw[6], Ab[36];
        const double* blk = d->efc_blk + 36 * r;
        for (int i = 0; i < dim; i++) {
          res[i] = (tree_dot(d->K + (size_t)(r + i) * nv, d->w, nv) + d->efc_R[r + i] * d->efc_f[r + i]) +
                   d->efc_b[r + i];
          old[i] = d->efc_f[r + i];
          for (int j = 0; j < dim; j++) Ab[i * dim + j] = blk[i * dim + j];
          Ab[i * dim + i] = Ab[i * dim + i] + d->efc_R[r + i];
        }
        double fn = old[0] - res[0] * d->efc_ARinv[r];
        if (fn < 0.0) fn = 0.0;
        double dn = fn - old[0];
        nw[0] = fn;
        if (fn < O_MINVAL) {
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
          qcqp(nf, Ac, bq, d->efc_mu + 5 * r, fn, nw + 1);
        }
        double del[6];
        for (int i = 0; i < dim; i++) del[i] = nw[i] - old[i];
        double dc = cost_change(dim, Ab, del, res);
        if (dc > 1e-10) {
          for (int i = 0; i < dim; i++) { nw[i] = old[i]; del[i] = 0.0; }
          dc = 0.0;
        }
        improvement = improvement - dc;
        for (int i = 0; i < dim; i++) d->efc_f[r + i] = nw[i];
        for (int k = 0; k < nv; k++) {
          double s = d->w[k];
          for (int i = 0; i < dim; i++) s = s + d->K[(size_t)(r + i) * nv + k] * del[i];
          d->w[k] = s;
        }
        r += dim;
      }
    }
    if (improvement * scale < m->tolerance) { it++; break; }
  }
  d->iters += it;
}

/* noslip (MuJoCo mj_solNoSlip restated): PGS over friction dims only,
 * unregularized, normal forces fixed; u = G^T f must be current. */
static void noslip(const Mdl* md, Dat* d) {
  const mgs_model_desc* m = md->m;
  int nv = m->nv, ne = d->nefc;
  /* MuJoCo engine_solver.c: scale = 1 / (m->stat.meaninertia * mjMAX(1, nv)) with
   * stat.meaninertia the mean diagonal of M at qpos0 (mj_setConst) */
  double scale = 1.0 / (m->meaninertia * (double)(nv > 1 ? nv : 1));
  /* noslip: friction dims only, unregularized, normal forces fixed */
  for (int ns = 0; ns < m->noslip_iterations && ne > 0; ns++) {
    double improvement = 0.0;
    /* the noslip cost drops the regulariser: count its removal at iteration 0 */
    if (ns == 0)
      for (int r = 0; r < ne; r++) improvement = improvement + ((0.5 * d->efc_f[r]) * d->efc_f[r]) * d->efc_R[r];
    for (int r = 0; r < ne;) {
      int t = d->efc_type[r];
      if (t == MGS_EFC_FRICTION) {
        const double* Gr = d->K + (size_t)r * nv;
        double res = tree_dot(Gr, d->w, nv) + d->efc_b[r];
        double fo = d->efc_f[r];
        double fnew[1] = {fo - res * d->efc_Ainv[r]};
        project_block(d, r, fnew);
        double delta = fnew[0] - fo;
        double ch = cost_change1(d->efc_A[r], delta, res);
        if (ch > 1e-10) { delta = 0.0; ch = 0.0; }
        improvement = improvement - ch;
        if (delta != 0.0) {
          d->efc_f[r] = fnew[0];
          for (int k = 0; k < nv; k++) d->w[k] = d->w[k] + Gr[k] * delta;
        }
        r += 1;
      } else if (t == MGS_EFC_CONTACT && d->efc_dim[r] > 1) {
        int dim = d->efc_dim[r];
        int nf = dim - 1;
        const double* blk = d->efc_blk + 36 * r;
        double res[5], old[5], Ac[25], bq[5], nw[5], del[5];
        for (int i = 0; i < nf; i++) {
          res[i] = tree_dot(d->K + (size_t)(r + 1 + i) * nv, d->w, nv) + d->efc_b[r + 1 + i];
          old[i] = d->efc_f[r + 1 + i];
        }
        for (int i = 0; i < nf; i++) {
          double s = res[i];
          for (int j = 0; j < nf; j++) {
            Ac[i * nf + j] = blk[(1 + i) * dim + 1 + j];
            s = s - Ac[i * nf + j] * old[j];
          }
          bq[i] = s;
        }
        if (d->efc_f[r] < O_MINVAL) for (int i = 0; i < nf; i++) nw[i] = 0.0;
        else qcqp(nf, Ac, bq, d->efc_mu + 5 * r, d->efc_f[r], nw);
        for (int i = 0; i < nf; i++) del[i] = nw[i] - old[i];
        double dc = cost_change(nf, Ac, del, res);
        if (dc > 1e-10) {
          for (int i = 0; i < nf; i++) { nw[i] = old[i]; del[i] = 0.0; }
          dc = 0.0;
        }
        improvement = improvement - dc;
        for (int i = 0; i < nf; i++) d->efc_f[r + 1 + i] = nw[i];
        for (int k = 0; k < nv; k++) {
          double s = d->w[k];
          for (int i = 0; i < nf; i++) s = s + d->K[(size_t)(r + 1 + i) * nv + k] * del[i];
          d->w[k] = s;
        }
        r += dim;
      } else {
        r += (t == MGS_EFC_CONTACT) ? d->efc_dim[r] : 1;
      }
    }
    if (improvement * scale < m->noslip_tolerance) break;
  }
}

/* qacc = qacc_smooth + L^-T D^-1/2 u_main ;  qfrc_constraint = L D^1/2 u.
 * u_main is the main solver's u: MuJoCo's mj_fwdConstraint saves
 * qacc_warmstart before mj_solNoSlip runs, and qacc feeds nothing but the
 * warmstart (implicitfast integrates qfrc_smooth + qfrc_constraint). */
static void finalize_solution(const Mdl* md, Dat* d, const double* u_main) {
  int nv = md->m->nv;
  double z[128];
  for (int i = nv - 1; i >= 0; i--) {
    double s = u_main[i] * d->isD[i];
    for (int k = nv - 1; k > i; k--) s = fma(-d->L[k * nv + i], z[k], s);   /* k descending (kernel order) */
    z[i] = s;
  }
  double t[128];
  for (int i = 0; i < nv; i++) t[i] = d->w[i] * d->sD[i];
  for (int i = 0; i < nv; i++) {
    double s = t[i];
    for (int k = 0; k < i; k++) s = fma(d->L[i * nv + k], t[k], s);
    d->qfrc_constraint[i] = s;
    d->qacc[i] = d->qacc_smooth[i] + z[i];
  }
}

/* ---------------------------------------------------------------------- */
/* Newton solver on the primal (MuJoCo mj_solNewton restated), in whitened
 * coordinates w = D^1/2 L^T qacc, where the Gauss cost is 1/2||w - w0||^2 and
 * every constraint row is jar = G_r.w - aref.  The soft-constraint cost of a
 * row block is the convex conjugate of the dual (PGS) problem:
 *   s(jar) = max_{f in K} (-f.jar - 1/2 f'Rf),   z = -R^-1/2 jar,  y = Proj_{R^1/2 K}(z),
 *   f = R^-1/2 y,  s = y.z - 1/2|y|^2  (= 1/2|y|^2 for cones),
 * which for elliptic contacts with R_t = R_n mu0^2/(impratio mu_j^2) is the
 * isotropic second-order cone |y_t| <= mu' y_n, mu' = mu0/sqrt(impratio)
 * (MuJoCo's "mu = friction[0]/sqrt(impratio)").  Reductions over dofs use
 * tree_dot (lanes over dofs), reductions over rows use tree_rows (lanes over
 * rows, rows >= 64 pre-added to row mod 64 in ascending order). */
static double tree_rows(const double* v, int ne) {
  double leaf[64], one[64];
  int n = ne < 64 ? ne : 64;
  if (n <= 0) return 0.0;
  for (int k = 0; k < n; k++) {
    /* lane k holds rows k, k + 64, k + 128, k + 192 (kernel Frc): summed in that order */
    double s = v[k];
    for (int h = 1; h < 4; h++)
      if (k + 64 * h < ne) s = s + v[k + 64 * h];
    leaf[k] = s;
    one[k] = 1.0;
  }
  /* tree_dot multiplies by 1.0: exact */
  return tree_dot(leaf, one, n);
}

#define ST_OFF 0
#define ST_QUAD 1
#define ST_CONE 2
#define ST_SAT 3

/* evaluate row r (or the block starting at r) at violations jr[];
 * writes forces f[], returns cost; state per row; hb = Hessian block (dim x dim) for cones */
static double row_eval(const Dat* d, int r, const double* jr, double* f, int* st, double* hb, double* cq) {
  int t = d->efc_type[r];
  if (t == MGS_EFC_EQUALITY) {
    double Dr = d->efc_Dr[r];
    f[0] = -jr[0] * Dr;
    st[0] = ST_QUAD;
    return ((0.5 * Dr) * jr[0]) * jr[0];
  }
  if (t == MGS_EFC_LIMIT || (t == MGS_EFC_CONTACT && d->efc_dim[r] == 1)) {
    double Dr = d->efc_Dr[r];
    if (jr[0] < 0.0) {
      f[0] = -jr[0] * Dr;
      st[0] = ST_QUAD;
      return ((0.5 * Dr) * jr[0]) * jr[0];
    }
    f[0] = 0.0;
    st[0] = ST_OFF;
    return 0.0;
  }
  if (t == MGS_EFC_FRICTION) {
    double z = -jr[0] * d->efc_isR[r];
    double lim = d->efc_floss[r] * d->efc_sqR[r];
    double y = z;
    st[0] = ST_QUAD;
    if (z > lim) { y = lim; st[0] = ST_SAT; }
    else if (z < -lim) { y = -lim; st[0] = ST_SAT; }
    f[0] = y * d->efc_isR[r];
    return y * z - 0.5 * (y * y);
  }
  /* elliptic contact block */
  int dim = d->efc_dim[r];
  double mup = d->efc_mup[r];
  double z[6], y[6];
  for (int a = 0; a < dim; a++) z[a] = -jr[a] * d->efc_isR[r + a];
  double t2 = 0.0;
  for (int a = 1; a < dim; a++) t2 = t2 + z[a] * z[a];
  double tn = sqrt(t2);
  int zone;
  double yn = 0.0, itn = 0.0, sc = 0.0;
  if (tn <= mup * z[0]) {
    zone = ST_QUAD;
    for (int a = 0; a < dim; a++) y[a] = z[a];
  } else if (mup * tn <= -z[0]) {
    zone = ST_OFF;
    for (int a = 0; a < dim; a++) y[a] = 0.0;
  } else {
    zone = ST_CONE;
    /* k1 = 1 / (1 + mu'^2) per block; one reciprocal of |z_t| per evaluation */
    yn = (z[0] + mup * tn) * d->efc_k1[r];
    itn = 1.0 / tn;
    sc = (mup * yn) * itn;
    y[0] = yn;
    for (int a = 1; a < dim; a++) y[a] = sc * z[a];
  }
  double c = 0.0;
  for (int a = 0; a < dim; a++) {
    f[a] = y[a] * d->efc_isR[r + a];
    st[a] = zone;
    c = c + y[a] * y[a];
  }
  if (cq && zone == ST_CONE) {
    /* cone curvature: k1 = 1/(1+mu'^2), k2 = mu' yn / |z_t|, e = z_t / |z_t| */
    cq[0] = d->efc_k1[r];
    cq[1] = sc;
    for (int a = 1; a < dim; a++) cq[1 + a] = z[a] * itn;
  }
  if (hb && zone == ST_CONE) {
    double k1 = d->efc_k1[r];
    double k2 = sc;
    double v[6], e[6];
    v[0] = 1.0;
    e[0] = 0.0;
    for (int a = 1; a < dim; a++) { e[a] = z[a] * itn; v[a] = mup * e[a]; }
    for (int a = 0; a < dim; a++)
      for (int b = 0; b < dim; b++) {
        double P = (k1 * v[a]) * v[b];
        if (a >= 1 && b >= 1) P = P + k2 * ((a == b ? 1.0 : 0.0) - e[a] * e[b]);
        hb[a * dim + b] = (d->efc_isR[r + a] * d->efc_isR[r + b]) * P;
      }
  }
  return 0.5 * c;
}

/* jar = G w - aref ; forces, states, cone Hessian blocks ; returns total cost */
static double newton_eval(const Mdl* md, Dat* d, const double* w, const double* w0) {
  int nv = md->m->nv, ne = d->nefc;
  double q[128], cr[256];
  for (int k = 0; k < nv; k++) q[k] = w[k] - w0[k];
  double gauss = 0.5 * tree_dot(q, q, nv);
  for (int r = 0; r < ne; r++) {
    const double* Gr = d->K + (size_t)r * nv;
    double s = 0.0;
    for (int k = 0; k < nv; k++) s = fma(Gr[k], w[k], s);
    d->efc_jar[r] = s - d->efc_aref[r];
  }
  for (int r = 0; r < ne;) {
    int dim = (d->efc_type[r] == MGS_EFC_CONTACT) ? d->efc_dim[r] : 1;
    cr[r] = row_eval(d, r, d->efc_jar + r, d->efc_f + r, d->efc_state + r, d->efc_hb + 36 * r, NULL);
    for (int a = 1; a < dim; a++) cr[r + a] = 0.0;
    r += dim;
  }
  return gauss + tree_rows(cr, ne);
}

static void newton_grad(const Dat* d, int nv, const double* w, const double* w0, double* g) {
  for (int k = 0; k < nv; k++) {
    double s = 0.0;
    for (int r = 0; r < d->nefc; r++) s = fma(d->K[(size_t)r * nv + k], d->efc_f[r], s);
    g[k] = (w[k] - w0[k]) - s;
  }
}

/* line-search derivatives at step alpha along direction with jv = G dir */
static void ls_eval(const Dat* d, double alpha, double A1, double A2, double* d1, double* d2) {
  int ne = d->nefc;
  double c1[256], c2[256];
  for (int r = 0; r < ne;) {
    int dim = (d->efc_type[r] == MGS_EFC_CONTACT) ? d->efc_dim[r] : 1;
    double jr[6], f[6], cq[8];
    int st[6];
    for (int a = 0; a < dim; a++) jr[a] = d->efc_jar[r + a] + alpha * d->efc_jv[r + a];
    row_eval(d, r, jr, f, st, NULL, cq);
    double s1 = 0.0, s2 = 0.0;
    if (dim == 1) {
      s1 = -f[0] * d->efc_jv[r];
      if (st[0] == ST_QUAD) s2 = (d->efc_jv[r] * d->efc_Dr[r]) * d->efc_jv[r];
    } else {
      for (int a = 0; a < dim; a++) s1 = s1 - f[a] * d->efc_jv[r + a];
      if (st[0] == ST_QUAD) {
        for (int a = 0; a < dim; a++) s2 = s2 + (d->efc_jv[r + a] * d->efc_Dr[r + a]) * d->efc_jv[r + a];
      } else if (st[0] == ST_CONE) {
        /* jv' hb jv in closed form: u_a = jv_a / sqrt(R_a),
         * s2 = k1 (v.u)^2 + k2 (|u_t|^2 - (e.u_t)^2),  v = (1, mu' e) */
        double mup = d->efc_mup[r];
        double u[6];
        for (int a = 0; a < dim; a++) u[a] = d->efc_jv[r + a] * d->efc_isR[r + a];
        double vu = u[0], eu = 0.0, uu = 0.0;
        for (int a = 1; a < dim; a++) {
          vu = vu + (mup * cq[1 + a]) * u[a];
          eu = eu + cq[1 + a] * u[a];
          uu = uu + u[a] * u[a];
        }
        s2 = (cq[0] * vu) * vu + cq[1] * (uu - eu * eu);
      }
    }
    c1[r] = s1;
    c2[r] = s2;
    for (int a = 1; a < dim; a++) { c1[r + a] = 0.0; c2[r + a] = 0.0; }
    r += dim;
  }
  *d1 = (A1 + alpha * A2) + tree_rows(c1, ne);
  *d2 = A2 + tree_rows(c2, ne);
}

static void solve_newton(const Mdl* md, Dat* d) {
  const mgs_model_desc* m = md->m;
  int nv = m->nv, ne = d->nefc;
  /* MuJoCo engine_solver.c: scale = 1 / (m->stat.meaninertia * mjMAX(1, nv)) with
   * stat.meaninertia the mean diagonal of M at qpos0 (mj_setConst) */
  double scale = 1.0 / (m->meaninertia * (double)(nv > 1 ? nv : 1));
  /* per-row constants */
  for (int r = 0; r < ne; r++) {
    double sq = sqrt(d->efc_R[r]);
    d->efc_sqR[r] = sq;
    d->efc_isR[r] = 1.0 / sq;
    d->efc_Dr[r] = 1.0 / d->efc_R[r];
  }
  for (int r = 0; r < ne;) {
    int dim = (d->efc_type[r] == MGS_EFC_CONTACT) ? d->efc_dim[r] : 1;
    if (dim > 1) {
      double mup = d->efc_mu[5 * r] / sqrt(m->impratio);
      d->efc_mup[r] = mup;
      d->efc_k1[r] = 1.0 / (1.0 + mup * mup);
    }
    r += dim;
  }
  /* whitened smooth and warmstart accelerations: W(a)_i = sD_i (a_i + sum_{k>i} L_ki a_k) */
  double w0[MGS_MAX_NV], w[MGS_MAX_NV], g[MGS_MAX_NV], dir[MGS_MAX_NV], HDinv[MGS_MAX_NV], HDv[MGS_MAX_NV];
  static __thread double H[MGS_MAX_NV * MGS_MAX_NV], HL[MGS_MAX_NV * MGS_MAX_NV];   /* 2 x 128 KB: per thread, off the stack */
  for (int i = 0; i < nv; i++) {
    double s = d->qacc_smooth[i], s2 = d->qacc_ws[i];
    for (int k = i + 1; k < nv; k++) s = fma(d->L[k * nv + i], d->qacc_smooth[k], s);
    for (int k = i + 1; k < nv; k++) s2 = fma(d->L[k * nv + i], d->qacc_ws[k], s2);
    w0[i] = s * d->sD[i];
    w[i] = s2 * d->sD[i];
  }
  double C = 0.0;
  if (ne > 0) {
    double cws = newton_eval(md, d, w, w0);
    double c0 = newton_eval(md, d, w0, w0);
    if (cws < c0) C = newton_eval(md, d, w, w0);
    else { for (int k = 0; k < nv; k++) w[k] = w0[k]; C = c0; }
  } else {
    for (int k = 0; k < nv; k++) w[k] = w0[k];
  }
  newton_grad(d, nv, w, w0, g);
  int it = 0;
  for (it = 0; it < m->iterations && ne > 0; it++) {
    /* Hessian I + G' W G with W block diagonal: Dr on quad rows, the cone
       Hessian block on cone blocks, 0 on inactive rows.  X = W G row by row
       (x = 0.0 + sum_a G_{lead+a,i} w_a), then H_ij = (i == j) + an fma chain
       over the rows in ascending order of G_rj X_ri: the kernel computes the
       sum with v_mfma_f64_16x16x4 k-steps, which round once per row (probed
       bit-exactly on MI355X, tools/probes/mfma_f64_check.py). */
    for (int r = 0; r < ne; r++) {
      int t = d->efc_type[r], st = d->efc_state[r];
      double wv[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
      int lead = r, nd = 0;
      if (st == ST_QUAD) {
        wv[0] = d->efc_Dr[r];
        nd = 1;
      } else if (st == ST_CONE && t == MGS_EFC_CONTACT) {
        lead = r;
        while (lead > 0 && d->efc_type[lead - 1] == MGS_EFC_CONTACT && d->efc_con[lead - 1] == d->efc_con[r] &&
               r - lead < 5)
          lead--;
        int dim = d->efc_dim[r], bp = r - lead;
        const double* hb = d->efc_hb + 36 * lead;
        for (int a = 0; a < dim; a++) wv[a] = hb[a * dim + bp];
        nd = dim;
      }
      for (int i = 0; i < nv; i++) {
        double x = 0.0;
        for (int a = 0; a < nd; a++) x = x + d->K[(size_t)(lead + a) * nv + i] * wv[a];
        d->hX[(size_t)r * nv + i] = x;
      }
    }
    for (int i = 0; i < nv; i++)
      for (int j = 0; j <= i; j++) {
        double s = 0.0;
        for (int r = 0; r < ne; r++) s = fma(d->K[(size_t)r * nv + j], d->hX[(size_t)r * nv + i], s);
        H[i * nv + j] = (i == j ? 1.0 : 0.0) + s;
        H[j * nv + i] = H[i * nv + j];
      }
    ldl_factor(nv, H, HL, HDinv, HDv);
    ldl_solve(nv, HL, HDinv, g, dir);
    for (int k = 0; k < nv; k++) dir[k] = -dir[k];
    for (int r = 0; r < ne; r++) {
      const double* Gr = d->K + (size_t)r * nv;
      double s = 0.0;
      for (int k = 0; k < nv; k++) s = fma(Gr[k], dir[k], s);
      d->efc_jv[r] = s;
    }
    double q[MGS_MAX_NV];
    for (int k = 0; k < nv; k++) q[k] = w[k] - w0[k];
    double A1 = tree_dot(q, dir, nv);
    double A2 = tree_dot(dir, dir, nv);
    /* exact line search: 1-D Newton with bracketing on the cost derivative */
    double p0, q0, alpha = 0.0;
    ls_eval(d, 0.0, A1, A2, &p0, &q0);
    if (p0 < 0.0) {
      double lo = 0.0, hi = 0.0;
      int hi_ok = 0;
      alpha = -p0 / q0;
      for (int ls = 0; ls < m->ls_iterations; ls++) {
        double p, qq;
        ls_eval(d, alpha, A1, A2, &p, &qq);
        if (fabs(p) < m->ls_tolerance * (-p0)) break;
        if (p < 0.0) lo = alpha;
        else { hi = alpha; hi_ok = 1; }
        double an = alpha - p / qq;
        if (!(an > lo) || (hi_ok && !(an < hi))) an = hi_ok ? 0.5 * (lo + hi) : 2.0 * alpha;
        alpha = an;
      }
    }
    if (!(alpha > 0.0)) { it++; break; }
    for (int k = 0; k < nv; k++) w[k] = w[k] + alpha * dir[k];
    double Cn = newton_eval(md, d, w, w0);
    newton_grad(d, nv, w, w0, g);
    double improvement = scale * (C - Cn);
    C = Cn;
    double gn = scale * sqrt(tree_dot(g, g, nv));
    if (improvement < m->tolerance || gn < m->tolerance) { it++; break; }
  }
  d->iters += it;
  /* u = G^T f */
  for (int k = 0; k < nv; k++) {
    double s = 0.0;
    for (int r = 0; r < ne; r++) s = fma(d->K[(size_t)r * nv + k], d->efc_f[r], s);
    d->w[k] = s;
  }
}

static void solve(const Mdl* md, Dat* d) {
  if (md->m->solver == 0) solve_pgs_main(md, d);
  else solve_newton(md, d);
  double u_main[128];
  memcpy(u_main, d->w, sizeof(double) * md->m->nv);
  noslip(md, d);
  finalize_solution(md, d, u_main);
}

/* ------------------------------------------------------------------------ */
/* forward: kinematics + collision (+ dynamics and solver when full != 0) */
static void forward(const Mdl* md, Dat* d, int full) {
  const mgs_model_desc* m = md->m;
  int nv = m->nv;
  kinematics(md, d);
  com_pos(md, d);
  collision(md, d);
  if (!full) return;
  crb(md, d);
  ldl_factor(nv, d->M, d->L, d->Dinv, d->Dv);
  for (int k = 0; k < nv; k++) {
    d->sD[k] = sqrt(d->Dv[k]);
    d->isD[k] = 1.0 / d->sD[k];
  }
  actuation(md, d);
  passive(md, d);
  rne(md, d);
  for (int k = 0; k < nv; k++)
    d->qfrc_smooth[k] = (d->qfrc_passive[k] - d->qfrc_bias[k]) + d->qfrc_actuator[k];
  ldl_solve(nv, d->L, d->Dinv, d->qfrc_smooth, d->qacc_smooth);
  make_constraints(md, d);
  solve(md, d);
}

/* implicitfast velocity update + position integration */
static void integrate(const Mdl* md, Dat* d) {
  const mgs_model_desc* m = md->m;
  int nv = m->nv;
  double dt = m->timestep;
  /* qDeriv: dof damping + actuator velocity gains (skipped when force clamped) */
  for (int i = 0; i < nv * nv; i++) d->qDeriv[i] = 0.0;
  const double* damp = DA(md, dof_damping);
  for (int k = 0; k < nv; k++) d->qDeriv[k * nv + k] = -damp[k];
  const int32_t *gtype = IA(md, actuator_gaintype), *btype = IA(md, actuator_biastype);
  const int32_t* flim = IA(md, actuator_forcelimited);
  const double *gain = DA(md, actuator_gainprm), *bias = DA(md, actuator_biasprm);
  const double* frange = DA(md, actuator_forcerange);
  for (int u = 0; u < m->nu; u++) {
    double f = d->act_force[u];
    if (flim[u] && (f <= frange[2 * u] || f >= frange[2 * u + 1])) continue;
    double dv = 0.0;
    if (btype[u] == MGS_BIAS_AFFINE) dv = dv + bias[3 * u + 2];
    if (gtype[u] == MGS_GAIN_AFFINE) dv = dv + gain[3 * u + 2] * d->ctrl[u];
    if (dv == 0.0) continue;
    const double* mom = d->act_moment + u * nv;
    for (int i = 0; i < nv; i++) {
      if (mom[i] == 0.0) continue;
      for (int j = 0; j < nv; j++)
        d->qDeriv[i * nv + j] = d->qDeriv[i * nv + j] + mom[i] * (mom[j] * dv);
    }
  }
  for (int i = 0; i < nv * nv; i++) d->MI[i] = d->M[i] - dt * d->qDeriv[i];
  ldl_factor(nv, d->MI, d->LI, d->DIinv, d->Dv);
  double rhs[128] = {0}, qa[128];
  for (int k = 0; k < nv; k++) rhs[k] = d->qfrc_smooth[k] + d->qfrc_constraint[k];
  ldl_solve(nv, d->LI, d->DIinv, rhs, qa);
  for (int k = 0; k < nv; k++) d->qvel[k] = d->qvel[k] + dt * qa[k];
  const int32_t *jtype = IA(md, jnt_type), *jq = IA(md, jnt_qposadr), *jd = IA(md, jnt_dofadr);
  for (int j = 0; j < m->njnt; j++) {
    int a = jq[j], v = jd[j];
    if (jtype[j] == MGS_JNT_FREE) {
      d->qpos[a] = d->qpos[a] + dt * d->qvel[v];
      d->qpos[a + 1] = d->qpos[a + 1] + dt * d->qvel[v + 1];
      d->qpos[a + 2] = d->qpos[a + 2] + dt * d->qvel[v + 2];
      double ax[3] = {d->qvel[v + 3], d->qvel[v + 4], d->qvel[v + 5]};
      double nrm = normalize3(ax);
      double qr[4], qn[4];
      axisangle2quat(qr, ax, dt * nrm);
      quatmul(qn, d->qpos + a + 3, qr);
      normalize4(qn);
      d->qpos[a + 3] = qn[0]; d->qpos[a + 4] = qn[1]; d->qpos[a + 5] = qn[2]; d->qpos[a + 6] = qn[3];
    } else {
      d->qpos[a] = d->qpos[a] + dt * d->qvel[v];
    }
  }
  for (int k = 0; k < nv; k++) d->qacc_ws[k] = d->qacc[k];
  d->time = d->time + dt;
  /* actuator state (mj_advance: act += dt act_dot), a mujoco.pid integral then
   * clamped to |ki integral| <= imax */
  const int32_t* aadr = IA(md, actuator_actadr);
  const double* pid = DA(md, actuator_pidprm);
  for (int u = 0; u < m->nu && m->nact > 0; u++) {
    if (gtype[u] != MGS_GAIN_PID) continue;
    const double* pp = pid + 5 * u;
    int k = aadr[u];
    if (pp[4] >= 0.0) {
      d->act[k] = d->act[k] + dt * d->act_dot[k];
      k++;
    }
    if (pp[1] != 0.0) {
      double v = d->act[k] + dt * d->act_dot[k];
      if (pp[3] >= 0.0) {
        const double lim = pp[3] / fabs(pp[1]);
        if (v < -lim) v = -lim;
        if (v > lim) v = lim;
      }
      d->act[k] = v;
    }
  }
}

static void step(const Mdl* md, Dat* d) {
  forward(md, d, 1);
  integrate(md, d);
}

static int obj_contact(const Mdl* md, const Dat* d) {
  const int32_t* side = IA(md, geom_side);
  for (int c = 0; c < d->ncon; c++) {
    int s1 = side[d->con_g1[c]], s2 = side[d->con_g2[c]];
    if ((s1 < 0 && s2 > 0) || (s1 > 0 && s2 < 0)) return 1;
  }
  return 0;
}

/* clutter_table.py:237-252: a gripper geom against the table or past it */
static int obj_contact_incl(const Mdl* md, const Dat* d) {
  const int32_t* side = IA(md, geom_side);
  for (int c = 0; c < d->ncon; c++) {
    int s1 = side[d->con_g1[c]], s2 = side[d->con_g2[c]];
    if ((s1 < 0 && s2 >= 0) || (s1 >= 0 && s2 < 0)) return 1;
  }
  return 0;
}

/* the contact predicates on a given contact list (tests: pinned against the
 * reference's check_* functions on scripted contacts, tests/golden/
 * make_golden_more.py): pairs = n (geom1, geom2) collision-geom indices;
 * predicate MGS_PRED_ANY_CONTACT / PARTITION / PARTITION_INCL */
int oracle_contact_predicate(const mgs_model_desc* desc, const int32_t* I, const double* D, const int32_t* pairs,
                             int n, int predicate) {
  Mdl md = {desc, I, D};
  Dat d;
  memset(&d, 0, sizeof(d));
  int g1[64], g2[64];
  if (n > 64) n = 64;
  for (int c = 0; c < n; c++) { g1[c] = pairs[2 * c]; g2[c] = pairs[2 * c + 1]; }
  d.ncon = n;
  d.con_g1 = g1;
  d.con_g2 = g2;
  if (predicate == MGS_PRED_ANY_CONTACT) return n != 0;
  return predicate == MGS_PRED_PARTITION_INCL ? obj_contact_incl(&md, &d) : obj_contact(&md, &d);
}

static void reset(const Mdl* md, Dat* d, const double* qpos_init, const double* mpos, const double* mquat) {
  const mgs_model_desc* m = md->m;
  memcpy(d->qpos, qpos_init, sizeof(double) * m->nq);
  memcpy(d->qvel, DA(md, qvel0), sizeof(double) * m->nv);
  memcpy(d->qacc_ws, DA(md, qacc_ws0), sizeof(double) * m->nv);
  memset(d->ctrl, 0, sizeof(double) * (m->nu > 0 ? m->nu : 1));
  for (int k = 0; k < m->nact; k++) { d->act[k] = DA(md, act0)[k]; d->act_dot[k] = 0.0; }
  for (int k = 0; k < 3; k++) d->mocap_pos[k] = mpos ? mpos[k] : 0.0;
  for (int k = 0; k < 4; k++) d->mocap_quat[k] = mquat[k];
  d->time = 0.0;
  d->overflow = 0;
  d->iters = 0;
  for (int k = 0; k < O_CERT; k++) d->cert[O_CERT_W * k] = -1.0;
}

/* ------------------------------------------------------------------------ */
/* exported API (ctypes) */
int oracle_abi_version(void) { return MGS_ABI_VERSION; }

int oracle_collision_free(const mgs_model_desc* desc, const int32_t* I, const double* D, int n,
                          const double* qpos_init, const double* mocap_pos, const double* mocap_quat,
                          int predicate, uint8_t* out, int nthreads) {
  Mdl md = {desc, I, D};
  (void)nthreads;
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1)
  {
    Dat* d = dat_alloc(&md);
    /* the masks skip multiccd (kernel collision(mccd 0)): its contacts repeat
     * a pair that already has one, so no mask predicate changes, and they
     * cannot crowd a later pair's first contact out of the capacity */
    d->mask_only = 1;
#pragma omp for schedule(dynamic, 4)
    for (int i = 0; i < n; i++) {
      reset(&md, d, qpos_init + (size_t)i * desc->nq, mocap_pos + 3 * i, mocap_quat + 4 * i);
      forward(&md, d, 0);
      int hit = (predicate == MGS_PRED_ANY_CONTACT) ? (d->ncon != 0)
                : (predicate == MGS_PRED_PARTITION_INCL) ? obj_contact_incl(&md, d) : obj_contact(&md, d);
      out[i] = (uint8_t)(hit ? 0 : 1);
    }
    dat_free(d);
  }
  return 0;
}

static void rollout_batch(const mgs_model_desc* desc, const int32_t* I, const double* D,
                          const mgs_schedule* sc, int n, const double* qpos_init,
                          const double* mocap_quat, const double* phase_start, const double* phase_target,
                          uint8_t* label, int32_t* fail_step, double* obj_qpos, int32_t* stats,
                          const double* vstate_init, double* state_out, int nthreads) {
  Mdl md = {desc, I, D};
  int np = sc->nphase;
  int obj_qposadr = sc->obj_qposadr;
  int nq = desc->nq, nv = desc->nv, na = desc->nact;
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1)
  {
    Dat* d = dat_alloc(&md);
#pragma omp for schedule(dynamic, 1)
    for (int i = 0; i < n; i++) {
      const double* ps = phase_start + (size_t)i * np * 3;
      const double* pt = phase_target + (size_t)i * np * 3;
      reset(&md, d, qpos_init + (size_t)i * nq, ps, mocap_quat + 4 * i);
      if (vstate_init) {
        const double* vs = vstate_init + (size_t)i * (2 * nv + na);
        memcpy(d->qvel, vs, sizeof(double) * nv);
        memcpy(d->qacc_ws, vs + nv, sizeof(double) * nv);
        if (na > 0) memcpy(d->act, vs + 2 * nv, sizeof(double) * na);
      }
      int ok = 1, gstep = 0, fstep = -1, maxcon = 0, maxefc = 0, sumcon = 0, sumefc = 0;
      for (int p = 0; p < np && ok; p++) {
        for (int u = 0; u < desc->nu; u++) d->ctrl[u] = sc->ctrl[p * 32 + u];
        int ns = sc->nsteps[p];
        for (int t = 0; t < ns && ok; t++) {
          double frac = (double)t / (double)ns;
          for (int k = 0; k < 3; k++) d->mocap_pos[k] = ps[3 * p + k] + (pt[3 * p + k] - ps[3 * p + k]) * frac;
          step(&md, d);
          if (d->ncon > maxcon) maxcon = d->ncon;
          if (d->nefc > maxefc) maxefc = d->nefc;
          sumcon += d->ncon;
          sumefc += d->nefc;
          /* divergence guard (mj_checkPos / mj_checkVel / mj_checkAcc): stop, label 0 */
          {
            int bad = 0;
            for (int k = 0; k < nq; k++) bad |= !(fabs(d->qpos[k]) <= MGS_MAXVAL);
            for (int k = 0; k < nv; k++) bad |= !(fabs(d->qvel[k]) <= MGS_MAXVAL) || !(fabs(d->qacc_ws[k]) <= MGS_MAXVAL);
            if (bad) { ok = 0; fstep = gstep; d->overflow |= MGS_FLAG_DIVERGED; break; }
          }
          if (sc->vclip > 0.0)
            for (int k = 0; k < nv; k++) {
              if (d->qvel[k] > sc->vclip) d->qvel[k] = sc->vclip;
              if (d->qvel[k] < -sc->vclip) d->qvel[k] = -sc->vclip;
            }
          int ce = sc->check_every[p];
          int tc = t + sc->check_offset[p];
          if (ce > 0 && tc > 0 && (tc % ce) == 0 && !obj_contact(&md, d)) { ok = 0; fstep = gstep; }
          gstep++;
        }
        if (ok && sc->check_at_end[p] && !obj_contact(&md, d)) { ok = 0; fstep = gstep - 1; }
      }
      if (label) label[i] = (uint8_t)ok;
      if (fail_step) fail_step[i] = fstep;
      if (obj_qpos && obj_qposadr >= 0)
        for (int k = 0; k < 7; k++) obj_qpos[7 * i + k] = d->qpos[obj_qposadr + k];
      if (stats) {
        int32_t* st = stats + MGS_NSTATS * i;
        st[0] = maxcon; st[1] = maxefc; st[2] = d->overflow; st[3] = d->iters; st[4] = sumcon; st[5] = sumefc;
      }
      if (state_out) {
        double* so = state_out + (size_t)i * (nq + 2 * nv + na);
        memcpy(so, d->qpos, sizeof(double) * nq);
        memcpy(so + nq, d->qvel, sizeof(double) * nv);
        memcpy(so + nq + nv, d->qacc_ws, sizeof(double) * nv);
        if (na > 0) memcpy(so + nq + 2 * nv, d->act, sizeof(double) * na);
      }
    }
    dat_free(d);
  }
}

int oracle_rollout(const mgs_model_desc* desc, const int32_t* I, const double* D,
                   const mgs_schedule* sc, int n, const double* qpos_init,
                   const double* mocap_quat, const double* phase_start, const double* phase_target,
                   uint8_t* label, int32_t* fail_step, double* obj_qpos, int32_t* stats, int nthreads) {
  rollout_batch(desc, I, D, sc, n, qpos_init, mocap_quat, phase_start, phase_target, label, fail_step, obj_qpos,
                stats, NULL, NULL, nthreads);
  return 0;
}

/* mgs_simulate restated: the rollout loop from per-state (qpos, qvel,
 * warmstart, act), final state out (n * (nq + 2nv + nact)) */
int oracle_simulate_batch(const mgs_model_desc* desc, const int32_t* I, const double* D,
                          const mgs_schedule* sc, int n, const double* qpos_init, const double* vstate_init,
                          const double* mocap_quat, const double* phase_start, const double* phase_target,
                          double* state_out, int32_t* stats, int nthreads) {
  mgs_schedule s = *sc;   /* no contact checks: a free simulation never stops early */
  for (int p = 0; p < MGS_MAX_PHASES; p++) { s.check_every[p] = 0; s.check_at_end[p] = 0; }
  rollout_batch(desc, I, D, &s, n, qpos_init, mocap_quat, phase_start, phase_target, NULL, NULL, NULL, stats,
                vstate_init, state_out, nthreads);
  return 0;
}

/* Antipodal ray casting (mgs_antipodal_contacts, csrc/mgs_sampler.hip; the
 * reference's trimesh intersects_location in antipodal.py:117-145): Moller-
 * Trumbore per triangle, valid hits at distance >= eps, the k-th valid hit,
 * k = min(floor(u * count), count - 1), +dir hits before -dir hits. */
static int o_ray_tri(const double* o, const double* d, const double* T, double* tout) {
  double e1[3], e2[3], p[3], tv[3], q[3];
  for (int k = 0; k < 3; k++) { e1[k] = T[3 + k] - T[k]; e2[k] = T[6 + k] - T[k]; }
  p[0] = d[1] * e2[2] - d[2] * e2[1];
  p[1] = d[2] * e2[0] - d[0] * e2[2];
  p[2] = d[0] * e2[1] - d[1] * e2[0];
  double det = (e1[0] * p[0] + e1[1] * p[1]) + e1[2] * p[2];
  if (!(fabs(det) > 1e-12)) return 0;
  double inv = 1.0 / det;
  for (int k = 0; k < 3; k++) tv[k] = o[k] - T[k];
  double u = ((tv[0] * p[0] + tv[1] * p[1]) + tv[2] * p[2]) * inv;
  q[0] = tv[1] * e1[2] - tv[2] * e1[1];
  q[1] = tv[2] * e1[0] - tv[0] * e1[2];
  q[2] = tv[0] * e1[1] - tv[1] * e1[0];
  double w = ((q[0] * d[0] + q[1] * d[1]) + q[2] * d[2]) * inv;
  double t = ((e2[0] * q[0] + e2[1] * q[1]) + e2[2] * q[2]) * inv;
  if (u >= 0.0 && w >= 0.0 && u + w <= 1.0 && t > 0.0) { *tout = t; return 1; }
  return 0;
}

static int o_ray_valid(const double* o, const double* d, double t, double eps, double* loc) {
  double s = 0.0;
  for (int k = 0; k < 3; k++) {
    loc[k] = o[k] + t * d[k];
    double r = loc[k] - o[k];
    s = s + r * r;
  }
  return sqrt(s) >= eps;
}

int oracle_antipodal_contacts(const double* tri, int ntri, int n, const double* origin, const double* dir,
                              const double* u_choice, double eps, double* out_second, int32_t* out_nvalid,
                              int nthreads) {
#pragma omp parallel for num_threads(nthreads > 0 ? nthreads : 1) schedule(static)
  for (int i = 0; i < n; i++) {
    const double* o = origin + 3 * i;
    double dp[3] = {dir[3 * i], dir[3 * i + 1], dir[3 * i + 2]}, dm[3] = {-dp[0], -dp[1], -dp[2]};
    int cnt[2] = {0, 0};
    for (int s = 0; s < 2; s++)
      for (int j = 0; j < ntri; j++) {
        double t, loc[3];
        if (o_ray_tri(o, s ? dm : dp, tri + 9 * j, &t) && o_ray_valid(o, s ? dm : dp, t, eps, loc)) cnt[s]++;
      }
    int total = cnt[0] + cnt[1];
    double sel[3] = {0, 0, 0};
    if (total > 0) {
      double fk = floor(u_choice[i] * (double)total);
      int kth = fk < (double)(total - 1) ? (int)fk : total - 1;
      int s = kth < cnt[0] ? 0 : 1, kk = s ? kth - cnt[0] : kth, seen = 0;
      for (int j = 0; j < ntri && seen <= kk; j++) {
        double t, loc[3];
        if (o_ray_tri(o, s ? dm : dp, tri + 9 * j, &t) && o_ray_valid(o, s ? dm : dp, t, eps, loc)) {
          if (seen == kk) { sel[0] = loc[0]; sel[1] = loc[1]; sel[2] = loc[2]; }
          seen++;
        }
      }
    }
    out_nvalid[i] = total;
    for (int k = 0; k < 3; k++) out_second[3 * i + k] = sel[k];
  }
  return 0;
}

/* Debug/KAT helper: run nsteps with a fixed mocap and ctrl from an initial
 * state, recording qpos after every step (nsteps * nq) and ncon per step. */
int oracle_trace(const mgs_model_desc* desc, const int32_t* I, const double* D, const double* qpos_init,
                 const double* mocap_pos, const double* mocap_quat, const double* ctrl, int nsteps,
                 double* qpos_trace, int32_t* ncon_trace, double* qvel_out) {
  Mdl md = {desc, I, D};
  Dat* d = dat_alloc(&md);
  reset(&md, d, qpos_init, mocap_pos, mocap_quat);
  for (int u = 0; u < desc->nu; u++) d->ctrl[u] = ctrl[u];
  for (int s = 0; s < nsteps; s++) {
    step(&md, d);
    if (qpos_trace) memcpy(qpos_trace + (size_t)s * desc->nq, d->qpos, sizeof(double) * desc->nq);
    if (ncon_trace) ncon_trace[s] = d->ncon;
  }
  if (qvel_out) memcpy(qvel_out, d->qvel, sizeof(double) * desc->nv);
  dat_free(d);
  return 0;
}

/* Debug helper: contacts of one configuration (after kinematics+collision). */
int oracle_contacts(const mgs_model_desc* desc, const int32_t* I, const double* D, const double* qpos,
                    const double* mocap_pos, const double* mocap_quat, int maxc, double* pos, double* frame,
                    double* dist, int32_t* geoms) {
  Mdl md = {desc, I, D};
  Dat* d = dat_alloc(&md);
  reset(&md, d, qpos, mocap_pos, mocap_quat);
  forward(&md, d, 0);
  int nc = d->ncon < maxc ? d->ncon : maxc;
  for (int c = 0; c < nc; c++) {
    memcpy(pos + 3 * c, d->con_pos + 3 * c, 3 * sizeof(double));
    memcpy(frame + 9 * c, d->con_frame + 9 * c, 9 * sizeof(double));
    dist[c] = d->con_dist[c];
    geoms[2 * c] = d->con_g1[c];
    geoms[2 * c + 1] = d->con_g2[c];
  }
  int r = d->ncon;
  dat_free(d);
  return r;
}

/* unit test hook for the shared numeric primitives */
void oracle_sincos(const double* x, int n, double* s, double* c) {
  for (int i = 0; i < n; i++) o_sincos(x[i], s + i, c + i);
}

/* unit test hook for the canonical lane reduction */
double oracle_tree_dot(const double* a, const double* b, int n) { return tree_dot(a, b, n); }

/* Debug hook: one forward() at a given state with a given solver; returns
 * nefc and copies efc_f (nefc), qacc (nv), types/dims and the Newton/PGS
 * iteration count; optionally the rows' G, aref, R | b, and pos | margin |
 * diagApprox | vel (4 nefc). */
int oracle_forward_debug(const mgs_model_desc* desc, const int32_t* I, const double* D, const double* qpos,
                         const double* qvel, const double* qacc_ws, const double* mocap_pos,
                         const double* mocap_quat, const double* ctrl, int solver, double* f_out, double* qacc_out,
                         int32_t* type_out, int32_t* iters_out, double* G_out, double* aref_out, double* R_out,
                         double* pos_out) {
  mgs_model_desc m2 = *desc;
  m2.solver = solver;
  Mdl md = {&m2, I, D};
  Dat* d = dat_alloc(&md);
  reset(&md, d, qpos, mocap_pos, mocap_quat);
  memcpy(d->qvel, qvel, sizeof(double) * desc->nv);
  memcpy(d->qacc_ws, qacc_ws, sizeof(double) * desc->nv);
  for (int u = 0; u < desc->nu; u++) d->ctrl[u] = ctrl[u];
  forward(&md, d, 1);
  int ne = d->nefc;
  memcpy(f_out, d->efc_f, sizeof(double) * ne);
  memcpy(qacc_out, d->qacc, sizeof(double) * desc->nv);
  for (int r = 0; r < ne; r++) type_out[r] = d->efc_type[r] * 16 + d->efc_dim[r];
  if (G_out) memcpy(G_out, d->K, sizeof(double) * ne * desc->nv);
  if (aref_out) memcpy(aref_out, d->efc_aref, sizeof(double) * ne);
  if (R_out) { memcpy(R_out, d->efc_R, sizeof(double) * ne); memcpy(R_out + ne, d->efc_b, sizeof(double) * ne); }
  if (pos_out) {   /* efc_pos, efc_margin, efc_diagApprox, efc_vel */
    memcpy(pos_out, d->efc_pos, sizeof(double) * ne);
    memcpy(pos_out + ne, d->efc_margin, sizeof(double) * ne);
    memcpy(pos_out + 2 * ne, d->efc_dA, sizeof(double) * ne);
    memcpy(pos_out + 3 * ne, d->efc_vel, sizeof(double) * ne);
  }
  *iters_out = d->iters;
  dat_free(d);
  return ne;
}
