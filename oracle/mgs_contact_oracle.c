/* mgs_contact_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker of
 * csrc/mgs_contact.hip; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline may call it).
 *
 * Sequential C restatement of the reference's contact-based dexterous-hand
 * sampler (ContactBasedDiff, mgs/sampler/contact.py):
 *   - farthest_point_sampling (mgs/sampler/kin/jax_util.py:182-203)
 *   - seed neighbourhoods: nearest seed (contact.py:226-228) and the random
 *     pick of ntip admissible seeds (contact.py:199-214)
 *   - the AdamW fit (contact.py:98-158 update/loss_fn, 254-280 the initial
 *     assignment and the 150-iteration loop) over the forward kinematics of
 *     forward_kinematic_point_transform (mgs/sampler/kin/base.py:80-113,
 *     quaternion algebra jax_util.py:22-120) and the permutation assignment
 *     find_best_assignment_and_reorder_targets (jax_util.py:205-224).
 *
 * Parity: the reference runs in JAX float32 with jax.random keys, flax/optax;
 * none of JAX, flax or optax is installed here, so this restatement (float64,
 * splitmix64 keys) is PARITY UNPINNED against the reference.  The gradient is
 * the exact derivative of the forward computation (forward mode over the
 * joints, reverse over the Gram-Schmidt rotation), checked against finite
 * differences in tests/test_contact_sampler.py; the optimiser restates
 * optax.adamw (scale_by_adam -> add_decayed_weights -> scale(-lr)).
 * The device kernels follow these expressions one for one (-ffp-contract=off),
 * so GPU == oracle is bit-exact. */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/mgs_gpu.h"

void oracle_sincos(const double* x, int n, double* s, double* c);

/* quaternion_raw_multiply_jax (jax_util.py:22-39), left-to-right sums */
static void qmul(double* o, const double* a, const double* b) {
  o[0] = ((a[0] * b[0] - a[1] * b[1]) - a[2] * b[2]) - a[3] * b[3];
  o[1] = ((a[0] * b[1] + a[1] * b[0]) + a[2] * b[3]) - a[3] * b[2];
  o[2] = ((a[0] * b[2] - a[1] * b[3]) + a[2] * b[0]) + a[3] * b[1];
  o[3] = ((a[0] * b[3] + a[1] * b[2]) - a[2] * b[1]) + a[3] * b[0];
}

/* quaternion_apply_jax (jax_util.py:85-101): (q (0, v) q^-1)[1:], q^-1 = conj */
static void qrot(double* o, const double* q, const double* v) {
  double p[4] = {0.0, v[0], v[1], v[2]}, t[4], r[4];
  double c[4] = {q[0], -q[1], -q[2], -q[3]};
  qmul(t, q, p);
  qmul(r, t, c);
  o[0] = r[1]; o[1] = r[2]; o[2] = r[3];
}

/* d/dtheta of q(theta) v q(theta)^-1 given dq: dq v q* + q v dq* */
static void qrot_d(double* o, const double* q, const double* dq, const double* v) {
  double p[4] = {0.0, v[0], v[1], v[2]}, t[4], r1[4], r2[4];
  double c[4] = {q[0], -q[1], -q[2], -q[3]}, dc[4] = {dq[0], -dq[1], -dq[2], -dq[3]};
  qmul(t, dq, p);
  qmul(r1, t, c);
  qmul(t, q, p);
  qmul(r2, t, dc);
  o[0] = r1[1] + r2[1]; o[1] = r1[2] + r2[2]; o[2] = r1[3] + r2[3];
}

/* transform_points_jax: rotate then translate */
static void tapply(double* o, const double* T, const double* v) {
  double r[3];
  qrot(r, T, v);
  o[0] = r[0] + T[4]; o[1] = r[1] + T[5]; o[2] = r[2] + T[6];
}

/* se3_raw_mupltiply (jax_util.py:109-114) */
static void compose(double* o, const double* A, const double* B) {
  double q[4], t[3];
  qmul(q, A, B);
  tapply(t, A, B + 4);
  o[0] = q[0]; o[1] = q[1]; o[2] = q[2]; o[3] = q[3];
  o[4] = t[0]; o[5] = t[1]; o[6] = t[2];
}

/* the joint's dynamic transform and its theta-derivative:
 * quaternion_from_axis_angle (jax_util.py:125-130) and translation dir*theta */
static void joint_tf(const mgs_kin_desc* K, int i, double th, double* J, double* dq) {
  const double* a = K->joint_tf[i] + 3;
  double n = sqrt((a[0] * a[0] + a[1] * a[1]) + a[2] * a[2]);
  double ax = a[0] / n, ay = a[1] / n, az = a[2] / n;
  double h = th / 2.0, s, c;
  oracle_sincos(&h, 1, &s, &c);
  J[0] = c; J[1] = ax * s; J[2] = ay * s; J[3] = az * s;
  J[4] = K->joint_tf[i][0] * th; J[5] = K->joint_tf[i][1] * th; J[6] = K->joint_tf[i][2] * th;
  dq[0] = -0.5 * s; dq[1] = ax * (0.5 * c); dq[2] = ay * (0.5 * c); dq[3] = az * (0.5 * c);
}

/* forward kinematics of tip a's chain: the three tip-frame points (contact,
 * origin, normal point) in the hand frame (X[3][3]) and, when dX != NULL,
 * their derivatives with respect to the chain's joints (dX[s][3][3]) */
static void tip_fk(const mgs_kin_desc* K, int a, const double* th, double X[3][3],
                   double dX[MGS_KIN_MAXCHAIN][3][3]) {
  int L = K->chain_len[a];
  double W[7] = {1.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  double A[MGS_KIN_MAXCHAIN][7], J[MGS_KIN_MAXCHAIN][7], dq[MGS_KIN_MAXCHAIN][4];
  for (int s = 0; s < L; s++) {
    int i = K->chain[a][s];
    compose(A[s], W, K->kin_tf[i]);
    joint_tf(K, i, th[i], J[s], dq[s]);
    compose(W, A[s], J[s]);
  }
  const double zero[3] = {0.0, 0.0, 0.0};
  const double* P[3] = {K->tip_point[a], zero, K->tip_normal[a]};
  for (int p = 0; p < 3; p++) {
    tapply(X[p], W, P[p]);
    if (!dX) continue;
    double y[3] = {P[p][0], P[p][1], P[p][2]};
    for (int s = L - 1; s >= 0; s--) {
      int i = K->chain[a][s];
      double z[3], t1[3];
      qrot_d(z, J[s], dq[s], y);
      z[0] = z[0] + K->joint_tf[i][0]; z[1] = z[1] + K->joint_tf[i][1]; z[2] = z[2] + K->joint_tf[i][2];
      qrot(dX[s][p], A[s], z);
      tapply(t1, J[s], y);
      tapply(y, K->kin_tf[i], t1);
    }
  }
}

/* rotation_6d_to_matrix (jax_util.py:147-155): rows b1, b2, b3 */
static void gs6(const double* r, double* R, double* n1o, double* n2o, double* dd) {
  double n1 = sqrt((r[0] * r[0] + r[1] * r[1]) + r[2] * r[2]);
  double b1[3] = {r[0] / n1, r[1] / n1, r[2] / n1};
  double d = (b1[0] * r[3] + b1[1] * r[4]) + b1[2] * r[5];
  double c[3] = {r[3] - d * b1[0], r[4] - d * b1[1], r[5] - d * b1[2]};
  double n2 = sqrt((c[0] * c[0] + c[1] * c[1]) + c[2] * c[2]);
  double b2[3] = {c[0] / n2, c[1] / n2, c[2] / n2};
  R[0] = b1[0]; R[1] = b1[1]; R[2] = b1[2];
  R[3] = b2[0]; R[4] = b2[1]; R[5] = b2[2];
  R[6] = b1[1] * b2[2] - b1[2] * b2[1];
  R[7] = b1[2] * b2[0] - b1[0] * b2[2];
  R[8] = b1[0] * b2[1] - b1[1] * b2[0];
  if (n1o) { *n1o = n1; *n2o = n2; *dd = d; }
}

static void world(const double* R, const double* p, const double* x, double* o) {
  for (int i = 0; i < 3; i++) o[i] = ((R[3 * i] * x[0] + R[3 * i + 1] * x[1]) + R[3 * i + 2] * x[2]) + p[i];
}

/* find_best_assignment_and_reorder_targets: the first permutation of least
 * summed distance; out[a] = T[perm[a]] */
static void assign(const mgs_kin_desc* K, const double (*X)[3], const double* T, double* out) {
  int nt = K->ntip;
  double D[MGS_KIN_MAXTIP][MGS_KIN_MAXTIP];
  for (int a = 0; a < nt; a++)
    for (int b = 0; b < nt; b++) {
      double d0 = X[a][0] - T[3 * b], d1 = X[a][1] - T[3 * b + 1], d2 = X[a][2] - T[3 * b + 2];
      D[a][b] = sqrt((d0 * d0 + d1 * d1) + d2 * d2);
    }
  int best = 0;
  double bc = INFINITY;
  for (int k = 0; k < K->nperm; k++) {
    double c = 0.0;
    for (int a = 0; a < nt; a++) c = c + D[a][K->perm[k][a]];
    if (c < bc) { bc = c; best = k; }
  }
  for (int a = 0; a < nt; a++)
    for (int j = 0; j < 3; j++) out[3 * a + j] = T[3 * K->perm[best][a] + j];
}

/* loss and gradient at the parameters prm (6-D rotation, position, joints)
 * against the target pool T (re-assigned here, as loss_fn does every step) */
static double loss_grad(const mgs_kin_desc* K, const double* prm, const double* T, const double* N, double* g) {
  int nd = K->ndof, nt = K->ntip;
  double R[9], n1, n2, dd, th[MGS_KIN_MAXDOF], As[3 * MGS_KIN_MAXTIP];
  double X[MGS_KIN_MAXTIP][3][3], dX[MGS_KIN_MAXTIP][MGS_KIN_MAXCHAIN][3][3];
  const double inv3n = 1.0 / (3.0 * nt);
  gs6(prm, R, &n1, &n2, &dd);
  for (int i = 0; i < nd; i++) th[i] = prm[9 + i];
  for (int a = 0; a < nt; a++) tip_fk(K, a, th, X[a], dX[a]);
  double Pw[MGS_KIN_MAXTIP][3], fn[MGS_KIN_MAXTIP][3];
  for (int a = 0; a < nt; a++) {
    double o[3], q[3];
    world(R, prm + 6, X[a][0], Pw[a]);
    world(R, prm + 6, X[a][1], o);
    world(R, prm + 6, X[a][2], q);
    for (int k = 0; k < 3; k++) fn[a][k] = q[k] - o[k];
  }
  assign(K, (const double(*)[3])Pw, T, As);
  /* loss = mean((target - p)^2) + w_cos * mean(0.5 (1 - n_surface . n_finger)) */
  double sq = 0.0, lc = 0.0;
  for (int a = 0; a < nt; a++)
    for (int k = 0; k < 3; k++) { double e = As[3 * a + k] - Pw[a][k]; sq = sq + e * e; }
  for (int a = 0; a < nt; a++) {
    double cs = (N[3 * a] * fn[a][0] + N[3 * a + 1] * fn[a][1]) + N[3 * a + 2] * fn[a][2];
    lc = lc + 0.5 * (1.0 - cs);
  }
  double loss = sq * inv3n + K->w_cos * (lc / nt);
  /* world-frame point / finger-normal gradients, then R, p, joints */
  double gP[MGS_KIN_MAXTIP][3], gF[MGS_KIN_MAXTIP][3];
  for (int a = 0; a < nt; a++)
    for (int k = 0; k < 3; k++) {
      gP[a][k] = (2.0 * (Pw[a][k] - As[3 * a + k])) * inv3n;
      gF[a][k] = (K->w_cos * (-0.5 * N[3 * a + k])) / nt;
    }
  double gR[9];
  for (int i = 0; i < 3; i++)
    for (int j = 0; j < 3; j++) {
      double s = 0.0;
      for (int a = 0; a < nt; a++) s = (s + gP[a][i] * X[a][0][j]) + gF[a][i] * (X[a][2][j] - X[a][1][j]);
      gR[3 * i + j] = s;
    }
  for (int k = 0; k < 3; k++) {
    double s = 0.0;
    for (int a = 0; a < nt; a++) s = s + gP[a][k];
    g[6 + k] = s;
  }
  for (int i = 0; i < nd; i++) g[9 + i] = 0.0;
  for (int a = 0; a < nt; a++) {
    double hP[3], hF[3];     /* hand-frame gradients R^T g */
    for (int j = 0; j < 3; j++) {
      hP[j] = (R[j] * gP[a][0] + R[3 + j] * gP[a][1]) + R[6 + j] * gP[a][2];
      hF[j] = (R[j] * gF[a][0] + R[3 + j] * gF[a][1]) + R[6 + j] * gF[a][2];
    }
    for (int s = 0; s < K->chain_len[a]; s++) {
      const double* d0 = dX[a][s][0];
      const double* d1 = dX[a][s][1];
      const double* d2 = dX[a][s][2];
      double t0 = (hP[0] * d0[0] + hP[1] * d0[1]) + hP[2] * d0[2];
      double t1 = (hF[0] * (d2[0] - d1[0]) + hF[1] * (d2[1] - d1[1])) + hF[2] * (d2[2] - d1[2]);
      g[9 + K->chain[a][s]] = g[9 + K->chain[a][s]] + (t0 + t1);
    }
  }
  /* Gram-Schmidt backward: rows b1 = R[0:3], b2 = R[3:6], b3 = b1 x b2 */
  const double *b1 = R, *b2 = R + 3, *g3 = gR + 6;
  double gb1[3], gb2[3];
  gb1[0] = gR[0] + (b2[1] * g3[2] - b2[2] * g3[1]);
  gb1[1] = gR[1] + (b2[2] * g3[0] - b2[0] * g3[2]);
  gb1[2] = gR[2] + (b2[0] * g3[1] - b2[1] * g3[0]);
  gb2[0] = gR[3] + (g3[1] * b1[2] - g3[2] * b1[1]);
  gb2[1] = gR[4] + (g3[2] * b1[0] - g3[0] * b1[2]);
  gb2[2] = gR[5] + (g3[0] * b1[1] - g3[1] * b1[0]);
  double pb2 = (b2[0] * gb2[0] + b2[1] * gb2[1]) + b2[2] * gb2[2];
  double gc[3];
  for (int k = 0; k < 3; k++) gc[k] = (gb2[k] - b2[k] * pb2) / n2;
  double gd = -((gc[0] * b1[0] + gc[1] * b1[1]) + gc[2] * b1[2]);
  double ga2[3];
  for (int k = 0; k < 3; k++) {
    gb1[k] = (gb1[k] - dd * gc[k]) + gd * prm[3 + k];
    ga2[k] = gc[k] + gd * b1[k];
  }
  double pb1 = (b1[0] * gb1[0] + b1[1] * gb1[1]) + b1[2] * gb1[2];
  for (int k = 0; k < 3; k++) {
    g[k] = (gb1[k] - b1[k] * pb1) / n1;
    g[3 + k] = ga2[k];
  }
  return loss;
}

/* one candidate: initial assignment, iters AdamW steps */
static void optimize_one(const mgs_kin_desc* K, const double* R0, const double* p0, const double* T0,
                         const double* N, double* oR, double* op, double* oj, double* oloss) {
  int nd = K->ndof, nt = K->ntip, np = 9 + nd;
  double prm[9 + MGS_KIN_MAXDOF], m[9 + MGS_KIN_MAXDOF], v[9 + MGS_KIN_MAXDOF], g[9 + MGS_KIN_MAXDOF];
  double T[3 * MGS_KIN_MAXTIP];
  /* initial fingertip positions with the initial (non-orthonormal) rotation */
  double Xw[MGS_KIN_MAXTIP][3];
  for (int a = 0; a < nt; a++) {
    double X[3][3];
    tip_fk(K, a, K->pregrasp, X, NULL);
    world(R0, p0, X[0], Xw[a]);
  }
  assign(K, (const double(*)[3])Xw, T0, T);
  /* params: 6-D rotation (first two rows of R0), position, joints */
  for (int j = 0; j < 6; j++) prm[j] = R0[j];
  for (int j = 0; j < 3; j++) prm[6 + j] = p0[j];
  for (int i = 0; i < nd; i++) prm[9 + i] = K->pregrasp[i];
  for (int j = 0; j < np; j++) { m[j] = 0.0; v[j] = 0.0; }
  double b1t = 1.0, b2t = 1.0, loss = 0.0;
  for (int it = 0; it < K->iters; it++) {
    loss = loss_grad(K, prm, T, N, g);
    /* optax.adamw: moments, bias correction, decoupled weight decay, -lr */
    b1t = b1t * K->b1;
    b2t = b2t * K->b2;
    double c1 = 1.0 - b1t, c2 = 1.0 - b2t;
    for (int j = 0; j < np; j++) {
      m[j] = (1.0 - K->b1) * g[j] + K->b1 * m[j];
      v[j] = (1.0 - K->b2) * (g[j] * g[j]) + K->b2 * v[j];
      double mh = m[j] / c1, vh = v[j] / c2;
      double u = mh / (sqrt(vh + K->eps_root) + K->eps);
      u = u + K->weight_decay * prm[j];
      prm[j] = prm[j] + (-K->lr) * u;
    }
    for (int i = 0; i < nd; i++) {
      double x = prm[9 + i];
      if (x < K->range[i][0]) x = K->range[i][0];
      if (x > K->range[i][1]) x = K->range[i][1];
      prm[9 + i] = x;
    }
  }
  gs6(prm, oR, NULL, NULL, NULL);
  for (int j = 0; j < 3; j++) op[j] = prm[6 + j];
  for (int i = 0; i < nd; i++) oj[i] = prm[9 + i];
  if (oloss) *oloss = loss;
}

void oracle_contact_optimize(const mgs_kin_desc* K, int n, const double* rot_init, const double* pos_init,
                             const double* targets, const double* normals, double* out_rot, double* out_pos,
                             double* out_joints, double* out_loss, int nthreads) {
  int nt = K->ntip;
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads > 0 ? nthreads : 1)
  for (int c = 0; c < n; c++)
    optimize_one(K, rot_init + 9 * (size_t)c, pos_init + 3 * (size_t)c, targets + 3 * nt * (size_t)c,
                 normals + 3 * nt * (size_t)c, out_rot + 9 * (size_t)c, out_pos + 3 * (size_t)c,
                 out_joints + (size_t)K->ndof * c, out_loss ? out_loss + c : NULL);
}

/* hand-frame fingertip points (contact, origin, normal point) and their joint
 * derivatives for one joint vector: the FK the optimiser differentiates */
void oracle_contact_fk(const mgs_kin_desc* K, const double* th, double* X, double* dX) {
  for (int a = 0; a < K->ntip; a++) {
    double Xa[3][3], dXa[MGS_KIN_MAXCHAIN][3][3];
    tip_fk(K, a, th, Xa, dXa);
    memcpy(X + 9 * a, Xa, sizeof(Xa));
    memcpy(dX + 9 * MGS_KIN_MAXCHAIN * a, dXa, sizeof(dXa));
  }
}

/* loss and gradient at one parameter vector for a target pool T (the
 * finite-difference check of the gradient) */
double oracle_contact_loss_grad(const mgs_kin_desc* K, const double* prm, const double* T, const double* N,
                                double* grad) {
  return loss_grad(K, prm, T, N, grad);
}

/* splitmix64 (Steele, Lea, Flood 2014): the key of seed pair (i, j) */
static uint64_t splitmix64(uint64_t x) {
  x = x + 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
static double key_uniform(uint64_t seed, uint64_t ctr) {
  return (double)(splitmix64(seed ^ splitmix64(ctr)) >> 11) * (1.0 / 9007199254740992.0);
}

/* (value, index) lexicographic order: a before b */
static int lex_less(double va, int ia, double vb, int ib) { return va < vb || (va == vb && ia < ib); }

void oracle_contact_seeds(const double* S, int k, double radius, uint64_t rng_seed, int ntip, int32_t* out_nn,
                          int32_t* out_sel, int nthreads) {
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
  for (int i = 0; i < k; i++) {
    double n0v = INFINITY, n1v = INFINITY;
    int n0i = 0x7fffffff, n1i = 0x7fffffff;
    double tv[MGS_KIN_MAXTIP];
    int ti[MGS_KIN_MAXTIP], cnt = 0;
    for (int j = 0; j < k; j++) {
      double d0 = S[3 * j] - S[3 * i], d1 = S[3 * j + 1] - S[3 * i + 1], d2 = S[3 * j + 2] - S[3 * i + 2];
      double d = sqrt((d0 * d0 + d1 * d1) + d2 * d2);
      /* two smallest (d, j) */
      if (lex_less(d, j, n1v, n1i)) {
        if (lex_less(d, j, n0v, n0i)) { n1v = n0v; n1i = n0i; n0v = d; n0i = j; }
        else { n1v = d; n1i = j; }
      }
      double key = (d < radius) ? key_uniform(rng_seed, (uint64_t)i * (uint64_t)k + (uint64_t)j) : -INFINITY;
      /* ntip largest (key, j), kept ascending */
      if (cnt < ntip || lex_less(tv[0], ti[0], key, j)) {
        int p;
        if (cnt < ntip) { p = cnt++; }
        else { for (p = 0; p + 1 < cnt; p++) { tv[p] = tv[p + 1]; ti[p] = ti[p + 1]; } p = cnt - 1; }
        while (p > 0 && lex_less(key, j, tv[p - 1], ti[p - 1])) { tv[p] = tv[p - 1]; ti[p] = ti[p - 1]; p--; }
        tv[p] = key; ti[p] = j;
      }
    }
    /* one seed: no second-nearest; the reference's sorted_indices[:, 1]
       (sampler/contact.py:213-214) clamps to column 0, the seed itself */
    out_nn[i] = n1i == 0x7fffffff ? n0i : n1i;
    /* fewer seeds than ntip (k < ntip): the empty slots take the seed itself */
    for (int a = 0; a < ntip; a++) out_sel[(size_t)i * ntip + a] = a < cnt ? ti[a] : i;
  }
}

void oracle_contact_fps(const double* x, int n, int k, int32_t* out) {
  double* dist = (double*)malloc(sizeof(double) * (size_t)(n > 0 ? n : 1));
  for (int j = 0; j < n; j++) dist[j] = INFINITY;
  if (k > 0) out[0] = 0;
  for (int i = 1; i < k; i++) {
    const double* l = x + 3 * (size_t)out[i - 1];
    int bi = 0;
    double bv = -INFINITY;
    for (int j = 0; j < n; j++) {
      double d0 = x[3 * j] - l[0], d1 = x[3 * j + 1] - l[1], d2 = x[3 * j + 2] - l[2];
      double d = (d0 * d0 + d1 * d1) + d2 * d2;
      if (d < dist[j]) dist[j] = d;
      if (dist[j] > bv) { bv = dist[j]; bi = j; }
    }
    out[i] = bi;
  }
  free(dist);
}
