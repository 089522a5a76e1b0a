// mgs_contact.hip -- the contact-based dexterous-hand sampler on the MI355X
// (reference: ContactBasedDiff.generate_grasps, mgs/sampler/contact.py:176-297,
// whose fit runs as a jitted, vmapped JAX/optax program):
//
//   mgs_fps_kernel        farthest_point_sampling (kin/jax_util.py:182-203):
//                         one workgroup of 1024 lanes carries the running
//                         minimum distances of all surface points through the
//                         k sequential picks; (value, index) argmax per wave
//                         by shuffles, across waves through LDS.
//   mgs_seeds_kernel      per seed: nearest other seed (contact.py:226-228)
//                         and the ntip largest random keys among seeds within
//                         the radius (contact.py:199-214); one lane per seed,
//                         the seed set streamed through LDS tiles.
//   mgs_contact_opt_kernel  the AdamW fit (contact.py:98-158, 254-280): one
//                         lane per candidate; forward kinematics of every
//                         fingertip chain (kin/base.py:80-113), the
//                         permutation assignment (jax_util.py:205-224), the
//                         loss and its exact gradient (joint derivatives by
//                         forward mode along each chain, the 6-D rotation by
//                         reverse mode through Gram-Schmidt), optax.adamw.
//
// Every expression follows oracle/mgs_contact_oracle.c one for one
// (-ffp-contract=off, the shared polynomial sincos), so GPU == oracle is
// bit-exact.  float64 throughout (the reference computes in JAX float32).

#define MGS_FPS_THREADS 1024
#define MGS_SEED_TILE 256

// ---------------------------------------------------------------------------
// farthest point sampling
DEVI void fps_take(double& bv, int& bi, double v, int i) {
  if (v > bv || (v == bv && i < bi)) { bv = v; bi = i; }
}

__global__ void __launch_bounds__(MGS_FPS_THREADS)
mgs_fps_kernel(const double* __restrict__ x, int n, int k, double* __restrict__ dist, int32_t* __restrict__ out) {
  __shared__ double wv[MGS_FPS_THREADS / WAVE];
  __shared__ int wi[MGS_FPS_THREADS / WAVE];
  __shared__ int last;
  const int t = threadIdx.x, lane = t & (WAVE - 1), w = t >> 6;
  for (int j = t; j < n; j += MGS_FPS_THREADS) dist[j] = INFINITY;
  if (t == 0) { last = 0; if (k > 0) out[0] = 0; }
  __syncthreads();
  for (int i = 1; i < k; i++) {
    const int li = last;
    const double lx = x[3 * li], ly = x[3 * li + 1], lz = x[3 * li + 2];
    double bv = -INFINITY;
    int bi = 0x7fffffff;
    for (int j = t; j < n; j += MGS_FPS_THREADS) {
      double d0 = x[3 * j] - lx, d1 = x[3 * j + 1] - ly, d2 = x[3 * j + 2] - lz;
      double d = (d0 * d0 + d1 * d1) + d2 * d2;
      double c = dist[j];
      if (d < c) { c = d; dist[j] = d; }
      if (c > bv) { bv = c; bi = j; }          // ascending j within the lane: first max
    }
#pragma unroll
    for (int s = 1; s < WAVE; s <<= 1) {
      double ov = __shfl_xor(bv, s);
      int oi = __shfl_xor(bi, s);
      fps_take(bv, bi, ov, oi);
    }
    if (lane == 0) { wv[w] = bv; wi[w] = bi; }
    __syncthreads();
    if (t == 0) {
      double v = wv[0];
      int b = wi[0];
      for (int q = 1; q < MGS_FPS_THREADS / WAVE; q++) fps_take(v, b, wv[q], wi[q]);
      if (b == 0x7fffffff) b = 0;
      out[i] = b;
      last = b;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
// seed neighbourhoods
DEVI uint64_t splitmix64(uint64_t x) {
  x = x + 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
DEVI double key_uniform(uint64_t seed, uint64_t ctr) {
  return (double)(splitmix64(seed ^ splitmix64(ctr)) >> 11) * (1.0 / 9007199254740992.0);
}
DEVI bool lex_less(double va, int ia, double vb, int ib) { return va < vb || (va == vb && ia < ib); }

__global__ void __launch_bounds__(MGS_SEED_TILE)
mgs_seeds_kernel(const double* __restrict__ S, int k, double radius, uint64_t rng_seed, int ntip,
                 int32_t* __restrict__ out_nn, int32_t* __restrict__ out_sel) {
  __shared__ double tile[3 * MGS_SEED_TILE];
  const int i = blockIdx.x * MGS_SEED_TILE + threadIdx.x;
  const bool act = i < k;
  double sx = 0.0, sy = 0.0, sz = 0.0;
  if (act) { sx = S[3 * i]; sy = S[3 * i + 1]; sz = S[3 * i + 2]; }
  double n0v = INFINITY, n1v = INFINITY;
  int n0i = 0x7fffffff, n1i = 0x7fffffff;
  double tv[MGS_KIN_MAXTIP];
  int ti[MGS_KIN_MAXTIP], cnt = 0;
  for (int base = 0; base < k; base += MGS_SEED_TILE) {
    __syncthreads();
    for (int q = threadIdx.x; q < 3 * MGS_SEED_TILE; q += MGS_SEED_TILE) {
      int g = 3 * base + q;
      tile[q] = g < 3 * k ? S[g] : 0.0;
    }
    __syncthreads();
    if (!act) continue;
    int m = k - base < MGS_SEED_TILE ? k - base : MGS_SEED_TILE;
    for (int q = 0; q < m; q++) {
      int j = base + q;
      double d0 = tile[3 * q] - sx, d1 = tile[3 * q + 1] - sy, d2 = tile[3 * q + 2] - sz;
      double d = sqrt((d0 * d0 + d1 * d1) + d2 * d2);
      if (lex_less(d, j, n1v, n1i)) {
        if (lex_less(d, j, n0v, n0i)) { n1v = n0v; n1i = n0i; n0v = d; n0i = j; }
        else { n1v = d; n1i = j; }
      }
      double key = (d < radius) ? key_uniform(rng_seed, (uint64_t)i * (uint64_t)k + (uint64_t)j) : -INFINITY;
      if (cnt < ntip || lex_less(tv[0], ti[0], key, j)) {
        int p;
        if (cnt < ntip) { p = cnt++; }
        else { for (p = 0; p + 1 < cnt; p++) { tv[p] = tv[p + 1]; ti[p] = ti[p + 1]; } p = cnt - 1; }
        while (p > 0 && lex_less(key, j, tv[p - 1], ti[p - 1])) { tv[p] = tv[p - 1]; ti[p] = ti[p - 1]; p--; }
        tv[p] = key; ti[p] = j;
      }
    }
  }
  if (act) {
    // one seed: no second-nearest; the reference's sorted_indices[:, 1]
    // (sampler/contact.py:213-214) clamps to column 0, the seed itself
    out_nn[i] = n1i == 0x7fffffff ? n0i : n1i;
    // fewer seeds than ntip (k < ntip): the empty slots take the seed itself
    for (int a = 0; a < ntip; a++) out_sel[(size_t)i * ntip + a] = a < cnt ? ti[a] : i;
  }
}

// ---------------------------------------------------------------------------
// the AdamW fit: quaternion algebra of kin/jax_util.py:22-130
DEVI void c_qmul(double* o, const double* a, const double* b) {
  o[0] = ((a[0] * b[0] - a[1] * b[1]) - a[2] * b[2]) - a[3] * b[3];
  o[1] = ((a[0] * b[1] + a[1] * b[0]) + a[2] * b[3]) - a[3] * b[2];
  o[2] = ((a[0] * b[2] - a[1] * b[3]) + a[2] * b[0]) + a[3] * b[1];
  o[3] = ((a[0] * b[3] + a[1] * b[2]) - a[2] * b[1]) + a[3] * b[0];
}
DEVI void c_qrot(double* o, const double* q, const double* v) {
  double p[4] = {0.0, v[0], v[1], v[2]}, t[4], r[4];
  double c[4] = {q[0], -q[1], -q[2], -q[3]};
  c_qmul(t, q, p);
  c_qmul(r, t, c);
  o[0] = r[1]; o[1] = r[2]; o[2] = r[3];
}
DEVI void c_qrot_d(double* o, const double* q, const double* dq, const double* v) {
  double p[4] = {0.0, v[0], v[1], v[2]}, t[4], r1[4], r2[4];
  double c[4] = {q[0], -q[1], -q[2], -q[3]}, dc[4] = {dq[0], -dq[1], -dq[2], -dq[3]};
  c_qmul(t, dq, p);
  c_qmul(r1, t, c);
  c_qmul(t, q, p);
  c_qmul(r2, t, dc);
  o[0] = r1[1] + r2[1]; o[1] = r1[2] + r2[2]; o[2] = r1[3] + r2[3];
}
DEVI void c_tapply(double* o, const double* T, const double* v) {
  double r[3];
  c_qrot(r, T, v);
  o[0] = r[0] + T[4]; o[1] = r[1] + T[5]; o[2] = r[2] + T[6];
}
DEVI void c_compose(double* o, const double* A, const double* B) {
  double q[4], t[3];
  c_qmul(q, A, B);
  c_tapply(t, A, B + 4);
  o[0] = q[0]; o[1] = q[1]; o[2] = q[2]; o[3] = q[3];
  o[4] = t[0]; o[5] = t[1]; o[6] = t[2];
}
DEVI void c_joint_tf(const mgs_kin_desc& K, int i, double th, double* J, double* dq) {
  const double* a = K.joint_tf[i] + 3;
  double n = sqrt((a[0] * a[0] + a[1] * a[1]) + a[2] * a[2]);
  double ax = a[0] / n, ay = a[1] / n, az = a[2] / n;
  double h = th / 2.0, s, c;
  k_sincos(h, &s, &c);
  J[0] = c; J[1] = ax * s; J[2] = ay * s; J[3] = az * s;
  J[4] = K.joint_tf[i][0] * th; J[5] = K.joint_tf[i][1] * th; J[6] = K.joint_tf[i][2] * th;
  dq[0] = -0.5 * s; dq[1] = ax * (0.5 * c); dq[2] = ay * (0.5 * c); dq[3] = az * (0.5 * c);
}

// forward kinematics of tip a: hand-frame contact, origin and normal points;
// with hP / hF given, also accumulates the joint gradient
// g[joint] += hP . dX_contact + hF . (dX_normal - dX_origin)   (oracle loss_grad)
DEVI void c_tip_fk(const mgs_kin_desc& K, int a, const double* th, double (*X)[3], const double* hP,
                   const double* hF, double* gj) {
  int L = K.chain_len[a];
  double W[7] = {1.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  double A[MGS_KIN_MAXCHAIN][7], J[MGS_KIN_MAXCHAIN][7], dq[MGS_KIN_MAXCHAIN][4];
  for (int s = 0; s < L; s++) {
    int i = K.chain[a][s];
    c_compose(A[s], W, K.kin_tf[i]);
    c_joint_tf(K, i, th[i], J[s], dq[s]);
    c_compose(W, A[s], J[s]);
  }
  const double zero[3] = {0.0, 0.0, 0.0};
  const double* P[3] = {K.tip_point[a], zero, K.tip_normal[a]};
  if (!hP) {
    for (int p = 0; p < 3; p++) c_tapply(X[p], W, P[p]);
    return;
  }
  double dX[MGS_KIN_MAXCHAIN][3][3];
  for (int p = 0; p < 3; p++) {
    double y[3] = {P[p][0], P[p][1], P[p][2]};
    for (int s = L - 1; s >= 0; s--) {
      int i = K.chain[a][s];
      double z[3], t1[3];
      c_qrot_d(z, J[s], dq[s], y);
      z[0] = z[0] + K.joint_tf[i][0]; z[1] = z[1] + K.joint_tf[i][1]; z[2] = z[2] + K.joint_tf[i][2];
      c_qrot(dX[s][p], A[s], z);
      c_tapply(t1, J[s], y);
      c_tapply(y, K.kin_tf[i], t1);
    }
  }
  for (int s = 0; s < L; s++) {
    const double* d0 = dX[s][0];
    const double* d1 = dX[s][1];
    const double* d2 = dX[s][2];
    double t0 = (hP[0] * d0[0] + hP[1] * d0[1]) + hP[2] * d0[2];
    double t1 = (hF[0] * (d2[0] - d1[0]) + hF[1] * (d2[1] - d1[1])) + hF[2] * (d2[2] - d1[2]);
    gj[K.chain[a][s]] = gj[K.chain[a][s]] + (t0 + t1);
  }
}

DEVI void c_gs6(const double* r, double* R, double* n1o, double* n2o, double* dd) {
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
DEVI void c_world(const double* R, const double* p, const double* x, double* o) {
  for (int i = 0; i < 3; i++) o[i] = ((R[3 * i] * x[0] + R[3 * i + 1] * x[1]) + R[3 * i + 2] * x[2]) + p[i];
}
DEVI void c_assign(const mgs_kin_desc& K, const double (*X)[3], const double* T, double* out) {
  int nt = K.ntip;
  double D[MGS_KIN_MAXTIP][MGS_KIN_MAXTIP];
  for (int a = 0; a < nt; a++)
    for (int b = 0; b < nt; b++) {
      double d0 = X[a][0] - T[3 * b], d1 = X[a][1] - T[3 * b + 1], d2 = X[a][2] - T[3 * b + 2];
      D[a][b] = sqrt((d0 * d0 + d1 * d1) + d2 * d2);
    }
  int best = 0;
  double bc = INFINITY;
  for (int k = 0; k < K.nperm; k++) {
    double c = 0.0;
    for (int a = 0; a < nt; a++) c = c + D[a][K.perm[k][a]];
    if (c < bc) { bc = c; best = k; }
  }
  for (int a = 0; a < nt; a++)
    for (int j = 0; j < 3; j++) out[3 * a + j] = T[3 * K.perm[best][a] + j];
}

DEVI double c_loss_grad(const mgs_kin_desc& K, const double* prm, const double* T, const double* N, double* g) {
  int nd = K.ndof, nt = K.ntip;
  double R[9], n1, n2, dd, th[MGS_KIN_MAXDOF], As[3 * MGS_KIN_MAXTIP];
  double X[MGS_KIN_MAXTIP][3][3];
  const double inv3n = 1.0 / (3.0 * nt);
  c_gs6(prm, R, &n1, &n2, &dd);
  for (int i = 0; i < nd; i++) th[i] = prm[9 + i];
  for (int a = 0; a < nt; a++) c_tip_fk(K, a, th, X[a], nullptr, nullptr, nullptr);
  double Pw[MGS_KIN_MAXTIP][3], fn[MGS_KIN_MAXTIP][3];
  for (int a = 0; a < nt; a++) {
    double o[3], q[3];
    c_world(R, prm + 6, X[a][0], Pw[a]);
    c_world(R, prm + 6, X[a][1], o);
    c_world(R, prm + 6, X[a][2], q);
    for (int k = 0; k < 3; k++) fn[a][k] = q[k] - o[k];
  }
  c_assign(K, Pw, T, As);
  double sq = 0.0, lc = 0.0;
  for (int a = 0; a < nt; a++)
    for (int k = 0; k < 3; k++) { double e = As[3 * a + k] - Pw[a][k]; sq = sq + e * e; }
  for (int a = 0; a < nt; a++) {
    double cs = (N[3 * a] * fn[a][0] + N[3 * a + 1] * fn[a][1]) + N[3 * a + 2] * fn[a][2];
    lc = lc + 0.5 * (1.0 - cs);
  }
  double loss = sq * inv3n + K.w_cos * (lc / nt);
  double gP[MGS_KIN_MAXTIP][3], gF[MGS_KIN_MAXTIP][3];
  for (int a = 0; a < nt; a++)
    for (int k = 0; k < 3; k++) {
      gP[a][k] = (2.0 * (Pw[a][k] - As[3 * a + k])) * inv3n;
      gF[a][k] = (K.w_cos * (-0.5 * N[3 * a + k])) / nt;
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
    double hP[3], hF[3], Xs[3][3];
    for (int j = 0; j < 3; j++) {
      hP[j] = (R[j] * gP[a][0] + R[3 + j] * gP[a][1]) + R[6 + j] * gP[a][2];
      hF[j] = (R[j] * gF[a][0] + R[3 + j] * gF[a][1]) + R[6 + j] * gF[a][2];
    }
    c_tip_fk(K, a, th, Xs, hP, hF, g + 9);
  }
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

__global__ void __launch_bounds__(64)
mgs_contact_opt_kernel(const mgs_kin_desc* __restrict__ Kp, int n, const double* __restrict__ rot_init,
                       const double* __restrict__ pos_init, const double* __restrict__ targets,
                       const double* __restrict__ normals, double* __restrict__ out_rot,
                       double* __restrict__ out_pos, double* __restrict__ out_joints, double* __restrict__ out_loss) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  const mgs_kin_desc& K = *Kp;
  const int nd = K.ndof, nt = K.ntip, np = 9 + nd;
  const double* R0 = rot_init + 9 * (size_t)c;
  const double* p0 = pos_init + 3 * (size_t)c;
  const double* T0 = targets + 3 * nt * (size_t)c;
  double N[3 * MGS_KIN_MAXTIP];
  for (int q = 0; q < 3 * nt; q++) N[q] = normals[3 * nt * (size_t)c + q];
  double prm[9 + MGS_KIN_MAXDOF], m[9 + MGS_KIN_MAXDOF], v[9 + MGS_KIN_MAXDOF], g[9 + MGS_KIN_MAXDOF];
  double T[3 * MGS_KIN_MAXTIP];
  {
    double Xw[MGS_KIN_MAXTIP][3], R0l[9], p0l[3], T0l[3 * MGS_KIN_MAXTIP];
    for (int q = 0; q < 9; q++) R0l[q] = R0[q];
    for (int q = 0; q < 3; q++) p0l[q] = p0[q];
    for (int q = 0; q < 3 * nt; q++) T0l[q] = T0[q];
    for (int a = 0; a < nt; a++) {
      double X[3][3];
      c_tip_fk(K, a, K.pregrasp, X, nullptr, nullptr, nullptr);
      c_world(R0l, p0l, X[0], Xw[a]);
    }
    c_assign(K, Xw, T0l, T);
    for (int j = 0; j < 6; j++) prm[j] = R0l[j];
    for (int j = 0; j < 3; j++) prm[6 + j] = p0l[j];
  }
  for (int i = 0; i < nd; i++) prm[9 + i] = K.pregrasp[i];
  for (int j = 0; j < np; j++) { m[j] = 0.0; v[j] = 0.0; }
  double b1t = 1.0, b2t = 1.0, loss = 0.0;
  for (int it = 0; it < K.iters; it++) {
    loss = c_loss_grad(K, prm, T, N, g);
    b1t = b1t * K.b1;
    b2t = b2t * K.b2;
    double c1 = 1.0 - b1t, c2 = 1.0 - b2t;
    for (int j = 0; j < np; j++) {
      m[j] = (1.0 - K.b1) * g[j] + K.b1 * m[j];
      v[j] = (1.0 - K.b2) * (g[j] * g[j]) + K.b2 * v[j];
      double mh = m[j] / c1, vh = v[j] / c2;
      double u = mh / (sqrt(vh + K.eps_root) + K.eps);
      u = u + K.weight_decay * prm[j];
      prm[j] = prm[j] + (-K.lr) * u;
    }
    for (int i = 0; i < nd; i++) {
      double x = prm[9 + i];
      if (x < K.range[i][0]) x = K.range[i][0];
      if (x > K.range[i][1]) x = K.range[i][1];
      prm[9 + i] = x;
    }
  }
  double R[9];
  c_gs6(prm, R, nullptr, nullptr, nullptr);
  for (int q = 0; q < 9; q++) out_rot[9 * (size_t)c + q] = R[q];
  for (int j = 0; j < 3; j++) out_pos[3 * (size_t)c + j] = prm[6 + j];
  for (int i = 0; i < nd; i++) out_joints[(size_t)nd * c + i] = prm[9 + i];
  if (out_loss) out_loss[c] = loss;
}
