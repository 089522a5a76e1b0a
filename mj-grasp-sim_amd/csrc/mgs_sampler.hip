// mgs_sampler.hip -- antipodal grasp-candidate ray casting on the MI355X
// (reference: mgs/sampler/antipodal.py:96-172, AntipodalGraspGenerator.
// generate_grasps).  For every sampled surface point the reference casts the
// sampled direction and its negative through the object mesh (trimesh
// intersects_location, all hits), keeps hits at distance >= eps and picks one
// uniformly at random; with none it falls back to a random offset.  The host
// draws every random number (surface points, von Mises-Fisher directions, the
// choice uniform u); this kernel does the O(points x triangles) part: it counts
// the valid hits of both rays and returns the k-th, k = min(floor(u * n), n - 1),
// in the order (+d hits by triangle index, then -d hits by triangle index).
//
// One thread per point, 256 points per workgroup; triangles are staged through
// LDS in tiles of 256 (9 doubles each, 18 KB) that every thread of the
// workgroup tests its two rays against.  Two sweeps: count, then select.
// Arithmetic follows oracle_antipodal_contacts (oracle/mgs_oracle.c) expression
// for expression (-ffp-contract=off), so results are bit-identical.

#define MGS_RAY_TILE 256

DEVI int ray_tri(const double* o, const double* d, const double* T, double* tout) {
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
  if (u >= 0.0 && w >= 0.0 && u + w <= 1.0 && t > 0.0) {
    *tout = t;
    return 1;
  }
  return 0;
}

// hit location o + t d and whether it lies at least eps from the origin
DEVI int ray_valid(const double* o, const double* d, double t, double eps, double* loc) {
  double s = 0.0;
  for (int k = 0; k < 3; k++) {
    loc[k] = o[k] + t * d[k];
    double r = loc[k] - o[k];
    s = s + r * r;
  }
  return sqrt(s) >= eps;
}

__global__ void __launch_bounds__(256)
mgs_antipodal_kernel(const double* __restrict__ tri, int ntri, int n, const double* __restrict__ origin,
                     const double* __restrict__ dir, const double* __restrict__ u_choice, double eps,
                     double* __restrict__ out_second, int32_t* __restrict__ out_nvalid) {
  __shared__ double tile[MGS_RAY_TILE * 9];
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  bool act = i < n;
  double o[3] = {0, 0, 0}, dp[3] = {1, 0, 0}, dm[3] = {-1, 0, 0};
  if (act)
    for (int k = 0; k < 3; k++) { o[k] = origin[3 * i + k]; dp[k] = dir[3 * i + k]; dm[k] = -dp[k]; }
  int cnt_p = 0, cnt_m = 0;
  // sweep 1: count valid hits of both rays
  for (int base = 0; base < ntri; base += MGS_RAY_TILE) {
    int m = ntri - base < MGS_RAY_TILE ? ntri - base : MGS_RAY_TILE;
    __syncthreads();
    for (int k = threadIdx.x; k < m * 9; k += blockDim.x) tile[k] = tri[(size_t)base * 9 + k];
    __syncthreads();
    if (act)
      for (int j = 0; j < m; j++) {
        double t, loc[3];
        if (ray_tri(o, dp, tile + 9 * j, &t) && ray_valid(o, dp, t, eps, loc)) cnt_p++;
        if (ray_tri(o, dm, tile + 9 * j, &t) && ray_valid(o, dm, t, eps, loc)) cnt_m++;
      }
  }
  int total = cnt_p + cnt_m;
  int kth = -1;
  if (act && total > 0) {
    double fk = floor(u_choice[i] * (double)total);
    kth = fk < (double)(total - 1) ? (int)fk : total - 1;
  }
  // sweep 2: the kth valid hit (+d hits first, then -d hits, each by triangle index)
  double sel[3] = {0, 0, 0};
  int want_p = kth >= 0 && kth < cnt_p;
  int kk = want_p ? kth : kth - cnt_p;
  int seen = 0;
  for (int base = 0; base < ntri; base += MGS_RAY_TILE) {
    int m = ntri - base < MGS_RAY_TILE ? ntri - base : MGS_RAY_TILE;
    __syncthreads();
    for (int k = threadIdx.x; k < m * 9; k += blockDim.x) tile[k] = tri[(size_t)base * 9 + k];
    __syncthreads();
    if (act && kth >= 0 && seen <= kk)
      for (int j = 0; j < m; j++) {
        double t, loc[3];
        const double* d = want_p ? dp : dm;
        if (ray_tri(o, d, tile + 9 * j, &t) && ray_valid(o, d, t, eps, loc)) {
          if (seen == kk) { sel[0] = loc[0]; sel[1] = loc[1]; sel[2] = loc[2]; }
          seen++;
          if (seen > kk) break;
        }
      }
  }
  if (act) {
    out_nvalid[i] = total;
    for (int k = 0; k < 3; k++) out_second[3 * i + k] = sel[k];
  }
}
