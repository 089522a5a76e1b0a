// ldl_probe.hip -- register-row LDL^T factor of an SPD matrix: column
// broadcasts by v_readlane (the kernels' ldl_factor_regs) against the same
// right-looking loop with the column broadcast through LDS (one ds_write of
// l_cj d_j per lane, uniform-address reads).  Same products in the same order,
// so the factors must be bit-identical; prints the shader-clock ticks per
// factor of each.  One wave per workgroup, one workgroup per CU.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/probes/ldl_probe tools/probes/ldl_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#ifndef NV
#define NV 58
#endif
#define REPS 64

__device__ __attribute__((always_inline)) inline double readlane_d(double x, int l) {
  int lo = __builtin_amdgcn_readlane(__double2loint(x), l);
  int hi = __builtin_amdgcn_readlane(__double2hiint(x), l);
  return __hiloint2double(hi, lo);
}

template <int MODE>
__global__ void __launch_bounds__(64) factor(const double* A, double* out, unsigned long long* ticks) {
  __shared__ double bc[64];
  const int lane = __lane_id();
  const int li = lane < NV ? lane : 0;
  double r[NV];
  unsigned long long t0 = 0, acc = 0;
  for (int rep = 0; rep < REPS; rep++) {
#pragma unroll
    for (int k = 0; k < NV; k++) r[k] = A[li * NV + k];
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int j = 0; j < NV; j++) {
      double dj = readlane_d(r[j], j);
      double inv = 1.0 / dj;
      if (lane > j) r[j] = r[j] * inv;
      double v = r[j] * dj;
      if (MODE == 0 || MODE == 2 || MODE == 6) {
#pragma unroll
        for (int c = j + 1; c < NV; c++) {
          double w = readlane_d(v, c);
          r[c] = __builtin_fma(-r[j], w, r[c]);
          // MODE 6: each broadcast and its FMA a scheduling region of their own
          if (MODE == 6) __builtin_amdgcn_sched_barrier(0);
        }
      } else if (MODE == 5) {
        // ds_bpermute broadcast (VGPR result, no SGPR)
#pragma unroll
        for (int c = j + 1; c < NV; c++) {
          int lo = __builtin_amdgcn_ds_bpermute(c << 2, __double2loint(v));
          int hi = __builtin_amdgcn_ds_bpermute(c << 2, __double2hiint(v));
          double w = __hiloint2double(hi, lo);
          r[c] = __builtin_fma(-r[j], w, r[c]);
          if (((c - j) & 7) == 0) __builtin_amdgcn_sched_barrier(0);
        }
      } else {
        bc[lane] = v;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
#pragma unroll
        for (int c = j + 1; c < NV; c++) {
          double w = bc[c];
          r[c] = __builtin_fma(-r[j], w, r[c]);
          // MODE 4: at most eight broadcasts in flight
          if (MODE == 4 && ((c - j) & 7) == 0) __builtin_amdgcn_sched_barrier(0);
          if (MODE == 7 && ((c - j) & 3) == 0) __builtin_amdgcn_sched_barrier(0);
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
      }
      // MODE 2, 3, 4: nothing of one column is scheduled into another
      if (MODE >= 2) __builtin_amdgcn_sched_barrier(0);
    }
    acc += __builtin_amdgcn_s_memtime() - t0;
  }
  if (blockIdx.x == 0) {
#pragma unroll
    for (int k = 0; k < NV; k++)
      if (lane < NV) out[lane * NV + k] = r[k];
    if (lane == 0) ticks[MODE] = acc / REPS;
  }
}

int main() {
  static double A[NV * NV], B[NV * NV];
  // SPD: M = C C^T + NV I
  for (int i = 0; i < NV; i++)
    for (int j = 0; j < NV; j++) {
      double s = 0.0;
      for (int k = 0; k < NV; k++) s += ((i * 7 + k * 3) % 11 - 5) * 0.1 * (((j * 7 + k * 3) % 11 - 5) * 0.1);
      A[i * NV + j] = s + (i == j ? NV : 0.0);
    }
  double *dA, *d0, *d1;
  unsigned long long *dt, t[8];
  hipMalloc(&dA, sizeof(A));
  hipMalloc(&d0, sizeof(A));
  hipMalloc(&d1, sizeof(A));
  hipMalloc(&dt, sizeof(t));
  hipMemcpy(dA, A, sizeof(A), hipMemcpyHostToDevice);
  static const char* names[8] = {"readlane", "LDS", "readlane+sched_barrier", "LDS+sched_barrier",
                                 "LDS+sched_barrier/8", "bpermute/8", "readlane+barrier/1", "LDS+barrier/4"};
  int same = 1;
  for (int m = 0; m < 8; m++) {
    for (int it = 0; it < 3; it++) {
      if (m == 0) hipLaunchKernelGGL(factor<0>, dim3(256), dim3(64), 0, 0, dA, m ? d1 : d0, dt);
      if (m == 1) hipLaunchKernelGGL(factor<1>, dim3(256), dim3(64), 0, 0, dA, d1, dt);
      if (m == 2) hipLaunchKernelGGL(factor<2>, dim3(256), dim3(64), 0, 0, dA, d1, dt);
      if (m == 3) hipLaunchKernelGGL(factor<3>, dim3(256), dim3(64), 0, 0, dA, d1, dt);
      if (m == 4) hipLaunchKernelGGL(factor<4>, dim3(256), dim3(64), 0, 0, dA, d1, dt);
      if (m == 5) hipLaunchKernelGGL(factor<5>, dim3(256), dim3(64), 0, 0, dA, d1, dt);
      if (m == 6) hipLaunchKernelGGL(factor<6>, dim3(256), dim3(64), 0, 0, dA, d1, dt);
      if (m == 7) hipLaunchKernelGGL(factor<7>, dim3(256), dim3(64), 0, 0, dA, d1, dt);
    }
    if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed\n"); return 1; }
    if (m == 0) { hipMemcpy(A, d0, sizeof(A), hipMemcpyDeviceToHost); continue; }
    hipMemcpy(B, d1, sizeof(B), hipMemcpyDeviceToHost);
    // compare the lower triangles (the factor); the upper entries are scratch
    for (int i = 0; i < NV; i++)
      for (int k = 0; k <= i; k++)
        if (memcmp(&A[i * NV + k], &B[i * NV + k], sizeof(double)) != 0) same = 0;
  }
  hipMemcpy(t, dt, sizeof(t), hipMemcpyDeviceToHost);
  for (int m = 0; m < 8; m++) printf("nv %d: %-24s %llu ticks per factor\n", NV, names[m], t[m]);
  printf("nv %d: factors %s\n", NV, same ? "bit-identical" : "DIFFER");
  return same ? 0 : 1;
}
