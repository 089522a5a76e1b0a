// Probe: numerics (which rounding order) and timing of v_mfma_f64_16x16x4_f64
// for one wave.  Writes A, B, C, D to mfma_f64.bin for tools/probes/mfma_f64_check.py.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
typedef double v4d __attribute__((ext_vector_type(4)));

__global__ void run(const double* A, const double* B, const double* C, double* D, int ntile,
                    unsigned long long* t) {
  int l = threadIdx.x;
  for (int q = 0; q < ntile; q++) {
    const double* a = A + q * 64; const double* b = B + q * 64; const double* c = C + q * 256;
    // A[i][k] at a[i*4+k]; B[k][j] at b[k*16+j]; C/D[i][j] at [i*16+j]
    double av = a[(l & 15) * 4 + (l >> 4)];
    double bv = b[(l >> 4) * 16 + (l & 15)];
    v4d cv;
    for (int r = 0; r < 4; r++) cv[r] = c[((l >> 4) + 4 * r) * 16 + (l & 15)];
    v4d dv = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, cv, 0, 0, 0);
    for (int r = 0; r < 4; r++) D[q * 256 + ((l >> 4) + 4 * r) * 16 + (l & 15)] = dv[r];
  }
  // timing: 64 dependent MFMAs on one accumulator; 64 over 4 independent accumulators
  double av = A[l], bv = B[l];
  v4d c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 64; i++) c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, c0, 0, 0, 0);
  asm volatile("s_nop 7\n s_nop 7" ::: "memory");
  double s0 = c0[0];
  asm volatile("" :: "v"(s0));
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 16; i++) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, c3, 0, 0, 0);
  }
  double s1 = c0[0] + c1[1] + c2[2] + c3[3];
  asm volatile("" :: "v"(s1));
  unsigned long long t2 = __builtin_amdgcn_s_memtime();
  if (l == 0) { t[0] = t1 - t0; t[1] = t2 - t1; }
  D[ntile * 256 + l] = s0 + s1;
}

int main() {
  const int NT = 400;
  size_t na = NT * 64, nc = NT * 256;
  double *hA = new double[na], *hB = new double[na], *hC = new double[nc], *hD = new double[nc + 64];
  srand(12345);
  auto rnd = [](int tile) {
    double u = (rand() + 1.0) / (RAND_MAX + 2.0), v = (rand() + 1.0) / (RAND_MAX + 2.0);
    double g = sqrt(-2 * log(u)) * cos(6.283185307179586 * v);
    int e = (tile % 4 == 0) ? 0 : (rand() % 41) - 20;
    return ldexp(g, e);
  };
  for (int q = 0; q < NT; q++) {
    for (int i = 0; i < 64; i++) { hA[q * 64 + i] = (q < 2) ? (double)((i * 7) % 13 - 6) : rnd(q); hB[q * 64 + i] = (q < 2) ? (double)((i * 5) % 11 - 5) : rnd(q); }
    for (int i = 0; i < 256; i++) hC[q * 256 + i] = (q < 2) ? (double)(i % 9) : ((q % 3 == 0) ? 0.0 : rnd(q));
  }
  double *A, *B, *C, *D; unsigned long long* T;
  hipMalloc(&A, na * 8); hipMalloc(&B, na * 8); hipMalloc(&C, nc * 8); hipMalloc(&D, (nc + 64) * 8); hipMalloc(&T, 16);
  hipMemcpy(A, hA, na * 8, hipMemcpyHostToDevice); hipMemcpy(B, hB, na * 8, hipMemcpyHostToDevice);
  hipMemcpy(C, hC, nc * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(run, dim3(1), dim3(64), 0, 0, A, B, C, D, NT, T);
  hipDeviceSynchronize();
  unsigned long long ht[2];
  hipMemcpy(hD, D, nc * 8, hipMemcpyDeviceToHost); hipMemcpy(ht, T, 16, hipMemcpyDeviceToHost);
  printf("64 dependent mfma_f64_16x16x4: %llu cycles (%.1f each); 64 over 4 accumulators: %llu (%.1f each)\n",
         ht[0], ht[0] / 64.0, ht[1], ht[1] / 64.0);
  FILE* f = fopen("gpurun_out/mfma_f64.bin", "wb");
  int nt = NT; fwrite(&nt, 4, 1, f);
  fwrite(hA, 8, na, f); fwrite(hB, 8, na, f); fwrite(hC, 8, nc, f); fwrite(hD, 8, nc, f);
  fclose(f);
  return 0;
}
