// Microbenchmark: issue/latency of the instruction classes the rollout kernel
// is made of, for ONE wave per SIMD (the kernel's occupancy).  Dev tool.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP10(x) x x x x x x x x x x
#define REP100(x) REP10(REP10(x))

__global__ void probe(unsigned long long* out, double* buf) {
  __shared__ double lds[1024];
  int lane = threadIdx.x;
  for (int i = lane; i < 1024; i += 64) lds[i] = 1.0 + i;
  __syncthreads();
  double a = buf[lane], b = buf[lane + 64], c = buf[lane + 128], e = buf[lane + 192];
  double a1 = a, a2 = a, a3 = a, a4 = a, a5 = a, a6 = a, a7 = a;
  unsigned long long t0, t1, r0, r1;
  int k = 0;
  // 0: clock ratio: s_memtime vs s_memrealtime (100 MHz) over a spin
  t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 0; i < 20000; i++) asm volatile("s_nop 7");
  t1 = __builtin_amdgcn_s_memtime(); r1 = __builtin_amdgcn_s_memrealtime();
  out[k++] = t1 - t0; out[k++] = r1 - r0;
  // 2: 100 dependent v_add_f64
  t0 = __builtin_amdgcn_s_memtime();
  REP100(asm volatile("v_add_f64 %0, %0, %1" : "+v"(a) : "v"(b));)
  asm volatile("s_waitcnt 0" ::: "memory");
  t1 = __builtin_amdgcn_s_memtime(); out[k++] = t1 - t0;
  // 3: 100 independent v_add_f64 (8 chains)
  t0 = __builtin_amdgcn_s_memtime();
  REP10(asm volatile("v_add_f64 %0, %0, %8\n v_add_f64 %1, %1, %8\n v_add_f64 %2, %2, %8\n v_add_f64 %3, %3, %8\n v_add_f64 %4, %4, %8\n v_add_f64 %5, %5, %8\n v_add_f64 %6, %6, %8\n v_add_f64 %7, %7, %8\n v_add_f64 %0, %0, %8\n v_add_f64 %1, %1, %8"
      : "+v"(a), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));)
  t1 = __builtin_amdgcn_s_memtime(); out[k++] = t1 - t0;
  // 4: 100 dependent v_fma_f64
  t0 = __builtin_amdgcn_s_memtime();
  REP100(asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a) : "v"(b), "v"(c));)
  t1 = __builtin_amdgcn_s_memtime(); out[k++] = t1 - t0;
  // 5: 100 independent v_fma_f64
  t0 = __builtin_amdgcn_s_memtime();
  REP10(asm volatile("v_fma_f64 %0, %0, %8, %9\n v_fma_f64 %1, %1, %8, %9\n v_fma_f64 %2, %2, %8, %9\n v_fma_f64 %3, %3, %8, %9\n v_fma_f64 %4, %4, %8, %9\n v_fma_f64 %5, %5, %8, %9\n v_fma_f64 %6, %6, %8, %9\n v_fma_f64 %7, %7, %8, %9\n v_fma_f64 %0, %0, %8, %9\n v_fma_f64 %1, %1, %8, %9"
      : "+v"(a), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b), "v"(c));)
  t1 = __builtin_amdgcn_s_memtime(); out[k++] = t1 - t0;
  // 6: 100 dependent v_mul_f64
  t0 = __builtin_amdgcn_s_memtime();
  REP100(asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a) : "v"(e));)
  t1 = __builtin_amdgcn_s_memtime(); out[k++] = t1 - t0;
  // 7: 100 independent v_add_u32
  int i0 = lane, i1 = lane, i2 = lane, i3 = lane;
  t0 = __builtin_amdgcn_s_memtime();
  REP10(asm volatile("v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4\n v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4\n v_add_u32 %2, %2, %4\n v_add_u32 %3, %3, %4\n v_add_u32 %0, %0, %4\n v_add_u32 %1, %1, %4"
      : "+v"(i0), "+v"(i1), "+v"(i2), "+v"(i3) : "v"(lane));)
  t1 = __builtin_amdgcn_s_memtime(); out[k++] = t1 - t0;
  // 8: 20 dependent ds_read_b64 (pointer chase through lds as index)
  int idx = lane & 7;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 20; i++) { double v = lds[idx]; idx = ((int)v) & 7; asm volatile("" : "+v"(idx)); }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  t1 = __builtin_amdgcn_s_memtime(); out[k++] = t1 - t0;
  // 9: 100 dependent readlane round trips: s = readlane(v); v = v + s
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 100; i++) {
    int lo = __builtin_amdgcn_readlane(__double2loint(a), 3), hi = __builtin_amdgcn_readlane(__double2hiint(a), 3);
    a = a + __hiloint2double(hi, lo);
    asm volatile("" : "+v"(a));
  }
  t1 = __builtin_amdgcn_s_memtime(); out[k++] = t1 - t0;
  // 10: 100 v_rcp_f64 dependent
  t0 = __builtin_amdgcn_s_memtime();
  REP100(asm volatile("v_rcp_f64 %0, %0" : "+v"(c));)
  t1 = __builtin_amdgcn_s_memtime(); out[k++] = t1 - t0;
  // 11: 10 IEEE f64 divisions (compiler sequence), dependent
  double q = e;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 10; i++) { q = b / q; asm volatile("" : "+v"(q)); }
  t1 = __builtin_amdgcn_s_memtime(); out[k++] = t1 - t0;
  // 12: 10 sqrt f64 dependent
  double sq = e;
  t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 10; i++) { sq = sqrt(sq + 2.0); asm volatile("" : "+v"(sq)); }
  t1 = __builtin_amdgcn_s_memtime(); out[k++] = t1 - t0;
  // 13: 100 independent ds_read_b64 broadcast, then wait
  double acc[8];
  t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = 0;
  for (int j = 0; j < 100; j += 8) {
#pragma unroll
    for (int i = 0; i < 8; i++) { double v; asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(0), "i"(i * 8)); acc[i] += 0; asm volatile("" :: "v"(v)); }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  t1 = __builtin_amdgcn_s_memtime(); out[k++] = t1 - t0;
  // 14: v_cndmask_b32 dependent x100
  t0 = __builtin_amdgcn_s_memtime();
  REP100(asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(i0) : "v"(i1));)
  t1 = __builtin_amdgcn_s_memtime(); out[k++] = t1 - t0;
  // 15: 100 independent readlane (to distinct SGPRs), consumed once at the end
  {
    int src = i0;
    int acc_s = 0;
    t0 = __builtin_amdgcn_s_memtime();
#pragma unroll
    for (int j = 0; j < 100; j++) acc_s += __builtin_amdgcn_readlane(src, j & 63) * (j + 1);
    asm volatile("" :: "s"(acc_s));
    t1 = __builtin_amdgcn_s_memtime(); out[k++] = t1 - t0;
    i0 += acc_s;
  }
  // 16: 50 ds_read_b128 broadcast (independent), then wait
  t0 = __builtin_amdgcn_s_memtime();
  for (int j = 0; j < 50; j += 5) {
#pragma unroll
    for (int i = 0; i < 5; i++) { double v0, v1; asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(*(__attribute__((ext_vector_type(2))) double*)&v0) : "v"(0), "i"(i * 16)); }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  t1 = __builtin_amdgcn_s_memtime(); out[k++] = t1 - t0;
  // 17: 100 ds_read_b64 with per-lane consecutive addresses (no broadcast)
  t0 = __builtin_amdgcn_s_memtime();
  for (int j = 0; j < 100; j += 10) {
#pragma unroll
    for (int i = 0; i < 10; i++) { double v; asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(lane * 8), "i"(i * 8)); }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  t1 = __builtin_amdgcn_s_memtime(); out[k++] = t1 - t0;
  // 18: 100 ds_write_b64
  t0 = __builtin_amdgcn_s_memtime();
  for (int j = 0; j < 100; j += 10) {
#pragma unroll
    for (int i = 0; i < 10; i++) asm volatile("ds_write_b64 %0, %1 offset:%2" :: "v"(lane * 8), "v"(a), "i"(i * 8 + 4096));
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  t1 = __builtin_amdgcn_s_memtime(); out[k++] = t1 - t0;
  // 19: 100 ds_bpermute_b32 independent
  t0 = __builtin_amdgcn_s_memtime();
  for (int j = 0; j < 100; j += 10) {
#pragma unroll
    for (int i = 0; i < 10; i++) { int v; asm volatile("ds_bpermute_b32 %0, %1, %2" : "=v"(v) : "v"(((lane + i) & 63) * 4), "v"(i1)); }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  t1 = __builtin_amdgcn_s_memtime(); out[k++] = t1 - t0;
  // 20: 100 dependent DPP row_shr:1 v_add_f32-free moves (v_mov_b32_dpp)
  t0 = __builtin_amdgcn_s_memtime();
  REP100(i1 = __builtin_amdgcn_update_dpp(0, i1, 0x111, 0xf, 0xf, false);)
  asm volatile("" :: "v"(i1));
  t1 = __builtin_amdgcn_s_memtime(); out[k++] = t1 - t0;
  // 21: 100 s_add_u32 dependent (scalar)
  int sv = __builtin_amdgcn_readfirstlane(lane);
  t0 = __builtin_amdgcn_s_memtime();
  REP100(asm volatile("s_add_u32 %0, %0, 3" : "+s"(sv));)
  t1 = __builtin_amdgcn_s_memtime(); out[k++] = t1 - t0;
  i0 += sv;
  // 22: 20 dependent global loads (pointer chase, L1/L2-resident 2 KB buffer)
  {
    int gi = lane & 7;
    const int* gb = (const int*)(buf + 256);
    t0 = __builtin_amdgcn_s_memtime();
    for (int j = 0; j < 20; j++) { gi = gb[gi]; asm volatile("" : "+v"(gi)); }
    t1 = __builtin_amdgcn_s_memtime(); out[k++] = t1 - t0;
    i0 += gi;
  }
  // 23: 20 dependent global loads, uniform address (scalar-loadable) via volatile vector path
  {
    int gi = 0;
    const int* gb = (const int*)(buf + 256);
    t0 = __builtin_amdgcn_s_memtime();
    for (int j = 0; j < 20; j++) { gi = __builtin_amdgcn_readfirstlane(gb[gi + (lane & 0)]); }
    t1 = __builtin_amdgcn_s_memtime(); out[k++] = t1 - t0;
    i0 += gi;
  }
  if (lane == 0) out[31] = (unsigned long long)(a + a1 + a2 + a3 + a4 + a5 + a6 + a7 + c + q + sq + i0 + i1 + i2 + i3 + idx + acc[0]);
  buf[lane] = a + b;
}

int main() {
  unsigned long long* d_out; double* d_buf;
  hipMalloc(&d_out, 32 * 8); hipMalloc(&d_buf, 2048 * 8);
  double h[256]; for (int i = 0; i < 256; i++) h[i] = 1.0 + 1e-3 * i;
  hipMemcpy(d_buf, h, sizeof(h), hipMemcpyHostToDevice);
  int hi[512]; for (int i = 0; i < 512; i++) hi[i] = (i * 37 + 11) % 64;
  hipMemcpy(d_buf + 256, hi, sizeof(hi), hipMemcpyHostToDevice);
  for (int it = 0; it < 2; it++) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d_out, d_buf);
    hipDeviceSynchronize();
  }
  unsigned long long o[32];
  hipMemcpy(o, d_out, sizeof(o), hipMemcpyDeviceToHost);
  double ratio = (double)o[0] / (double)o[1];
  printf("memtime ticks per realtime tick (100MHz): %.2f -> memtime clock %.0f MHz\n", ratio, ratio * 100);
  const char* names[] = {"", "", "100 dep v_add_f64", "100 indep v_add_f64", "100 dep v_fma_f64", "100 indep v_fma_f64",
                         "100 dep v_mul_f64", "100 indep v_add_u32", "20 dep ds_read_b64", "100 readlane x2 + add_f64",
                         "100 dep v_rcp_f64", "10 dep f64 div", "10 dep f64 sqrt", "100 indep ds_read_b64", "100 dep v_cndmask", "100 indep readlane_b32", "50 ds_read_b128 bcast",
                         "100 ds_read_b64 per-lane", "100 ds_write_b64", "100 ds_bpermute_b32", "100 dep dpp mov",
                         "100 dep s_add_u32", "20 dep global loads", "20 dep global (readfirstlane)"};
  for (int i = 2; i < 24; i++) printf("%-28s %6llu ticks  (%.1f per op)\n", names[i], o[i], o[i] / (i == 8 || i == 22 || i == 23 ? 20.0 : (i == 11 || i == 12) ? 10.0 : i == 16 ? 50.0 : 100.0));
  return 0;
}
