// mgs_inst.hip -- one dof count's kernel instantiations of libmgs_gpu.so.
//
// Compiled once per entry of the library's dof list (-DMGS_INST_NV=<nv>, in
// parallel; mgs_capi.hip holds the C-ABI and dispatches on the model's nv
// through mgs_kernels_nv<nv>()).  These are the runtime-layout kernels (model
// description and LDS offsets read from the launch arguments); a model with a
// specialised code object attached (mgs_special.hip) launches that instead.
#include <hip/hip_runtime.h>

#ifdef MGS_WIDE
#define MGS_RPL 4
#ifndef MGS_G_LDS          /* -DMGS_G_LDS: the wide build with G kept in LDS (experiments) */
#define MGS_G_GLOBAL 1
#endif
#endif
#define MGS_TEMPLATES_ONLY
#include "mgs_kernels.hip"
#include "mgs_launch.h"

#ifndef MGS_INST_NV
#error "mgs_inst.hip is compiled with -DMGS_INST_NV=<nv>"
#endif

namespace {
void launch_collision(dim3 grid, size_t shmem, hipStream_t st, const CollisionArgs& a) {
  hipLaunchKernelGGL(mgs_collision_kernel<MGS_INST_NV>, grid, dim3(64), shmem, st, a.md, a.md.I, a.md.D, a.lay, a.n,
                     a.qpos_init, a.mocap_pos, a.mocap_quat, a.predicate, a.out);
}
void launch_rollout(dim3 grid, size_t shmem, hipStream_t st, const RolloutArgs& a) {
  hipLaunchKernelGGL(mgs_rollout_kernel<MGS_INST_NV>, grid, dim3(64), shmem, st, a.md, a.md.I, a.md.D, a.lay, a.sc,
                     a.n, a.qpos_init, a.mocap_quat, a.phase_start, a.phase_target, a.active, a.label, a.fail_step,
                     a.obj_qpos, a.stats, a.vstate_init, a.state_out, a.list, a.list_count, a.resume_out,
                     a.resume_in, a.mask_mpos, a.mask_pred, a.mask_out, a.queue, a.ovf_count, a.ovf_list);
}
#ifdef MGS_PROFILE
int prof_read(unsigned long long* acc) {
  unsigned long long v[64], z[64] = {0};
  if (hipMemcpyFromSymbol(v, HIP_SYMBOL(g_prof), sizeof(v)) != hipSuccess) return -1;
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(z)) != hipSuccess) return -1;
  for (int k = 0; k < 64; k++) acc[k] += v[k];
  return 0;
}
#endif
const KernelSet kset = {launch_collision, launch_rollout, (const void*)mgs_collision_kernel<MGS_INST_NV>,
                        (const void*)mgs_rollout_kernel<MGS_INST_NV>,
#ifdef MGS_PROFILE
                        prof_read
#else
                        nullptr
#endif
};
}  // namespace

template <>
const KernelSet* mgs_kernels_nv<MGS_INST_NV>() { return &kset; }
