// mgs_special.hip -- a model-specialised code object.
//
// Compiled per model (mgs/core/special.py: hipcc --genco --offload-arch=gfx950
// -DMGS_SPECIAL="<header>" [-DMGS_WIDE]) with the header that carries the
// model's description and LDS layout as constants; loaded at run time with
// hipModuleLoad by mgs_model_attach_special (mgs_capi.hip), which first reads
// the baked description and layout back from the object (mgs_special_desc,
// mgs_special_words, mgs_special_abi) and compares them with the model's.
//
// The kernels are the rollout / collision kernels of mgs_kernels.hip
// instantiated at the model's dof count with SL = 1 (every LDS view and every
// model size / table offset a compile-time constant).  Any dof count up to 64
// can be specialised, and up to 128 with two dofs per lane (-DMGS_DPL=2, the
// wide flavour), so models the library has no instantiation for (clutter
// piles of any size, other grippers) run through these objects.
#include <hip/hip_runtime.h>

#ifdef MGS_WIDE
#define MGS_RPL 4
#define MGS_G_GLOBAL 1
#endif
#define MGS_TEMPLATES_ONLY
#include "mgs_kernels.hip"

#ifndef MGS_SPECIAL
#error "mgs_special.hip is compiled with -DMGS_SPECIAL=<generated header>"
#endif

// kernel symbols by role: an escalation engine's object (mgs/core/special.py,
// role "escalation": -DMGS_SPECIAL_ESC) names its kernels *_esc, so a trace
// tells the capacity escalation's re-runs from the main launches
// (mgs_model_attach_special accepts either)
#ifdef MGS_SPECIAL_ESC
#define MGS_SPECIAL_COLLISION mgs_special_collision_esc
#define MGS_SPECIAL_ROLLOUT mgs_special_rollout_esc
#else
#define MGS_SPECIAL_COLLISION mgs_special_collision
#define MGS_SPECIAL_ROLLOUT mgs_special_rollout
#endif

extern "C" {

// what the object was compiled for, read back by mgs_model_attach_special
// (not const: const namespace-scope variables have internal linkage and would
// not be visible to hipModuleGetGlobal)
__device__ int mgs_special_abi = MGS_ABI_VERSION;
__device__ int mgs_special_rows_per_lane = MGS_RPL;
__device__ int mgs_special_maxdim = MGS_MAXDIM;
__device__ int mgs_special_max_nv = MGS_MAXNV;   // 64, or 128 with two dofs per lane (-DMGS_DPL=2)
static_assert(MGS_SL_NV <= MGS_MAXNV, "a model of more than 64 dofs is specialised with -DMGS_DPL=2");
__device__ mgs_model_desc mgs_special_desc = mgs_sl_desc;
__device__ int mgs_special_words[L_COUNT + U_COUNT + 4] = MGS_SL_WORDS_INIT;

__global__ void __launch_bounds__(64)
MGS_SPECIAL_COLLISION(Mdl mdarg, const int32_t* __restrict__ mI, const double* __restrict__ mD, Lay lay, int n,
                      const double* __restrict__ qpos_init, const double* __restrict__ mocap_pos,
                      const double* __restrict__ mocap_quat, int predicate, uint8_t* __restrict__ out) {
  extern __shared__ double smem[];
  collision_entry<MGS_SL_NV, 1>(smem, mdarg, mI, mD, lay, n, qpos_init, mocap_pos, mocap_quat, predicate, out);
}

__global__ void __launch_bounds__(64) MGS_ROLL_ATTR
MGS_SPECIAL_ROLLOUT(Mdl mdarg, const int32_t* __restrict__ mI, const double* __restrict__ mD, Lay lay,
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
  rollout_entry<MGS_SL_NV, 1>(smem, mdarg, mI, mD, lay, sc, n, qpos_init, mocap_quat, phase_start, phase_target,
                              active, label, fail_step, obj_qpos, stats, vstate_init, state_out, list, list_count,
                              resume_out, resume_in, mask_mpos, mask_pred, mask_out, queue, ovf_count, ovf_list);
}

}  // extern "C"
