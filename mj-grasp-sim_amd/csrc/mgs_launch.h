// mgs_launch.h -- host-side launch interface between the C-ABI translation unit
// (mgs_capi.hip) and the per-dof-count kernel instantiations (mgs_inst.hip),
// which are compiled as separate translation units in parallel.  Include after
// mgs_kernels.hip (Mdl, Lay).
#pragma once

struct CollisionArgs {
  Mdl md;
  Lay lay;
  int n;
  const double *qpos_init, *mocap_pos, *mocap_quat;
  int predicate;
  uint8_t* out;
};

struct RolloutArgs {
  Mdl md;
  Lay lay;
  mgs_schedule sc;
  int n;
  const double *qpos_init, *mocap_quat, *phase_start, *phase_target;
  const uint8_t* active;
  uint8_t* label;
  int32_t* fail_step;
  double* obj_qpos;
  int32_t* stats;
  const double* vstate_init;
  double* state_out;
  const int32_t* list;
  int32_t* list_count;       // list header (MGS_LIST_HEADER words, see mgs_rollout_list_device)
  double* resume_out;
  const double* resume_in;
  const double* mask_mpos;   // fused collision mask (mgs_mask_rollout_device): mocap positions,
  int mask_pred;             // predicate
  uint8_t* mask_out;         // and the mask written per candidate (nullptr: no fused mask)
  uint32_t* queue;           // work-queue counter pair (nullptr: one workgroup per candidate)
  int32_t* ovf_count;        // overflow list the capped candidates append to (nullptr: none):
  int32_t* ovf_list;         // its header (count first) and its entries
};

// one dof count's runtime-layout kernels: launchers (64 lanes per workgroup,
// grid and dynamic LDS from the caller) and the kernel handles for attributes
struct KernelSet {
  void (*collision)(dim3 grid, size_t shmem, hipStream_t st, const CollisionArgs& a);
  void (*rollout)(dim3 grid, size_t shmem, hipStream_t st, const RolloutArgs& a);
  const void* collision_fn;
  const void* rollout_fn;
  int (*prof_read)(unsigned long long* acc);   // MGS_PROFILE builds: add and clear the stage timers
};

// defined (specialised) in mgs_inst.hip for each dof count of the library
template <int NV>
const KernelSet* mgs_kernels_nv();
