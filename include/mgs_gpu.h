/*
 * mgs_gpu.h — C-ABI of libmgs_gpu.so, the MI355X batched grasp-evaluation engine.
 *
 * The reference (freiberg-roman/mj-grasp-sim) has no FFI of its own: its hot
 * path calls the MuJoCo 3.2.2 C library through the `mujoco` Python bindings,
 * one candidate at a time.  Each entry point below replaces a group of those
 * binding calls for a whole batch of grasp candidates:
 *
 *   mgs_model_create      <- mujoco.MjModel.from_xml_string + mujoco.MjData
 *                            (mgs/env/gravityless_object_grasping.py:67-71);
 *                            the MJCF is compiled host-side by mgs.core.mjcf
 *                            into the flat model described by mgs_model_desc.
 *   mgs_collision_free    <- per-candidate mj_resetData / set_qpos / set_pose /
 *                            mj_forward / `data.ncon != 0`
 *                            (mgs/env/gravityless_object_grasping.py:90-125,
 *                             mgs/core/simualtion.py:45-49, mgs/gripper/base.py:48-59)
 *   mgs_rollout           <- per-candidate close_gripper_at + lift + shake loop of
 *                            grasp_stability_evaluation_from_joints
 *                            (mgs/env/gravityless_object_grasping.py:127-295,
 *                             mgs/gripper/robotiq2f85.py:240-244), each step one
 *                            mujoco.mj_step, each check check_contact_with_object
 *                            (:309-320).
 *
 * Conventions: all pointers are host pointers to C-contiguous arrays owned by
 * the caller (the library copies in/out).  Functions return 0 on success and a
 * negative MGS_E* code on failure; mgs_last_error() returns a thread-local
 * message.  One mgs_batch is used by one host thread at a time; a batch is bound
 * to one HIP device (one process per GPU for multi-GPU runs).
 *
 * The compiled model is two flat buffers (int32 and float64).  mgs_model_desc
 * holds the sizes, the physics options and, for every array, its offset into
 * the int buffer (fields named i_*) or the double buffer (fields named d_*).
 * The Python side builds this struct by parsing this header, so the field list
 * below is the single source of truth.
 */
#ifndef MGS_GPU_H_
#define MGS_GPU_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MGS_ABI_VERSION 23
#define MGS_NSTATS 6
/* largest dof count: 64 for the libraries' kernels (one dof per lane), 128
   for model-specialised code objects (two dofs per lane, ABI 22) */
#define MGS_MAX_NV 128

/* error codes */
#define MGS_OK 0
#define MGS_EINVAL (-1)
#define MGS_EHIP (-2)
#define MGS_ECAPACITY (-3)
#define MGS_ENOMEM (-4)
#define MGS_EQUEUE (-5)     /* a rotating launch's ring protocol timed out (an expired spin, see
                               mgs_queue_stats): a candidate may have been lost; the outputs of
                               that launch are not valid (the rings are reset) */

/* joint types (MuJoCo mjtJoint numbering) */
#define MGS_JNT_FREE 0
#define MGS_JNT_BALL 1
#define MGS_JNT_SLIDE 2
#define MGS_JNT_HINGE 3

/* equality types (MuJoCo mjtEq numbering) */
#define MGS_EQ_CONNECT 0
#define MGS_EQ_WELD 1
#define MGS_EQ_JOINT 2

/* actuator transmission / gain / bias types (MuJoCo numbering) */
#define MGS_TRN_JOINT 0
#define MGS_TRN_TENDON 3
#define MGS_GAIN_FIXED 0
#define MGS_GAIN_AFFINE 1
#define MGS_GAIN_PID 16            /* MuJoCo's mujoco.pid actuator plugin (ABI 21): force from the
                                      actuator_pidprm gains and the actuator's act state, see below */
#define MGS_BIAS_NONE 0
#define MGS_BIAS_AFFINE 1

/* constraint row kinds (efc) */
#define MGS_EFC_EQUALITY 0
#define MGS_EFC_FRICTION 1
#define MGS_EFC_LIMIT 2
#define MGS_EFC_CONTACT 3

/* stats[:, 2] flags */
#define MGS_FLAG_CONTACTS 1        /* contacts exceeded ncon_max at some step (re-run wider) */
#define MGS_FLAG_ROWS 2            /* constraint rows exceeded nefc_max (re-run wider) */
#define MGS_FLAG_CAPACITY 3        /* either capacity flag */
#define MGS_FLAG_DIVERGED 4        /* qpos / qvel / qacc NaN or beyond 1e10 (MuJoCo mj_checkPos /
                                      mj_checkVel / mj_checkAcc, mjMAXVAL): the candidate stops, label 0 */
#define MGS_FLAG_PAUSED 8          /* reached mgs_schedule.pause_step unfinished: stopped there with a
                                      resume record (fail_step -4), continued by a later launch */
#define MGS_MAXVAL 1e10

/* fail_step values below -1 (label 0): -2 collision-mask reject (not simulated), -3 stopped at a
 * capacity overflow with a resume record, -4 paused at mgs_schedule.pause_step, and
 * MGS_FAIL_YIELDED: the sentinel a yielding candidate writes before it joins the launch's rotation
 * ring (ABI 20).  Its continuation overwrites it, so it survives a launch only if the candidate was
 * lost -- never in a correct run; callers of the device entries treat it as an error. */
#define MGS_FAIL_YIELDED (-5)

/* narrowphase of a geom pair (pair_kind).  With ccd_mode 0 only the first two
 * occur; with ccd_mode 1 / 2 the pairs follow MuJoCo 3.2.2's collision table
 * (engine_collision_driver.c mjCOLLISIONFUNC; geom1 has the smaller MuJoCo geom
 * type, as mj_collideGeoms orders them; ABI 23) */
#define MGS_PAIR_CONVEX 0          /* mjc_Convex: MPR (ccd_mode 0: + feature clipping; 1: + multiccd) */
#define MGS_PAIR_BOXBOX 1          /* box-box separating-axis collider (mjc_BoxBox role) */
#define MGS_PAIR_CONVEX_SMOOTH 2   /* mjc_Convex with a sphere in the pair: one MPR contact (no multiccd) */
#define MGS_PAIR_SPHERE_SPHERE 3   /* mjc_SphereSphere  (1 contact) */
#define MGS_PAIR_SPHERE_CAPSULE 4  /* mjc_SphereCapsule (1) */
#define MGS_PAIR_CAPSULE_CAPSULE 5 /* mjc_CapsuleCapsule (1; 2 for parallel axes) */
#define MGS_PAIR_SPHERE_BOX 6      /* mjc_SphereBox (1) */
#define MGS_PAIR_CAPSULE_BOX 7     /* mjc_CapsuleBox (1 or 2) */
#define MGS_PAIR_SPHERE_CYLINDER 8 /* mjc_SphereCylinder (1) */

/* ccd_mode: how convex pairs make contacts */
#define MGS_CCD_R5 0               /* round 5's contract: MPR + face clipping (<= 4 points), rounded geoms
                                      as hull (+) ball (kept for the contact-set study) */
#define MGS_CCD_MULTI 1            /* MuJoCo 3.2.2 restated: libccd's MPR penetration (point-triangle
                                      depth, tetrahedron barycentre position) + multiccd (4 perturbed
                                      MPRs, <= 5 contacts); analytic primitive colliders */
#define MGS_CCD_SINGLE 2           /* the same without the multiccd flag: one MPR contact per pair */

/* predicate for the collision pre-filter */
#define MGS_PRED_ANY_CONTACT 0     /* data.ncon != 0            (gravityless :306-307) */
#define MGS_PRED_PARTITION 1       /* gripper geom vs geom past the partition (gravityless
                                      check_contact_with_object :309-320; clutter check_gripper_contact) */
#define MGS_PRED_PARTITION_INCL 2  /* gripper geom vs the partition geom or past it
                                      (clutter check_gripper_collision, clutter_table.py:237-252) */

typedef struct mgs_model_desc {
  /* sizes */
  int32_t nq;
  int32_t nv;
  int32_t nbody;
  int32_t njnt;
  int32_t ngeom;      /* collision geoms only, in MuJoCo geom order */
  int32_t nhull;
  int32_t nhullvert;
  int32_t npair;      /* statically admissible collision pairs */
  int32_t neq;
  int32_t ntendon;
  int32_t nwrap;
  int32_t nu;
  int32_t nmocap;
  int32_t nact;       /* actuator state (mjData.act) entries: 2 per mujoco.pid actuator (ABI 21) */
  int32_t npid;       /* mujoco.pid actuators (MGS_GAIN_PID), with or without act entries (ABI 23) */
  int32_t maxcondim;  /* largest contact dimension of the admissible pairs: 1, 3, 4 or 6 (condim 6:
                         torsional and rolling friction; runs through a specialised code object) */
  int32_t g_rows_hbm; /* 1: the whitened constraint rows G of each candidate live in a batch-owned
                         HBM buffer instead of LDS (always so in the wide library; in the main
                         library an option of the specialised code objects, which are then built
                         with -DMGS_G_GLOBAL; the library kernels refuse it) */
  int32_t ncon_max;   /* contact capacity per candidate (set by host) */
  int32_t nefc_max;   /* constraint-row capacity per candidate (set by host) */
  int32_t maxhullvert;
  /* options (MuJoCo <option>) */
  int32_t iterations;
  int32_t noslip_iterations;
  int32_t cone;       /* 1 = elliptic (the only cone supported) */
  int32_t integrator; /* 2 = implicitfast (the only integrator supported) */
  int32_t solver;     /* MuJoCo mjtSolver numbering: 0 = PGS, 2 = Newton (MuJoCo's default) */
  int32_t ls_iterations;
  int32_t ccd_mode;       /* MGS_CCD_*: the collision table and the convex pairs' contacts (ABI 23) */
  int32_t ccd_iterations; /* MuJoCo opt.ccd_iterations (50): MPR penetration refinement cap */
  double ls_tolerance;
  double timestep;
  double impratio;
  double tolerance;
  double noslip_tolerance;
  double mpr_tolerance;
  double meaninertia; /* MuJoCo stat.meaninertia: mean diagonal of M at qpos0 (mj_setConst);
                         the solvers' tolerance scale is 1 / (meaninertia * max(1, nv)) */
  double gravity[3];
  /* body arrays: int */
  int32_t i_body_parentid;
  int32_t i_body_rootid;
  int32_t i_body_mocapid;
  int32_t i_body_jntnum;
  int32_t i_body_jntadr;
  int32_t i_body_dofnum;
  int32_t i_body_dofadr;
  int32_t i_body_lastdof;   /* last dof in the body's kinematic chain, -1 if none */
  int32_t i_body_dofmask;   /* 2 (4 when nv > 64): bit d set if dof d moves the body (dofs 0-31, 32-63, ...) */
  int32_t i_body_depth;     /* tree depth (world 0); entry [nbody] = max depth */
  int32_t i_body_childadr;  /* first entry of the body's children in body_child */
  int32_t i_body_childnum;  /* number of children */
  int32_t i_body_child;     /* children grouped by parent, decreasing body index */
  /* body arrays: double */
  int32_t d_body_pos;       /* 3 */
  int32_t d_body_quat;      /* 4 */
  int32_t d_body_ipos;      /* 3 */
  int32_t d_body_iquat;     /* 4 */
  int32_t d_body_mass;      /* 1 */
  int32_t d_body_inertia;   /* 3 */
  int32_t d_body_gravcomp;  /* 1: gravity compensation (ABI 21): the body's weight times this,
                               cancelled through a force at its centre of mass (passive force) */
  int32_t d_body_invweight0; /* 2: translational, rotational (MuJoCo mj_setConst) */
  int32_t d_dof_invweight0;  /* nv (indexed by dof) */
  /* joints */
  int32_t i_jnt_type;
  int32_t i_jnt_qposadr;
  int32_t i_jnt_dofadr;
  int32_t i_jnt_bodyid;
  int32_t i_jnt_limited;
  int32_t d_jnt_pos;        /* 3 */
  int32_t d_jnt_axis;       /* 3 */
  int32_t d_jnt_range;      /* 2 */
  int32_t d_jnt_solref;     /* 2 */
  int32_t d_jnt_solimp;     /* 5 */
  int32_t d_jnt_margin;     /* 1 */
  int32_t d_jnt_stiffness;  /* 1 */
  /* dofs */
  int32_t i_dof_bodyid;
  int32_t i_dof_jntid;
  int32_t i_dof_parentid;
  int32_t d_dof_armature;
  int32_t d_dof_damping;
  int32_t d_dof_frictionloss;
  int32_t d_dof_solref;     /* 2 */
  int32_t d_dof_solimp;     /* 5 */
  int32_t d_qpos0;          /* nq */
  int32_t d_qvel0;          /* nv: initial qvel of every candidate (0; a clutter scene's env_state) */
  int32_t d_qacc_ws0;       /* nv: initial qacc_warmstart (0; a clutter scene's env_state) */
  int32_t d_qpos_spring;    /* nq */
  /* collision geoms */
  int32_t i_geom_bodyid;
  int32_t i_geom_hullid;
  int32_t i_geom_side;      /* -1 before the partition geom, 0 the partition geom, +1 after */
  int32_t d_geom_pos;       /* 3 */
  int32_t d_geom_quat;      /* 4 */
  int32_t d_geom_aabb;      /* 6: local box center (3), half sizes (3) */
  int32_t d_geom_radius;    /* 1: rounding radius; the geom is its hull (+) a ball of this
                               radius (sphere: 1 vertex, capsule: 2 vertices on z; 0 otherwise) */
  int32_t d_geom_rbound;    /* 1: largest vertex norm of the geom's hull (geom frame): bounds how
                               far a rotation moves its supports (separation certificates) */
  int32_t d_geom_cyl;       /* 2: cylinder radius and half-height, (0, 0) for other geoms (ABI
                               18).  A cylinder's supports and contact features are the exact
                               ones; its hull, a 16-sided prism inscribed in it (rim vertices
                               on the true circle), serves the broadphase and the cap polygon */
  int32_t d_geom_size;      /* 3: MuJoCo geom_size (sphere r; capsule r, half-length; box half sizes;
                               cylinder r, half-height): the analytic colliders (ABI 23) */
  /* convex hulls */
  int32_t i_hull_vertadr;
  int32_t i_hull_vertnum;
  int32_t d_hull_vert;      /* 3 * nhullvert, in geom frame; per hull x[n], y[n], z[n] */
  int32_t d_hull_center;    /* 3 * nhull, MPR interior point in geom frame (the geom origin, as
                               MuJoCo's ccd centre geom_xpos; meshes are recentred on their COM) */
  /* admissible pairs with mixed contact parameters */
  int32_t i_pair_geom1;
  int32_t i_pair_geom2;
  int32_t i_pair_condim;
  int32_t i_pair_kind;      /* MGS_PAIR_*: the pair's collider (see above) */
  int32_t d_pair_friction;  /* 5 */
  int32_t d_pair_solref;    /* 2 */
  int32_t d_pair_solimp;    /* 5 */
  int32_t d_pair_margin;    /* 1 */
  /* equality constraints */
  int32_t i_eq_type;
  int32_t i_eq_obj1id;
  int32_t i_eq_obj2id;
  int32_t d_eq_data;        /* 11 */
  int32_t d_eq_solref;      /* 2 */
  int32_t d_eq_solimp;      /* 5 */
  /* fixed tendons */
  int32_t i_tendon_adr;
  int32_t i_tendon_num;
  int32_t i_wrap_dofid;
  int32_t i_wrap_qposadr;
  int32_t d_wrap_coef;
  /* actuators */
  int32_t i_actuator_trntype;
  int32_t i_actuator_trnid;
  int32_t i_actuator_gaintype;
  int32_t i_actuator_biastype;
  int32_t i_actuator_ctrllimited;
  int32_t i_actuator_forcelimited;
  int32_t d_actuator_gainprm;   /* 3 */
  int32_t d_actuator_biasprm;   /* 3 */
  int32_t d_actuator_ctrlrange; /* 2 */
  int32_t d_actuator_forcerange;/* 2 */
  int32_t d_actuator_gear;      /* 1 */
  int32_t d_actuator_moment;    /* nu x nv: the actuator moment rows (joint: gear at the joint's dof;
                                   fixed tendon: 0 + sum of wrap coef x gear in wrap order), constant
                                   for these transmissions (round 5: the wide build reads them here) */
  int32_t i_actuator_actadr;    /* first act entry of the actuator, -1 if it has none */
  int32_t d_act0;               /* nact: the act state every candidate starts from (mj_resetData: 0;
                                   ClutterTableEnv: the scene state's, clutter_table.py:290-291) */
  int32_t d_actuator_pidprm;    /* 5: kp, ki, kd, imax, slewmax of a MGS_GAIN_PID actuator (imax,
                                   slewmax < 0: not set).  Restated from MuJoCo's mujoco.pid plugin
                                   semantics (parity unpinned: its source is not here): setpoint =
                                   ctrl clamped to ctrlrange, then, with slewmax, to within
                                   slewmax * dt of the previous setpoint (act entry 2); error =
                                   setpoint - actuator length; force = kp error + kd (setpoint rate -
                                   actuator velocity) + ki integral, clamped to forcerange, where the
                                   integral (act entry 1) advances by error * dt, clamped so that
                                   |ki integral| <= imax.  The act entries advance with the step
                                   (mj_advance: act += dt * act_dot). */
  /* buffer lengths (elements) */
  int32_t isize;
  int32_t dsize;
} mgs_model_desc;

/* Rollout schedule: a sequence of phases (close, lift, back, right, left ...).
 * During phase p, step t (0-based) the mocap position is
 *     start + (target - start) * (t / nsteps)          (per component, fp64)
 * with per-candidate start/target given to mgs_rollout; ctrl is held at
 * ctrl[p*32 .. p*32+nu).  After step t, if check_every > 0 and t + off > 0 and
 * (t + off) % check_every == 0 (off = check_offset[p]), the gripper-object
 * contact predicate is evaluated on
 * the contacts of that step; if check_at_end, it is evaluated after the last
 * step.  The first failed check ends the candidate with label 0.            */
#define MGS_MAX_PHASES 8
typedef struct mgs_schedule {
  int32_t nphase;
  int32_t obj_qposadr;   /* qpos address of the object free joint reported in obj_qpos (-1: none) */
  int32_t nsteps[MGS_MAX_PHASES];
  int32_t check_every[MGS_MAX_PHASES];
  int32_t check_at_end[MGS_MAX_PHASES];
  int32_t check_offset[MGS_MAX_PHASES];  /* check after step t if (t + off) > 0 and (t + off) % check_every == 0:
                                            0 = gravityless lift (:216), 1 = clutter lift ((t+1) % 100, :313) */
  double ctrl[MGS_MAX_PHASES * 32];
  double vclip;          /* > 0: clip every qvel entry to [-vclip, vclip] after each step
                            (ClutterTableEnv.gen_clutter, clutter_table.py:215-221); 0 = off */
  int32_t pause_step;    /* > 0 (with resume records): a candidate that has executed this many
                            steps (global step count, resumed runs included) stops before the
                            next one with its resume record, MGS_FLAG_PAUSED and fail_step -4,
                            so a long batch runs as time slices of several launches (ABI 18);
                            0 = run to the end */
  int32_t capped_continue; /* 1: with resume records, a candidate over the contact / row capacity
                            runs on capped and flagged instead of stopping (the last stage of an
                            escalation); 0 = stop there (fail_step -3) */
  int32_t yield_every;   /* > 0 (with resume records, on a work-queue launch): in-launch rotation
                            (ABI 19).  Every yield_every steps a candidate checks whether another
                            one waits for a slot (not started yet, or yielded); if so it writes
                            its resume record, joins the launch's ring of yielded candidates and
                            its workgroup takes the waiting one.  A launch with more rollouts
                            than resident workgroups then runs them round robin and ends about
                            one slice after the last one finishes; outputs are those of one
                            uninterrupted run (the record is the complete state).  0 = off */
} mgs_schedule;

/* per-candidate rollout outputs */
typedef struct mgs_rollout_out {
  uint8_t* label;          /* n: 1 = every check passed */
  int32_t* fail_step;      /* n: global step index of the failed check, -1 if none */
  double* obj_qpos;        /* n * 7: object free-joint qpos when the candidate stopped (may be NULL) */
  int32_t* stats;          /* n * MGS_NSTATS: max ncon, max nefc, overflow flags, total solver
                              iterations, sum of ncon and sum of nefc over executed steps (may be NULL) */
  double* resume;          /* n * (nq + 2 nv + nact + MGS_RESUME_EXTRA), may be NULL.  When set, a candidate
                              that exceeds the contact / row capacity stops at that step (fail_step
                              -3) and its record holds the state entering it (qpos, qvel,
                              qacc_warmstart, time) and the schedule position / partial stats, from
                              which mgs_rollout_resume continues it with more capacity */
} mgs_rollout_out;
#define MGS_RESUME_EXTRA 10        /* time, phase, step in phase, global step, max ncon, max nefc,
                                      sum ncon, sum nefc, solver iterations, flags.  A record is
                                      qpos (nq), qvel (nv), qacc_warmstart (nv), act (nact), then
                                      these (ABI 21: act) */

typedef struct mgs_model mgs_model;
typedef struct mgs_batch mgs_batch;

int mgs_abi_version(void);
const char* mgs_last_error(void);

/* Upload a compiled model; ibuf/dbuf hold desc->isize int32 and desc->dsize doubles. */
int mgs_model_create(const mgs_model_desc* desc, const int32_t* ibuf, const double* dbuf,
                     int device, mgs_model** out);
void mgs_model_free(mgs_model* model);

/* Per-candidate LDS working set (bytes) the kernels would use for this model
 * description, i.e. at its ncon_max / nefc_max capacity; host-only (no device
 * needed).  The host picks the contact/row capacity with it: a CU holds
 * floor(160 KiB / bytes) candidates in flight. */
int mgs_model_lds_bytes(const mgs_model_desc* desc, int64_t* out_bytes);
/* The LDS carve-up itself (offsets in doubles: the persistent arrays, the
 * time-multiplexed U views, then ncon_max, nefc_max, nv, total), host-only.
 * Writes at most cap words and their count to *nwords.  A model-specialised
 * code object bakes exactly these words (mgs/core/special.py). */
int mgs_model_layout(const mgs_model_desc* desc, int32_t* out, int cap, int32_t* nwords);
/* Attach a model-specialised code object: mgs_special.hip compiled for this
 * model (hipcc --genco with the header mgs/core/special.py generates from the
 * model description and mgs_model_layout), in which every LDS view, size,
 * table offset and option is a compile-time constant.  The object's baked ABI
 * version, library flavour (rows per lane), description and layout are read
 * back and must equal this model's, else MGS_EINVAL and nothing changes.  From
 * then on the model's collision and rollout launches use its kernels; a dof
 * count without a library instantiation (mgs_supports_nv == 0) runs only
 * this way.  Stage timers of an MGS_PROFILE object: mgs_model_prof_read. */
int mgs_model_attach_special(mgs_model* model, const char* code_object_path);
/* 1 if a specialised code object is attached, 0 if the runtime-offset kernels run. */
int mgs_model_special(const mgs_model* model);

/* Capacity limits of this library build: constraint rows per candidate
 * (libmgs_gpu.so 128, libmgs_gpu_wide.so 256) and whether a kernel is
 * instantiated for a dof count (1/0). */
int mgs_max_rows(void);
int mgs_supports_nv(int nv);
/* constraint rows per lane of this build's kernels (2 main, 4 wide): the
 * flavour a specialised code object must be compiled for (-DMGS_WIDE if 4) */
int mgs_rows_per_lane(void);

/* Device buffers for up to `capacity` candidates. */
int mgs_batch_open(mgs_model* model, int capacity, mgs_batch** out);
void mgs_batch_close(mgs_batch* batch);

/* Collision pre-filter (grasp_collision_mask).  qpos_init: n * nq initial qpos of
 * every candidate (host applies set_qpos / set_pose semantics); mocap_pos n*3,
 * mocap_quat n*4 (wxyz).  out_free[i] = 1 if the candidate is collision free. */
int mgs_collision_free(mgs_batch* batch, int n, const double* qpos_init,
                       const double* mocap_pos, const double* mocap_quat,
                       int predicate, uint8_t* out_free);

/* Same on device-resident inputs (HBM), asynchronous on `stream` (a
 * hipStream_t, NULL = default stream); d_out_free: n bytes on the device. */
int mgs_collision_free_device(mgs_batch* batch, int n, const double* d_qpos_init,
                              const double* d_mocap_pos, const double* d_mocap_quat,
                              int predicate, uint8_t* d_out_free, void* stream);

/* Close -> lift -> shake rollout.  phase_start / phase_target: n * nphase * 3
 * mocap endpoints per candidate and phase. */
int mgs_rollout(mgs_batch* batch, const mgs_schedule* sched, int n,
                const double* qpos_init, const double* mocap_quat,
                const double* phase_start, const double* phase_target,
                mgs_rollout_out* out);

/* mgs_rollout continuing each candidate from its resume record (n records as
 * returned in mgs_rollout_out.resume by a capped run of the same candidates,
 * same schedule): GravitylessObjectGrasping.rollout's capacity escalation. */
int mgs_rollout_resume(mgs_batch* batch, const mgs_schedule* sched, int n, const double* qpos_init,
                       const double* mocap_quat, const double* phase_start, const double* phase_target,
                       const double* resume, mgs_rollout_out* out);

/* Same as mgs_rollout but with inputs already resident on the device (device
 * pointers, same layouts); outputs stay on the device.  Used to time the
 * kernel with inputs in HBM.  stream may be NULL (default stream).
 * d_active (n bytes, may be NULL = all): candidates with d_active[i] == 0 are
 * not simulated (the collision-mask rejects of filter_to_stable.py:39-44):
 * label 0, fail_step -2, obj_qpos = the initial object pose, stats 0. */
int mgs_rollout_device(mgs_batch* batch, const mgs_schedule* sched, int n,
                       const double* d_qpos_init, const double* d_mocap_quat,
                       const double* d_phase_start, const double* d_phase_target,
                       const uint8_t* d_active, uint8_t* d_label, int32_t* d_fail_step,
                       double* d_obj_qpos, int32_t* d_stats, void* stream);

/* Capacity escalation on the device (GravitylessObjectGrasping.rollout's
 * re-run of the candidates that overflowed the contact / constraint-row
 * capacity, with no host round trip).  A device list is a header of
 * MGS_LIST_HEADER int32 words -- [0] count, [1] workgroup exits (internal),
 * [2] the count the last mgs_rollout_list_device over it ran, [3] reserved --
 * followed by up to n int32 candidate indices (arrival order; each re-run is
 * independent of the order).  A header starts zeroed (the caller's
 * allocation) and mgs_rollout_list_device leaves words 0 and 1 zeroed again,
 * so one header serves launch after launch with no fill in between (ABI 17).
 *
 * mgs_overflow_list_device zeroes words 0 and 1 of *d_count and writes the
 * indices i < n with stats[i * MGS_NSTATS + 2] & flag_mask into d_list,
 * asynchronously on `stream`.  mgs_rollout_list_device re-runs exactly the
 * listed candidates (as mgs_rollout_device would, outputs written at their
 * indices, other entries untouched) with `grid` workgroups that loop over the
 * list, so an empty or short list costs a handful of workgroups instead of one
 * per batch entry; d_count is the list's header, grid <= the batch capacity. */
#define MGS_LIST_HEADER 4
int mgs_overflow_list_device(int n, const int32_t* d_stats, int flag_mask, int32_t* d_count, int32_t* d_list,
                             void* stream);
int mgs_rollout_list_device(mgs_batch* batch, const mgs_schedule* sched, int n, int32_t* d_count,
                            const int32_t* d_list, int grid, const double* d_qpos_init, const double* d_mocap_quat,
                            const double* d_phase_start, const double* d_phase_target, const double* d_resume_in,
                            uint8_t* d_label, int32_t* d_fail_step, double* d_obj_qpos, int32_t* d_stats,
                            void* stream);
/* mgs_rollout_device that stops each overflowing candidate at the overflowing
 * step and writes its resume record to d_resume_out (n records, see
 * mgs_rollout_out.resume); mgs_rollout_list_device with d_resume_in != NULL
 * continues the listed candidates from those records (the capped run and the
 * wider one are identical up to that step), so the escalation costs only the
 * remaining steps.  d_ovf (may be NULL; ABI 17): a device list (header +
 * n entries, see above) each capacity-capped candidate appends itself to, so
 * mgs_rollout_list_device(d_count = d_ovf, d_list = d_ovf + MGS_LIST_HEADER)
 * can follow with no list kernel in between. */
int mgs_rollout_resumable_device(mgs_batch* batch, const mgs_schedule* sched, int n, const double* d_qpos_init,
                                 const double* d_mocap_quat, const double* d_phase_start,
                                 const double* d_phase_target, const uint8_t* d_active, uint8_t* d_label,
                                 int32_t* d_fail_step, double* d_obj_qpos, int32_t* d_stats, double* d_resume_out,
                                 int32_t* d_ovf, void* stream);
/* The collision mask and the rollout in one launch (ABI 15): each workgroup
 * computes its candidate's mask exactly as mgs_collision_free_device does
 * (qpos_init, mocap_pos, mocap_quat, predicate) into d_free_out[i], and a
 * collision-free candidate then runs mgs_rollout_resumable_device's rollout in
 * the same workgroup (rejects get mgs_rollout_device's reject outputs), so no
 * rollout waits for a separate mask launch.  The pair the reference runs as
 * grasp_collision_mask then grasp_stability_evaluation_from_joints on the
 * collision-free subset (mgs/cli/filter_to_stable.py:39-50); outputs are those
 * of the two separate calls, bit for bit.  d_resume_out and d_ovf (the
 * overflow list, as in mgs_rollout_resumable_device) may be NULL. */
int mgs_mask_rollout_device(mgs_batch* batch, const mgs_schedule* sched, int n, const double* d_qpos_init,
                            const double* d_mocap_pos, const double* d_mocap_quat, const double* d_phase_start,
                            const double* d_phase_target, int predicate, uint8_t* d_free_out, uint8_t* d_label,
                            int32_t* d_fail_step, double* d_obj_qpos, int32_t* d_stats, double* d_resume_out,
                            int32_t* d_ovf, void* stream);
/* Launch shape of the rollout calls above (ABI 16).  A rollout over n
 * candidates runs as a work queue: the grid is the number of rollout
 * workgroups the device holds at once (occupancy at this model's LDS size x
 * CUs) and each workgroup takes the next candidate index from a counter when
 * its previous rollout ends, so rejected, early-failing and full-length
 * candidates pack the slots; outputs are independent of the order.  Returns
 * that grid (n if n is smaller, or in mode 0 of mgs_rollout_queue: one
 * workgroup per candidate); needs the device. */
int mgs_rollout_grid(mgs_batch* batch, int n);
/* The rollout workgroups the device holds at once for this model (occupancy
 * at its LDS size x CUs; -1 if unknown), the grid of a work-queue launch in
 * mode 1, without opening a batch (ABI 23). */
int mgs_model_resident(mgs_model* model);
/* In-launch rotation counters of a batch (ABI 19), cumulative over its
 * launches: out[0] yields (a candidate handed its slot to a waiting one),
 * out[1] expired ring spins (0 unless the rotation protocol is broken; see
 * mgs_schedule.yield_every).  Synchronises the device.  The synchronous
 * entries (mgs_rollout, mgs_rollout_resume) check out[1] after their launch
 * themselves and fail with MGS_EQUEUE if it grew (ABI 20); callers of the
 * device entries check it (or the MGS_FAIL_YIELDED sentinel) after theirs.
 * The rotation rings are sized for the largest n a batch has launched with
 * rotation (grown, with a device synchronisation, when a launch's n exceeds
 * it), whatever the batch capacity. */
int mgs_queue_stats(mgs_batch* batch, uint64_t* out);
/* Execution spans of the batch's work-queue rollout launches (round 5), from
 * the device's 100 MHz real-time counter: the workgroup that takes candidate 0
 * records the start, the last workgroup to leave records the end, in the
 * launch's queue header.  Writes up to cap spans (ms) of the launches completed
 * since the previous call, in queue-slot order (the slots cycle through 64
 * headers, so call at least every 64 launches), sets *count, and clears the
 * spans it returned.  *overwritten (may be NULL; ABI 23): the launches since
 * the previous call whose spans were lost to that cycling (0 if none).  Synchronises the device.  (bench.py: the per-launch
 * duration of the roofline line, the kernel-trace duration without a
 * profiler.) */
int mgs_queue_spans(mgs_batch* batch, double* out_ms, int cap, int* count, int* overwritten);
/* Rollout launch mode for this process; returns the previous one and leaves it
 * unchanged if mode < 0.  0: one workgroup per candidate; 1 (default): the work
 * queue on the resident grid; k >= 2: the queue on at most k workgroups (tests
 * exercise the queue with small batches this way).  MGS_QUEUE in the
 * environment sets the initial mode. */
int mgs_rollout_queue(int mode);

/* Antipodal candidate ray casting (AntipodalGraspGenerator.generate_grasps,
 * mgs/sampler/antipodal.py:96-172, trimesh intersects_location): for each of
 * n surface points, cast dir and -dir from origin through the ntri triangles
 * (tri: ntri * 9, vertices v0 v1 v2), keep hits at distance >= eps, and return
 * the k-th, k = min(floor(u_choice * count), count - 1), in the order (+dir hits
 * by triangle index, -dir hits by triangle index).  out_nvalid[i] = count (0:
 * the caller applies the reference's random-offset fallback).  Host pointers;
 * synchronous on `device`; kernel_ms (may be NULL) = kernel duration. */
int mgs_antipodal_contacts(int device, const double* tri, int ntri, int n, const double* origin,
                           const double* dir, const double* u_choice, double eps, double* out_second,
                           int32_t* out_nvalid, double* kernel_ms);

/* Free simulation of n states (scene settling: ClutterTableEnv.gen_clutter /
 * is_stable / settle, clutter_table.py:157-222): the rollout loop of `sched`
 * with its contact checks ignored (a free simulation never stops early),
 * starting from qpos_init (n * nq) and, when vstate_init is not NULL,
 * per-state qvel, qacc_warmstart and act (n * (2nv + nact): qvel, warmstart,
 * act; NULL = the model's qvel0 / qacc_ws0 and act 0).  state_out receives
 * n * (nq + 2nv + nact): final qpos, qvel, qacc_warmstart, act.  stats (may be NULL): n * MGS_NSTATS as in
 * mgs_rollout_out; stats[i * MGS_NSTATS + 2] != 0 means state i exceeded the
 * contact / row capacity at some step and should be re-run wider.  Host
 * pointers (mgs_simulate) or device pointers on a stream (mgs_simulate_device,
 * n <= the batch capacity). */
int mgs_simulate(mgs_batch* batch, const mgs_schedule* sched, int n, const double* qpos_init,
                 const double* vstate_init, const double* mocap_quat, const double* phase_start,
                 const double* phase_target, double* state_out, int32_t* stats);
int mgs_simulate_device(mgs_batch* batch, const mgs_schedule* sched, int n, const double* d_qpos_init,
                        const double* d_vstate_init, const double* d_mocap_quat, const double* d_phase_start,
                        const double* d_phase_target, double* d_state_out, int32_t* d_stats, void* stream);

/* ---------------------------------------------------------------------------
 * Contact-based dexterous-hand sampler (ContactBasedDiff.generate_grasps,
 * mgs/sampler/contact.py:176-297): farthest-point seeds, local contact-target
 * selection, and a batched AdamW fit of the hand pose (6-D rotation, position)
 * and joints so that the fingertip contact points reach the targets
 * (contact.py:98-158 update/loss_fn; forward kinematics
 * mgs/sampler/kin/base.py:80-113; assignment mgs/sampler/kin/jax_util.py:205-224).
 * The kinematic model is data (mgs/sampler/kin/shadow.py:17-223).  Host
 * pointers, synchronous on `device`; kernel_ms (may be NULL) = kernel time. */
#define MGS_KIN_MAXDOF 24
#define MGS_KIN_MAXTIP 5
#define MGS_KIN_MAXCHAIN 6
#define MGS_KIN_MAXPERM 120
typedef struct mgs_kin_desc {
  int32_t ndof, ntip, nperm, iters;
  int32_t chain_len[MGS_KIN_MAXTIP];                 /* dofs from the palm to tip a */
  int32_t chain[MGS_KIN_MAXTIP][MGS_KIN_MAXCHAIN];   /* dof indices, root first */
  int32_t perm[MGS_KIN_MAXPERM][MGS_KIN_MAXTIP];     /* itertools.permutations order */
  double kin_tf[MGS_KIN_MAXDOF][7];                  /* parent -> joint frame: wxyz, xyz */
  double joint_tf[MGS_KIN_MAXDOF][6];                /* prismatic direction, revolute axis */
  double range[MGS_KIN_MAXDOF][2];
  double pregrasp[MGS_KIN_MAXDOF];
  double tip_point[MGS_KIN_MAXTIP][3];               /* chosen contact point, tip frame */
  double tip_normal[MGS_KIN_MAXTIP][3];              /* contact normal point, tip frame */
  double lr, b1, b2, eps, eps_root, weight_decay;    /* optax.adamw(lr) */
  double w_cos;                                      /* weight of the normal-alignment term */
} mgs_kin_desc;

/* sizeof(mgs_kin_desc) as compiled (the Python mirror checks its layout) */
int mgs_kin_desc_size(void);

/* farthest_point_sampling (jax_util.py:182-203): k indices into points (n * 3),
 * out_idx[0] = 0, each next index the first argmax of the running minimum
 * squared distance to the chosen set. */
int mgs_contact_fps(int device, const double* points, int n, int k, int32_t* out_idx, double* kernel_ms);

/* Per seed i of k seeds (seeds: k * 3): out_nn[i] = the nearest other seed
 * (argsort(dists)[:, 1], contact.py:226-228) and out_sel[i * ntip ...] = the
 * ntip largest random keys among seeds within `radius` (non-admissible keys
 * -inf), in ascending stable-argsort order (contact.py:201-210).  The keys are
 * splitmix64(rng_seed, i * k + j) uniforms in [0, 1) (the reference draws them
 * with jax.random.uniform, which is not restated). */
int mgs_contact_seeds(int device, const double* seeds, int k, double radius, uint64_t rng_seed, int ntip,
                      int32_t* out_nn, int32_t* out_sel, double* kernel_ms);

/* The AdamW fit of n candidates: rot_init (n * 9, the initial rotation matrix,
 * row-major), pos_init (n * 3), targets / normals (n * ntip * 3, the offset
 * contact targets and their surface normals in selection order).  The initial
 * fingertip-target assignment uses rot_init (contact.py:254-278); the loop
 * re-assigns every iteration (loss_fn).  Outputs: out_rot (n * 9, rows of the
 * Gram-Schmidt matrix of the final 6-D rotation), out_pos (n * 3), out_joints
 * (n * ndof, clipped to the ranges), out_loss (n, may be NULL: the loss at the
 * last iteration). */
int mgs_contact_optimize(int device, const mgs_kin_desc* kin, int n, const double* rot_init, const double* pos_init,
                         const double* targets, const double* normals, double* out_rot, double* out_pos,
                         double* out_joints, double* out_loss, double* kernel_ms);

/* Duration (ms) of the last rollout kernel launch, measured with HIP events
 * on the launch stream (waits for it). */
double mgs_last_kernel_ms(mgs_batch* batch);

/* Same for the last collision-mask kernel launch. */
double mgs_last_collision_ms(mgs_batch* batch);

#ifdef __cplusplus
}
#endif
#endif /* MGS_GPU_H_ */
