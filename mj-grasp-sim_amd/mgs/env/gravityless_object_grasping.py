"""Batched drop-in for GravitylessObjectGrasping
(reference: mgs/env/gravityless_object_grasping.py:34-321).

Same constructor and hot-path methods as the reference:

    env = GravitylessObjectGrasping(gripper, obj)
    mask  = env.grasp_collision_mask(poses, joints)                       # :90-125
    label = env.grasp_stability_evaluation_from_joints(poses, joints, ...) # :127-295

but every candidate of the batch is evaluated at once on the MI355X through
libmgs_gpu.so (mgs.core.engine).  The host side reproduces the reference's
bookkeeping exactly, because it defines the inputs of the physics:

  * pose processing `poses[i] @ b2c` through float32 SE3Pose (:117, :162);
  * `set_qpos(joints[i], get_joint_idxs(names))` with MuJoCo's
    mj_name2id == -1 -> jnt_qposadr[-1] behaviour (simualtion.py:37-49);
  * `set_pose`: free-joint qpos and mocap from the processed pose (base.py:48-59);
  * the mocap trajectory of close / lift / back / right / left, including the
    float32 re-cast of the mocap pose before the shake (:229-233) and the
    left-shake restart from the pre-right position (:264-272);
  * the check cadence (`t > 0 and t % 100 == 0` during lift, one check after
    each phase) and the `enough_stable` first-K rule (:151-156).

Only the physics (every mj_step / mj_forward and the contact predicates) runs
on the GPU.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional

import numpy as np

from mgs.core.abi import MGS
from mgs.core.mjcf import CompiledModel, compile_xml
from mgs.gripper.base import MjShakableOpenCloseGripper
from mgs.obj.base import CollisionMeshObject
from mgs.util.geo.transforms import SE3Pose

# stats[:, 2] flags that a wider re-run resolves (contacts / rows over capacity);
# MGS_FLAG_DIVERGED (a diverged state) is final
FLAG_CAPACITY = MGS["MGS_FLAG_CAPACITY"]

# Environment template: options, ground box and geom order restated from the
# reference (gravityless_object_grasping.py:34-54).  Geom order is
# gripper < geom:ground < object, which the contact predicate relies on.
XML = r"""
<mujoco>
    <compiler angle="radian" autolimits="true" />
    <option integrator="implicitfast" timestep="0.001"/>
    <compiler discardvisual="false"/>
    <option noslip_iterations="1"> </option>
    <option><flag multiccd="enable"/> </option>
    <option cone="elliptic" impratio="3" timestep="0.001" noslip_iterations="2" noslip_tolerance="1e-8" tolerance="1e-8"/>
    <option gravity="0 0 0" />
    {gripper}
    <worldbody>
        <body name="body:ground" pos="0.0 0 -1.0">
           <geom name="geom:ground" pos="0 0 0" size="1.0 1.0 0.02" type="box" density="500"/>
        </body>
    </worldbody>
    {object}
</mujoco>
"""

# Named rollout horizons.  ref8000 is the reference's own
# schedule; h200 keeps its phase structure (back = right = shake_steps,
# left = 2 * shake_steps, lift checked at a fixed cadence) scaled to 200 steps.
HORIZONS = {
    "ref8000": dict(close_steps=3000, nstep_lift=3000, shake_steps=500, lift_check_every=100),
    "h200": dict(close_steps=76, nstep_lift=76, shake_steps=12, lift_check_every=25),
}


@dataclass
class RolloutPlan:
    """Everything the GPU needs for one batch of rollouts (host-computed)."""
    nsteps: List[int]
    check_every: List[int]
    check_at_end: List[int]
    ctrl: List[np.ndarray]
    qpos_init: np.ndarray      # (n, nq)
    mocap_quat: np.ndarray     # (n, 4)
    phase_start: np.ndarray    # (n, nphase, 3)
    phase_target: np.ndarray   # (n, nphase, 3)
    obj_qposadr: int
    check_offset: Optional[List[int]] = None    # per phase, see mgs_schedule (0 when None)

    @property
    def horizon(self):
        return int(sum(self.nsteps))

    def subset(self, idx) -> "RolloutPlan":
        return RolloutPlan(self.nsteps, self.check_every, self.check_at_end, self.ctrl,
                           self.qpos_init[idx], self.mocap_quat[idx], self.phase_start[idx],
                           self.phase_target[idx], self.obj_qposadr, self.check_offset)


class _SimView:
    """Minimal stand-in for the reference's MjSimulation attributes used by
    gripper helpers (`sim.model.nu`, `sim.get_joint_idxs`)."""

    def __init__(self, env):
        self.model = env.model
        self.get_joint_idxs = env.get_joint_idxs


class GravitylessObjectGrasping:
    def __init__(self, gripper: MjShakableOpenCloseGripper, obj: CollisionMeshObject,
                 device: int = 0, ncon_max: int = 20, nefc_max: Optional[int] = None):
        self.gripper = gripper
        self.obj = obj
        self.gripper_xml, self.gripper_assets = gripper.to_xml()
        self.object_xml, self.object_assets = obj.to_xml()
        self.model_xml = XML.format(gripper=self.gripper_xml, object=self.object_xml)
        self.model: CompiledModel = compile_xml(self.model_xml, {**self.gripper_assets, **self.object_assets})
        self.device = device
        self.ncon_max = ncon_max
        self._nefc_max = nefc_max
        self._engine = None
        self._sim = _SimView(self)

    # -- reference helpers ---------------------------------------------------
    def get_joint_idxs(self, joint_list: List[str]) -> List[int]:
        return [self.model.jnt_qposadr_by_name(j) for j in joint_list]

    def get_object_qposadr(self) -> int:
        return self.get_joint_idxs(["{}:joint".format(self.obj.name)])[0]

    @property
    def nefc_max(self) -> int:
        """Constraint-row capacity of the main engine (default: mgs.core.engine.
        auto_capacity, the most candidates in flight per CU for ncon_max)."""
        if self._nefc_max is None:
            from mgs.core.engine import auto_capacity
            self._nefc_max = auto_capacity(self.model, self.ncon_max)[1]
        return self._nefc_max

    @property
    def capacity(self):
        return self.ncon_max, self.nefc_max

    @property
    def engine(self):
        if self._engine is None:
            from mgs.core.engine import Engine
            self._engine = Engine(self.model, device=self.device, ncon_max=self.ncon_max, nefc_max=self.nefc_max,
                                  g_rows_hbm="auto")
        return self._engine

    def engine_for(self, ncon_max: int):
        """Engine with a larger per-candidate contact capacity (overflow re-runs)."""
        if ncon_max == self.ncon_max:
            return self.engine
        if not hasattr(self, "_wide"):
            self._wide = {}
        if ncon_max not in self._wide:
            from mgs.core.engine import Engine
            # the few overflowing candidates: a specialised object only if one is
            # cached (compiling one would cost more than the re-run)
            self._wide[ncon_max] = Engine(self.model, device=self.device, ncon_max=ncon_max, specialize="cached",
                                          role="escalation")
        return self._wide[ncon_max]

    # in-launch rotation (mgs_schedule.yield_every, ABI 19): a batch with more
    # rollouts than resident workgroups runs them round robin in slices of this
    # many steps, so the launch ends about one slice after its last rollout
    # finishes instead of one whole rollout after its last one started
    YIELD_EVERY = 32
    # explicit time slices by relaunch (rollout(slices=k)): every k-th part of
    # the horizon is its own launch (pause_step); the default is one launch
    SLICES = 1

    # A call of a few rollouts (the stability call of filter_to_stable: the
    # collision-free part of one candidate file) is one round of them, i.e. its
    # heaviest rollout's latency.  The G-rows-in-LDS object (four per CU) steps
    # faster than the eight-per-CU one that holds the throughput: it finishes
    # calls of up to about 1.25-1.5 x its resident grid sooner (1173 rollouts:
    # 58.4 vs 59.5 ms; 1536: 61.2 vs 59.9; 2048: 68.7 vs 61.7;
    # profiles/r05lat_latency_engine.txt).  Same results bit for bit
    # (both objects are the oracle's arithmetic).
    LATENCY_ROUNDS = 1.25

    @property
    def latency_engine(self):
        """the main capacity's G-rows-in-LDS engine when the main engine keeps
        its rows in HBM and that object is cached, else None"""
        main = self.engine
        # (keyed by the main engine: a copied env with a rebuilt engine builds its own)
        if getattr(self, "_latency_for", None) is not main:
            self._latency_for, self._latency_engine = main, None
            if int(main.desc.g_rows_hbm):
                from mgs.core.engine import Engine
                e = Engine(self.model, device=self.device, ncon_max=self.ncon_max, nefc_max=self.nefc_max,
                           g_rows_hbm=False, specialize="cached")
                self._latency_engine = e if e.specialized() else None
        return self._latency_engine

    def engine_for_rollouts(self, n: int):
        """the engine a rollout call of n candidates runs on (LATENCY_ROUNDS;
        the latency engine's grid under the current queue mode, read per call)"""
        le = self.latency_engine
        if le is not None and 0 < n <= self.LATENCY_ROUNDS * le.queue_grid(1 << 30):
            return le
        return self.engine

    # the escalation's last capacity: 128 contacts / 256 rows (the wide
    # library's rows), as ClutterTableEnv; MuJoCo has no cap, so a candidate
    # still over it fails the call (sliced_rollout, on_capacity="raise")
    MAX_NCON = 128

    def rollout(self, plan: "RolloutPlan", max_ncon: Optional[int] = None, slices: Optional[int] = None,
                yield_every: Optional[int] = None, on_capacity: str = "raise"):
        """engine.rollout with capacity escalation, in-launch rotation and
        optional time slices by relaunch (sliced_rollout below), on the engine
        that finishes a call of this size first (engine_for_rollouts)."""
        return sliced_rollout(plan, self.engine_for_rollouts(len(plan.qpos_init)), self.engine_for, self.ncon_max,
                              self.MAX_NCON if max_ncon is None else max_ncon,
                              self.SLICES if slices is None else slices,
                              yield_every=self.YIELD_EVERY if yield_every is None else yield_every,
                              on_capacity=on_capacity)

    # -- host-side bookkeeping (exactly the reference's arithmetic) ------------
    def _check_inputs(self, poses, joints, check_width=True):
        if len(poses) != len(joints):
            raise ValueError(
                f"Number of poses ({len(poses)}) must match number of joint configurations ({len(joints)}).")
        if check_width and joints.shape[1] != len(self.gripper.get_actuator_joint_names()):
            raise ValueError(
                f"Joints array has incorrect dimension ({joints.shape[1]}), expected "
                f"{len(self.gripper.get_actuator_joint_names())}.")

    def initial_state(self, poses: SE3Pose, joints: np.ndarray):
        """(qpos_init (n,nq), mocap_pos (n,3), mocap_quat (n,4), processed pose)."""
        n = len(poses)
        b2c = self.gripper.base_to_contact_transform()
        proc = poses @ b2c if n > 0 else poses
        idxs = self.get_joint_idxs(self.gripper.get_actuator_joint_names())
        qpos = np.tile(self.model.qpos0, (n, 1))
        jj = np.asarray(joints, dtype=np.float64)
        for k, a in enumerate(idxs):      # sequential: duplicate indices -> last wins
            qpos[:, a] = jj[:, k]
        fj = self.get_joint_idxs(["freejoint"])[0]
        vec = proc.to_vec(layout="pq", type="wxyz") if n > 0 else np.zeros((0, 7), np.float32)
        qpos[:, fj:fj + 3] = vec[:, :3]
        qpos[:, fj + 3:fj + 7] = vec[:, 3:]
        mocap_pos = vec[:, :3].astype(np.float64)
        mocap_quat = vec[:, 3:].astype(np.float64)
        return qpos, mocap_pos, mocap_quat, proc

    def rollout_plan(self, poses: SE3Pose, joints: np.ndarray, nstep_lift=3000, lift_dist=0.1,
                     shake_steps=500, shake_dist=0.02, close_steps=None, lift_check_every=100) -> RolloutPlan:
        qpos, mocap_pos, mocap_quat, proc = self.initial_state(poses, joints)
        n = len(poses)
        close_steps = self.gripper.close_steps if close_steps is None else close_steps
        # close: mocap = pose (close_gripper_at), held
        p_close = mocap_pos.copy()
        # lift (:205-214): only z moves; x, y keep the mocap value
        start_lift = p_close.copy()
        target_lift = start_lift.copy()
        target_lift[:, 2] = start_lift[:, 2] + lift_dist
        t_last = nstep_lift - 1
        after_lift = start_lift.copy()
        after_lift[:, 2] = start_lift[:, 2] + (target_lift[:, 2] - start_lift[:, 2]) * (t_last / nstep_lift)
        # shake frame from the float32 mocap pose (:229-236)
        cur = SE3Pose(np.copy(after_lift), np.copy(mocap_quat), "wxyz")
        rot = cur.to_mat()[:, :3, :3]
        back_dir = rot @ np.array([0, 0, -1.0])
        right_dir = rot @ np.array([0, 1.0, 0])
        left_dir = rot @ np.array([0, -1.0, 0])
        target_back = cur.pos + back_dir * shake_dist
        start_back = after_lift.copy()
        s_last = shake_steps - 1
        after_back = start_back + (target_back - start_back) * (s_last / shake_steps)
        target_right = target_back + right_dir * shake_dist
        start_right = after_back.copy()
        # left restarts from the pre-right position (:266-272)
        target_left = start_right + left_dir * (2 * shake_dist)
        start_left = start_right.copy()
        starts = np.stack([p_close, start_lift, start_back, start_right, start_left], axis=1)
        targets = np.stack([p_close, target_lift, target_back, target_right, target_left], axis=1)
        ctrl_close = np.asarray(self.gripper.close_ctrl(self._sim), dtype=np.float64)
        return RolloutPlan(
            nsteps=[close_steps, nstep_lift, shake_steps, shake_steps, 2 * shake_steps],
            check_every=[0, lift_check_every, 0, 0, 0],
            check_at_end=[1, 1, 1, 1, 1],
            ctrl=[ctrl_close] * 5,
            qpos_init=qpos, mocap_quat=mocap_quat,
            phase_start=np.ascontiguousarray(starts), phase_target=np.ascontiguousarray(targets),
            obj_qposadr=self.get_object_qposadr())

    # -- hot path --------------------------------------------------------------
    def grasp_collision_mask(self, poses: SE3Pose, joints: np.ndarray) -> np.ndarray:
        self._check_inputs(poses, joints)
        if len(poses) == 0:
            return np.zeros(0, dtype=bool)
        qpos, mocap_pos, mocap_quat, _ = self.initial_state(poses, joints)
        return self.engine.collision_free(qpos, mocap_pos, mocap_quat, predicate="any")

    def grasp_stability_evaluation_from_joints(self, poses: SE3Pose, joints: np.ndarray,
                                               nstep_lift: int = 3000, lift_dist: float = 0.1,
                                               shake_steps: int = 500, shake_dist: float = 0.02,
                                               enough_stable=None, *, close_steps: Optional[int] = None,
                                               lift_check_every: int = 100, return_details: bool = False):
        self._check_inputs(poses, joints, check_width=False)
        if len(poses) == 0:
            return np.zeros(0, dtype=bool)
        plan = self.rollout_plan(poses, joints, nstep_lift, lift_dist, shake_steps, shake_dist,
                                 close_steps=close_steps, lift_check_every=lift_check_every)
        res = self.rollout(plan)
        labels = apply_enough_stable(res["label"].astype(bool), enough_stable)
        if return_details:
            res["label"] = labels
            return res
        return labels

    def evaluate(self, poses: SE3Pose, joints: np.ndarray, horizon: str = "ref8000", enough_stable=None):
        """collision mask + rollout of the collision-free candidates (the
        filter_to_stable.py:39-50 pipeline) with a named horizon."""
        h = HORIZONS[horizon]
        mask = self.grasp_collision_mask(poses, joints)
        stable = np.zeros(len(poses), dtype=bool)
        idx = np.nonzero(mask)[0]
        if len(idx):
            stable[idx] = self.grasp_stability_evaluation_from_joints(
                poses[idx], joints[idx], nstep_lift=h["nstep_lift"], shake_steps=h["shake_steps"],
                enough_stable=enough_stable, close_steps=h["close_steps"],
                lift_check_every=h["lift_check_every"])
        return mask, stable


def apply_enough_stable(labels: np.ndarray, enough_stable) -> np.ndarray:
    """Reference :151-156 -- once `enough_stable` candidates passed, the rest
    are reported False without simulation.  Equivalent post-hoc rule: keep the
    first K True labels."""
    labels = np.asarray(labels, dtype=bool).copy()
    if enough_stable is None:
        return labels
    cum = np.cumsum(labels)
    labels[(cum > enough_stable)] = False
    return labels


class CapacityError(RuntimeError):
    """candidates still over the contact / row capacity at the escalation's
    last stage: their labels would come from a capped contact set, which
    MuJoCo (no cap) never makes -- the call fails instead"""

    def __init__(self, idx, max_ncon):
        self.candidates = np.asarray(idx)
        super().__init__(f"{len(idx)} candidate(s) still exceed the contact / row capacity at max_ncon={max_ncon} "
                         f"(first {self.candidates[:8].tolist()}); their contact sets would be capped.  Raise "
                         f"max_ncon or pass on_capacity='capped' to accept flagged, capped results")


def sliced_rollout(plan: "RolloutPlan", engine, engine_for, cap: int, max_ncon: int, slices: int = 1,
                   yield_every: int = 0, on_capacity: str = "raise"):
    """A batch's rollouts on `engine` (capacity `cap` contacts) with capacity
    escalation and time slices; results equal one launch at unlimited capacity.

    Capacity: MuJoCo has no contact cap, the kernel's per-candidate contact
    arrays do (ncon_max, LDS-resident).  A candidate that exceeds it
    (stats[:, 2] & FLAG_CAPACITY) stops at that step and is continued from the
    state entering it on engine_for(2 cap) -- the capped and the wider run are
    identical up to there -- until none overflows or max_ncon is reached; its
    results replace the capped run's.  A candidate still over the capacity at
    max_ncon raises CapacityError (on_capacity="raise", the default: no label
    from a capped contact set is ever returned); on_capacity="capped" lets the
    last stage run on capped and flagged (res['overflow'] counts them).

    Rotation (yield_every > 0): inside each launch, a candidate that has run
    yield_every steps hands its slot to a waiting one (mgs_schedule.yield_every),
    so the launch ends about one slice after its last rollout finishes.

    Slices by relaunch (slices > 1): the horizon is cut into `slices`
    launches: every unfinished candidate stops at the slice boundary with a
    resume record (MGS_FLAG_PAUSED) and the next launch continues the
    survivors (one host round trip per slice; profiles/r04b_api.txt).

    Records carry the complete state, so either way the results equal one
    uninterrupted launch's bit for bit."""
    if on_capacity not in ("raise", "capped"):
        raise ValueError(f"on_capacity must be 'raise' or 'capped', not {on_capacity!r}")
    n = len(plan.qpos_init)
    H = plan.horizon
    slices = max(1, min(int(slices), max(H, 1)))
    bounds = [int(round(H * (j + 1) / slices)) for j in range(slices - 1)] + [0]
    capped_ok = on_capacity == "capped"
    last_cap = cap >= max_ncon and capped_ok
    res = engine.rollout(plan, resumable=True, pause_step=bounds[0], capped_continue=last_cap,
                         yield_every=yield_every)
    rec = res.pop("resume")
    live = np.arange(n)
    for j, b in enumerate(bounds):
        if j > 0:
            sub = engine.rollout(plan.subset(live), resumable=True, resume_from=rec[live], pause_step=b,
                                 capped_continue=last_cap, yield_every=yield_every)
            for k in ("label", "fail_step", "obj_qpos", "stats"):
                res[k][live] = sub[k]
            rec[live] = sub["resume"]
        flags = res["stats"][live, 2]
        ov = live[(flags & FLAG_CAPACITY) != 0] if not last_cap else live[:0]
        c = cap
        while len(ov) and c < max_ncon:
            c = min(2 * c, max_ncon)
            last = c >= max_ncon and capped_ok
            sub = engine_for(c).rollout(plan.subset(ov), resumable=True, resume_from=rec[ov], capped_continue=last,
                                        yield_every=yield_every)
            for k in ("label", "fail_step", "obj_qpos", "stats"):
                res[k][ov] = sub[k]
            keep = np.nonzero(sub["stats"][:, 2] & FLAG_CAPACITY)[0] if not last else np.zeros(0, np.int64)
            rec[ov[keep]] = sub["resume"][keep]
            ov = ov[keep]
        if len(ov) and not capped_ok:
            raise CapacityError(ov, max_ncon)
        live = live[(flags & MGS["MGS_FLAG_PAUSED"]) != 0]
        if not len(live):
            break
    res["overflow"] = int(((res["stats"][:, 2] & FLAG_CAPACITY) != 0).sum()) if n else 0
    return res
