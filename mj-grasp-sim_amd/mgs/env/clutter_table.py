"""Batched drop-in for ClutterTableEnv's grasp evaluation
(reference: mgs/env/clutter_table.py:60-399).

Same constructor, scene dict (`to_dict` / `from_dict`), integration-state
vector (`get_state` / `set_state`, MuJoCo's mjSTATE_INTEGRATION layout of the
reference model) and hot-path methods:

    env = ClutterTableEnv.from_dict(scene)
    mask   = env.grasp_collision_mask(poses, joints)                   # :330-367
    stable = env.grasp_stable_mask(poses, joints, env_state, ...)      # :272-321

with every candidate of the batch simulated at once on the MI355X (the wide
library: 4 constraint rows per lane, contact-rich piles).  The host keeps the
reference's bookkeeping: the in-bounds box of the collision mask (:344-354),
`mj_setState(env_state)` before each candidate (:290-291, :356), set_qpos /
set_pose from the float32 pose @ base_to_contact (:296-300), the gripper's
close phase (3000 steps), the 0.3 m lift checked when (t + 1) % 100 == 0
(:304-315) with check_gripper_contact, and the `enough_stable` prefix.

Bodies the reference keeps weightless and contact-free -- the scan camera
(`gravcomp="1"`, a free joint only moved for rendering, :46-50) and objects
taken out with `remove_obj` (contype = conaffinity = 0, gravcomp 1, :127-137)
-- exert no force on anything and feel none, so they are compiled as static
bodies at their state pose; the state vector keeps their slots.
"""
from __future__ import annotations

import xml.etree.ElementTree as Et
from copy import deepcopy
from typing import List, Optional

import numpy as np

from mgs.core.abi import MGS
from mgs.core.mjcf import CompiledModel, compile_xml
from mgs.env.gravityless_object_grasping import RolloutPlan, apply_enough_stable, sliced_rollout
from mgs.util.geo.transforms import SE3Pose

# stats[:, 2] flags that a wider re-run resolves (contacts / rows over capacity);
# MGS_FLAG_DIVERGED (a diverged state) is final
FLAG_CAPACITY = MGS["MGS_FLAG_CAPACITY"]

# clutter_table.py:41-79, restated (lights and the camera element are render-only)
XML = r"""
<mujoco>
    <compiler angle="radian" autolimits="true" />
    <option integrator="implicitfast" timestep="0.001"/>
    <compiler discardvisual="false"/>
    <option noslip_iterations="3"> </option>
    <option><flag multiccd="enable"/> </option>
    <option cone="elliptic" gravity="0 0 -9.81" impratio="3" timestep="0.001" noslip_iterations="3" noslip_tolerance="1e-10" tolerance="1e-10"/>
    {gripper}
    <worldbody>
        <body name="body:table" pos="0.0 0 -0.02">
           <geom name="geom:table" pos="0 0 0" size="10 10 0.02" type="box" density="500" friction="1.0 0.1 0.1"/>
        </body>
        <body name="body:camera" pos="{camera_pos}" quat="{camera_quat}">
          <geom name="geom:camera" size="0.01"/>
        </body>
        <body name="base_origin" pos="0.0 0.0 -0.025" quat="1.0 0.0 0 0">
          <geom name="geom:base_origin" size="0.01"/>
        </body>
        <body name="body:wall_top" pos="0.0 1.0 0.1">
           <geom name="geom:wall_top" pos="0 0 0" size="1.0 0.02 0.2" type="box" density="500"/>
        </body>
        <body name="body:wall_right" pos="1.0 0.0 0.1">
           <geom name="geom:wall_right" pos="0 0 0" size="0.02 1.0 0.2" type="box" density="500"/>
        </body>
        <body name="body:wall_bottom" pos="0.0 -1.0 0.1">
           <geom name="geom:wall_bottom" pos="0 0 0" size="1.0 0.02 0.2" type="box" density="500"/>
        </body>
        <body name="body:wall_left" pos="-1.0 0.0 0.1">
           <geom name="geom:wall_left" pos="0 0 0" size="0.02 1.0 0.2" type="box" density="500"/>
        </body>
    </worldbody>
    {objects}
</mujoco>
"""

CAMERA_QPOS0 = np.array([0.0, 0.0, -1.0, 1.0, 0.0, 0.0, 0.0])   # :46


def _frozen_object_xml(xml_bytes: bytes, qpos7) -> bytes:
    """an object include with its free joint removed, its geoms contact-free and
    its body placed at qpos7 (remove_obj + gravcomp: static in effect)."""
    root = Et.fromstring(xml_bytes)
    for body in root.iter("body"):
        for j in list(body):
            if j.tag in ("joint", "freejoint"):
                body.remove(j)
        for g in body.iter("geom"):
            g.set("contype", "0")
            g.set("conaffinity", "0")
        body.set("pos", " ".join(repr(float(x)) for x in qpos7[:3]))
        body.set("quat", " ".join(repr(float(x)) for x in qpos7[3:7]))
        break
    return Et.tostring(root)


class ClutterTableEnv:
    def __init__(self, gripper, objects: list, scene_randomization=True, device: int = 0,
                 ncon_max: int = 64, nefc_max: Optional[int] = None):
        self.gripper = gripper
        self.objects = list(objects)
        self.object_names = [o.name for o in self.objects]
        self.object_ids = [o.object_id for o in self.objects]
        self.device = device
        self.ncon_max = ncon_max
        self._nefc_max = nefc_max
        self.removed = set()                     # names of objects taken out (remove_obj)
        self.gripper_xml, self.gripper_assets = gripper.to_xml()
        self.object_xml_assets = [o.to_xml() for o in self.objects]
        # reference-model state layout: gripper joints, camera free joint, objects
        probe = self._compile(camera_qpos=CAMERA_QPOS0, frozen={})
        self._gripper_nq = probe.jnt_qposadr_by_name(f"{self.object_names[0]}:joint") if self.objects else probe.nq
        self._gripper_nv = int(probe.jnt_dofadr[probe.jnt_names.index(f"{self.object_names[0]}:joint")]) \
            if self.objects else probe.nv
        self.ref_nq = probe.nq + 7
        self.ref_nv = probe.nv + 6
        self._check_kernel(probe.nv)
        self.nbody = probe.nbody
        self.neq = len(probe.eq_type)
        self.nu = probe.nu
        self.na = int(probe.nact)                # actuator state (the gripper's mujoco.pid actuators)
        self._state = self._initial_state(probe)
        self._model_key = None
        self._model = None
        self._engines = {}

    def _check_kernel(self, nv):
        """the kernels hold up to 128 dofs (lanes over dofs: one per lane up to
        64, two per lane beyond, in a model-specialised code object compiled on
        first use, mgs.core.special); fail here, with the largest pile, rather
        than at the first simulation"""
        from mgs.core.engine import MAX_NV
        if nv > MAX_NV:
            g = self._gripper_nv
            raise ValueError(
                f"no GPU kernel for this scene: {len(self.objects) - len(self.removed)} free objects with this "
                f"gripper give nv={nv}; the kernels hold at most {MAX_NV} dofs, i.e. piles of at most "
                f"{(MAX_NV - g) // 6} free objects for this gripper")

    # -- state vector (mjSTATE_INTEGRATION of the reference model) ------------
    def _sizes(self):
        return [("time", 1), ("qpos", self.ref_nq), ("qvel", self.ref_nv), ("act", self.na),
                ("qacc_warmstart", self.ref_nv),
                ("ctrl", self.nu), ("qfrc_applied", self.ref_nv), ("xfrc_applied", 6 * self.nbody),
                ("eq_active", self.neq), ("mocap_pos", 3), ("mocap_quat", 4)]

    def state_size(self) -> int:
        return sum(n for _, n in self._sizes())

    def split_state(self, state) -> dict:
        state = np.asarray(state, dtype=np.float64)
        if state.shape != (self.state_size(),):
            raise ValueError(f"env_state has {state.shape[0] if state.ndim else 0} entries, expected "
                             f"{self.state_size()} (mjSTATE_INTEGRATION of this scene)")
        out, o = {}, 0
        for k, n in self._sizes():
            out[k] = state[o:o + n]
            o += n
        return out

    def join_state(self, parts: dict) -> np.ndarray:
        return np.concatenate([np.asarray(parts[k], np.float64).reshape(n) for k, n in self._sizes()])

    def _initial_state(self, cm: CompiledModel) -> np.ndarray:
        gq, gv = self._gripper_nq, self._gripper_nv
        qpos = np.concatenate([cm.qpos0[:gq], CAMERA_QPOS0, cm.qpos0[gq:]])
        mp = cm.body_pos[cm.body_names.index("mocap")]
        mq = cm.body_quat[cm.body_names.index("mocap")]
        return self.join_state(dict(time=[0.0], qpos=qpos, qvel=np.zeros(self.ref_nv), act=np.zeros(self.na),
                                    qacc_warmstart=np.zeros(self.ref_nv), ctrl=np.zeros(self.nu),
                                    qfrc_applied=np.zeros(self.ref_nv), xfrc_applied=np.zeros(6 * self.nbody),
                                    eq_active=np.ones(self.neq), mocap_pos=mp, mocap_quat=mq))

    def get_state(self) -> np.ndarray:
        return self._state.copy()

    def set_state(self, state) -> None:
        self.split_state(state)
        self._state = np.asarray(state, np.float64).copy()

    # -- ref layout <-> compiled (reduced) model -----------------------------
    def _obj_slices(self):
        """(name, ref qpos slice, ref qvel slice) of every object."""
        gq, gv = self._gripper_nq, self._gripper_nv
        return [(n, slice(gq + 7 + 7 * i, gq + 14 + 7 * i), slice(gv + 6 + 6 * i, gv + 12 + 6 * i))
                for i, n in enumerate(self.object_names)]

    def _reduce(self, vec, which):
        """ref-layout qpos / qvel -> the compiled model's (camera and removed objects dropped)."""
        gq, gv = self._gripper_nq, self._gripper_nv
        head = vec[:gq] if which == "q" else vec[:gv]
        parts = [head]
        for n, qs, vs in self._obj_slices():
            if n not in self.removed:
                parts.append(vec[qs] if which == "q" else vec[vs])
        return np.concatenate(parts)

    def _compile(self, camera_qpos, frozen: dict) -> CompiledModel:
        objs_xml, assets = "", {}
        for o, (oxml, oassets) in zip(self.objects, self.object_xml_assets):
            oassets = dict(oassets)
            if o.name in frozen:
                key = next(iter(oassets))
                oassets[key] = _frozen_object_xml(oassets[key], frozen[o.name])
            objs_xml += oxml
            assets.update(oassets)
        xml = XML.format(gripper=self.gripper_xml, objects=objs_xml,
                         camera_pos=" ".join(repr(float(x)) for x in camera_qpos[:3]),
                         camera_quat=" ".join(repr(float(x)) for x in camera_qpos[3:7]))
        return compile_xml(xml, {**self.gripper_assets, **assets})

    def model_for(self, state) -> CompiledModel:
        """compiled model of this scene for an integration state: static camera and
        removed objects at their state poses, qvel0 / qacc_ws0 = the state's."""
        parts = self.split_state(state)
        q = parts["qpos"]
        gq = self._gripper_nq
        cam = q[gq:gq + 7]
        frozen = {n: q[qs] for n, qs, _ in self._obj_slices() if n in self.removed}
        key = (tuple(np.round(cam, 15)), tuple((n, tuple(v)) for n, v in sorted(frozen.items())))
        if key != self._model_key:
            self._model = self._compile(cam, frozen)
            self._check_kernel(self._model.nv)      # remove_obj lowers nv by 6 per object
            self._model_key = key
            self._engines = {}
        cm = self._model
        cm.qvel0 = self._reduce(parts["qvel"], "v")
        cm.qacc_ws0 = self._reduce(parts["qacc_warmstart"], "v")
        cm.act0 = np.array(parts["act"], np.float64)
        return cm

    @property
    def model(self) -> CompiledModel:
        return self.model_for(self._state)

    def engine_for_state(self, state, ncon_max=None):
        from mgs.core.engine import Engine
        cm = self.model_for(state)
        nc = self.ncon_max if ncon_max is None else ncon_max
        key = (nc, cm.qvel0.tobytes(), cm.qacc_ws0.tobytes(), cm.act0.tobytes())
        if key not in self._engines:
            self._engines = {k: v for k, v in self._engines.items() if k[1:] == key[1:]}
            # escalation capacities re-run few candidates: specialised only if cached
            self._engines[key] = Engine(cm, device=self.device, ncon_max=nc, nefc_max=self.rows_for(cm, nc),
                                        specialize=None if nc == self.ncon_max else "cached",
                                        role="main" if nc == self.ncon_max else "escalation",
                                        g_rows_hbm="auto" if nc == self.ncon_max else None)
        return self._engines[key]

    def rows_for(self, cm, nc):
        """constraint rows of the engine at nc contacts: the env's nefc_max if
        one was given; at the main capacity the rows that keep the most pile
        candidates per CU (auto_capacity: two per CU at 64 contacts and about
        190 rows), whose overflow the escalation continues wider;
        an escalation capacity's engine the library's worst case (None)"""
        from mgs.core.engine import auto_capacity
        if self._nefc_max is not None:
            return self._nefc_max
        if nc != self.ncon_max:
            return None
        key = (nc, cm.nv, len(cm.pair_condim), len(cm.eq_type))
        if getattr(self, "_rows_key", None) != key:
            self._rows_key, self._rows = key, auto_capacity(cm, nc)[1]
        return self._rows

    # -- reference helpers ---------------------------------------------------
    def get_joint_idxs(self, joint_list: List[str]) -> List[int]:
        """qpos addresses in the reference model's layout (the camera joint
        follows the gripper's)."""
        cm = self.model
        out = []
        for j in joint_list:
            a = cm.jnt_qposadr_by_name(j)
            out.append(a + 7 if a >= self._gripper_nq else a)
        return out

    def remove_obj(self, obj):
        """clutter_table.py:127-137: the object stops colliding and floats."""
        self.removed.add(obj.name)
        self._model_key = None

    def get_obj_pose(self, object_name: str) -> SE3Pose:
        q = self.split_state(self._state)["qpos"]
        qs = dict((n, s) for n, s, _ in self._obj_slices())[object_name]
        return SE3Pose(np.copy(q[qs][:3]), np.copy(q[qs][3:7]), "wxyz")

    def get_object(self, object_name: str):
        for o in self.objects:
            if o.name == object_name:
                return o
        return None

    # -- scene dict (:369-399) ------------------------------------------------
    def to_dict(self):
        cm = self.model
        ng = int(cm.ngeom_all) if hasattr(cm, "ngeom_all") else len(cm.geom_bodyid)
        gravcomp = np.zeros(self.nbody)
        gravcomp[cm.body_names.index("body:camera")] = 1.0
        contype = np.ones(ng, np.int32)
        for o in self.removed:
            gravcomp[cm.body_names.index(o)] = 1.0
        state = {"geom_conaffinity": contype.copy(), "geom_contype": contype, "geom_rgba": np.ones((ng, 4)),
                 "body_gravcomp": gravcomp, "state": self.get_state(),
                 "removed_objects": sorted(self.removed)}
        return {"gripper": deepcopy(self.gripper), "objects": deepcopy(self.objects), "env_state": state}

    @classmethod
    def from_dict(cls, state_dict, **kw):
        gripper, obj_list, state = state_dict["gripper"], state_dict["objects"], state_dict["env_state"]
        env = cls(gripper, obj_list, scene_randomization=False, **kw)
        env.set_state(state["state"])
        removed = set(state.get("removed_objects", []))
        if not removed and "body_gravcomp" in state:
            probe = env.model
            for o in obj_list:
                b = probe.body_names.index(o.name)
                if b < len(state["body_gravcomp"]) and state["body_gravcomp"][b] > 0:
                    removed.add(o.name)
        env.removed = removed
        env._model_key = None
        return env

    # -- host bookkeeping ------------------------------------------------------
    def _initial_qpos(self, poses: SE3Pose, joints: np.ndarray, state):
        """per candidate: mj_setState(state) -> set_qpos(joints) -> set_pose(pose @ b2c)
        in the compiled model's layout; returns (qpos, mocap_pos, mocap_quat)."""
        cm = self.model_for(state)
        parts = self.split_state(state)
        n = len(poses)
        q0 = self._reduce(parts["qpos"], "q")
        qpos = np.tile(q0, (n, 1))
        idxs = [cm.jnt_qposadr_by_name(j) for j in self.gripper.get_actuator_joint_names()]
        jj = np.asarray(joints, dtype=np.float64)
        for k, a in enumerate(idxs):          # sequential: duplicate indices -> last wins
            qpos[:, a] = jj[:, k]
        proc = poses @ self.gripper.base_to_contact_transform()
        vec = proc.to_vec(layout="pq", type="wxyz")
        fj = cm.jnt_qposadr_by_name("freejoint")
        qpos[:, fj:fj + 3] = vec[:, :3]
        qpos[:, fj + 3:fj + 7] = vec[:, 3:]
        return qpos, vec[:, :3].astype(np.float64), vec[:, 3:].astype(np.float64)

    def _check_inputs(self, poses, joints):
        if len(poses) != len(joints):
            raise ValueError(f"Number of poses ({len(poses)}) must match number of joint configurations "
                             f"({len(joints)}).")

    # -- hot path --------------------------------------------------------------
    def grasp_collision_mask(self, poses: SE3Pose, joints: np.ndarray) -> np.ndarray:
        """clutter_table.py:330-367: out-of-bounds poses are rejected, the rest are
        collision-free unless a gripper geom touches the table or anything past it."""
        self._check_inputs(poses, joints)
        n = len(poses)
        if n == 0:
            return np.zeros(0, dtype=bool)
        inb = self.in_bounds(poses)
        out = np.zeros(n, dtype=bool)
        idx = np.nonzero(inb)[0]
        if len(idx):
            q, mp, mq = self._initial_qpos(poses[idx], joints[idx], self._state)
            out[idx] = self.engine_for_state(self._state).collision_free(q, mp, mq, predicate="partition_incl")
        return out

    @staticmethod
    def in_bounds(poses: SE3Pose) -> np.ndarray:
        """the reference's workspace box of the collision mask (:344-354)"""
        p = poses.pos
        return (p[..., 0] < 0.25) & (p[..., 0] > -0.25) & (p[..., 1] < 0.25) & (p[..., 1] > -0.25) & \
            (p[..., 2] < 1.0) & (p[..., 2] > 0.0)

    def stable_plan(self, poses: SE3Pose, joints: np.ndarray, env_state, nstep_lift=3000, lift_dist=0.3,
                    close_steps=None) -> RolloutPlan:
        q, mp, mq = self._initial_qpos(poses, joints, env_state)
        close_steps = self.gripper.close_steps if close_steps is None else close_steps
        start_lift = mp.copy()
        target_lift = mp.copy()
        target_lift[:, 2] = start_lift[:, 2] + lift_dist
        ctrl = np.asarray(self.gripper.close_ctrl(self), dtype=np.float64)
        return RolloutPlan(nsteps=[close_steps, nstep_lift], check_every=[0, 100], check_at_end=[0, 0],
                           ctrl=[ctrl, ctrl], qpos_init=q, mocap_quat=mq,
                           phase_start=np.ascontiguousarray(np.stack([mp, start_lift], 1)),
                           phase_target=np.ascontiguousarray(np.stack([mp, target_lift], 1)),
                           obj_qposadr=-1, check_offset=[0, 1])

    # in-launch rotation and explicit relaunch slices, as GravitylessObjectGrasping
    YIELD_EVERY = 32
    SLICES = 1

    def rollout(self, plan: RolloutPlan, env_state, max_ncon: int = 128, slices: Optional[int] = None,
                yield_every: Optional[int] = None, on_capacity: str = "raise"):
        """engine rollout with contact-capacity escalation (continued from the
        overflowing step), in-launch rotation and optional time slices by
        relaunch, as GravitylessObjectGrasping.rollout (sliced_rollout; a
        candidate still over max_ncon raises CapacityError unless
        on_capacity="capped")."""
        return sliced_rollout(plan, self.engine_for_state(env_state),
                              lambda c: self.engine_for_state(env_state, ncon_max=c), self.ncon_max, max_ncon,
                              self.SLICES if slices is None else slices,
                              yield_every=self.YIELD_EVERY if yield_every is None else yield_every,
                              on_capacity=on_capacity)

    def grasp_stable_mask(self, poses: SE3Pose, joints: np.ndarray, env_state, nstep_lift: int = 3000,
                          lift_dist: float = 0.3, enough_stable=None, *, close_steps: Optional[int] = None,
                          return_details: bool = False):
        """clutter_table.py:272-321."""
        self._check_inputs(poses, joints)
        if len(poses) == 0:
            return np.zeros(0, dtype=bool)
        plan = self.stable_plan(poses, joints, env_state, nstep_lift, lift_dist, close_steps)
        res = self.rollout(plan, env_state)
        labels = apply_enough_stable(res["label"].astype(bool), enough_stable)
        if return_details:
            res["label"] = labels
            return res
        return labels

    # -- scene generation (:155-222), many scenes at once -----------------------
    def _expand(self, ref_vec, reduced, which):
        """compiled-model qpos / qvel -> the reference layout (the camera and removed
        objects keep their ref_vec entries)."""
        out = np.array(ref_vec, dtype=np.float64).copy()
        h = self._gripper_nq if which == "q" else self._gripper_nv
        out[:h] = reduced[:h]
        o = h
        for name, qs, vs in self._obj_slices():
            if name in self.removed:
                continue
            sl = qs if which == "q" else vs
            w = sl.stop - sl.start
            out[sl] = reduced[o:o + w]
            o += w
        return out

    def free_plan(self, states, nsteps: int):
        """RolloutPlan of a free simulation of integration states (rows of
        `states`): ctrl and mocap held at the first state's, plus the per-state
        initial (qvel | qacc_warmstart | act) in the compiled model's layout."""
        parts = [self.split_state(s) for s in states]
        q = np.stack([self._reduce(p["qpos"], "q") for p in parts])
        vs = np.stack([np.concatenate([self._reduce(p["qvel"], "v"), self._reduce(p["qacc_warmstart"], "v"),
                                       p["act"]]) for p in parts])
        mp = np.ascontiguousarray(np.stack([p["mocap_pos"] for p in parts])[:, None, :])
        mq = np.ascontiguousarray(np.stack([p["mocap_quat"] for p in parts]))
        plan = RolloutPlan(nsteps=[int(nsteps)], check_every=[0], check_at_end=[0],
                           ctrl=[np.array(parts[0]["ctrl"], np.float64)], qpos_init=q, mocap_quat=mq,
                           phase_start=mp, phase_target=mp.copy(), obj_qposadr=-1)
        return plan, vs

    def apply_free(self, states, res, nsteps: int):
        """write a free simulation's final (qpos, qvel, qacc_warmstart) back into
        the states; time advances by nsteps timesteps, added one at a time as
        mj_step does."""
        out = np.array(states, dtype=np.float64, copy=True)
        dt = float(self.model_for(out[0]).options["timestep"])
        t = out[:, 0].copy()
        for _ in range(int(nsteps)):
            t += dt
        for i in range(len(out)):
            p = dict(self.split_state(out[i]))
            p = dict(p, time=t[i:i + 1], qpos=self._expand(p["qpos"], res["qpos"][i], "q"),
                     qvel=self._expand(p["qvel"], res["qvel"][i], "v"),
                     qacc_warmstart=self._expand(p["qacc_warmstart"], res["qacc_warmstart"][i], "v"),
                     act=res["act"][i] if "act" in res else p["act"])
            out[i] = self.join_state(p)
        return out

    def simulate_states(self, states, nsteps: int, vclip: float = 0.0, max_ncon: int = 128,
                        ncon_max: Optional[int] = None):
        """advance integration states by `nsteps` mj_step each, all at once on the
        GPU (mgs_simulate; one wave per state).  vclip > 0 clips every qvel entry
        to +-vclip after each step.  States that exceed the contact capacity are
        re-run at twice the capacity (as GravitylessObjectGrasping.rollout);
        `last_overflow` counts those still over at max_ncon.  ncon_max (default
        the env's) sets the starting capacity: a smaller one with auto-sized rows
        (engine.auto_capacity) keeps more piles in flight per CU."""
        states = np.atleast_2d(np.asarray(states, dtype=np.float64))
        if len(states) == 0 or nsteps <= 0:
            return states.copy()
        plan, vs = self.free_plan(states, nsteps)
        cap = self.ncon_max if ncon_max is None else int(ncon_max)
        res = self._sim_engine(states[0], cap).simulate(plan, vstate=vs, vclip=vclip)
        ov = np.nonzero(res["stats"][:, 2] & FLAG_CAPACITY)[0]
        while len(ov) and cap < max_ncon:
            cap = min(2 * cap, max_ncon)
            sub = self.engine_for_state(states[0], ncon_max=cap).simulate(plan.subset(ov), vstate=vs[ov],
                                                                          vclip=vclip)
            for k in res:
                res[k][ov] = sub[k]
            ov = ov[np.nonzero(sub["stats"][:, 2] & FLAG_CAPACITY)[0]]
        self.last_overflow = len(ov)
        # states whose run is not MuJoCo's: contacts / rows still truncated at
        # max_ncon, or a diverged state (MGS_FLAG_DIVERGED); callers treat them as
        # unstable rather than keep a truncated pile
        self.last_bad = res["stats"][:, 2] != 0
        return self.apply_free(states, res, nsteps)

    def _sim_engine(self, state, ncon_max):
        """engine for a free simulation starting at capacity ncon_max: the env's own
        capacity uses engine_for_state; a smaller one gets auto-sized rows."""
        if ncon_max == self.ncon_max or self._nefc_max is not None:
            return self.engine_for_state(state, ncon_max=ncon_max)
        from mgs.core.engine import Engine, auto_capacity
        cm = self.model_for(state)
        key = ("sim", ncon_max)
        if key not in self._engines:
            self._engines[key] = Engine(cm, device=self.device, ncon_max=ncon_max,
                                        nefc_max=auto_capacity(cm, ncon_max)[1])
        return self._engines[key]

    def gen_clutter_states(self, n_scenes: int, rng=None, steps_each: int = 900, steps_final: int = 9000,
                           vclip: float = 50.0, ncon_max: Optional[int] = None):
        """gen_clutter (:197-222) for n_scenes piles at once: one random drop pose
        per scene at (0, 0, 0.8) (scipy Rotation.random), shared by its objects;
        each object in turn is placed there with every qvel zeroed and
        `steps_each` steps run, then `steps_final` steps settle the pile; qvel is
        clipped to +-vclip after every step (the reference clips before the next
        step: the same trajectory, except that the final qvel is clipped too).
        Returns the (n_scenes, state_size) integration states."""
        from scipy.spatial.transform import Rotation
        rng = np.random.default_rng(rng)
        xyzw = Rotation.random(int(n_scenes), random_state=rng).as_quat().reshape(-1, 4)
        drop = np.concatenate([np.tile([0.0, 0.0, 0.8], (len(xyzw), 1)), xyzw[:, [3, 0, 1, 2]]], axis=1)
        states = np.tile(self._state, (len(xyzw), 1))
        q0, v0 = 1, 1 + self.ref_nq
        bad = np.zeros(len(states), bool)
        self.last_bad = None
        for _, qs, _ in self._obj_slices():
            states[:, q0 + qs.start:q0 + qs.stop] = drop
            states[:, v0:v0 + self.ref_nv] = 0.0
            states = self.simulate_states(states, steps_each, vclip, ncon_max=ncon_max)
            bad |= self._last_bad(len(states))
        states = self.simulate_states(states, steps_final, vclip, ncon_max=ncon_max)
        self.last_bad_scenes = bad | self._last_bad(len(states))
        return states

    def _last_bad(self, n):
        """the bad-state mask of the last simulate_states call, consumed (zeros
        if the call left none, e.g. a substituted simulator)"""
        b = getattr(self, "last_bad", None)
        self.last_bad = None
        return np.zeros(n, bool) if b is None or len(b) != n else np.asarray(b, bool)

    def gen_clutter(self, rng=None, **kw):
        """clutter_table.py:197-222 on this env's state."""
        self._state = self.gen_clutter_states(1, rng, **kw)[0]

    def settle(self):
        """clutter_table.py:157-158: 10000 free steps."""
        self._state = self.simulate_states(self._state, 10000)[0]

    def is_stable_states(self, states, rounds: int = 10, steps: int = 100, tol: float = 5e-3):
        """is_stable (:160-195) for many states: `rounds` x `steps` free steps, per
        object the summed |position change| of every chunk; a state is stable if
        the largest sum is < tol.  Returns (stable, largest sum, advanced states)."""
        states = np.atleast_2d(np.asarray(states, dtype=np.float64))
        delta = np.zeros((len(states), len(self.object_names)))
        bad = np.zeros(len(states), bool)
        self.last_bad = None
        for _ in range(rounds):
            new = self.simulate_states(states, steps)
            bad |= self._last_bad(len(states))
            for k, (_, qs, _) in enumerate(self._obj_slices()):
                a = 1 + qs.start
                delta[:, k] += np.sum(np.abs(new[:, a:a + 3] - states[:, a:a + 3]), axis=1)
            states = new
        mx = np.max(delta, axis=1, initial=0.0)
        # a truncated (capacity) or diverged run is not a stable pile
        return (mx < tol) & ~bad, mx, states

    def is_stable(self) -> bool:
        """clutter_table.py:160-195 (advances this env's state like the reference)."""
        ok, _, st = self.is_stable_states(self._state)
        self._state = st[0]
        return bool(ok[0])
