"""Host logic of the envs' rollout driver (mgs.env.gravityless_object_grasping.
sliced_rollout: capacity escalation from resume records, time slices by
relaunch, the rotation setting) against a fake engine with the C-ABI's
semantics (mgs_schedule.pause_step / capped_continue / yield_every, resume
records, MGS_FLAG_CAPACITY / MGS_FLAG_PAUSED, fail_step -3 / -4).  CPU only:
the kernels' side of the same contract is GPU-tested bit for bit
(tests/test_gpu_parity.py: time slices, rotation, escalation)."""
import numpy as np
import pytest

from mgs.core.abi import MGS
from mgs.env.gravityless_object_grasping import RolloutPlan, sliced_rollout

CAP, PAUSED, NS = MGS["MGS_FLAG_CAPACITY"], MGS["MGS_FLAG_PAUSED"], MGS["MGS_NSTATS"]
H = 60


class FakeEngine:
    """candidate i needs need[i, t] contacts at step t and fails at fail_at[i]
    (-1: never); a record is [step, sumcon]; calls are logged"""

    def __init__(self, need, fail_at, cap, log):
        self.need, self.fail_at, self.cap, self.log = need, fail_at, cap, log

    def rollout(self, plan, resumable=False, resume_from=None, pause_step=0, capped_continue=False, yield_every=0):
        ids = plan.qpos_init[:, 0].astype(int)
        self.log.append(dict(cap=self.cap, n=len(ids), pause=pause_step, yield_every=yield_every,
                             resumed=resume_from is not None))
        n = len(ids)
        out = dict(label=np.zeros(n, bool), fail_step=np.zeros(n, np.int32), obj_qpos=np.zeros((n, 7)),
                   stats=np.zeros((n, NS), np.int32), resume=np.zeros((n, 4)))
        for k, i in enumerate(ids):
            t0, sc = (int(resume_from[k, 0]), int(resume_from[k, 1])) if resume_from is not None else (0, 0)
            # a paused record keeps its flags (without the pause); an
            # escalation's record starts afresh (the C-ABI's resume semantics)
            rf = int(resume_from[k, 2]) if resume_from is not None else 0
            flags, label, fs = (rf & ~PAUSED) if rf & PAUSED else 0, True, -1
            t = t0
            while t < H:
                if pause_step > 0 and t >= pause_step:
                    flags |= PAUSED
                    out["resume"][k] = (t, sc, flags, 0)
                    label, fs = False, -4
                    break
                if self.need[i, t] > self.cap:
                    flags |= CAP
                    if not capped_continue:
                        out["resume"][k] = (t, sc, flags, 0)
                        label, fs = False, -3
                        break
                sc += int(min(self.need[i, t], self.cap))
                if t == self.fail_at[i]:
                    label, fs = False, t
                    break
                t += 1
            out["label"][k] = label
            out["fail_step"][k] = fs
            out["obj_qpos"][k] = i + np.arange(7)
            out["stats"][k, 2] = flags
            out["stats"][k, 4] = sc
        return out


def _case(seed, n=40):
    rng = np.random.default_rng(seed)
    need = rng.integers(0, 10, (n, H))
    need[rng.random((n, H)) < 0.03] = rng.integers(10, 50)      # rare spikes past the main capacity
    fail_at = np.where(rng.random(n) < 0.4, rng.integers(0, H, n), -1)
    q = np.zeros((n, 3))
    q[:, 0] = np.arange(n)
    z = np.zeros((n, 5, 3))
    plan = RolloutPlan(nsteps=[H], check_every=[0], check_at_end=[1], ctrl=[np.zeros(1)], qpos_init=q,
                       mocap_quat=np.zeros((n, 4)), phase_start=z, phase_target=z, obj_qposadr=0)
    return need, fail_at, plan


@pytest.mark.parametrize("seed", [0, 1, 2])
@pytest.mark.parametrize("slices", [1, 2, 3, 7])
def test_sliced_rollout_equals_one_uncapped_run(seed, slices):
    need, fail_at, plan = _case(seed)
    log = []
    ref = FakeEngine(need, fail_at, 10 ** 6, []).rollout(plan)
    engines = {}

    def engine_for(c):
        return engines.setdefault(c, FakeEngine(need, fail_at, c, log))
    res = sliced_rollout(plan, engine_for(10), engine_for, 10, 80, slices, yield_every=32)
    assert res["overflow"] == 0
    for k in ("label", "fail_step", "obj_qpos"):
        assert np.array_equal(res[k], ref[k]), k
    assert np.array_equal(res["stats"][:, 4], ref["stats"][:, 4])
    assert not (res["stats"][:, 2] & (CAP | PAUSED)).any()
    # every launch carried the rotation setting; the escalation grew the capacity
    assert all(c["yield_every"] == 32 for c in log)
    assert any(c["cap"] > 10 for c in log)
    main = [c for c in log if c["cap"] == 10]
    assert 1 <= len(main) <= slices and all(c["resumed"] for c in main[1:])


def test_escalation_past_max_ncon_raises():
    """a candidate still over the largest capacity fails the
    call (CapacityError naming it) instead of returning a label from a capped
    contact set; the last stage stops it (no capped_continue)"""
    from mgs.env.gravityless_object_grasping import CapacityError
    need, fail_at, plan = _case(3)
    need[5, 20] = 500
    fail_at[5] = -1
    engines = {}
    log = []

    def engine_for(c):
        return engines.setdefault(c, FakeEngine(need, fail_at, c, log))
    with pytest.raises(CapacityError) as ei:
        sliced_rollout(plan, engine_for(10), engine_for, 10, 40, 1)
    assert 5 in ei.value.candidates.tolist()
    assert max(c["cap"] for c in log) == 40
    # every candidate the escalation could hold is below 40: raising the cap resolves it
    res = sliced_rollout(plan, engine_for(10), engine_for, 10, 640, 1)
    assert res["overflow"] == 0 and not res["stats"][5, 2] & CAP


def test_escalation_stops_at_max_ncon_when_capped_is_accepted():
    """on_capacity="capped" (opt-in): the candidate runs on capped and flagged
    (capped_continue on the last stage), counted in res['overflow']"""
    need, fail_at, plan = _case(3)
    need[5, 20] = 500
    fail_at[5] = -1
    engines = {}
    log = []

    def engine_for(c):
        return engines.setdefault(c, FakeEngine(need, fail_at, c, log))
    res = sliced_rollout(plan, engine_for(10), engine_for, 10, 40, 1, on_capacity="capped")
    assert res["overflow"] >= 1 and res["stats"][5, 2] & CAP
    assert res["label"][5] and res["fail_step"][5] == -1
    assert max(c["cap"] for c in log) == 40


@pytest.mark.parametrize("slices", [2, 3, 7])
def test_capped_slices_keep_capacity_flags(slices):
    """the last escalation stage from the first launch (cap >=
    max_ncon, capped_continue) with slices: a capped candidate that pauses keeps
    FLAG_CAPACITY through the relaunch, so res['overflow'] equals one launch's"""
    need, fail_at, plan = _case(4)
    one = sliced_rollout(plan, FakeEngine(need, fail_at, 10, []), None, 10, 10, 1, on_capacity="capped")
    assert one["overflow"] > 0
    res = sliced_rollout(plan, FakeEngine(need, fail_at, 10, []), None, 10, 10, slices, on_capacity="capped")
    assert res["overflow"] == one["overflow"]
    for k in ("label", "fail_step", "obj_qpos", "stats"):
        assert np.array_equal(res[k], one[k]), k
