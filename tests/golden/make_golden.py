#!/usr/bin/env python3
"""Generate golden vectors by importing the REFERENCE's own numpy code (build container only).

The reference package cannot be imported as a package here (gym_so100/__init__.py:1 imports
gymnasium; env.py:1-6 imports gymnasium/dm_control/gym, all absent).  Its numpy-only modules are
loaded by file path, with minimal stubs standing in for the absent third-party *imports* only
(dm_control.suite.base.Task's before_step -> physics.set_control, gymnasium.Env/spaces
constructors).  Every value below is computed by reference code:

  unnormalize_so100 / SO100Task.before_step  gym_so100/constants.py:44-47,78-86; tasks/single_arm.py:33-38
  sample_so100_box_pose                      gym_so100/utils.py:18-29
  get_reward (3 tasks)                       gym_so100/tasks/single_arm.py:149-215,246-285,322-380
  get_observation + _format_raw_obs          tasks/single_arm.py:82-114; env.py:130-146
  SO100Env.step terminated/is_success        gym_so100/env.py:172-182
  SO100GoalEnv.compute_reward/_is_success    gym_so100/env.py:341-358

Outputs small .npz fixtures (no pickle) next to this script.  The GPU box never runs this.
"""
import importlib.util
import json
import os
import sys
import types

import numpy as np

REF = os.environ.get("SO100_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
MODEL = os.path.join(HERE, "..", "..", "gym-so100-c_amd", "gym_so100", "assets", "so100_model.json")


def _stub_modules():
    class Task:  # dm_control.suite.base.Task: before_step forwards to physics.set_control
        def __init__(self, random=None):
            self._random = random

        def before_step(self, action, physics):
            physics.set_control(action)

        def initialize_episode(self, physics):
            pass

    class Env:  # gymnasium.Env surface used by env.py
        def __init__(self, *a, **k):
            pass

        def reset(self, seed=None, options=None):
            pass

    class Box:
        def __init__(self, low=None, high=None, shape=None, dtype=None):
            self.low, self.high, self.shape, self.dtype = low, high, shape, dtype

    class Dict(dict):
        pass

    mods = {}
    for name in ["dm_control", "dm_control.suite", "dm_control.suite.base", "dm_control.mujoco",
                 "dm_control.rl", "dm_control.rl.control", "gymnasium", "gymnasium.spaces", "gym",
                 "gymnasium.envs", "gymnasium.envs.registration"]:
        mods[name] = types.ModuleType(name)
    mods["dm_control.suite.base"].Task = Task
    mods["dm_control"].mujoco = mods["dm_control.mujoco"]
    mods["dm_control.rl"].control = mods["dm_control.rl.control"]
    mods["gymnasium"].Env = Env
    mods["gymnasium"].spaces = mods["gymnasium.spaces"]
    mods["gymnasium.spaces"].Box = Box
    mods["gymnasium.spaces"].Dict = Dict
    mods["gymnasium.envs.registration"].register = lambda **k: None
    sys.modules.update(mods)


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    m = importlib.util.module_from_spec(spec)
    sys.modules[name] = m
    spec.loader.exec_module(m)
    return m


def load_reference():
    _stub_modules()
    pkg = types.ModuleType("gym_so100")
    pkg.__path__ = [os.path.join(REF, "gym_so100")]
    sys.modules["gym_so100"] = pkg
    tasks = types.ModuleType("gym_so100.tasks")
    tasks.__path__ = [os.path.join(REF, "gym_so100", "tasks")]
    sys.modules["gym_so100.tasks"] = tasks
    c = _load("gym_so100.constants", os.path.join(REF, "gym_so100", "constants.py"))
    u = _load("gym_so100.utils", os.path.join(REF, "gym_so100", "utils.py"))
    t = _load("gym_so100.tasks.single_arm", os.path.join(REF, "gym_so100", "tasks", "single_arm.py"))
    e = _load("gym_so100.env", os.path.join(REF, "gym_so100", "env.py"))
    return c, u, t, e


class FakePhysics:
    """Exposes exactly the mjData/mjModel surface the reference task code reads."""
    SITES = ["cube_site", "ee_site", "bin_center"]

    def __init__(self, geom_names, cube, ee, bin_center, contacts, qpos=None, qvel=None):
        self._geom_names = geom_names
        phys = self

        class _Site:
            def __init__(self, i):
                self.id = i

        class _Model:
            def site(self, name):
                return _Site(FakePhysics.SITES.index(name))

            def id2name(self, i, kind):
                assert kind == "geom"
                return phys._geom_names[i]

        class _Con:
            def __init__(self, g1, g2):
                self.geom1, self.geom2 = g1, g2

        class _Data:
            pass

        self.model = _Model()
        self.data = _Data()
        self.data.site_xpos = np.array([cube, ee, bin_center], dtype=np.float64)
        self.data.ncon = len(contacts)
        self.data.contact = [_Con(a, b) for a, b in contacts]
        self.data.qpos = np.zeros(13) if qpos is None else np.asarray(qpos, dtype=np.float64)
        self.data.qvel = np.zeros(12) if qvel is None else np.asarray(qvel, dtype=np.float64)
        self.ctrl = None

    def set_control(self, a):
        self.ctrl = np.array(a, copy=True)

    def render(self, height, width, camera_id):
        return np.zeros((height, width, 3), np.uint8)


def main():
    c, u, t, e = load_reference()
    model = json.load(open(MODEL))
    geom_names = [g["name"] for g in model["geoms"]]
    pairs = [(p["g1"], p["g2"]) for p in model["pairs"]]
    # bin_center exactly as MuJoCo forms site_xpos: body pos + site pos (so100_transfer_cube.xml:16,23)
    bin_center = np.array([-0.2, 0.7, 0.001]) + np.array([0.0, 0.0, 0.02])
    rng = np.random.default_rng(20251015)
    out = {}

    # ---------------- 1. action un-normalisation with float32 write-back ----------------
    grid = np.linspace(-1.0, 1.0, 41)
    acts = [np.full(6, v) for v in grid]
    acts += [np.full(6, v) for v in (-2.0, -1.0000001, 1.0000001, 2.0, 1e-8, -1e-8)]
    acts += list(rng.uniform(-1.2, 1.2, size=(200, 6)))
    acts = np.asarray(acts, dtype=np.float32)
    ctrl = []
    task = t.SO100CubeToBinTask(observation_width=4, observation_height=3)
    for a in acts:
        ph = FakePhysics(geom_names, np.zeros(3), np.zeros(3), bin_center, [])
        task.before_step(a, ph)
        ctrl.append(ph.ctrl)
    out["unnorm_action"] = acts
    out["unnorm_ctrl"] = np.asarray(ctrl)
    assert out["unnorm_ctrl"].dtype == np.float32

    # ---------------- 2. cube spawn per seed (numpy legacy MT19937) ----------------
    seeds = np.concatenate([np.arange(0, 1024), np.arange(1000, 1000 + 64), [4095, 65535, 1000 + 65535,
                            123456789, 2**31 - 1, 2**32 - 1]]).astype(np.uint64)
    out["spawn_seed"] = seeds
    out["spawn_pose"] = np.asarray([u.sample_so100_box_pose(int(s)) for s in seeds])

    # ---------------- 3. reward ladders for the three tasks ----------------
    bmin = bin_center + np.array([-0.06, -0.06, 0.0])
    bmax = bin_center + np.array([0.06, 0.06, 0.03])
    cubes = []
    # random f32 positions around and inside the bin, and on the table
    cubes += list(rng.uniform([-0.30, 0.60, 0.0], [-0.10, 0.80, 0.09], size=(300, 3)))
    cubes += list(rng.uniform([-0.25, 0.30, 0.0], [-0.15, 0.60, 0.06], size=(60, 3)))
    # exact boundary probes of the strict inequalities (single_arm.py:80,184-186,356-358)
    for axis in range(3):
        for bound, off in ((bmin, +0.01), (bmax, -0.01), (bmin, 0.0), (bmax, 0.0)):
            x0 = np.float32(bound[axis] + off)
            for k in range(-3, 4):
                x = x0
                for _ in range(abs(k)):
                    x = np.nextafter(x, np.float32(np.inf if k > 0 else -np.inf), dtype=np.float32)
                p = np.array([-0.2, 0.7, 0.035], dtype=np.float32)
                p[axis] = x
                cubes.append(p)
    cubes = np.asarray(cubes, dtype=np.float32).astype(np.float64)
    dists = np.array([0.0, 0.01, 0.03, 0.049, 0.0505, 0.07, 0.099, 0.101, 0.2, 0.299, 0.301, 0.45, 0.499,
                      0.501, 0.6, 0.699, 0.701, 0.9])
    contact_sets = [
        [], [0], [4], [0, 4], [3, 7], [8], [0, 8], [5, 8], [13], [0, 13], [9], [2, 9, 13], [1, 6, 8, 13],
        [10, 11], [7, 12], [8, 13],
    ]
    rc, re, rb, rr = [], [], [], []
    for i, cube in enumerate(cubes):
        d = dists[i % len(dists)]
        v = rng.normal(size=3)
        v /= np.linalg.norm(v)
        ee = np.asarray(cube + d * v, dtype=np.float32).astype(np.float64)
        cs = contact_sets[(i * 7) % len(contact_sets)]
        bits = 0
        for p in cs:
            bits |= 1 << p
        contacts = [pairs[p] for p in cs]
        row = []
        for cls in (t.SO100CubeToBinTask, t.SO100TouchCubeTask, t.SO100TouchCubeSparseTask):
            tk = cls(observation_width=4, observation_height=3)
            ph = FakePhysics(geom_names, cube, ee, bin_center, contacts)
            row.append(float(tk.get_reward(ph)))
        rc.append(cube); re.append(ee); rb.append(bits); rr.append(row)
    out["reward_cube"] = np.asarray(rc)
    out["reward_ee"] = np.asarray(re)
    out["reward_bits"] = np.asarray(rb, dtype=np.uint32)
    out["reward_value"] = np.asarray(rr)     # columns: cube_to_bin, touch_cube, touch_cube_sparse

    # ---------------- 4. observation packing (so100_state) + step() termination ----------------
    obs_in, obs_out, term = [], [], []
    for i in range(32):
        qpos = rng.uniform(-2, 2, size=13)
        cube = rng.uniform(-0.3, 0.1, size=3)
        ee = rng.uniform(-0.3, 0.1, size=3)
        ph = FakePhysics(geom_names, cube, ee, bin_center, [], qpos=qpos)
        raw = task.get_observation(ph)
        fake = types.SimpleNamespace(obs_type="so100_state")
        obs = e.SO100Env._format_raw_obs(fake, raw)
        obs_in.append(np.concatenate([qpos, cube, ee]))
        obs_out.append(obs)
    for r in (0.0, 1.0, 2.0, 2.5, 3.0, 4.0, 3.9999999):
        fake_env = types.SimpleNamespace(step=lambda a, r=r: (None, r, None, {}))
        fake = types.SimpleNamespace(_env=fake_env, _format_raw_obs=lambda raw: raw)
        _, rew, terminated, truncated, info = e.SO100Env.step(fake, np.zeros(6, np.float32))
        term.append([r, float(terminated), float(truncated), float(info["is_success"])])
    out["obs_in"] = np.asarray(obs_in)
    out["obs_out"] = np.asarray(obs_out)
    out["step_term"] = np.asarray(term)

    # ---------------- 5. GoalEnv sparse reward ----------------
    ach = rng.uniform(-0.3, 0.8, size=(64, 3)).astype(np.float32)
    des = ach + (rng.normal(size=(64, 3)) * rng.choice([0.001, 0.004, 0.02], size=(64, 1))).astype(np.float32)
    fake = types.SimpleNamespace(distance_threshold=0.01)
    out["goal_achieved"] = ach
    out["goal_desired"] = des
    out["goal_reward_batch"] = e.SO100GoalEnv.compute_reward(fake, ach, des, {})
    out["goal_reward_single"] = np.asarray([e.SO100GoalEnv.compute_reward(fake, a, d, {}) for a, d in zip(ach, des)])
    out["goal_success"] = np.asarray([bool(e.SO100GoalEnv._is_success(fake, a, d)) for a, d in zip(ach, des)])

    path = os.path.join(HERE, "golden_task.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
