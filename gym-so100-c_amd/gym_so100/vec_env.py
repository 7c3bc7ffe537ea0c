"""Batched SO-ARM100 envs on one MI355X: torch-ROCm tensors in, torch-ROCm tensors out.

``SO100VecEnv`` is the batched form of the reference's ``SO100Env`` (gym_so100/env.py:26-185) and
``SO100GoalEnv`` (env.py:188-409): N independent envs stepped by one HIP launch per env step
(csrc/so100_step.hip).  Semantics kept from the reference:

* actions [N,6] in [-1,1], un-normalised per joint with float32 write-back (single_arm.py:33-38);
* 10 physics substeps per env step (control_timestep 0.02 / timestep 0.002, env.py:120-127);
* reward ladders of the three tasks (single_arm.py), ``terminated = is_success = reward == 4``
  (env.py:175), TimeLimit truncation at 700 / 300 steps (gym_so100/__init__.py:7,17,27);
* so100_state observation = [box, bin, ee, qpos[:6]] float32 (env.py:137-145);
* so100_pixels_agent_pos observation = {"pixels": top camera uint8 [N,H,W,3], "agent_pos": qpos[:6]}
  (env.py:130-136), rendered on the device by render.CameraRenderer (csrc/so100_render.hip);
* GoalEnv: sparse reward 0/-1 at 0.01 m, terminated = success, own 300-step truncation, lifted-goal
  curriculum for the first 5000 steps (env.py:322-353, 372-406);
* reset(seed=s) reproduces ``RandomState(s)`` cube spawns bit-for-bit (utils.py:18-29).

Auto-reset follows the SB3/gymnasium-vector convention: when an env finishes, ``obs`` already holds
the first observation of the next episode and ``info["final_observation"]`` the last one of the
finished episode (mask in ``info["_final_observation"]``).

With pixel observations an env that finishes is stepped, its terminal image drawn into
``final_pixels``, then reset by the masked reset kernel (the same spawn and episode counter as the
in-kernel auto-reset) and drawn again: ``info["final_observation"]`` is then {"pixels", "agent_pos"}.

Output tensors are persistent device buffers overwritten by the next ``step``/``reset``; clone them if
you keep them across calls.
"""
import ctypes

import numpy as np

from . import _native
from .model import NOBS, NQ, NV, build_model
from .constants import GOAL_MAX_EPISODE_STEPS

_MAX_STEPS = {"so100_cube_to_bin": 700, "so100_touch_cube": 300, "so100_touch_cube_sparse": 300,
              "so100_goal": GOAL_MAX_EPISODE_STEPS}


def _torch():
    import torch
    return torch


def _splitmix64(x):
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def _hash_uniform(seed, ids, field):
    """U[0,1) per global env id from a counter-based hash (splitmix64), independent of sharding."""
    with np.errstate(over="ignore"):
        key = _splitmix64(np.uint64(seed & 0xFFFFFFFFFFFFFFFF) ^ (ids * np.uint64(0x100000001B3)) ^
                          np.uint64(field * 0xD1B54A32D192ED03 & 0xFFFFFFFFFFFFFFFF))
    return (key >> np.uint64(40)).astype(np.float64) / float(1 << 24)


class SO100VecEnv:
    """N parallel SO-ARM100 envs on one GPU.

    Args:
        num_envs: number of envs on this device.
        task: "so100_cube_to_bin" | "so100_touch_cube" | "so100_touch_cube_sparse" | "so100_goal".
        obs_type: "so100_state" (15 floats) or "so100_pixels_agent_pos" (the reference's registered
            default: top-camera image + joint positions; GoalEnv: the flattened form of env.py:267-270).
        observation_width, observation_height: image size for pixel observations (env.py:34-35).
        variant: "joint" (so100_transfer_cube.xml, the registered envs) or "ee" (so100_transfer_cube_ee.xml:
            a weld equality pulls ee_site to each env's mocap pose ``self.mocap`` [N,7], set with
            ``set_mocap``; teleop_ee.py drives the same inputs).
        device: torch device string ("cuda:0").
        seed: base seed for in-kernel (auto-)reset spawns.
        max_episode_steps: TimeLimit; default per task as registered by the reference.
        autoreset: reset finished envs inside the step kernel.
        domain_randomization: None or dict(mass=(lo,hi), friction=(lo,hi), action_noise=sigma):
            per-env cube mass / friction scales (fixed per env) + Gaussian action noise.
        env_offset: global index of this shard's first env (multi-GPU sharding); in-kernel seeds use
            the global env id so trajectories do not depend on the number of GPUs.
        iterations: solver iterations per substep, PGS sweeps or Newton steps (default: the model's 100,
            MuJoCo's default).
        solver: "newton" (default: MuJoCo's default solver, which the reference's model runs; the
            unique minimiser of the constraint problem) or "pgs" (north_star's projected Gauss-Seidel).
        debug: allocate the [N, 160] diagnostics buffer (contacts, forces, solver iterations; layout:
            include/so100.h SO100_DBG_STRIDE).  While it is passed (``debug_enabled``, default True) the
            fused step launches its debug build; set ``debug_enabled = False`` to run the product build.
        reward64: also keep the reward in float64 (``self.reward64``), as the reference returns it; the
            float32 ``reward`` rounds the dense TouchCube shaping (the other ladders are exact in float32).
        convex: the collider of the mesh pairs (the cube, bin boxes and finger pads against the link hulls, the
            links against each other and the Base): "epa" (default: GJK + EPA, MuJoCo 3.3.3's default native
            convex collider: the minimum penetration) or "mpr" (libccd's MPR, MuJoCo's mjDSBL_NATIVECCD path).
        episode_stats: keep device-side episode statistics (RecordEpisodeStatistics): the running float64
            return ``ep_return`` [N], the last finished episode's (return, length) ``ep_final`` [N,2] and the
            per-env totals ``ep_accum`` [N,4] (episodes, successes, sum of returns, sum of lengths), written
            by the step kernel's epilogue; ``info["episode"]`` then carries r / l of the envs that finished
            (mask ``info["_episode"]``), and ``episode_statistics()`` reduces the totals on demand.
        nsubstep: physics substeps per env step (default: the reference's 10, control_timestep / timestep);
            1 makes an env step one mj_step + the final mj_step1 (the parity tests' per-substep checks).
    """

    def __init__(self, num_envs, task="so100_cube_to_bin", obs_type="so100_state", device="cuda:0", seed=0,
                 max_episode_steps=None, autoreset=True, domain_randomization=None, env_offset=0,
                 iterations=None, debug=False, solver="newton", observation_width=640, observation_height=480,
                 variant="joint", reward64=False, nsubstep=None, convex="epa", episode_stats=False):
        torch = _torch()
        if obs_type not in ("so100_state", "so100_pixels_agent_pos"):
            raise NotImplementedError(f"obs_type={obs_type!r}: 'so100_state' or 'so100_pixels_agent_pos'")
        if task not in _native.TASKS:
            raise NotImplementedError(task)    # env.py:117-118
        self.lib = _native.load()
        self.num_envs = int(num_envs)
        self.task = task
        self.obs_type = obs_type
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise ValueError("SO100VecEnv runs on a HIP device (torch 'cuda' device on ROCm)")
        self.autoreset = bool(autoreset)
        self.max_episode_steps = _MAX_STEPS[task] if max_episode_steps is None else int(max_episode_steps)
        self.base_seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.env_offset = int(env_offset)
        self.solver = solver
        self.variant = variant
        self.model = build_model(iterations=iterations, solver=solver, variant=variant, nsubstep=nsubstep, convex=convex)
        dev_index = self.device.index if self.device.index is not None else torch.cuda.current_device()
        self._handle = self.lib.so100_create(ctypes.byref(self.model), self.num_envs, dev_index)
        if not self._handle:
            raise RuntimeError("so100_create failed: " + self.lib.so100_last_error().decode())
        _native.check(self.lib.so100_configure(self._handle, _native.TASKS[task], self.max_episode_steps,
                                               ctypes.c_uint64(self.base_seed), self.env_offset), "so100_configure")
        n, d = self.num_envs, self.device
        f32, i32 = torch.float32, torch.int32
        self.qpos = torch.zeros(n, NQ, dtype=f32, device=d)
        self.qvel = torch.zeros(n, NV, dtype=f32, device=d)
        self.qacc_warmstart = torch.zeros(n, NV, dtype=f32, device=d)
        self.elapsed = torch.zeros(n, dtype=i32, device=d)
        self.episode = torch.zeros(n, dtype=i32, device=d)
        self.actions = torch.zeros(n, 6, dtype=f32, device=d)
        self.obs = torch.zeros(n, NOBS, dtype=f32, device=d)
        self.reward = torch.zeros(n, dtype=f32, device=d)
        self.terminated = torch.zeros(n, dtype=torch.bool, device=d)
        self.truncated = torch.zeros(n, dtype=torch.bool, device=d)
        self.success = torch.zeros(n, dtype=torch.bool, device=d)
        self.diverged = torch.zeros(n, dtype=torch.bool, device=d)
        self.final_obs = torch.zeros(n, NOBS, dtype=f32, device=d)
        self.contact_bits = torch.zeros(n, dtype=i32, device=d)
        # contacts the 16-per-env cap left out in the last step (MuJoCo has no cap: 0 is the bar)
        self.ncon_dropped = torch.zeros(n, dtype=i32, device=d)
        self.is_goal = task == "so100_goal"
        self.achieved_goal = torch.zeros(n, 3, dtype=f32, device=d) if self.is_goal else None
        self.desired_goal = torch.zeros(n, 3, dtype=f32, device=d) if self.is_goal else None
        self.total_steps = torch.zeros(n, dtype=i32, device=d) if self.is_goal else None
        self.debug = torch.zeros(n, _native.SO100_DBG_STRIDE, dtype=f32, device=d) if debug else None
        self.reward64 = torch.zeros(n, dtype=torch.float64, device=d) if reward64 else None
        f64 = torch.float64
        self.ep_return = torch.zeros(n, dtype=f64, device=d) if episode_stats else None
        self.ep_final = torch.zeros(n, 2, dtype=f64, device=d) if episode_stats else None
        self.ep_accum = torch.zeros(n, 4, dtype=f64, device=d) if episode_stats else None
        self.mocap = None
        if variant == "ee":          # mj_resetData's mocap pose: the mocap body's (so_arm100_ee.xml:155)
            m0 = list(self.model.mocap_pos0) + list(self.model.mocap_quat0)
            self.mocap = torch.tensor(m0, dtype=f32, device=d).repeat(n, 1).contiguous()
        self.dr_params = None
        self._flags = _native.SO100_FLAG_AUTORESET if self.autoreset else 0
        if domain_randomization:
            self.set_domain_randomization(**domain_randomization)
        self._buf = _native.SO100Buffers()
        self._fill_buffers()
        self._seeds = torch.zeros(n, dtype=i32, device=d)
        self._mask = torch.zeros(n, dtype=torch.uint8, device=d)
        self.pixels = self.final_pixels = self.renderer = None
        if obs_type == "so100_pixels_agent_pos":
            from .render import CameraRenderer
            self.renderer = CameraRenderer(self, observation_width, observation_height)
            self.pixels = self.renderer.pixels
            self.final_pixels = torch.zeros_like(self.pixels) if self.autoreset else None

    # ------------------------------------------------------------------ plumbing
    def _fill_buffers(self):
        P = _native.ptr
        b = self._buf
        for name in ("qpos", "qvel", "qacc_warmstart", "elapsed", "episode", "obs", "reward", "terminated",
                     "truncated", "success", "final_obs", "diverged", "contact_bits", "achieved_goal",
                     "desired_goal", "total_steps", "dr_params", "debug", "mocap", "reward64", "ncon_dropped",
                     "ep_return", "ep_final", "ep_accum"):
            setattr(b, name, P(getattr(self, name)))
        if not getattr(self, "_debug_enabled", True):
            b.debug = None
        b.action = P(self.actions) if getattr(self, "_action_ref", None) is None else P(self._action_ref)

    def set_mocap(self, pos, quat=None, mask=None):
        """EE variant: the mocap target pose of every env (pos [N,3], quat [N,4] wxyz; the data.mocap_pos /
        data.mocap_quat that teleop_ee.py:52-98 edits), or of the envs in mask."""
        torch = _torch()
        if self.mocap is None:
            raise ValueError("set_mocap needs variant='ee'")
        p = torch.as_tensor(pos, dtype=torch.float32, device=self.device).reshape(-1, 3)
        q = None if quat is None else torch.as_tensor(quat, dtype=torch.float32, device=self.device).reshape(-1, 4)
        if mask is None:
            self.mocap[:, :3] = p
            if q is not None:
                self.mocap[:, 3:] = q
        else:
            m = torch.as_tensor(mask, device=self.device).bool()
            self.mocap[m, :3] = p if p.shape[0] != self.num_envs else p[m]
            if q is not None:
                self.mocap[m, 3:] = q if q.shape[0] != self.num_envs else q[m]

    def _stream(self):
        return _native.stream_ptr(_torch(), self.device)

    def set_domain_randomization(self, mass=(0.8, 1.2), friction=(0.8, 1.2), action_noise=0.05, seed=None):
        """Per-env cube mass scale, contact friction scale (fixed per env) and action-noise sigma.

        The scales are a counter-based hash of (seed, global env id), so an env draws the same parameters
        whatever the sharding (configs[4]: 32,768 envs over 4 GPUs)."""
        torch = _torch()
        s = self.base_seed if seed is None else int(seed)
        ids = np.arange(self.env_offset, self.env_offset + self.num_envs, dtype=np.uint64)
        p = torch.zeros(self.num_envs, 4, dtype=torch.float32)
        p[:, 0] = torch.from_numpy(mass[0] + (mass[1] - mass[0]) * _hash_uniform(s, ids, 1))
        p[:, 1] = torch.from_numpy(friction[0] + (friction[1] - friction[0]) * _hash_uniform(s, ids, 2))
        p[:, 2] = float(action_noise)
        self.dr_params = p.to(self.device)
        self._flags |= _native.SO100_FLAG_DR
        if hasattr(self, "_buf"):
            self._fill_buffers()

    # ------------------------------------------------------------------ API
    def reset(self, seed=None, mask=None):
        """Reset all envs (or those with mask[i] true).

        seed: None -> in-kernel seeds from (base seed, global env id, episode);
              int s -> env i uses RandomState(s + i) exactly like SB3's VecEnv.seed(s);
              sequence/array/tensor of N ints -> per-env RandomState seeds.
        """
        torch = _torch()
        seeds_p = None
        if seed is not None:
            if isinstance(seed, (int, np.integer)):
                s = (int(seed) + np.arange(self.num_envs, dtype=np.int64)) & 0xFFFFFFFF
            else:
                s = np.asarray(seed.cpu() if hasattr(seed, "cpu") else seed, dtype=np.int64).reshape(-1) & 0xFFFFFFFF
                if s.shape[0] != self.num_envs:
                    raise ValueError("need one seed per env")
            self._seeds.copy_(torch.from_numpy(s.astype(np.uint32).view(np.int32)))
            seeds_p = _native.ptr(self._seeds)
        mask_p = None
        if mask is not None:
            m = mask if isinstance(mask, torch.Tensor) else torch.as_tensor(np.asarray(mask))
            self._mask.copy_(m.to(self.device).to(torch.uint8))
            mask_p = _native.ptr(self._mask)
        _native.check(self.lib.so100_reset(self._handle, ctypes.byref(self._buf), mask_p, seeds_p, self._stream()),
                      "so100_reset")
        if self.renderer is not None:
            self.renderer.render()
        info = {"is_success": torch.zeros_like(self.success)}
        return self._observation(), info

    def step(self, actions):
        """actions: [N,6] (torch tensor on any device, or numpy) in [-1, 1]."""
        torch = _torch()
        if getattr(self, "_action_ref", None) is not None:
            self._action_ref = None
            self._buf.action = _native.ptr(self.actions)
        if isinstance(actions, torch.Tensor):
            if actions.shape != (self.num_envs, 6):
                raise ValueError(f"actions must be [{self.num_envs}, 6], got {tuple(actions.shape)}")
            if actions.device == self.device and actions.dtype == torch.float32 and actions.is_contiguous():
                if actions.data_ptr() != self.actions.data_ptr():
                    self.actions.copy_(actions)
            else:
                self.actions.copy_(actions.to(self.device, torch.float32))
        else:
            a = np.asarray(actions, dtype=np.float32)
            if a.shape != (self.num_envs, 6):
                raise ValueError(f"actions must be [{self.num_envs}, 6], got {a.shape}")
            self.actions.copy_(torch.from_numpy(a))
        if self.renderer is None:
            _native.check(self.lib.so100_step(self._handle, ctypes.byref(self._buf), self._flags, self._stream()),
                          "so100_step")
            done = self.terminated | self.truncated
        else:
            done = self._step_pixels()
        info = {"is_success": self.success, "diverged": self.diverged, "contact_bits": self.contact_bits,
                "ncon_dropped": self.ncon_dropped}
        if self.autoreset:
            info["final_observation"] = self.final_obs if self.renderer is None else \
                {"pixels": self.final_pixels, "agent_pos": self.final_obs[:, 9:15]}
            info["_final_observation"] = done
        if self.is_goal:
            info["TimeLimit.truncated"] = self.truncated
        if self.ep_final is not None:                  # RecordEpisodeStatistics' info["episode"] / "_episode"
            info["episode"] = {"r": self.ep_final[:, 0], "l": self.ep_final[:, 1]}
            info["_episode"] = done
        return self._observation(), self.reward, self.terminated, self.truncated, info

    def set_action_buffer(self, actions):
        """Point the kernel's action input at a resident [N,6] float32 device tensor (zero copy).
        The tensor must stay alive until the next call; ``step()`` copies into ``self.actions``."""
        torch = _torch()
        if actions.shape != (self.num_envs, 6) or actions.dtype != torch.float32 or not actions.is_contiguous() \
                or actions.device != self.device:
            raise ValueError("action buffer must be a contiguous float32 [N,6] tensor on the env's device")
        self._action_ref = actions
        self._buf.action = _native.ptr(actions)

    def _step_pixels(self):
        """Pixel observations: step without the in-kernel reset, draw the terminal images of finished envs,
        reset them with the masked reset kernel (same seeds/episode counters as the in-kernel reset), then
        draw every env.  All on the current stream, no host synchronisation."""
        s = self._stream()
        flags = self._flags & ~_native.SO100_FLAG_AUTORESET
        _native.check(self.lib.so100_step(self._handle, ctypes.byref(self._buf), flags, s), "so100_step")
        done = self.terminated | self.truncated
        if self.autoreset:
            self.final_obs.copy_(self.obs)
            self._mask.copy_(done)
            self.renderer.render(out=self.final_pixels, mask=self._mask)
            _native.check(self.lib.so100_reset(self._handle, ctypes.byref(self._buf), _native.ptr(self._mask), None,
                                               s), "so100_reset")
        self.renderer.render()
        return done

    def episode_statistics(self, clear=False):
        """Totals of the episodes finished since construction (or the last ``clear``), reduced over the envs
        on the device and read once: episodes, successes, success_rate, mean_return, mean_length."""
        if self.ep_accum is None:
            raise ValueError("episode statistics need episode_stats=True")
        t = self.ep_accum.sum(dim=0).cpu().tolist()
        if clear:
            self.ep_accum.zero_()
        n = t[0]
        return {"episodes": int(n), "successes": int(t[1]), "success_rate": t[1] / n if n else float("nan"),
                "mean_return": t[2] / n if n else float("nan"), "mean_length": t[3] / n if n else float("nan")}

    def step_async_raw(self):
        """Launch one env step on the current stream using the actions already in ``self.actions``
        (no argument handling, no output views) — the benchmark's hot loop."""
        self.lib.so100_step(self._handle, ctypes.byref(self._buf), self._flags, self._stream())

    def _observation(self):
        if self.renderer is not None:
            agent_pos = self.obs[:, 9:15]                       # qpos[:6] float32 (single_arm.py:45-50)
            if self.is_goal:                                     # _flatten_observation (env.py:267-270)
                flat = self.pixels.reshape(self.num_envs, -1).to(_torch().float32).div_(255.0)
                return {"observation": _torch().cat([flat, agent_pos], dim=1), "achieved_goal": self.achieved_goal,
                        "desired_goal": self.desired_goal}
            return {"pixels": self.pixels, "agent_pos": agent_pos}
        if self.is_goal:
            return {"observation": self.obs, "achieved_goal": self.achieved_goal, "desired_goal": self.desired_goal}
        return self.obs

    def compute_reward(self, achieved_goal, desired_goal, info=None):
        """Batched sparse GoalEnv reward on the device (env.py:341-353)."""
        torch = _torch()
        a = torch.as_tensor(achieved_goal, dtype=torch.float32, device=self.device).reshape(-1, 3).contiguous()
        d = torch.as_tensor(desired_goal, dtype=torch.float32, device=self.device).reshape(-1, 3).contiguous()
        out = torch.empty(a.shape[0], dtype=torch.float32, device=self.device)
        _native.check(self.lib.so100_goal_reward(self._handle, a.shape[0], _native.ptr(a), _native.ptr(d),
                                                 _native.ptr(out), self._stream()), "so100_goal_reward")
        return out

    # state access (checkpoint / teacher-forced parity tests)
    def get_state(self):
        return {"qpos": self.qpos.clone(), "qvel": self.qvel.clone(), "qacc_warmstart": self.qacc_warmstart.clone(),
                "elapsed": self.elapsed.clone(), "episode": self.episode.clone()}

    def set_state(self, qpos, qvel, qacc_warmstart=None, elapsed=None, episode=None):
        torch = _torch()
        self.qpos.copy_(torch.as_tensor(qpos, dtype=torch.float32))
        self.qvel.copy_(torch.as_tensor(qvel, dtype=torch.float32))
        if qacc_warmstart is not None:
            self.qacc_warmstart.copy_(torch.as_tensor(qacc_warmstart, dtype=torch.float32))
        if elapsed is not None:
            self.elapsed.copy_(torch.as_tensor(elapsed, dtype=torch.int32))
        if episode is not None:
            self.episode.copy_(torch.as_tensor(episode, dtype=torch.int32))

    # standalone ops exposed for parity tests
    def eval_reward(self, task, cube_site, ee_site, pair_bits):
        torch = _torch()
        c = torch.as_tensor(cube_site, dtype=torch.float32, device=self.device).contiguous()
        e = torch.as_tensor(ee_site, dtype=torch.float32, device=self.device).contiguous()
        b = torch.as_tensor(np.asarray(pair_bits, dtype=np.uint32).view(np.int32), device=self.device).contiguous()
        out = torch.empty(c.shape[0], dtype=torch.float32, device=self.device)
        _native.check(self.lib.so100_eval_reward(self._handle, _native.TASKS[task], c.shape[0], _native.ptr(c),
                                                 _native.ptr(e), _native.ptr(b), _native.ptr(out), self._stream()),
                      "so100_eval_reward")
        return out

    def spawn_pose(self, seeds):
        torch = _torch()
        s = np.asarray(seeds, dtype=np.int64) & 0xFFFFFFFF
        st = torch.as_tensor(s.astype(np.uint32).view(np.int32), device=self.device).contiguous()
        out = torch.empty(len(s), 7, dtype=torch.float64, device=self.device)
        _native.check(self.lib.so100_spawn_pose(self._handle, len(s), _native.ptr(st), _native.ptr(out),
                                                self._stream()), "so100_spawn_pose")
        return out

    def unnormalize(self, actions):
        torch = _torch()
        a = torch.as_tensor(actions, dtype=torch.float32, device=self.device).reshape(-1, 6).contiguous()
        out = torch.empty_like(a)
        _native.check(self.lib.so100_unnormalize(self._handle, a.shape[0], _native.ptr(a), _native.ptr(out),
                                                 self._stream()), "so100_unnormalize")
        return out

    # ---------------------------------------------------------------- benchmark instrumentation
    def profile_enable(self, max_steps):
        """Record HIP events around every stage/solver launch of the next max_steps steps (0 = off)."""
        _native.check(self.lib.so100_profile_enable(self._handle, int(max_steps)), "so100_profile_enable")

    def profile_read(self):
        """(solver_ms, solver_launches, stage_ms, stage_launches) summed since profile_enable; synchronises."""
        sm, sn, tm, tn = ctypes.c_double(0), ctypes.c_int(0), ctypes.c_double(0), ctypes.c_int(0)
        _native.check(self.lib.so100_profile_read(self._handle, ctypes.byref(sm), ctypes.byref(sn),
                                                  ctypes.byref(tm), ctypes.byref(tn)), "so100_profile_read")
        return sm.value, sn.value, tm.value, tn.value

    @property
    def fused(self):
        """True when a step is one fused kernel launch (Newton solver); False: the split stage/solver
        launches (always for PGS).  Set True / False to force a mode, None for auto (the default: fused at
        every size, SO100_FUSED_MAX=n splits above n envs; include/so100.h so100_set_step_mode)."""
        return bool(self.lib.so100_step_mode(self._handle))

    @fused.setter
    def fused(self, on):
        mode = -1 if on is None else (1 if on else 0)
        _native.check(self.lib.so100_set_step_mode(self._handle, mode), "so100_set_step_mode")

    @property
    def debug_enabled(self):
        """Whether steps write the debug buffer (and so launch the fused kernel's debug build)."""
        return self.debug is not None and getattr(self, "_debug_enabled", True)

    @debug_enabled.setter
    def debug_enabled(self, on):
        self._debug_enabled = bool(on)
        self._fill_buffers()

    @property
    def fused_build(self):
        """The fused kernel build the next fused step launches: 1 = debug build, 2 / 3 = the product build for
        2 / 3 waves per SIMD.  Set 2, 3 or 0 (auto, the default) to choose the product build
        (include/so100.h so100_set_fused_build); every build gives the same results bit for bit."""
        return int(self.lib.so100_fused_build(self._handle, 1 if self.debug_enabled else 0))

    @fused_build.setter
    def fused_build(self, waves):
        _native.check(self.lib.so100_set_fused_build(self._handle, int(waves or 0)), "so100_set_fused_build")

    def chunk_info(self):
        """(chunks, envs of chunk 0): the env split of a step; profile_read times chunk 0's launches."""
        k, n0 = ctypes.c_int(0), ctypes.c_int(0)
        _native.check(self.lib.so100_chunk_info(self._handle, ctypes.byref(k), ctypes.byref(n0)), "so100_chunk_info")
        return k.value, n0.value

    def pool_stats(self, reset=False):
        """The fused step's contact-record pool, summed over the steps since construction or the last
        reset: {"taken": entries taken (wave-substeps whose env lists passed the 16 held on chip), "none_free": entry
        requests that found none free (0 by construction: each XCD's pool holds an entry per wave it can hold
        resident), "entries_per_xcd": the pool's size}.  Synchronises the device."""
        out = (ctypes.c_uint64 * 3)()
        _native.check(self.lib.so100_pool_stats(self._handle, out, int(bool(reset))), "so100_pool_stats")
        return {"taken": int(out[0]), "none_free": int(out[1]), "entries_per_xcd": int(out[2])}

    def contact_count(self, accum):
        """accum (int64 device tensor, 1 element) += contacts in the last solver launch, summed over envs."""
        _native.check(self.lib.so100_contact_count(self._handle, _native.ptr(accum), self._stream()),
                      "so100_contact_count")

    def contact_counts(self):
        """int32 device tensor [N]: each env's contact count in the last solver launch (the last substep's list;
        up to SO100_NCON_MAX, the first 16 held on chip).  Zeros before the first solver launch (zero-initialised:
        the native call writes nothing until a launch has recorded counts)."""
        torch = _torch()
        out = torch.zeros(self.num_envs, dtype=torch.int32, device=self.device)
        _native.check(self.lib.so100_contact_counts(self._handle, _native.ptr(out), self._stream()),
                      "so100_contact_counts")
        return out

    def close(self):
        if getattr(self, "_handle", None):
            self.lib.so100_destroy(self._handle)
            self._handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
