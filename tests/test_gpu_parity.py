"""GPU parity: the HIP path (through the C-ABI) against the oracle and the reference's golden vectors.

Bars:
* task logic (unnormalize, spawn, reward ladders, obs packing, termination): bit-exact vs the
  reference's golden vectors;
* physics: teacher-forced single env steps from identical states vs the fp64 oracle.  The kernel
  computes in fp32, so the bar is the fp32 restatement of the same algorithm: the GPU's per-step
  error distribution must be within 2x (+1e-4) of the fp32-oracle's distribution on the same
  states, and qpos/qvel medians must be <= 1e-5 (abs / rel to 1+|v|).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def venv():
    from gym_so100 import SO100VecEnv
    env = SO100VecEnv(64, device="cuda:0", autoreset=False, debug=True, max_episode_steps=0)
    yield env
    env.close()


def _native_loaded():
    import gym_so100._native as n
    return n._lib is not None


# ----------------------------------------------------------------------------- task layer vs golden
def test_unnormalize_matches_reference(venv, golden):
    got = venv.unnormalize(torch.from_numpy(golden["unnorm_action"])).cpu().numpy()
    np.testing.assert_array_equal(got, golden["unnorm_ctrl"])
    assert _native_loaded()


def test_spawn_matches_reference_randomstate(venv, golden):
    got = venv.spawn_pose(golden["spawn_seed"]).cpu().numpy()
    np.testing.assert_array_equal(got, golden["spawn_pose"])


@pytest.mark.parametrize("col,task", [(0, "so100_cube_to_bin"), (1, "so100_touch_cube"), (2, "so100_touch_cube_sparse")])
def test_reward_matches_reference(venv, golden, col, task):
    cube = golden["reward_cube"].astype(np.float32)
    ee = golden["reward_ee"].astype(np.float32)
    got = venv.eval_reward(task, cube, ee, golden["reward_bits"]).cpu().numpy()
    want = golden["reward_value"][:, col].astype(np.float32)
    if col == 1:
        np.testing.assert_allclose(got, want, rtol=0, atol=1e-6)
    else:
        np.testing.assert_array_equal(got, want)


def test_goal_compute_reward_matches_reference(venv, golden):
    got = venv.compute_reward(golden["goal_achieved"], golden["goal_desired"]).cpu().numpy()
    np.testing.assert_array_equal(got, golden["goal_reward_batch"])


# ----------------------------------------------------------------------------- reset / obs
def test_reset_obs_matches_oracle(venv, model, oracle64):
    obs, _ = venv.reset(seed=1000)
    torch.cuda.synchronize()
    obs = obs.cpu().numpy()
    d = oracle64.new_data()
    for i in range(venv.num_envs):
        oracle64.reset(model, d, oracle64.spawn_pose(1000 + i))
        np.testing.assert_allclose(obs[i], oracle64.observe(model, d), rtol=0, atol=2e-7)
    qpos = venv.qpos.cpu().numpy()
    np.testing.assert_array_equal(qpos[:, :6], np.tile(np.float32(model.start_qpos[:]), (venv.num_envs, 1)))
    assert not venv.qvel.abs().sum().item()


# ----------------------------------------------------------------------------- physics, teacher-forced
def _set_mocap(d, mocap):
    for k in range(3):
        d.mocap_pos[k] = float(mocap[k])
    for k in range(4):
        d.mocap_quat[k] = float(mocap[3 + k])


def _teacher_forced(venv, model, oracle, steps, seed, mocap=None):
    n = venv.num_envs
    venv.reset(seed=seed)
    if mocap is not None:
        venv.set_mocap(mocap[:, :3], mocap[:, 3:])
    rng = np.random.default_rng(seed)
    d = oracle.new_data()
    qp_err, qv_err, rew_bad, bit_bad = [], [], 0, 0
    states = []
    for step in range(steps):
        qpos = venv.qpos.cpu().numpy().astype(np.float64)
        qvel = venv.qvel.cpu().numpy().astype(np.float64)
        warm = venv.qacc_warmstart.cpu().numpy().astype(np.float64)
        act = (rng.uniform(-1, 1, (n, 6)) if step % 20 < 10 else np.clip(rng.normal(0, 0.3, (n, 6)), -1, 1))
        act = act.astype(np.float32)
        _, rew, _, _, info = venv.step(torch.from_numpy(act).cuda())
        torch.cuda.synchronize()
        gq, gv = venv.qpos.cpu().numpy(), venv.qvel.cpu().numpy()
        gr, gb = rew.cpu().numpy(), info["contact_bits"].cpu().numpy().astype(np.uint32)
        for i in range(n):
            oracle.set_state(d, qpos[i], qvel[i], warm[i])
            if mocap is not None:
                _set_mocap(d, mocap[i])
            _, r, _ = oracle.env_step(model, d, 0, act[i])
            oq, ov, _, _ = oracle.get_state(d)
            qp_err.append(np.abs(oq - gq[i]).max())
            qv_err.append((np.abs(ov - gv[i]) / (1 + np.abs(ov))).max())
            rew_bad += abs(r - gr[i]) > 1e-6
            bit_bad += oracle.contact_bits(d) != gb[i]
            states.append((qpos[i], qvel[i], warm[i], act[i]) + ((mocap[i],) if mocap is not None else ()))
    return np.array(qp_err), np.array(qv_err), rew_bad, bit_bad, states


def _oracle_precision_floor(model, o64, o32, states):
    d64, d32 = o64.new_data(), o32.new_data()
    qp, qv = [], []
    for st in states:
        qpos, qvel, warm, act = st[:4]
        o64.set_state(d64, qpos, qvel, warm)
        o32.set_state(d32, qpos, qvel, warm)
        if len(st) > 4:
            _set_mocap(d64, st[4])
            _set_mocap(d32, st[4])
        o64.env_step(model, d64, 0, act)
        o32.env_step(model, d32, 0, act)
        a, b = o64.get_state(d64), o32.get_state(d32)
        qp.append(np.abs(a[0] - b[0]).max())
        qv.append((np.abs(a[1] - b[1]) / (1 + np.abs(a[1]))).max())
    return np.array(qp), np.array(qv)


@pytest.mark.parametrize("solver", ["newton", "pgs"])
def test_step_parity_teacher_forced(solver, oracle64, oracle32):
    from gym_so100 import SO100VecEnv
    from gym_so100.model import build_model
    model = build_model(solver=solver)
    venv = SO100VecEnv(64, device="cuda:0", autoreset=False, debug=True, max_episode_steps=0, solver=solver)
    qp, qv, rew_bad, bit_bad, states = _teacher_forced(venv, model, oracle64, steps=40, seed=1000)
    venv.close()
    fqp, fqv = _oracle_precision_floor(model, oracle64, oracle32, states)
    n = len(qv)
    print(f"\n[{solver}] GPU vs fp64 oracle over {n} env-steps: qpos abs median {np.median(qp):.2e} p99 {np.quantile(qp, .99):.2e}"
          f" | qvel rel median {np.median(qv):.2e} p99 {np.quantile(qv, .99):.2e} max {qv.max():.2e}"
          f" | within 1e-4: {np.mean(qv < 1e-4):.3f}")
    print(f"fp32 oracle vs fp64 oracle (precision floor): qvel rel median {np.median(fqv):.2e} "
          f"p99 {np.quantile(fqv, .99):.2e} max {fqv.max():.2e} | within 1e-4: {np.mean(fqv < 1e-4):.3f}")
    assert np.median(qp) <= 1e-5 and np.median(qv) <= 1e-5
    assert np.quantile(qv, 0.9) <= 2 * np.quantile(fqv, 0.9) + 1e-4
    assert np.quantile(qv, 0.99) <= 2 * np.quantile(fqv, 0.99) + 1e-4
    assert qv.max() <= 2 * fqv.max() + 1e-3
    assert np.mean(qv < 1e-4) >= np.mean(fqv < 1e-4) - 0.05
    assert rew_bad <= max(2, 0.005 * n)          # ladder flips only at contact on/off boundaries
    assert bit_bad <= max(4, 0.01 * n)


@pytest.mark.parametrize("solver", ["newton", "pgs"])
def test_free_flight_bit_close(solver, oracle64):
    """No contacts at all (cube in the air, arm high): GPU equals the fp64 oracle to fp32 rounding."""
    from gym_so100 import SO100VecEnv
    from gym_so100.model import build_model
    model = build_model(solver=solver)
    env = SO100VecEnv(8, device="cuda:0", autoreset=False, max_episode_steps=0, solver=solver)
    env.reset(seed=7)
    qpos = env.qpos.clone()
    qpos[:, 8] = 0.6
    env.set_state(qpos, torch.zeros_like(env.qvel))
    a = np.zeros((8, 6), np.float32)
    d = oracle64.new_data()
    q0 = env.qpos.cpu().numpy().astype(np.float64)
    env.step(torch.from_numpy(a).cuda())
    torch.cuda.synchronize()
    for i in range(8):
        oracle64.set_state(d, q0[i], np.zeros(12), np.zeros(12))
        oracle64.env_step(model, d, 0, a[i])
        oq, ov, _, _ = oracle64.get_state(d)
        np.testing.assert_allclose(env.qpos[i].cpu().numpy(), oq, atol=2e-6)
        np.testing.assert_allclose(env.qvel[i].cpu().numpy(), ov, atol=2e-4, rtol=1e-4)
    env.close()


# ----------------------------------------------------------------------------- size-independent properties
def test_full_size_invariants():
    """configs[1] size (4096 envs): finite state, unit quaternions, cube above the floor, obs layout."""
    from gym_so100 import SO100VecEnv
    env = SO100VecEnv(4096, device="cuda:0", seed=3)
    env.reset(seed=1000)
    g = torch.Generator(device="cuda").manual_seed(0)
    for _ in range(30):
        a = torch.rand(4096, 6, generator=g, device="cuda") * 2 - 1
        obs, rew, term, trunc, info = env.step(a)
    torch.cuda.synchronize()
    assert torch.isfinite(env.qpos).all() and torch.isfinite(env.qvel).all()
    qn = env.qpos[:, 9:13].norm(dim=1)
    assert torch.allclose(qn, torch.ones_like(qn), atol=1e-5)
    assert (env.qpos[:, 8] > -0.05).all()
    assert torch.equal(obs[:, 9:15], env.qpos[:, :6])
    assert torch.allclose(obs[:, 3:6], torch.tensor([-0.2, 0.7, 0.021], device="cuda").expand(4096, 3))
    assert not info["diverged"].any()
    assert set(torch.unique(rew).tolist()) <= {0.0, 1.0, 2.0, 2.5, 3.0, 4.0}
    env.close()


def test_autoreset_and_timelimit():
    from gym_so100 import SO100VecEnv
    env = SO100VecEnv(16, device="cuda:0", max_episode_steps=5, seed=11)
    env.reset(seed=0)
    a = torch.zeros(16, 6, device="cuda")
    for k in range(1, 6):
        obs, _, term, trunc, info = env.step(a)
        torch.cuda.synchronize()
        if k < 5:
            assert not trunc.any() and (env.elapsed == k).all()
    assert trunc.all() and info["_final_observation"].all()
    assert (env.elapsed == 0).all() and (env.episode == 2).all()   # reset() started episode 1
    # the new episode's spawn is the reference RandomState(seed) for the in-kernel episode seed
    assert not torch.equal(info["final_observation"], obs)
    assert torch.equal(obs[:, 9:15], env.qpos[:, :6])
    env.close()


def test_sharding_invariance():
    """Global env ids drive the in-kernel seeds: 2 shards of 8 == 1 shard of 16."""
    from gym_so100 import SO100VecEnv
    full = SO100VecEnv(16, device="cuda:0", seed=5, max_episode_steps=3)
    a0 = SO100VecEnv(8, device="cuda:0", seed=5, env_offset=0, max_episode_steps=3)
    a1 = SO100VecEnv(8, device="cuda:0", seed=5, env_offset=8, max_episode_steps=3)
    for e in (full, a0, a1):
        e.reset()
    g = torch.Generator(device="cuda").manual_seed(1)
    for _ in range(7):
        a = torch.rand(16, 6, generator=g, device="cuda") * 2 - 1
        full.step(a)
        a0.step(a[:8].contiguous())
        a1.step(a[8:].contiguous())
    torch.cuda.synchronize()
    assert torch.equal(full.qpos, torch.cat([a0.qpos, a1.qpos]))
    assert torch.equal(full.obs, torch.cat([a0.obs, a1.obs]))


@pytest.mark.parametrize("variant", ["joint", "ee"])
def test_chunking_invariance(monkeypatch, variant):
    """The env-range chunks of a step (concurrent streams, so100_capi.cpp) change nothing: 4 ragged
    chunks == 1 chunk, bitwise, through auto-resets and the solver's debug record.  The EE variant gives
    every env its own mocap target, so a chunk reading another chunk's targets (a per-env pointer left
    unshifted by offset_buffers) shows up as a mismatch."""
    from gym_so100 import SO100VecEnv
    n = 4160
    kw = dict(device="cuda:0", seed=4, max_episode_steps=5, debug=True, variant=variant)
    monkeypatch.setenv("SO100_CHUNKS", "1")
    one = SO100VecEnv(n, **kw)
    monkeypatch.setenv("SO100_CHUNKS", "4")
    four = SO100VecEnv(n, **kw)
    for e in (one, four):
        e.fused = False                  # chunks belong to the split path (a fused step is one launch)
    assert one.chunk_info() == (1, n)
    k, n0 = four.chunk_info()
    assert k == 4 and n0 < n
    for e in (one, four):
        e.reset()
    if variant == "ee":
        gm = torch.Generator(device="cuda").manual_seed(3)
        pos = one.mocap[:, :3] + (torch.rand(n, 3, generator=gm, device="cuda") - 0.5) * 0.08
        for e in (one, four):
            e.set_mocap(pos)
        assert pos[:, 0].unique().numel() > n // 2          # distinct per-env targets
    g = torch.Generator(device="cuda").manual_seed(2)
    for _ in range(12):
        a = torch.rand(n, 6, generator=g, device="cuda") * 2 - 1
        r1 = one.step(a)
        r4 = four.step(a)
        torch.cuda.synchronize()
        assert torch.equal(r1[1], r4[1]) and torch.equal(r1[2], r4[2]) and torch.equal(r1[3], r4[3])
    for name in ("qpos", "qvel", "qacc_warmstart", "obs", "debug"):
        assert torch.equal(getattr(one, name), getattr(four, name)), name
    one.close()
    four.close()


@pytest.mark.parametrize("variant,task,dr", [("joint", "so100_cube_to_bin", False), ("ee", "so100_touch_cube", False),
                                               ("joint", "so100_goal", True)])
def test_fused_step_matches_split(variant, task, dr):
    """The fused step kernel (one launch per env step, the Newton rows handed over in registers) gives the
    split path's results (per substep a stage and a Newton launch exchanging an HBM record) bit for bit:
    state, outputs, auto-resets and the debug record, with a ragged tail wave (n % 4 != 0)."""
    from gym_so100 import SO100VecEnv
    n = 1003
    kw = dict(task=task, device="cuda:0", seed=7, max_episode_steps=6, debug=True, variant=variant,
              domain_randomization=(dict(mass=(0.8, 1.2), friction=(0.8, 1.2), action_noise=0.05) if dr else None))
    fused, split = SO100VecEnv(n, **kw), SO100VecEnv(n, **kw)
    fused.fused, split.fused = True, False
    assert fused.fused and not split.fused
    for e in (fused, split):
        e.reset(seed=500)
    if variant == "ee":
        gm = torch.Generator(device="cuda").manual_seed(3)
        pos = fused.mocap[:, :3] + (torch.rand(n, 3, generator=gm, device="cuda") - 0.5) * 0.08
        for e in (fused, split):
            e.set_mocap(pos)
    g = torch.Generator(device="cuda").manual_seed(5)
    for _ in range(14):
        a = torch.rand(n, 6, generator=g, device="cuda") * 2 - 1
        rf, rs = fused.step(a), split.step(a)
        torch.cuda.synchronize()
        for x, y in zip(rf[1:4], rs[1:4]):
            assert torch.equal(x, y)
    for name in ("qpos", "qvel", "qacc_warmstart", "obs", "debug", "elapsed", "episode"):
        assert torch.equal(getattr(fused, name), getattr(split, name)), name
    fused.close()
    split.close()


def test_step_mode_switch():
    """PGS always runs split; auto mode (the default) runs fused up to 49,152 envs; the mode can be switched
    between steps (Newton), and the contact counter reads the record of the mode that ran."""
    from gym_so100 import SO100VecEnv
    big = SO100VecEnv(32768, device="cuda:0")
    assert big.fused and big.chunk_info() == (1, 32768)
    big.fused = False
    assert not big.fused and big.chunk_info()[0] == 4
    big.close()
    big = SO100VecEnv(65536, device="cuda:0")
    assert not big.fused and big.chunk_info()[0] == 4
    big.close()
    pgs = SO100VecEnv(8, device="cuda:0", solver="pgs")
    assert not pgs.fused
    pgs.fused = True
    assert not pgs.fused
    pgs.close()
    env = SO100VecEnv(8, device="cuda:0", debug=True)
    assert env.fused
    env.reset(seed=1)
    for _ in range(30):                                     # the cube lands on the table: contacts
        env.step(torch.zeros(8, 6, device="cuda"))
    counts = []
    for mode in (True, False, True, None):
        env.fused = mode
        env.step(torch.zeros(8, 6, device="cuda"))
        acc = torch.zeros(1, dtype=torch.int64, device="cuda")
        env.contact_count(acc)
        torch.cuda.synchronize()
        assert int(acc) == int(env.debug[:, 0].sum())      # the last substep's contact count
        counts.append(int(acc))
    assert torch.isfinite(env.qpos).all() and counts[0] > 0
    env.close()


def test_goal_env_semantics():
    from gym_so100 import SO100VecEnv
    env = SO100VecEnv(32, task="so100_goal", device="cuda:0", seed=2)
    obs, _ = env.reset(seed=100)
    torch.cuda.synchronize()
    dg, ag = obs["desired_goal"], obs["achieved_goal"]
    spawn = env.qpos[:, 6:8]
    # lifted-goal curriculum (env.py:324-330): within +-0.03 of the spawn xy, z in [0.01, 0.05]
    assert ((dg[:, :2] - spawn).abs() <= 0.03 + 1e-6).all()
    assert ((dg[:, 2] >= 0.01) & (dg[:, 2] <= 0.05)).all()
    a = torch.zeros(32, 6, device="cuda")
    o, r, term, trunc, info = env.step(a)
    torch.cuda.synchronize()
    dist = (o["achieved_goal"] - o["desired_goal"]).norm(dim=1)
    assert torch.equal(r, torch.where(dist < 0.01, 0.0, -1.0))
    assert torch.equal(term, dist < 0.01)
    assert (env.total_steps == 1).all()
    env.close()


def test_domain_randomization_changes_dynamics_deterministically():
    from gym_so100 import SO100VecEnv
    kw = dict(device="cuda:0", seed=9, domain_randomization=dict(mass=(0.8, 1.2), friction=(0.8, 1.2),
                                                                  action_noise=0.05))
    e1, e2 = SO100VecEnv(32, **kw), SO100VecEnv(32, **kw)
    e3 = SO100VecEnv(32, device="cuda:0", seed=9)
    for e in (e1, e2, e3):
        e.reset(seed=0)
    a = torch.zeros(32, 6, device="cuda")
    for _ in range(5):
        for e in (e1, e2, e3):
            e.step(a)
    torch.cuda.synchronize()
    assert torch.equal(e1.qpos, e2.qpos)
    assert not torch.equal(e1.qpos, e3.qpos)
    assert ((e1.dr_params[:, 0] >= 0.8) & (e1.dr_params[:, 0] <= 1.2)).all()


def test_single_env_api():
    from gym_so100 import SO100Env, SO100GoalEnv
    with pytest.raises(ValueError):
        SO100Env("so100_cube_to_bin")                  # the reference's default obs_type "pixels"
    env = SO100Env("so100_cube_to_bin", obs_type="so100_state")
    obs, info = env.reset(seed=0)
    assert obs.shape == (15,) and obs.dtype == np.float32 and info == {"is_success": False}
    obs, r, term, trunc, info = env.step(np.zeros(6, np.float32))
    assert obs.shape == (15,) and isinstance(r, float) and trunc is False and "is_success" in info
    g = SO100GoalEnv()
    o, _ = g.reset(seed=0)
    assert set(o) == {"observation", "achieved_goal", "desired_goal"}
    o, r, term, trunc, info = g.step(np.zeros(6, np.float32))
    assert r in (0.0, -1.0)
    rb = g.compute_reward(np.zeros((4, 3)), np.zeros((4, 3)) + 0.001, {})
    assert rb.dtype == np.float32 and (rb == 0).all()


def test_reward64_is_the_double_ladder(oracle64):
    """reward64 holds the reward in float64 as the reference returns it (env.py:174-182 passes the task's
    python float through); reward is its float32 rounding.  Dense TouchCube shaping (single_arm.py:149-215)
    is not representable in float32, so the two differ there; the float64 value equals the oracle's."""
    from gym_so100 import SO100VecEnv
    from gym_so100.model import build_model
    n = 64
    venv = SO100VecEnv(n, task="so100_touch_cube", device="cuda:0", autoreset=False, max_episode_steps=0,
                       reward64=True)
    venv.reset(seed=300)
    torch.cuda.synchronize()
    q0 = venv.qpos.cpu().numpy().astype(np.float64)
    a = np.random.default_rng(1).uniform(-1, 1, size=(n, 6)).astype(np.float32)
    venv.step(torch.from_numpy(a).cuda())
    torch.cuda.synchronize()
    r32, r64 = venv.reward.cpu().numpy(), venv.reward64.cpu().numpy()
    assert np.array_equal(r64.astype(np.float32), r32)
    assert (r64 != r32.astype(np.float64)).any()           # the dense shaping needs float64
    model, d = build_model(), oracle64.new_data()
    for i in range(n):
        oracle64.set_state(d, q0[i], np.zeros(12), np.zeros(12))
        _, r, _ = oracle64.env_step(model, d, 1, a[i])
        assert abs(r64[i] - r) <= 1e-5
    venv.close()


@pytest.mark.parametrize("solver", ["newton", "pgs"])
def test_heavy_contact_parity(solver, oracle64, oracle32):
    """Cube pressed into a bin corner: floor + two walls give up to 12 contacts, beyond the solver's 4
    on-chip slots — exercises the streamed-overflow contacts and the heavy-group first dispatch."""
    from gym_so100 import SO100VecEnv
    from gym_so100.model import build_model
    model = build_model(solver=solver)
    n = 32
    env = SO100VecEnv(n, device="cuda:0", autoreset=False, max_episode_steps=0, debug=True, solver=solver)
    env.reset(seed=5)
    rng = np.random.default_rng(7)
    qpos = env.qpos.cpu().numpy().astype(np.float64)
    pen = rng.uniform(2e-4, 1e-3, (n, 3))
    # bin inner faces (assets: bin_wall3 x = -0.14 - 0.005, bin_wall y = 0.76 - 0.005, floor top z = 0.001)
    qpos[:, 6] = -0.145 - 0.02 + pen[:, 0]
    qpos[:, 7] = 0.755 - 0.02 + pen[:, 1]
    qpos[:, 8] = 0.001 + 0.02 - pen[:, 2]
    ang = rng.uniform(-0.01, 0.01, n)
    qpos[:, 9:13] = np.stack([np.cos(ang / 2), np.zeros(n), np.zeros(n), np.sin(ang / 2)], 1)
    qvel = np.zeros((n, 12))
    qvel[:, 6:9] = rng.normal(0, 0.02, (n, 3))
    env.set_state(qpos.astype(np.float32), qvel.astype(np.float32), np.zeros((n, 12), np.float32))
    d64, d32 = oracle64.new_data(), oracle32.new_data()
    qv_err, qv_floor, ncon = [], [], []
    for step in range(3):
        q0 = env.qpos.cpu().numpy().astype(np.float64)
        v0 = env.qvel.cpu().numpy().astype(np.float64)
        w0 = env.qacc_warmstart.cpu().numpy().astype(np.float64)
        act = rng.uniform(-0.2, 0.2, (n, 6)).astype(np.float32)
        env.step(torch.from_numpy(act).cuda())
        torch.cuda.synchronize()
        gv = env.qvel.cpu().numpy()
        ncon.append(env.debug.cpu().numpy()[:, 0])
        for i in range(n):
            oracle64.set_state(d64, q0[i], v0[i], w0[i])
            oracle32.set_state(d32, q0[i], v0[i], w0[i])
            oracle64.env_step(model, d64, 0, act[i])
            oracle32.env_step(model, d32, 0, act[i])
            ov = oracle64.get_state(d64)[1]
            qv_err.append((np.abs(ov - gv[i]) / (1 + np.abs(ov))).max())
            qv_floor.append((np.abs(ov - oracle32.get_state(d32)[1]) / (1 + np.abs(ov))).max())
    qv_err, qv_floor, ncon = np.array(qv_err), np.array(qv_floor), np.concatenate(ncon)
    print(f"\n[{solver}] heavy contacts: GPU ncon mean {ncon.mean():.1f} max {ncon.max():.0f} | qvel rel GPU median "
          f"{np.median(qv_err):.2e} p90 {np.quantile(qv_err, .9):.2e} max {qv_err.max():.2e} | fp32 floor median "
          f"{np.median(qv_floor):.2e} p90 {np.quantile(qv_floor, .9):.2e} max {qv_floor.max():.2e}")
    assert (ncon > 4).mean() > 0.5                      # the overflow path is really exercised
    assert np.median(qv_err) <= 2 * np.median(qv_floor) + 1e-5
    assert np.quantile(qv_err, 0.9) <= 2 * np.quantile(qv_floor, 0.9) + 1e-4
    assert qv_err.max() <= 2 * qv_floor.max() + 1e-3
    env.close()


@pytest.mark.parametrize("solver", ["newton", "pgs"])
def test_hull_table_parity(solver, oracle64, oracle32):
    """Arm/jaw hulls resting on the table (pairs 14..22, condim 3): states made by the
    fp64 oracle driving the arm down onto the table, then teacher-forced GPU steps against it."""
    from gym_so100 import SO100VecEnv
    from gym_so100.model import NPAIR_BOX, PAIR_MPR0, build_model
    model = build_model(solver=solver)
    n = 24
    rng = np.random.default_rng(11)
    d = oracle64.new_data()
    states, targets = [], []
    lo, hi = np.array(model.action_lo[:]), np.array(model.action_hi[:])
    for i in range(n):
        oracle64.reset(model, d, np.array([2.0, 0.95, 0.6, 1, 0, 0, 0]))          # cube off the table: it falls
        # clear, so no cube resting at dist ~ 0 (its contacts flip between precisions)
        target = np.array([rng.uniform(-0.6, 0.6), rng.uniform(0.6, 1.2), rng.uniform(-1.2, -0.6),
                           rng.uniform(0.8, 1.5), rng.uniform(-1.5, 1.5), rng.uniform(-0.17, 1.0)])
        for k in range(6):
            d.ctrl[k] = target[k]
        for _ in range(400):
            oracle64.call("so100o_substep", model, d)
        q, v, w, _ = oracle64.get_state(d)
        states.append((q, v, w))
        targets.append((target - lo) / (hi - lo) * 2 - 1)      # keep pressing: the same targets as actions
    env = SO100VecEnv(n, device="cuda:0", autoreset=False, max_episode_steps=0, debug=True, solver=solver)
    env.reset(seed=3)
    env.set_state(np.array([s[0] for s in states], np.float32), np.array([s[1] for s in states], np.float32),
                  np.array([s[2] for s in states], np.float32))
    d64, d32 = oracle64.new_data(), oracle32.new_data()
    qv_err, qv_floor, hull_con, bit_bad, same = [], [], [], 0, []
    for step in range(4):
        q0 = env.qpos.cpu().numpy().astype(np.float64)
        v0 = env.qvel.cpu().numpy().astype(np.float64)
        w0 = env.qacc_warmstart.cpu().numpy().astype(np.float64)
        act = (np.array(targets) + rng.normal(0, 0.02, (n, 6))).astype(np.float32)
        _, _, _, _, info = env.step(torch.from_numpy(act).cuda())
        torch.cuda.synchronize()
        gv = env.qvel.cpu().numpy()
        dbg = env.debug.cpu().numpy()
        gb = info["contact_bits"].cpu().numpy().astype(np.uint32)
        for i in range(n):
            pairs = dbg[i, 48:48 + int(dbg[i, 0])]
            hull_con.append(int(((pairs >= NPAIR_BOX) & (pairs < PAIR_MPR0)).sum()))
            oracle64.set_state(d64, q0[i], v0[i], w0[i])
            oracle32.set_state(d32, q0[i], v0[i], w0[i])
            oracle64.env_step(model, d64, 0, act[i])
            oracle32.env_step(model, d32, 0, act[i])
            same.append(sorted(pairs.astype(int).tolist()) == sorted(d64.con[c].pair for c in range(d64.ncon)))
            ov = oracle64.get_state(d64)[1]
            qv_err.append((np.abs(ov - gv[i]) / (1 + np.abs(ov))).max())
            qv_floor.append((np.abs(ov - oracle32.get_state(d32)[1]) / (1 + np.abs(ov))).max())
            bit_bad += oracle64.contact_bits(d64) != gb[i]
    qv_err, qv_floor, hull_con, same = np.array(qv_err), np.array(qv_floor), np.array(hull_con), np.array(same)
    print(f"\n[{solver}] hull-table: GPU hull contacts per env mean {hull_con.mean():.2f} (envs with any: "
          f"{(hull_con > 0).mean():.2f}) | qvel rel GPU median {np.median(qv_err):.2e} p90 "
          f"{np.quantile(qv_err, .9):.2e} max {qv_err.max():.2e} | fp32 floor median {np.median(qv_floor):.2e} "
          f"p90 {np.quantile(qv_floor, .9):.2e} max {qv_floor.max():.2e} | contact-bit mismatches {bit_bad} | "
          f"contact-set flips {(~same).sum()} of {len(same)} (same-set p90 GPU {np.quantile(qv_err[same], .9):.2e}, "
          f"floor {np.quantile(qv_floor[same], .9):.2e})")
    assert (hull_con > 0).mean() > 0.5                 # the arm really rests on the table
    # a contact at dist ~ 0 can be in one precision's set and not the other's; PGS, unconverged at 100
    # sweeps on resting contacts, amplifies such a flip, so the tail bar applies to the states whose GPU
    # and oracle contact sets agree, and flips must stay rare
    assert (~same).mean() <= 0.1
    assert np.median(qv_err) <= 2 * np.median(qv_floor) + 1e-5
    assert np.quantile(qv_err[same], 0.9) <= 2 * np.quantile(qv_floor[same], 0.9) + 1e-4
    assert qv_err.max() <= 2 * qv_floor.max() + 1e-3
    assert bit_bad <= max(2, 0.05 * len(qv_err))
    env.close()


@pytest.mark.parametrize("solver", ["newton", "pgs"])
def test_pad_contact_parity(solver, oracle64, oracle32):
    """Finger pads against the table and the bin boxes (pairs 98..145, box-box, condim 3):
    states made by the fp64 oracle pressing the gripper onto the table top (two thirds of the envs) and
    into the bin (the rest), then teacher-forced GPU steps against it, with the pad contacts counted."""
    from gym_so100 import SO100VecEnv
    from gym_so100.model import PAIR_PAD0, build_model
    model = build_model(solver=solver)
    n = 24
    rng = np.random.default_rng(13)
    d = oracle64.new_data()
    over_bin = np.array([[0.72, -0.89, 2.15, -1.24, -1.38, -0.05], [0.7, -0.91, 1.85, -0.39, -0.2, 0.33]])
    states, targets = [], []
    lo, hi = np.array(model.action_lo[:]), np.array(model.action_hi[:])
    for i in range(n):
        oracle64.reset(model, d, np.array([0.4, 0.95, 0.6, 1, 0, 0, 0]))          # cube out of reach
        if i % 3 < 2:
            target = np.array([rng.uniform(-0.6, 0.6), rng.uniform(0.2, 1.3), rng.uniform(-1.4, -0.2),
                               rng.uniform(0.6, 1.6), rng.uniform(-1.5, 1.5), rng.uniform(-0.17, 1.5)])
        else:
            target = over_bin[i % 2] + rng.normal(0, 0.12, 6) + np.array([0, 0.15, 0, 0, 0, 0])
        target = np.clip(target, lo, hi)
        for k in range(6):
            d.ctrl[k] = target[k]
        for _ in range(400):
            oracle64.call("so100o_substep", model, d)
        q, v, w, _ = oracle64.get_state(d)
        states.append((q, v, w))
        targets.append((target - lo) / (hi - lo) * 2 - 1)      # keep pressing: the same targets as actions
    env = SO100VecEnv(n, device="cuda:0", autoreset=False, max_episode_steps=0, debug=True, solver=solver)
    env.reset(seed=3)
    env.set_state(np.array([s[0] for s in states], np.float32), np.array([s[1] for s in states], np.float32),
                  np.array([s[2] for s in states], np.float32))
    d64, d32 = oracle64.new_data(), oracle32.new_data()
    qv_err, qv_floor, pad_gpu, pad_ora = [], [], [], []
    for step in range(4):
        q0 = env.qpos.cpu().numpy().astype(np.float64)
        v0 = env.qvel.cpu().numpy().astype(np.float64)
        w0 = env.qacc_warmstart.cpu().numpy().astype(np.float64)
        act = (np.array(targets) + rng.normal(0, 0.02, (n, 6))).astype(np.float32)
        _, _, _, _, info = env.step(torch.from_numpy(act).cuda())
        torch.cuda.synchronize()
        gv = env.qvel.cpu().numpy()
        dbg = env.debug.cpu().numpy()
        for i in range(n):
            pairs = dbg[i, 48:48 + int(dbg[i, 0])]
            pad_gpu.append(int((pairs >= PAIR_PAD0).sum()))
            oracle64.set_state(d64, q0[i], v0[i], w0[i])
            oracle32.set_state(d32, q0[i], v0[i], w0[i])
            oracle64.env_step(model, d64, 0, act[i])
            oracle32.env_step(model, d32, 0, act[i])
            pad_ora.append(sum(d64.con[c].pair >= PAIR_PAD0 for c in range(d64.ncon)))
            ov = oracle64.get_state(d64)[1]
            qv_err.append((np.abs(ov - gv[i]) / (1 + np.abs(ov))).max())
            qv_floor.append((np.abs(ov - oracle32.get_state(d32)[1]) / (1 + np.abs(ov))).max())
    qv_err, qv_floor = np.array(qv_err), np.array(qv_floor)
    pad_gpu, pad_ora = np.array(pad_gpu), np.array(pad_ora)
    print(f"\n[{solver}] pads: GPU pad contacts per env mean {pad_gpu.mean():.2f} (envs with any: "
          f"{(pad_gpu > 0).mean():.2f}; oracle {pad_ora.mean():.2f}, count mismatches {(pad_gpu != pad_ora).sum()}) "
          f"| qvel rel GPU median {np.median(qv_err):.2e} p90 {np.quantile(qv_err, .9):.2e} max {qv_err.max():.2e} "
          f"| fp32 floor median {np.median(qv_floor):.2e} p90 {np.quantile(qv_floor, .9):.2e} max {qv_floor.max():.2e}")
    assert (pad_gpu > 0).sum() >= 10                    # the pads really touch the table / bin
    assert (pad_gpu != pad_ora).mean() <= 0.05           # the same pad contact sets (fp32 flips at dist ~ 0 aside)
    assert np.median(qv_err) <= 2 * np.median(qv_floor) + 1e-5
    assert np.quantile(qv_err, 0.9) <= 2 * np.quantile(qv_floor, 0.9) + 1e-4
    assert qv_err.max() <= 2 * qv_floor.max() + 1e-3
    env.close()


@pytest.mark.parametrize("solver", ["newton", "pgs"])
def test_mpr_contact_parity(solver, oracle64, oracle32):
    """Box-hull contacts through the MPR collider (pairs 23..76: the cube and the bin boxes against the
    arm/jaw hulls): states from fp64-oracle random-action rollouts that hold such
    contacts, then teacher-forced GPU steps against the oracle at the fp32 floor."""
    from gym_so100 import SO100VecEnv
    from gym_so100.model import PAIR_MPR0, PAIR_PAD0, NHULL, build_model
    model = build_model(solver=solver)
    rng = np.random.default_rng(21)
    d = oracle64.new_data()
    states, kinds = [], set()
    for e in range(128):
        oracle64.reset(model, d, oracle64.spawn_pose(2000 + e))
        for _ in range(200):
            oracle64.env_step(model, d, 0, rng.uniform(-1, 1, 6).astype(np.float32))
            pairs = [d.con[i].pair for i in range(d.ncon)]
            mp = [p for p in pairs if PAIR_MPR0 <= p < PAIR_PAD0]
            if mp and not d.ncon_dropped:
                q, v, w, _ = oracle64.get_state(d)
                states.append((q, v, w))
                kinds.update(p < PAIR_MPR0 + NHULL for p in mp)
                break
        if len(states) >= 48:
            break
    n = len(states)
    assert n >= 24 and kinds == {True, False}, (n, kinds)     # both cube-hull and bin-hull contacts
    env = SO100VecEnv(n, device="cuda:0", autoreset=False, max_episode_steps=0, debug=True, solver=solver)
    env.reset(seed=3)
    env.set_state(np.array([s[0] for s in states], np.float32), np.array([s[1] for s in states], np.float32),
                  np.array([s[2] for s in states], np.float32))
    d64, d32 = oracle64.new_data(), oracle32.new_data()
    qv_err, qv_floor, mpr_con = [], [], []
    for step in range(3):
        q0 = env.qpos.cpu().numpy().astype(np.float64)
        v0 = env.qvel.cpu().numpy().astype(np.float64)
        w0 = env.qacc_warmstart.cpu().numpy().astype(np.float64)
        act = rng.uniform(-1, 1, (n, 6)).astype(np.float32)
        env.step(torch.from_numpy(act).cuda())
        torch.cuda.synchronize()
        gv = env.qvel.cpu().numpy()
        dbg = env.debug.cpu().numpy()
        for i in range(n):
            pairs = dbg[i, 48:48 + int(dbg[i, 0])]
            mpr_con.append(int(((pairs >= PAIR_MPR0) & (pairs < PAIR_PAD0)).sum()))
            oracle64.set_state(d64, q0[i], v0[i], w0[i])
            oracle32.set_state(d32, q0[i], v0[i], w0[i])
            oracle64.env_step(model, d64, 0, act[i])
            oracle32.env_step(model, d32, 0, act[i])
            ov = oracle64.get_state(d64)[1]
            qv_err.append((np.abs(ov - gv[i]) / (1 + np.abs(ov))).max())
            qv_floor.append((np.abs(ov - oracle32.get_state(d32)[1]) / (1 + np.abs(ov))).max())
    qv_err, qv_floor, mpr_con = np.array(qv_err), np.array(qv_floor), np.array(mpr_con)
    print(f"\n[{solver}] box-hull (MPR): {n} envs, GPU MPR contacts per env mean {mpr_con.mean():.2f} (envs with any: "
          f"{(mpr_con > 0).mean():.2f}) | qvel rel GPU median {np.median(qv_err):.2e} p90 "
          f"{np.quantile(qv_err, .9):.2e} max {qv_err.max():.2e} | fp32 floor median {np.median(qv_floor):.2e} "
          f"p90 {np.quantile(qv_floor, .9):.2e} max {qv_floor.max():.2e}")
    assert (mpr_con[:n] > 0).mean() > 0.3              # the GPU collider sees the contacts too
    # MPR's fp32 branches (different portals) make the tail chaotic for ANY fp32 implementation: the
    # fp32 oracle and the GPU put their large deviations on different states, so the tail is compared by
    # its mass (share of env steps off by > 1e-4), not by a quantile of a 150-sample set
    assert np.median(qv_err) <= 2 * np.median(qv_floor) + 1e-5
    assert np.mean(qv_err > 1e-4) <= 1.5 * np.mean(qv_floor > 1e-4) + 0.05
    assert qv_err.max() <= 2 * qv_floor.max() + 1e-3
    env.close()


def test_newton_solver_parity(oracle64, oracle32):
    """MuJoCo's default solver (primal Newton, solver="newton"): teacher-forced GPU steps against the fp64
    oracle's Newton from random-action rollout states (contacts on the table, bin, gripper and hulls),
    at the fp32 floor (the fp32 oracle's Newton on the same states); 2-6 Newton steps per substep."""
    from gym_so100 import SO100VecEnv
    from gym_so100.model import build_model
    mn = build_model(solver="newton")
    n = 48
    rng = np.random.default_rng(31)
    d = oracle64.new_data()
    states = []
    for e in range(n):
        oracle64.reset(mn, d, oracle64.spawn_pose(4000 + e))
        for _ in range(int(rng.integers(10, 160))):
            oracle64.env_step(mn, d, 0, rng.uniform(-1, 1, 6).astype(np.float32))
        states.append(oracle64.get_state(d)[:3])
    env = SO100VecEnv(n, device="cuda:0", autoreset=False, max_episode_steps=0, debug=True, solver="newton")
    env.reset(seed=3)
    env.set_state(np.array([s[0] for s in states], np.float32), np.array([s[1] for s in states], np.float32),
                  np.array([s[2] for s in states], np.float32))
    d64, d32 = oracle64.new_data(), oracle32.new_data()
    qv_err, qv_floor, iters, ncon = [], [], [], []
    for step in range(3):
        q0 = env.qpos.cpu().numpy().astype(np.float64)
        v0 = env.qvel.cpu().numpy().astype(np.float64)
        w0 = env.qacc_warmstart.cpu().numpy().astype(np.float64)
        act = rng.uniform(-1, 1, (n, 6)).astype(np.float32)
        env.step(torch.from_numpy(act).cuda())
        torch.cuda.synchronize()
        gv = env.qvel.cpu().numpy()
        dbg = env.debug.cpu().numpy()
        iters += list(dbg[:, 1])
        ncon += list(dbg[:, 0])
        for i in range(n):
            oracle64.set_state(d64, q0[i], v0[i], w0[i])
            oracle32.set_state(d32, q0[i], v0[i], w0[i])
            oracle64.env_step(mn, d64, 0, act[i])
            oracle32.env_step(mn, d32, 0, act[i])
            ov = oracle64.get_state(d64)[1]
            qv_err.append((np.abs(ov - gv[i]) / (1 + np.abs(ov))).max())
            qv_floor.append((np.abs(ov - oracle32.get_state(d32)[1]) / (1 + np.abs(ov))).max())
    qv_err, qv_floor, iters, ncon = np.array(qv_err), np.array(qv_floor), np.array(iters), np.array(ncon)
    print(f"\nnewton: contacts/env {ncon.mean():.2f}, GPU Newton steps per substep mean {iters.mean():.2f} max "
          f"{iters.max():.0f} | qvel rel GPU median {np.median(qv_err):.2e} p90 {np.quantile(qv_err, .9):.2e} max "
          f"{qv_err.max():.2e} | fp32 floor median {np.median(qv_floor):.2e} p90 {np.quantile(qv_floor, .9):.2e} "
          f"max {qv_floor.max():.2e}")
    assert ncon.mean() > 1.0
    assert iters.max() <= 30 and iters.mean() < 10
    assert np.median(qv_err) <= 2 * np.median(qv_floor) + 1e-5
    assert np.quantile(qv_err, 0.9) <= 2 * np.quantile(qv_floor, 0.9) + 1e-4
    assert qv_err.max() <= 2 * qv_floor.max() + 1e-3
    env.close()


@pytest.mark.parametrize("solver", ["newton", "pgs"])
def test_goal_env_config3_size(solver):
    """configs[3] size (GoalEnv, 16,384 envs, randomized cube spawn): 40 steps with auto-reset keep the
    state finite and the dict-obs contract: achieved_goal = the cube site, sparse reward consistent with
    the goal distance, the lifted-goal curriculum box around each spawn."""
    from gym_so100 import SO100VecEnv
    n = 16384
    env = SO100VecEnv(n, task="so100_goal", device="cuda:0", seed=4, solver=solver)
    obs, _ = env.reset(seed=7)
    spawn = env.qpos[:, 6:8].clone()
    dg0 = obs["desired_goal"].clone()
    assert ((dg0[:, :2] - spawn).abs() <= 0.03 + 1e-6).all()
    g = torch.Generator(device="cuda").manual_seed(1)
    for _ in range(40):
        o, r, term, trunc, info = env.step(torch.rand(n, 6, generator=g, device="cuda") * 2 - 1)
        dist = (o["achieved_goal"] - o["desired_goal"]).norm(dim=1)
        ok = ~info["_final_observation"] if "_final_observation" in info else torch.ones_like(term)
        assert torch.equal(r[ok], torch.where(dist[ok] < 0.01, 0.0, -1.0))
    torch.cuda.synchronize()
    assert torch.isfinite(env.qpos).all() and torch.isfinite(env.qvel).all()
    assert torch.allclose(o["observation"][:, :3], o["achieved_goal"])
    assert (env.total_steps == 40).all()
    env.close()


@pytest.mark.parametrize("solver", ["newton", "pgs"])
def test_domain_randomization_config4_shard(solver):
    """configs[4] shard (32,768 DR envs over 4 GPUs = 8,192 per GPU): the shard at env_offset 8,192 draws
    the same per-env parameters and runs the same trajectories as those envs of a 16,384-env run."""
    from gym_so100 import SO100VecEnv
    dr = dict(mass=(0.8, 1.2), friction=(0.8, 1.2), action_noise=0.05)
    full = SO100VecEnv(16384, device="cuda:0", seed=6, domain_randomization=dr, solver=solver)
    shard = SO100VecEnv(8192, device="cuda:0", seed=6, domain_randomization=dr, env_offset=8192, solver=solver)
    full.reset(seed=[5000 + i for i in range(16384)])
    shard.reset(seed=[5000 + 8192 + i for i in range(8192)])
    assert torch.equal(full.dr_params[8192:], shard.dr_params)
    g = torch.Generator(device="cuda").manual_seed(2)
    for _ in range(10):
        a = torch.rand(16384, 6, generator=g, device="cuda") * 2 - 1
        full.step(a)
        shard.step(a[8192:].contiguous())
    torch.cuda.synchronize()
    assert torch.equal(full.qpos[8192:], shard.qpos)
    assert torch.isfinite(full.qpos).all()
    full.close()
    shard.close()


def _arm_contact_parity(solver, oracle64, oracle32, p0, p1, label, seed):
    """random arm configurations with a contact in pairs [p0, p1), the actuators holding them;
    teacher-forced GPU steps at the fp32 floor"""
    from gym_so100 import SO100VecEnv
    from gym_so100.model import build_model
    PAIR_SELF0, PAIR_BASE0 = p0, p1
    model = build_model(solver=solver)
    rng = np.random.default_rng(seed)
    lo_j = np.array([r[0] for r in model.jnt_range]); hi_j = np.array([r[1] for r in model.jnt_range])
    lo, hi = np.array(model.action_lo[:]), np.array(model.action_hi[:])
    d = oracle64.new_data()
    states, targets = [], []
    # 48 states: folded arms are chaotic (two fp32 runs of the MPR collider settle on different portals in
    # deep overlaps), so the quantiles of 24 states were noise-dominated (GPU / fp32-oracle median ratio
    # 2.7 on 24 states, 1.3 on 192: tests/dev/padlink_err.py)
    while len(states) < 48:
        arm = rng.uniform(lo_j, hi_j)
        oracle64.reset(model, d, np.array([0.4, 0.95, 0.6, 1, 0, 0, 0]))
        for k in range(6):
            d.qpos[k] = arm[k]
        oracle64.call("so100o_fwd_position", model, d)
        if any(PAIR_SELF0 <= d.con[i].pair < PAIR_BASE0 for i in range(d.ncon)) and not d.ncon_dropped:
            q, v, w, _ = oracle64.get_state(d)
            states.append((q, v * 0, w * 0))
            targets.append(np.clip((arm - lo) / (hi - lo) * 2 - 1, -1, 1))
    n = len(states)
    env = SO100VecEnv(n, device="cuda:0", autoreset=False, max_episode_steps=0, debug=True, solver=solver)
    env.reset(seed=3)
    env.set_state(np.array([s[0] for s in states], np.float32), np.array([s[1] for s in states], np.float32),
                  np.array([s[2] for s in states], np.float32))
    d64, d32 = oracle64.new_data(), oracle32.new_data()
    qv_err, qv_floor, self_con = [], [], []
    for step in range(3):
        q0 = env.qpos.cpu().numpy().astype(np.float64)
        v0 = env.qvel.cpu().numpy().astype(np.float64)
        w0 = env.qacc_warmstart.cpu().numpy().astype(np.float64)
        act = (np.array(targets) + rng.normal(0, 0.02, (n, 6))).astype(np.float32)
        env.step(torch.from_numpy(act).cuda())
        torch.cuda.synchronize()
        gv = env.qvel.cpu().numpy()
        dbg = env.debug.cpu().numpy()
        for i in range(n):
            pairs = dbg[i, 48:48 + int(dbg[i, 0])]
            self_con.append(int(((pairs >= PAIR_SELF0) & (pairs < PAIR_BASE0)).sum()))
            oracle64.set_state(d64, q0[i], v0[i], w0[i])
            oracle32.set_state(d32, q0[i], v0[i], w0[i])
            oracle64.env_step(model, d64, 0, act[i])
            oracle32.env_step(model, d32, 0, act[i])
            ov = oracle64.get_state(d64)[1]
            qv_err.append((np.abs(ov - gv[i]) / (1 + np.abs(ov))).max())
            qv_floor.append((np.abs(ov - oracle32.get_state(d32)[1]) / (1 + np.abs(ov))).max())
    qv_err, qv_floor, self_con = np.array(qv_err), np.array(qv_floor), np.array(self_con)
    print(f"\n[{solver}] {label}: GPU {label} contacts per env mean {self_con.mean():.2f} (envs with any: "
          f"{(self_con > 0).mean():.2f}) | qvel rel GPU median {np.median(qv_err):.2e} p90 "
          f"{np.quantile(qv_err, .9):.2e} max {qv_err.max():.2e} | fp32 floor median {np.median(qv_floor):.2e} "
          f"p90 {np.quantile(qv_floor, .9):.2e} max {qv_floor.max():.2e}")
    assert (self_con[:n] > 0).mean() > 0.5
    # the error distribution is bimodal (states with and without chaotic deep overlaps, ~3e-3 and ~2e-4), so a
    # median falls between the modes and moves with fp32 rounding: the floor's median on the same test came
    # out 2.7e-4 and 8.0e-5 for two GPU builds differing only in FK rounding (384-state runs of
    # tests/dev/padlink_err.py: GPU / fp32-oracle medians 0.6-1.4 per mode).  Bar: the GPU's median within
    # the fp32 restatement's upper quartile
    assert np.median(qv_err) <= 2 * np.quantile(qv_floor, 0.75) + 1e-5
    assert np.mean(qv_err > 1e-4) <= 1.5 * np.mean(qv_floor > 1e-4) + 0.05    # tail mass (MPR: see above)
    # the 95th percentile, not the maximum: in these deep overlaps a single state's two fp32 runs (GPU and
    # fp32 oracle) can settle on different MPR portals, so the maxima of 144 samples are single outliers
    # (pad-link, Newton: GPU max 0.33 vs the fp32 oracle's 0.08 with equal medians, 3.1e-3 / 3.4e-3)
    assert np.quantile(qv_err, 0.95) <= 2 * np.quantile(qv_floor, 0.95) + 1e-3
    env.close()


@pytest.mark.parametrize("solver", ["newton", "pgs"])
def test_self_collision_parity(solver, oracle64, oracle32):
    """Hull-hull self-collision (pairs 77..97): random arm configurations whose
    non-adjacent links overlap, the actuators holding them; teacher-forced GPU steps at the fp32 floor."""
    from gym_so100.model import PAIR_SELF0, PAIR_BASE0
    _arm_contact_parity(solver, oracle64, oracle32, PAIR_SELF0, PAIR_BASE0, "self-collision", 17)


@pytest.mark.parametrize("solver", ["newton", "pgs"])
def test_base_contact_parity(solver, oracle64, oracle32):
    """Link hulls against the static Base's hull (pairs 99..106 through MPR): random arm
    configurations folded into the Base, the actuators holding them; teacher-forced GPU steps."""
    from gym_so100.model import PAIR_BASE0, PAIR_PADLINK0
    _arm_contact_parity(solver, oracle64, oracle32, PAIR_BASE0, PAIR_PADLINK0, "Base", 19)


@pytest.mark.parametrize("solver", ["newton", "pgs"])
def test_pad_link_contact_parity(solver, oracle64, oracle32):
    """The finger pads against the arm's own link hulls (pairs 107..142 through MPR, round 2; with them
    the pair table is every pair MuJoCo's filters leave): random arm configurations folding a jaw onto a
    link, the actuators holding them; teacher-forced GPU steps at the fp32 floor."""
    from gym_so100.model import PAIR_PADLINK0, PAIR_PAD0
    _arm_contact_parity(solver, oracle64, oracle32, PAIR_PADLINK0, PAIR_PAD0, "pad-link", 23)


@pytest.mark.parametrize("solver", ["newton", "pgs"])
def test_cube_on_base_parity(solver, oracle64, oracle32):
    """The cube resting on the static Base (pair 98, box vs the Base hull through MPR, one contact):
    states made by the fp64 oracle dropping the cube onto the Base top, then teacher-forced GPU steps."""
    from gym_so100 import SO100VecEnv
    from gym_so100.model import PAIR_BASE0, build_model
    model = build_model(solver=solver)
    rng = np.random.default_rng(23)
    d = oracle64.new_data()
    states = []
    for i in range(16):
        dx, dy = rng.uniform(-0.02, 0.02, 2)
        q = np.array([1, 0, 0, rng.uniform(-0.3, 0.3)])
        oracle64.reset(model, d, np.array([-0.469 + dx, 0.5 + dy, 0.12, *(q / np.linalg.norm(q))]))
        for _ in range(300):
            oracle64.call("so100o_substep", model, d)
        states.append(oracle64.get_state(d)[:3])
    n = len(states)
    start = np.array([-1.0 + 2.0 * (model.start_qpos[k] - model.action_lo[k]) / (model.action_hi[k] - model.action_lo[k])
                      for k in range(6)], np.float32)
    env = SO100VecEnv(n, device="cuda:0", autoreset=False, max_episode_steps=0, debug=True, solver=solver)
    env.reset(seed=3)
    env.set_state(np.array([s[0] for s in states], np.float32), np.array([s[1] for s in states], np.float32),
                  np.array([s[2] for s in states], np.float32))
    d64, d32 = oracle64.new_data(), oracle32.new_data()
    qv_err, qv_floor, base_con = [], [], []
    for step in range(4):
        q0 = env.qpos.cpu().numpy().astype(np.float64)
        v0 = env.qvel.cpu().numpy().astype(np.float64)
        w0 = env.qacc_warmstart.cpu().numpy().astype(np.float64)
        act = np.tile(start, (n, 1))
        env.step(torch.from_numpy(act).cuda())
        torch.cuda.synchronize()
        gv = env.qvel.cpu().numpy()
        dbg = env.debug.cpu().numpy()
        for i in range(n):
            pairs = dbg[i, 48:48 + int(dbg[i, 0])]
            base_con.append(int((pairs == PAIR_BASE0).sum()))
            oracle64.set_state(d64, q0[i], v0[i], w0[i])
            oracle32.set_state(d32, q0[i], v0[i], w0[i])
            oracle64.env_step(model, d64, 0, act[i])
            oracle32.env_step(model, d32, 0, act[i])
            ov = oracle64.get_state(d64)[1]
            qv_err.append((np.abs(ov - gv[i]) / (1 + np.abs(ov))).max())
            qv_floor.append((np.abs(ov - oracle32.get_state(d32)[1]) / (1 + np.abs(ov))).max())
    qv_err, qv_floor, base_con = np.array(qv_err), np.array(qv_floor), np.array(base_con)
    print(f"\n[{solver}] cube on Base: GPU cube-Base contacts per env mean {base_con.mean():.2f} | qvel rel GPU "
          f"median {np.median(qv_err):.2e} p90 {np.quantile(qv_err, .9):.2e} max {qv_err.max():.2e} | fp32 floor "
          f"median {np.median(qv_floor):.2e} p90 {np.quantile(qv_floor, .9):.2e} max {qv_floor.max():.2e}")
    assert (base_con > 0).mean() > 0.8                     # the cube really rests on the Base
    assert np.median(qv_err) <= 2 * np.median(qv_floor) + 1e-5
    assert np.quantile(qv_err, 0.9) <= 2 * np.quantile(qv_floor, 0.9) + 1e-4
    assert qv_err.max() <= 2 * qv_floor.max() + 1e-3
    env.close()


@pytest.mark.parametrize("fused", [False, True])
def test_step_graph_replay_matches_eager(monkeypatch, fused):
    """so100_step replays a captured hipGraph of the step (split: the chunk fork/join included; fused: the
    one launch); SO100_GRAPH=0 launches eagerly.  Both must give bit-identical trajectories, across
    re-captures (new action buffer, flags)."""
    import torch
    from gym_so100 import SO100VecEnv
    n = 4096                                        # 4 chunks: the forked streams are captured too
    monkeypatch.setenv("SO100_GRAPH", "0")
    eager = SO100VecEnv(n, max_episode_steps=7, seed=3)
    monkeypatch.setenv("SO100_GRAPH", "1")
    graph = SO100VecEnv(n, max_episode_steps=7, seed=3)
    for e in (eager, graph):
        e.fused = fused
    assert eager.chunk_info()[0] == (1 if fused else 4)
    eager.reset(seed=9)
    graph.reset(seed=9)
    g = torch.Generator().manual_seed(1)
    other = torch.zeros(n, 6, device="cuda:0")
    for t in range(20):
        act = (torch.rand(n, 6, generator=g) * 2 - 1).cuda()
        if t == 10:                                 # a different action buffer: the graph is re-captured
            other.copy_(act)
            graph.set_action_buffer(other)
            eager.set_action_buffer(other)
        for e in (eager, graph):
            if t >= 10:
                e.step_async_raw()
            else:
                e.step(act)
        torch.cuda.synchronize()
        for name in ("qpos", "qvel", "qacc_warmstart", "obs", "reward", "terminated", "truncated", "elapsed", "episode"):
            assert torch.equal(getattr(eager, name), getattr(graph, name)), (t, name)


@pytest.mark.parametrize("solver", ["newton", "pgs"])
def test_ee_weld_parity(solver, oracle64, oracle32):
    """EE / mocap variant (so100_transfer_cube_ee.xml): per-env mocap targets within 4 cm and
    0.4 rad of the end effector's start frame; teacher-forced against the fp64 oracle, fp32-oracle bars."""
    from scipy.spatial.transform import Rotation
    from gym_so100 import SO100VecEnv
    from gym_so100.model import build_model
    model = build_model(solver=solver, variant="ee")
    n = 32
    venv = SO100VecEnv(n, device="cuda:0", autoreset=False, max_episode_steps=0, solver=solver, variant="ee")
    venv.reset(seed=77)
    torch.cuda.synchronize()
    d = oracle64.new_data()
    q0 = venv.qpos.cpu().numpy().astype(np.float64)
    rng = np.random.default_rng(5)
    mocap = np.zeros((n, 7))
    for i in range(n):
        oracle64.set_state(d, q0[i], np.zeros(12), np.zeros(12))
        oracle64.call("so100o_fwd_position", model, d)
        R = np.array(d.xmat[6][:]).reshape(3, 3)
        rot = Rotation.from_rotvec(rng.uniform(-0.4, 0.4, 3)) * Rotation.from_matrix(R)
        mocap[i, :3] = np.array(d.site_ee[:]) + rng.uniform(-0.04, 0.04, 3)
        mocap[i, 3:] = rot.as_quat()[[3, 0, 1, 2]]
    qp, qv, rew_bad, bit_bad, states = _teacher_forced(venv, model, oracle64, steps=30, seed=77, mocap=mocap)
    ee_gap = np.linalg.norm(venv.obs[:, 6:9].cpu().numpy() - mocap[:, :3], axis=1)
    venv.close()
    fqp, fqv = _oracle_precision_floor(model, oracle64, oracle32, states)
    print(f"\n[ee {solver}] qvel rel median {np.median(qv):.2e} p90 {np.quantile(qv, .9):.2e} max {qv.max():.2e}"
          f" (fp32 floor median {np.median(fqv):.2e} p90 {np.quantile(fqv, .9):.2e} max {fqv.max():.2e});"
          f" ee-target gap after 30 steps: median {np.median(ee_gap):.3f} m")
    assert np.median(qp) <= 1e-5 and np.median(qv) <= 1e-5
    assert np.quantile(qv, 0.9) <= 2 * np.quantile(fqv, 0.9) + 1e-4
    assert qv.max() <= 2 * fqv.max() + 1e-3
    assert np.median(ee_gap) < 0.04
