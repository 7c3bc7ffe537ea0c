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
# Every physics parity test below steps the kernels the product launches: the fused step's product builds
# (so100_fused_kernel<false, 2> and <false, 3>, include/so100.h so100_set_fused_build) and the split path,
# each from the same state with the debug buffer off, and then the debug build (so100_fused_kernel<true>),
# whose record gives the contact list, the per-contact forces and qacc.  The product kernels must equal the
# debug build bit for bit (state, reward, contact bits, dropped contacts), so the oracle comparisons grade the
# product path.  PGS runs split only (debug off vs on).
F_FLOOR = 1e-3        # N: floor of the per-contact force-error denominator (the cube weighs 0.49 N)
# m: a contact this close to zero depth (2 fp32 ulps of a 0.7 m coordinate) is a tie fp32 cannot resolve as fp64
# does: the GPU may see the point on the other side of the surface and drop (or add) the contact
NEAR0 = 1e-7


def _set_mocap(d, mocap):
    for k in range(3):
        d.mocap_pos[k] = float(mocap[k])
    for k in range(4):
        d.mocap_quat[k] = float(mocap[3 + k])


def _step_all_builds(env, act):
    """One env step from the env's current state through every product kernel and the debug build (see
    above); asserts bitwise equality and leaves the env in the stepped state.  Returns numpy (reward,
    contact_bits, ncon_dropped, debug record) of the step and the builds that ran."""
    a = torch.as_tensor(act, dtype=torch.float32).cuda()
    s0 = [t.clone() for t in (env.qpos, env.qvel, env.qacc_warmstart, env.elapsed, env.episode)]
    modes = [("fused", 2), ("fused", 3), ("split", 0)] if env.solver == "newton" else [("split", 0)]
    outs = []
    for kind, w in modes:
        env.set_state(*s0)
        env.debug_enabled = False
        env.fused = kind == "fused"
        env.fused_build = w
        if kind == "fused":
            assert env.fused and env.fused_build == w
        _, r, _, _, info = env.step(a)
        outs.append((f"{kind}{w or ''}", [t.clone() for t in (env.qpos, env.qvel, env.qacc_warmstart, r,
                                                               info["contact_bits"], info["ncon_dropped"])]))
    env.set_state(*s0)
    env.debug_enabled = True
    env.fused = None
    env.fused_build = 0
    if env.solver == "newton":
        assert env.fused and env.fused_build == 1          # the debug build
    _, r, _, _, info = env.step(a)
    ref = (env.qpos, env.qvel, env.qacc_warmstart, r, info["contact_bits"], info["ncon_dropped"])
    torch.cuda.synchronize()
    for name, o in outs:
        for k, (x, y) in enumerate(zip(o, ref)):
            assert torch.equal(x, y), (name, ("qpos", "qvel", "warmstart", "reward", "contact_bits", "ncon_dropped")[k])
    return (r.cpu().numpy(), info["contact_bits"].cpu().numpy().astype(np.uint32), info["ncon_dropped"].cpu().numpy(),
            env.debug.cpu().numpy(), [n for n, _ in outs])


def _gpu_solve(dbg_row):
    """(pairs, forces [ncon, 4], dof frictionloss forces, qacc) of the last solve from a debug record row
    (include/so100.h SO100_DBG_STRIDE layout: contacts 0..15 in the fixed fields, the rest of the list from
    SO100_DBG_OVF, 6 floats each)."""
    from gym_so100._native import SO100_DBG_OVF
    nc = int(dbg_row[0])
    n0 = min(nc, 16)
    f = np.zeros((nc, 4))
    pairs = np.zeros(nc, np.int64)
    f[:n0, 0] = dbg_row[32:32 + n0]
    f[:n0, 1:] = dbg_row[96:96 + 3 * 16].reshape(16, 3)[:n0]
    pairs[:n0] = dbg_row[48:48 + n0]
    if nc > 16:
        ov = dbg_row[SO100_DBG_OVF:SO100_DBG_OVF + 6 * (nc - 16)].reshape(nc - 16, 6)
        pairs[16:] = ov[:, 1]
        f[16:] = ov[:, 2:6]
    return pairs, f, dbg_row[76:88].astype(np.float64), dbg_row[4:16].astype(np.float64)


def _force_err(f, fo):
    """per-contact relative force error ||f - fo|| / max(||fo||, F_FLOOR)"""
    return np.linalg.norm(f - fo, axis=1) / np.maximum(np.linalg.norm(fo, axis=1), F_FLOOR)


def _rel(a, o):
    return (np.abs(a - o) / (1 + np.abs(o))).max()


class TF:
    """Results of teacher-forced steps: per env step the GPU's (product-kernel) error against the fp64
    oracle, and two floors on the same states: the fp32 oracle's error (the precision floor of the same
    algorithm in fp32) and the fp64 oracle's own response to a perturbation of its input state by one fp32
    rounding (relative N(0, 2^-24) on qpos and qvel: the problem's conditioning, which no fp32 implementation
    can beat and which bounds MuJoCo itself on fp32-rounded state).  Errors: qpos (abs), qvel and qacc (rel to
    1+|v|), per-contact forces (relative, contacts matched in order where both contact lists agree); plus the
    contact lists, dropped-contact counts, reward and contact-bit mismatches."""

    def __init__(self):
        self.qp, self.qv, self.fqp, self.fqv, self.qa, self.fqa = [], [], [], [], [], []
        # the ensemble floor (_tf_run ens=True): per env step the errors of ENS64 independent 1-ulp input perturbations
        # through the fp64 oracle and ENS32 more through the fp32 restatement, qvel and qacc [steps, ENS64 + ENS32] (fp64
        # members first), and the members' contact forces (lists equal to the fp64 oracle's).  A fixed budget per
        # state, run before and independently of the GPU's result: nothing in a floor depends on the error it grades
        self.eqv, self.eqa, self.eforce = [], [], []
        # (ens > 0) the fp32 restatement compiled with FMA contraction, as the GPU compiler contracts: a second fp32
        # rounding of the same algorithm, qvel and qacc per env step
        self.mqv, self.mqa = [], []
        self.pqv, self.pqa, self.pforce, self.psame = [], [], [], []
        self.force, self.fforce, self.same, self.fsame, self.pairs = [], [], [], [], []
        self.drop_gpu, self.drop_ora = [], []
        self.near0 = []       # the fp64 oracle's first position stage holds a contact at |dist| < NEAR0
        self.rew_bad = self.bit_bad = 0
        self.states = []
        self.builds = None

    def arrays(self):
        for k in ("qp", "qv", "fqp", "fqv", "qa", "fqa", "pqv", "pqa", "pforce", "psame", "force", "fforce", "same",
                  "fsame", "drop_gpu", "drop_ora", "near0", "eqv", "eqa", "eforce", "mqv", "mqa"):
            setattr(self, k, np.array(getattr(self, k)))
        return self

    def floor(self, name, q):
        """the largest of the floors' q-quantile (q = 1: maximum) for qv / qa / force: the fp32 restatement, the
        single 1-ulp perturbation and, where it ran, the ensemble of K perturbations"""
        f = {"qv": (self.fqv, self.pqv, self.eqv), "qa": (self.fqa, self.pqa, self.eqa),
             "force": (self.fforce, self.pforce, self.eforce)}[name]
        return max(np.quantile(np.ravel(x), q) if np.size(x) else 0.0 for x in f)

    def summary(self, label):
        q = lambda x, p: np.quantile(x, p) if len(x) else float("nan")
        trio = lambda x: f"{q(x, .5):.2e} / {q(x, .9):.2e} / {q(x, 1.0):.2e}"
        f = self.force
        return (f"[{label}] {len(self.qv)} env-steps (kernels {'/'.join(self.builds)} == debug build, bitwise) | "
                f"median / p90 / max: qvel rel GPU {trio(self.qv)} (fp32 oracle {trio(self.fqv)}; fp64 under a 1-ulp "
                f"input perturbation {trio(self.pqv)}), within 1e-4: {np.mean(self.qv < 1e-4):.3f} | qacc rel GPU "
                f"{trio(self.qa)} (floors {trio(self.fqa)}; {trio(self.pqa)}) | contact forces: {len(f)} contacts in "
                f"{self.same.mean():.3f} of steps with equal lists (fp32 oracle {self.fsame.mean():.3f}, perturbed fp64 "
                f"{self.psame.mean():.3f}), rel GPU {trio(f)} (floors {trio(self.fforce)}; {trio(self.pforce)}), within "
                f"1e-4: {np.mean(f < 1e-4) if len(f) else float('nan'):.3f} | dropped contacts GPU "
                f"{int(self.drop_gpu.sum())} oracle {int(self.drop_ora.sum())}")


def _tf_run(env, model, o64, o32, steps, act_fn, task=0, mocap=None, res=None, ens=False):
    """Teacher-forced steps: each starts the product kernels, the debug build and both oracles from the
    GPU's fp32 state (act_fn(step) -> [n, 6] float32 actions).  ens: also the ensemble floor (TF.eqv / eqa), ENS64
    independent 1-ulp perturbations of each state through the fp64 oracle and ENS32 through the fp32 restatement, and
    the FMA-contracted fp32 restatement on the state itself (TF.mqv / mqa).  The floors of a state are computed from
    the oracle runs alone, before the GPU's result is read."""
    res = res or TF()
    n = env.num_envs
    d64, d32, dp, dq = o64.new_data(), o32.new_data(), o64.new_data(), o64.new_data()
    prng = np.random.default_rng(12345)
    erng = np.random.default_rng(777)

    def setm(d, i):
        if mocap is not None:
            _set_mocap(d, mocap[i])

    def perturbed(i, q0, v0):
        return q0[i] * (1 + erng.normal(0, 2.0 ** -24, 13)), v0[i] * (1 + erng.normal(0, 2.0 ** -24, 12))

    for step in range(steps):
        q0 = env.qpos.cpu().numpy().astype(np.float64)
        v0 = env.qvel.cpu().numpy().astype(np.float64)
        w0 = env.qacc_warmstart.cpu().numpy().astype(np.float64)
        act = np.asarray(act_fn(step), np.float32)
        # the oracle side of every state first: the fp64 answer and every floor (single runs and the ensemble)
        ora = []
        for i in range(n):
            for o, d in ((o64, d64), (o32, d32)):
                o.set_state(d, q0[i], v0[i], w0[i])
                setm(d, i)
            o64.set_state(dp, q0[i] * (1 + prng.normal(0, 2.0 ** -24, 13)), v0[i] * (1 + prng.normal(0, 2.0 ** -24, 12)),
                          w0[i])
            setm(dp, i)
            o64.set_state(dq, q0[i], v0[i], w0[i])
            setm(dq, i)
            o64.call("so100o_fwd_position", model, dq)
            near0 = any(abs(dq.con[c].dist) < NEAR0 for c in range(dq.ncon))
            _, r, _ = o64.env_step(model, d64, task, act[i])
            o32.env_step(model, d32, task, act[i])
            o64.env_step(model, dp, task, act[i])
            oq, ov = o64.get_state(d64)[:2]
            fq, fv = o32.get_state(d32)[:2]
            s64, s32, sp = o64.last_solve(d64), o32.last_solve(d32), o64.last_solve(dp)
            o_ = dict(r=r, oq=oq, ov=ov, fq=fq, fv=fv, bits=o64.contact_bits(d64), s64=s64, s32=s32, sp=sp,
                      pv=o64.get_state(dp)[1], near0=near0)
            if ens:
                eq, ea, ef = [], [], []
                for _ in range(ENS64):
                    qp, vp = perturbed(i, q0, v0)
                    o64.set_state(dp, qp, vp, w0[i])
                    setm(dp, i)
                    o64.env_step(model, dp, task, act[i])
                    pe, fe, _, qae, _ = o64.last_solve(dp)
                    eq.append(_rel(o64.get_state(dp)[1], ov))
                    ea.append(_rel(qae, s64[3]))
                    if np.array_equal(pe, s64[0]) and len(pe):
                        ef += list(_force_err(fe, s64[1]))
                # fp32 rounding's own discrete flips (an EPA face-face witness, whose tie between coplanar facets fp32
                # breaks either way while fp64 resolves it one way) on this state
                for _ in range(ENS32):
                    qp, vp = perturbed(i, q0, v0)
                    o32.set_state(d32, qp, vp, w0[i])
                    setm(d32, i)
                    o32.env_step(model, d32, task, act[i])
                    eq.append(_rel(o32.get_state(d32)[1], ov))
                    pe, fe, _, qae, _ = o32.last_solve(d32)
                    ea.append(_rel(qae, s64[3]))
                    if np.array_equal(pe, s64[0]) and len(pe):
                        ef += list(_force_err(fe, s64[1]))
                om = _oracle32fma()
                dm = om.new_data()
                om.set_state(dm, q0[i], v0[i], w0[i])
                setm(dm, i)
                om.env_step(model, dm, task, act[i])
                o_.update(eq=eq, ea=ea, ef=ef, mqv=_rel(om.get_state(dm)[1], ov), mqa=_rel(om.last_solve(dm)[3], s64[3]))
            ora.append(o_)
        # then the GPU, graded against them
        gr, gb, gdrop, dbg, res.builds = _step_all_builds(env, act)
        gq, gv = env.qpos.cpu().numpy(), env.qvel.cpu().numpy()
        for i, o_ in enumerate(ora):
            p64, f64, fr64, qa64, nd64 = o_["s64"]
            p32, f32, fr32, qa32, _ = o_["s32"]
            pp, fp, _, qap, _ = o_["sp"]
            ov = o_["ov"]
            res.near0.append(o_["near0"])
            res.qp.append(np.abs(o_["oq"] - gq[i]).max())
            res.qv.append(_rel(gv[i], ov))
            res.fqp.append(np.abs(o_["oq"] - o_["fq"]).max())
            res.fqv.append(_rel(o_["fv"], ov))
            res.rew_bad += abs(o_["r"] - gr[i]) > 1e-6
            res.bit_bad += o_["bits"] != gb[i]
            gp, gf, gfr, gqa = _gpu_solve(dbg[i])
            res.pqv.append(_rel(o_["pv"], ov))
            res.qa.append(_rel(gqa, qa64))
            res.fqa.append(_rel(qa32, qa64))
            res.pqa.append(_rel(qap, qa64))
            res.fsame.append(np.array_equal(p32, p64))
            res.psame.append(np.array_equal(pp, p64))
            if np.array_equal(pp, p64) and len(pp):
                res.pforce += list(_force_err(fp, f64))
            res.pairs.append(gp)
            res.drop_gpu.append(int(gdrop[i]))
            res.drop_ora.append(nd64)
            same = np.array_equal(gp, p64)
            res.same.append(same)
            if same and np.array_equal(p32, p64) and len(gp):
                res.force += list(_force_err(gf, f64))
                res.fforce += list(_force_err(f32, f64))
            res.states.append((q0[i], v0[i], w0[i], act[i]) + ((mocap[i],) if mocap is not None else ()))
            if ens:
                res.eqv.append(o_["eq"])
                res.eqa.append(o_["ea"])
                res.eforce += o_["ef"]
                res.mqv.append(o_["mqv"])
                res.mqa.append(o_["mqa"])
    return res


_O32FMA = []


def _oracle32fma():
    if not _O32FMA:
        from oracle.oracle import Oracle
        _O32FMA.append(Oracle(32, fma=True))
    return _O32FMA[0]


def _new_env(n, solver, **kw):
    from gym_so100 import SO100VecEnv
    return SO100VecEnv(n, device="cuda:0", autoreset=False, max_episode_steps=0, debug=True, solver=solver, **kw)


def _set_states(env, states):
    env.set_state(np.array([s[0] for s in states], np.float32), np.array([s[1] for s in states], np.float32),
                  np.array([s[2] for s in states], np.float32))


def _force_bars(r, median_abs=None):
    """contact-force and qacc bars at the floors (the larger of the fp32 restatement's error and the fp64
    oracle's response to a 1-ulp input perturbation, TF): the GPU's median within 2x the floor's median
    (+1e-6), its p90 within 2x the floor's p90 (+1e-4); optionally an absolute median bar"""
    if len(r.force):
        assert np.median(r.force) <= 2 * r.floor("force", 0.5) + 1e-6
        assert np.quantile(r.force, 0.9) <= 2 * r.floor("force", 0.9) + 1e-4
        if median_abs is not None:
            assert np.median(r.force) <= median_abs
    assert np.median(r.qa) <= 2 * r.floor("qa", 0.5) + 1e-6
    assert np.quantile(r.qa, 0.9) <= 2 * r.floor("qa", 0.9) + 1e-4
    if len(r.force):
        # the force tail (which the median / p90 bars above leave unbounded): the share of contacts off by more than
        # 1e-4 against the floors' share; and, where the ensemble floor ran (its fp32 members' forces sample fp32
        # rounding's own spread of a contact's force, which one fp32 run cannot: PGS stopped at 100 sweeps on resting
        # contacts splits the force among redundant contacts by rounding), the p99 against the floors' p99
        share = lambda x: np.mean(np.asarray(x) > 1e-4) if np.size(x) else 0.0
        fshare = max(share(r.fforce), share(r.pforce), share(r.eforce))
        assert share(r.force) <= 1.5 * fshare + 0.03, (share(r.force), fshare)
        if len(r.eqv):
            assert np.quantile(r.force, 0.99) <= 2 * r.floor("force", 0.99) + 1e-3, (np.quantile(r.force, 0.99),
                                                                                      r.floor("force", 0.99))


@pytest.mark.parametrize("solver", ["newton", "pgs"])
def test_step_parity_teacher_forced(solver, oracle64, oracle32):
    """Random-action rollouts from RandomState spawns (the bench's workload): per step qpos / qvel / qacc and
    the per-contact forces of the GPU's product kernels against the fp64 oracle (north_star: 'per-step
    qpos/qvel/contact forces match CPU MuJoCo within 1e-4 rel'), at the fp32 floor."""
    from gym_so100.model import build_model
    model = build_model(solver=solver)
    env = _new_env(64, solver)
    env.reset(seed=1000)
    rng = np.random.default_rng(1000)
    act_fn = lambda step: (rng.uniform(-1, 1, (64, 6)) if step % 20 < 10 else np.clip(rng.normal(0, 0.3, (64, 6)), -1, 1))
    r = _tf_run(env, model, oracle64, oracle32, 40, act_fn).arrays()
    env.close()
    print("\n" + r.summary(f"{solver} random actions"))
    n = len(r.qv)
    assert np.median(r.qp) <= 1e-5 and np.median(r.qv) <= 1e-5
    assert np.quantile(r.qv, 0.9) <= 2 * r.floor("qv", 0.9) + 1e-4
    assert np.quantile(r.qv, 0.99) <= 2 * r.floor("qv", 0.99) + 1e-4
    assert r.qv.max() <= 2 * r.floor("qv", 1.0) + 1e-3
    assert np.mean(r.qv < 1e-4) >= min(np.mean(r.fqv < 1e-4), np.mean(r.pqv < 1e-4)) - 0.05
    assert r.rew_bad <= max(2, 0.005 * n)          # ladder flips only at contact on/off boundaries
    assert r.bit_bad <= max(4, 0.01 * n)
    # the last substep's contact list agrees with the fp64 oracle's as often as the fp32 oracle's does
    # (PGS: its 100-sweep truncation amplifies rounding within the step, so lists at dist ~ 0 flip)
    assert len(r.force) > 200 and r.same.mean() >= min(r.fsame.mean(), r.psame.mean()) - 0.03
    # north_star's 1e-4 at the median for the solver MuJoCo runs (PGS stops at 100 sweeps short of the
    # minimiser on resting contacts, so its forces carry the iteration error: floor bars only)
    _force_bars(r, median_abs=1e-4 if solver == "newton" else None)
    assert r.drop_gpu.sum() == 0 and r.drop_ora.sum() == 0


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
    # chunks belong to the split path (a fused step is one launch), whose workspaces are made when it is first
    # selected: while SO100_CHUNKS applies
    monkeypatch.setenv("SO100_CHUNKS", "1")
    one = SO100VecEnv(n, **kw)
    one.fused = False
    monkeypatch.setenv("SO100_CHUNKS", "4")
    four = SO100VecEnv(n, **kw)
    four.fused = False
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
    """PGS always runs split; auto mode (the default) runs fused at every size (65,536 envs included); the mode
    can be switched between steps (Newton), and the contact counter reads the record of the mode that ran."""
    from gym_so100 import SO100VecEnv
    big = SO100VecEnv(32768, device="cuda:0")
    assert big.fused and big.chunk_info() == (1, 32768)
    big.fused = False
    assert not big.fused and big.chunk_info()[0] == 4
    big.close()
    big = SO100VecEnv(65536, device="cuda:0")
    assert big.fused and big.chunk_info() == (1, 65536)
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
    on-chip slots -- exercises the streamed-overflow contacts, the J rows in LDS and the heavy-group first
    dispatch; per-contact forces against the oracle."""
    from gym_so100.model import build_model
    model = build_model(solver=solver)
    n = 32
    env = _new_env(n, solver)
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
    r = _tf_run(env, model, oracle64, oracle32, 3, lambda step: rng.uniform(-0.2, 0.2, (n, 6))).arrays()
    env.close()
    ncon = np.array([len(p) for p in r.pairs])
    print(f"\nGPU ncon mean {ncon.mean():.1f} max {ncon.max():.0f}; " + r.summary(f"{solver} heavy contacts"))
    assert (ncon > 4).mean() > 0.5 and ncon.max() > 8     # the overflow path and the LDS J rows really run
    assert np.median(r.qv) <= 2 * r.floor("qv", 0.5) + 1e-5
    assert np.quantile(r.qv, 0.9) <= 2 * r.floor("qv", 0.9) + 1e-4
    # the max over the env-steps without a zero-depth tie (a rotated cube's far corner exactly on a wall:
    # PGS, which does not converge on these redundant contacts in 100 sweeps, then distributes the forces
    # differently; Newton's minimiser is unique and needs no exclusion)
    keep = ~r.near0 if solver == "pgs" else np.ones(len(r.qv), bool)
    print(f"zero-depth ties (|dist| < {NEAR0} m at the first position stage): {int(r.near0.sum())} of {len(r.qv)}")
    assert keep.mean() >= 0.9
    assert r.qv[keep].max() <= 2 * r.floor("qv", 1.0) + 1e-3
    _force_bars(r)
    assert r.drop_gpu.sum() == 0 and r.drop_ora.sum() == 0


def _pressed_states(model, oracle64, n, rng, target_fn, cube_pose):
    """States made by the fp64 oracle driving the arm to target_fn(i) for 400 substeps (the cube parked at
    cube_pose); returns the states and the targets as normalised actions (keep pressing)."""
    d = oracle64.new_data()
    states, targets = [], []
    lo, hi = np.array(model.action_lo[:]), np.array(model.action_hi[:])
    for i in range(n):
        oracle64.reset(model, d, np.array(cube_pose))
        target = np.clip(target_fn(i), lo, hi)
        for k in range(6):
            d.ctrl[k] = target[k]
        for _ in range(400):
            oracle64.call("so100o_substep", model, d)
        q, v, w, _ = oracle64.get_state(d)
        states.append((q, v, w))
        targets.append((target - lo) / (hi - lo) * 2 - 1)
    return states, np.array(targets)


@pytest.mark.parametrize("solver", ["newton", "pgs"])
def test_hull_table_parity(solver, oracle64, oracle32):
    """Arm/jaw hulls resting on the table (pairs 14..22, condim 3): states made by the
    fp64 oracle driving the arm down onto the table, then teacher-forced GPU steps against it."""
    from gym_so100.model import NPAIR_BOX, PAIR_MPR0, build_model
    model = build_model(solver=solver)
    n = 24
    rng = np.random.default_rng(11)
    # the cube off the table: it falls clear, so no cube resting at dist ~ 0 (its contacts flip between precisions)
    states, targets = _pressed_states(model, oracle64, n, rng, lambda i: np.array(
        [rng.uniform(-0.6, 0.6), rng.uniform(0.6, 1.2), rng.uniform(-1.2, -0.6), rng.uniform(0.8, 1.5),
         rng.uniform(-1.5, 1.5), rng.uniform(-0.17, 1.0)]), [2.0, 0.95, 0.6, 1, 0, 0, 0])
    env = _new_env(n, solver)
    env.reset(seed=3)
    _set_states(env, states)
    r = _tf_run(env, model, oracle64, oracle32, 4, lambda step: targets + rng.normal(0, 0.02, (n, 6))).arrays()
    env.close()
    hull_con = np.array([int(((p >= NPAIR_BOX) & (p < PAIR_MPR0)).sum()) for p in r.pairs])
    same = r.same
    print(f"\nGPU hull contacts per env mean {hull_con.mean():.2f} (envs with any: {(hull_con > 0).mean():.2f}), "
          f"contact-list flips {(~same).sum()} of {len(same)}, contact-bit mismatches {r.bit_bad}; " +
          r.summary(f"{solver} hull-table"))
    assert (hull_con > 0).mean() > 0.5                 # the arm really rests on the table
    # a contact at dist ~ 0 can be in one precision's set and not the other's; PGS, unconverged at 100
    # sweeps on resting contacts, amplifies such a flip, so the tail bar applies to the states whose GPU
    # and oracle contact lists agree, and flips must stay rare
    assert (~same).mean() <= 0.1
    assert np.median(r.qv) <= 2 * r.floor("qv", 0.5) + 1e-5
    assert np.quantile(r.qv[same], 0.9) <= 2 * max(np.quantile(r.fqv[same], 0.9), np.quantile(r.pqv[same], 0.9)) + 1e-4
    # the maximum on the steps whose lists agree (round 6: the fp32 restatement no longer flips a contact on these
    # states, so its maximum stopped covering the GPU's own rare flips; a flip is bounded by the share bar above)
    assert r.qv[same].max() <= 2 * max(r.fqv[same].max(), r.pqv[same].max()) + 1e-3
    if (~same).any():
        print(f"flipped steps' qvel error: {np.sort(r.qv[~same])}")
    assert r.bit_bad <= max(2, 0.05 * len(r.qv))
    _force_bars(r)
    assert r.drop_gpu.sum() == 0 and r.drop_ora.sum() == 0


@pytest.mark.parametrize("solver", ["newton", "pgs"])
def test_pad_contact_parity(solver, oracle64, oracle32):
    """Finger pads against the table and the bin boxes (pairs 143..190, condim 3): states made
    by the fp64 oracle pressing the gripper onto the table top (two thirds of the envs) and into the bin (the
    rest), then teacher-forced GPU steps against it, with the pad contacts counted."""
    from gym_so100.model import PAIR_PAD0, build_model
    model = build_model(solver=solver)
    n = 24
    rng = np.random.default_rng(13)
    over_bin = np.array([[0.72, -0.89, 2.15, -1.24, -1.38, -0.05], [0.7, -0.91, 1.85, -0.39, -0.2, 0.33]])

    def target(i):
        if i % 3 < 2:
            return np.array([rng.uniform(-0.6, 0.6), rng.uniform(0.2, 1.3), rng.uniform(-1.4, -0.2),
                             rng.uniform(0.6, 1.6), rng.uniform(-1.5, 1.5), rng.uniform(-0.17, 1.5)])
        return over_bin[i % 2] + rng.normal(0, 0.12, 6) + np.array([0, 0.15, 0, 0, 0, 0])
    states, targets = _pressed_states(model, oracle64, n, rng, target, [0.4, 0.95, 0.6, 1, 0, 0, 0])
    env = _new_env(n, solver)
    env.reset(seed=3)
    _set_states(env, states)
    d64 = oracle64.new_data()
    r = _tf_run(env, model, oracle64, oracle32, 4, lambda step: targets + rng.normal(0, 0.02, (n, 6))).arrays()
    env.close()
    pad_gpu = np.array([int((p >= PAIR_PAD0).sum()) for p in r.pairs])
    pad_ora = []
    for st in r.states:                                  # the oracle's pad contacts of the same solves
        oracle64.set_state(d64, st[0], st[1], st[2])
        oracle64.env_step(model, d64, 0, st[3])
        pad_ora.append(int((oracle64.last_solve(d64)[0] >= PAIR_PAD0).sum()))
    pad_ora = np.array(pad_ora)
    print(f"\nGPU pad contacts per env mean {pad_gpu.mean():.2f} (envs with any: {(pad_gpu > 0).mean():.2f}; oracle "
          f"{pad_ora.mean():.2f}, count mismatches {(pad_gpu != pad_ora).sum()}); " + r.summary(f"{solver} pads"))
    assert (pad_gpu > 0).sum() >= 10                    # the pads really touch the table / bin
    assert (pad_gpu != pad_ora).mean() <= 0.05           # the same pad contact sets (fp32 flips at dist ~ 0 aside)
    assert np.median(r.qv) <= 2 * r.floor("qv", 0.5) + 1e-5
    assert np.quantile(r.qv, 0.9) <= 2 * r.floor("qv", 0.9) + 1e-4
    assert r.qv.max() <= 2 * r.floor("qv", 1.0) + 1e-3
    _force_bars(r)
    assert r.drop_gpu.sum() == 0 and r.drop_ora.sum() == 0


@pytest.mark.parametrize("solver,convex", [("newton", "epa"), ("pgs", "epa"), ("newton", "mpr"), ("pgs", "mpr")])
def test_mpr_contact_parity(solver, convex, oracle64, oracle32):
    """Box-hull contacts through the convex collider (pairs 23..76: the cube and the bin boxes against the
    arm/jaw hulls), GJK + EPA (MuJoCo 3.3.3's default) and libccd's MPR: states from fp64-oracle
    random-action rollouts that hold such contacts, then teacher-forced GPU steps against the oracle at the
    fp32 floor."""
    from gym_so100.model import PAIR_MPR0, PAIR_PAD0, NHULL, build_model
    model = build_model(solver=solver, convex=convex)
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
    env = _new_env(n, solver, convex=convex)
    env.reset(seed=3)
    _set_states(env, states)
    r = _tf_run(env, model, oracle64, oracle32, 3, lambda step: rng.uniform(-1, 1, (n, 6))).arrays()
    env.close()
    mpr_con = np.array([int(((p >= PAIR_MPR0) & (p < PAIR_PAD0)).sum()) for p in r.pairs])
    print(f"\n{n} envs, GPU convex contacts per env mean {mpr_con.mean():.2f} (envs with any: {(mpr_con > 0).mean():.2f}); "
          + r.summary(f"{solver} box-hull ({convex.upper()})"))
    assert (mpr_con[:n] > 0).mean() > 0.3              # the GPU collider sees the contacts too
    # MPR's fp32 branches (different portals) make the tail chaotic for ANY fp32 implementation: the
    # fp32 oracle and the GPU put their large deviations on different states, so the tail is compared by
    # its mass (share of env steps off by > 1e-4), not by a quantile of a 150-sample set
    assert np.median(r.qv) <= 2 * r.floor("qv", 0.5) + 1e-5
    assert np.mean(r.qv > 1e-4) <= 1.5 * max(np.mean(r.fqv > 1e-4), np.mean(r.pqv > 1e-4)) + 0.05
    assert r.qv.max() <= 2 * r.floor("qv", 1.0) + 1e-3
    if convex == "epa":
        _force_bars(r)
    else:
        # MPR's portal choice flips on a rounding, so which tenth of the contacts lands in the force tail changes
        # with any 1-ulp change of the trajectory: its tail is compared by mass, as qvel's above
        assert np.median(r.force) <= 2 * r.floor("force", 0.5) + 1e-6
        assert np.mean(r.force > 1e-4) <= 1.5 * max(np.mean(r.fforce > 1e-4), np.mean(r.pforce > 1e-4)) + 0.05
        assert np.median(r.qa) <= 2 * r.floor("qa", 0.5) + 1e-6
    assert r.drop_gpu.sum() == 0 and r.drop_ora.sum() == 0


def test_newton_solver_parity(oracle64, oracle32):
    """MuJoCo's default solver (primal Newton, solver="newton"): teacher-forced GPU steps against the fp64
    oracle's Newton from random-action rollout states (contacts on the table, bin, gripper and hulls),
    at the fp32 floor (the fp32 oracle's Newton on the same states); 2-6 Newton steps per substep."""
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
    env = _new_env(n, "newton")
    env.reset(seed=3)
    _set_states(env, states)
    iters = []

    def act_fn(step):
        if env.debug is not None and step > 0:
            iters.extend(env.debug.cpu().numpy()[:, 1])
        return rng.uniform(-1, 1, (n, 6))
    r = _tf_run(env, mn, oracle64, oracle32, 3, act_fn).arrays()
    iters.extend(env.debug.cpu().numpy()[:, 1])
    env.close()
    iters = np.array(iters)
    ncon = np.array([len(p) for p in r.pairs])
    print(f"\ncontacts/env {ncon.mean():.2f}, GPU Newton steps per substep mean {iters.mean():.2f} max {iters.max():.0f}; "
          + r.summary("newton rollout states"))
    assert ncon.mean() > 1.0
    assert iters.max() <= 30 and iters.mean() < 10
    assert np.median(r.qv) <= 2 * r.floor("qv", 0.5) + 1e-5
    assert np.quantile(r.qv, 0.9) <= 2 * r.floor("qv", 0.9) + 1e-4
    assert r.qv.max() <= 2 * r.floor("qv", 1.0) + 1e-3
    _force_bars(r, median_abs=1e-4)
    assert r.drop_gpu.sum() == 0 and r.drop_ora.sum() == 0


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


ENS64 = 8    # the ensemble floor: independent 1-ulp perturbations of each state through the fp64 oracle
ENS32 = 32   # ... and through the fp32 restatement


def _ensemble_bars(r, name="qv"):
    """The deep-fold gate (rounds 4-5): these states (links pushed centimetres into each other) are chaotic, so a
    single perturbation's maximum is a noisy bar that legal fp reorderings can cross.  The GPU's error distribution
    is graded against a floor computed per state from the oracles alone, with a fixed budget, before the GPU's result
    is read (_tf_run): ENS64 independent 1-ulp input perturbations through the fp64 oracle, ENS32 through the fp32
    restatement (fp32 rounding breaks discrete ties, e.g. an EPA face-face witness, that fp64 resolves one way), and
    the fp32 restatement host-compiled and FMA-contracted (the GPU's arithmetic; the contraction alone moves the fp32
    p99 up to 7x on these states, tools/dev/fp32_floor.py) on the state itself.  Bars: median, p90 and p99 within 2x
    the floor's (+1e-5 / 1e-4 / 1e-4); on the steps whose GPU and fp64 contact lists are equal, p99 within 2x the
    floor's on those steps (+1e-4); the tail mass (share off by more than 1e-4) within 1.5x the floor's (+0.03); and per
    state the GPU beyond every member of its own state (2x + 1e-5) at most as often as one member would be
    (1 / (members + 1))."""
    g = getattr(r, name)
    # the single fp32 runs: the restatement as compiled for the host and with FMA contraction (the GPU's arithmetic)
    f = np.maximum({"qv": r.fqv, "qa": r.fqa}[name], {"qv": r.mqv, "qa": r.mqa}[name])
    E = np.asarray({"qv": r.eqv, "qa": r.eqa}[name])
    assert E.shape[1] == ENS64 + ENS32
    fl = lambda q, m=slice(None): max(np.quantile(f[m], q), np.quantile(E[m].ravel(), q))
    assert np.median(g) <= 2 * fl(0.5) + 1e-5, (name, np.median(g), fl(0.5))
    assert np.quantile(g, 0.9) <= 2 * fl(0.9) + 1e-4, (name, np.quantile(g, 0.9), fl(0.9))
    assert np.quantile(g, 0.99) <= 2 * fl(0.99) + 1e-4, (name, np.quantile(g, 0.99), fl(0.99))
    same = np.asarray(r.same, bool)
    if same.sum() >= 10:
        assert np.quantile(g[same], 0.99) <= 2 * fl(0.99, same) + 1e-4, (name, np.quantile(g[same], 0.99), fl(0.99, same))
    tail = lambda x: np.mean(np.asarray(x) > 1e-4)
    assert tail(g) <= 1.5 * max(tail(f), tail(E.ravel())) + 0.03, (name, tail(g), tail(f), tail(E.ravel()))
    beyond = g > 2 * np.maximum(E.max(axis=1), f) + 1e-5
    assert beyond.mean() <= 1.0 / (E.shape[1] + 1), (name, beyond.mean())
    return beyond


def _arm_contact_parity(solver, oracle64, oracle32, p0, p1, label, seed, nsubstep=None, select=None):
    """random arm configurations with a contact in pairs [p0, p1) (or select(d)), the actuators holding them;
    teacher-forced GPU steps graded against the ensemble floor (_ensemble_bars) on qvel and qacc."""
    from gym_so100.model import build_model
    model = build_model(solver=solver, nsubstep=nsubstep)
    rng = np.random.default_rng(seed)
    lo_j = np.array([r[0] for r in model.jnt_range]); hi_j = np.array([r[1] for r in model.jnt_range])
    lo, hi = np.array(model.action_lo[:]), np.array(model.action_hi[:])
    d = oracle64.new_data()
    states, targets = [], []
    while len(states) < 48:
        arm = rng.uniform(lo_j, hi_j)
        oracle64.reset(model, d, np.array([0.4, 0.95, 0.6, 1, 0, 0, 0]))
        for k in range(6):
            d.qpos[k] = arm[k]
        oracle64.call("so100o_fwd_position", model, d)
        if (select(d) if select else any(p0 <= d.con[i].pair < p1 for i in range(d.ncon))) and not d.ncon_dropped:
            q, v, w, _ = oracle64.get_state(d)
            states.append((q, v * 0, w * 0))
            targets.append(np.clip((arm - lo) / (hi - lo) * 2 - 1, -1, 1))
    n = len(states)
    targets = np.array(targets)
    env = _new_env(n, solver, nsubstep=nsubstep)
    env.reset(seed=3)
    _set_states(env, states)
    r = _tf_run(env, model, oracle64, oracle32, 3, lambda step: targets + rng.normal(0, 0.02, (n, 6)), ens=True).arrays()
    env.close()
    cls = np.array([int(((p >= p0) & (p < p1)).sum()) for p in r.pairs])
    E = r.eqv
    print(f"\nGPU {label} contacts per env mean {cls.mean():.2f} (envs with any: {(cls > 0).mean():.2f}); "
          + r.summary(f"{solver} {label}" + (f", {nsubstep} substep per env step" if nsubstep else "")))
    q = lambda x, p: np.quantile(np.ravel(x), p)
    print(f"ensemble floor ({ENS64} fp64 + {ENS32} fp32 perturbations x {E.shape[0]} steps): qvel median / p90 / p99 / max "
          f"{q(E, .5):.2e} / {q(E, .9):.2e} / {q(E, .99):.2e} / {E.max():.2e} (fp64 members p99 {q(E[:, :ENS64], .99):.2e}, "
          f"fp32 {q(E[:, ENS64:], .99):.2e}; FMA fp32 p99 {q(r.mqv, .99):.2e}); GPU p99 {q(r.qv, .99):.2e}; "
          f"contact-list flips (GPU vs fp64 oracle, last substep): {int((~r.same).sum())} of {len(r.same)}")
    assert (cls > 0).mean() > 0.5
    # a contact one side sees and the other does not (a deep fold's vertex on another hull's boundary) is a
    # discrete flip fp32 cannot resolve as fp64 does: counted and kept rare
    assert r.same.mean() >= 0.9
    beyond = _ensemble_bars(r, "qv")
    _ensemble_bars(r, "qa")
    print(f"GPU steps beyond their state's whole ensemble (2x + 1e-5): {int(beyond.sum())} of {len(beyond)}")
    assert r.drop_gpu.sum() == 0 and r.drop_ora.sum() == 0     # every contact kept (no per-env cap, as MuJoCo)
    return r


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
    from gym_so100.model import PAIR_PADLINK0, PAIR_MOCAPHULL0
    _arm_contact_parity(solver, oracle64, oracle32, PAIR_PADLINK0, PAIR_MOCAPHULL0, "pad-link", 23)


@pytest.mark.parametrize("solver", ["newton", "pgs"])
def test_table_edge_parity(solver, oracle64, oracle32):
    """Arm hulls and finger pads against the table's edges and side faces (pairs 14..22 and 152..159, SURVEY §8 f.2;
    round 5): the table is a mesh, so MuJoCo collides these pairs through its convex collider at the minimum
    penetration.  Random arm poses whose first position stage holds a table contact with a non-vertical normal (a link
    or pad pushed into a side face, through GJK + EPA or the box-box SAT), the actuators holding them; teacher-forced
    GPU steps graded against the ensemble floor."""
    from gym_so100.model import NPAIR_BOX, NHULL, PAIR_PAD0, PAIR_PADBIN0, NPAIR
    table = lambda p: NPAIR_BOX <= p < NPAIR_BOX + NHULL or PAIR_PAD0 <= p < PAIR_PADBIN0

    def side(d):
        return any(table(d.con[i].pair) and abs(d.con[i].frame[2]) < 0.99 for i in range(d.ncon))
    r = _arm_contact_parity(solver, oracle64, oracle32, 0, NPAIR, "table-edge", 31, select=side)
    nside = np.array([int(sum(table(p) for p in ps)) for ps in r.pairs])
    print(f"GPU table contacts per env step: mean {nside.mean():.2f}")
    _force_bars(r)


@pytest.mark.parametrize("solver", ["newton", "pgs"])
@pytest.mark.parametrize("cls", ["self", "base", "padlink"])
def test_arm_contact_substep_parity(solver, cls, oracle64, oracle32):
    """The arm-contact classes one physics substep at a time (nsubstep = 1: an env step is one mj_step plus
    the final mj_step1).  Over the 10 substeps of an env step, these deep folds amplify an input
    perturbation of one fp32 rounding to 1e-3 (median) in the fp64 oracle itself (TF's perturbation floor;
    DESIGN.md §5), so per env step no fp32 implementation can hold 1e-4 there; per substep the problem is
    well conditioned at the median, and the GPU's product kernels must hold north_star's 1e-4 on qvel,
    qacc and the contact forces at the median (Newton, MuJoCo's solver), and the floors' bars in the tail."""
    from gym_so100.model import PAIR_SELF0, PAIR_BASE0, PAIR_PADLINK0, PAIR_MOCAPHULL0
    p0, p1, seed = {"self": (PAIR_SELF0, PAIR_BASE0, 17), "base": (PAIR_BASE0, PAIR_PADLINK0, 19),
                    "padlink": (PAIR_PADLINK0, PAIR_MOCAPHULL0, 23)}[cls]
    r = _arm_contact_parity(solver, oracle64, oracle32, p0, p1, cls, seed, nsubstep=1)
    _force_bars(r, median_abs=1e-4 if solver == "newton" else None)
    if solver == "newton":
        assert np.median(r.qv) <= 1e-4 and np.median(r.qa) <= 1e-4


@pytest.mark.parametrize("solver", ["newton", "pgs"])
@pytest.mark.parametrize("nsubstep", [1, None])
def test_overflow_contact_parity(solver, nsubstep, oracle64, oracle32):
    """Contact lists longer than the 16 an env holds on chip (round 4: no per-env cap, as MuJoCo): random arm
    poses whose first position stage holds more than 16 contacts (jaws and pads jammed into the bin walls, folds
    into the Base and the links; 17-73 contacts), the actuators holding them.  The contacts beyond 16 live in the
    env's HBM contact record (J, the rows, the solve's per-contact state); teacher-forced GPU steps against the
    fp64 oracle, which keeps every contact too, per substep (nsubstep = 1) and per env step.  No contact may be
    dropped by either side, and the per-contact forces of the whole list (debug record, SO100_DBG_OVF) are graded."""
    from gym_so100.model import NPAIR
    r = _arm_contact_parity(solver, oracle64, oracle32, 0, NPAIR, "overflow", 29, nsubstep=nsubstep,
                            select=lambda d: d.ncon > 16)
    ncon = np.array([len(p) for p in r.pairs])
    print(f"GPU contact-list length: mean {ncon.mean():.1f}, max {ncon.max()}, share > 16: {(ncon > 16).mean():.2f}")
    assert (ncon > 16).mean() > 0.5 and ncon.max() > 32       # the record's contacts really take part
    if nsubstep == 1:
        _force_bars(r, median_abs=1e-4 if solver == "newton" else None)
        if solver == "newton":
            assert np.median(r.qv) <= 1e-4 and np.median(r.qa) <= 1e-4


def _long_list_states(model, oracle64, n, seed=41):
    """random folded arm poses whose first position stage holds more than 16 contacts (17-73), with the actuator
    targets holding them"""
    rng = np.random.default_rng(seed)
    lo_j = np.array([r[0] for r in model.jnt_range]); hi_j = np.array([r[1] for r in model.jnt_range])
    lo, hi = np.array(model.action_lo[:]), np.array(model.action_hi[:])
    d = oracle64.new_data()
    states, targets = [], []
    while len(states) < n:
        arm = rng.uniform(lo_j, hi_j)
        oracle64.reset(model, d, np.array([0.4, 0.95, 0.6, 1, 0, 0, 0]))
        for k in range(6):
            d.qpos[k] = arm[k]
        oracle64.call("so100o_fwd_position", model, d)
        if d.ncon > 16:
            q, v, w, _ = oracle64.get_state(d)
            states.append((q, v * 0, w * 0))
            targets.append(np.clip((arm - lo) / (hi - lo) * 2 - 1, -1, 1))
    return states, targets, rng


def test_pool_contention_bitwise(oracle64):
    """The fused step's contact-record pool: an env whose list is longer than the 16 held on chip takes an
    HBM record of its XCD's pool for the substep.  1,024 envs (256 waves) all holding 17-73 contacts (random folded arm
    poses, tiled): every wave takes an entry every substep.  Round 6: the pool holds as many entries per XCD as the XCD
    can hold fused waves resident (here all 256 waves' worth: min(the grid's waves, 32 CUs x 12)), so no request finds
    the pool empty (so100_pool_stats' none_free, asserted 0) and no contact is dropped by construction; the fused 2- and
    3-wave builds equal the split path and the debug build bit for bit over 3 env steps."""
    from gym_so100.model import build_model
    model = build_model()
    states, targets, rng = _long_list_states(model, oracle64, 64)
    n = 1024
    env = _new_env(n, "newton")
    env.reset(seed=3)
    _set_states(env, [states[i % len(states)] for i in range(n)])
    act = np.array([targets[i % len(targets)] for i in range(n)], np.float32)
    st0 = env.pool_stats(reset=True)
    assert st0["entries_per_xcd"] >= n // 4            # every wave of the grid could hold an entry at once
    long_lists = []
    for step in range(3):
        _, _, ndrop, dbg, builds = _step_all_builds(env, act + rng.normal(0, 0.02, (n, 6)).astype(np.float32))
        assert int(ndrop.sum()) == 0
        long_lists.append(float((dbg[:, 0] > 16).mean()))
    st = env.pool_stats()
    env.close()
    print(f"\nbuilds {builds} == debug build, bitwise; share of envs with more than 16 contacts per step {long_lists}; "
          f"pool {st}")
    assert min(long_lists) > 0.5
    assert st["none_free"] == 0 and st["taken"] > 0


def test_pool_every_env_long_lists():
    """The pool at a size whose grid exceeds the resident waves (16,384 envs: 4,096 waves, 8 x 384 entries): every env
    holds more than 16 contacts (tiled folded poses), 3 env steps of the fused 3-wave product build.  No request finds
    the pool empty and no contact is dropped (by construction, not by timing: no wave ever waits for an entry)."""
    from gym_so100.model import build_model
    from oracle.oracle import Oracle
    from gym_so100 import SO100VecEnv
    model = build_model()
    states, targets, rng = _long_list_states(model, Oracle(64), 64, seed=43)
    n = 16384
    env = SO100VecEnv(n, device="cuda:0", autoreset=False, max_episode_steps=0)
    env.reset(seed=3)
    _set_states(env, [states[i % len(states)] for i in range(n)])
    act = torch.from_numpy(np.array([targets[i % len(targets)] for i in range(n)], np.float32)).cuda()
    env.pool_stats(reset=True)
    drops = 0
    for _ in range(3):
        env.step(act)
        drops += int(env.ncon_dropped.sum().item())
    st = env.pool_stats()
    counts = env.contact_counts().cpu().numpy()
    env.close()
    print(f"\n{n} envs, share with more than 16 contacts after 3 steps {np.mean(counts > 16):.2f}; pool {st}")
    assert st["entries_per_xcd"] == 384 and st["none_free"] == 0 and st["taken"] > 0
    assert drops == 0 and np.isfinite(counts).all()


def test_contact_record_memory():
    """The contact record by need: a 65,536-env fused-path env allocates its workspace (the contact counts, the
    separating-direction cache and the contact-record pool: 8 XCDs x 384 entries x 4 records x 288 KB = 3.5 GB, the
    most waves the chip holds resident; round 5's timing-dependent pool was 295 MB) in under 4 GiB (round 4's record per
    env took 18.9 GB)."""
    from gym_so100 import SO100VecEnv
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info()
    env = SO100VecEnv(65536, device="cuda:0")
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info()
    used = (free0 - free1) / 2 ** 30
    env.close()
    print(f"\n65,536 envs: {used:.2f} GiB of device memory (state tensors, workspace and the contact-record pool)")
    assert used < 4.0


@pytest.mark.parametrize("solver", ["newton", "pgs"])
def test_cube_on_base_parity(solver, oracle64, oracle32):
    """The cube resting on the static Base (pair 98, box vs the Base hull through MPR, one contact):
    states made by the fp64 oracle dropping the cube onto the Base top, then teacher-forced GPU steps."""
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
    env = _new_env(n, solver)
    env.reset(seed=3)
    _set_states(env, states)
    r = _tf_run(env, model, oracle64, oracle32, 4, lambda step: np.tile(start, (n, 1))).arrays()
    env.close()
    base_con = np.array([int((p == PAIR_BASE0).sum()) for p in r.pairs])
    print(f"\nGPU cube-Base contacts per env mean {base_con.mean():.2f}; " + r.summary(f"{solver} cube on Base"))
    assert (base_con > 0).mean() > 0.8                     # the cube really rests on the Base
    assert np.median(r.qv) <= 2 * r.floor("qv", 0.5) + 1e-5
    assert np.quantile(r.qv, 0.9) <= 2 * r.floor("qv", 0.9) + 1e-4
    assert r.qv.max() <= 2 * r.floor("qv", 1.0) + 1e-3
    _force_bars(r)


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
    from gym_so100.model import build_model
    model = build_model(solver=solver, variant="ee")
    n = 32
    venv = _new_env(n, solver, variant="ee")
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
    venv.set_mocap(mocap[:, :3], mocap[:, 3:])
    act_rng = np.random.default_rng(77)
    r = _tf_run(venv, model, oracle64, oracle32, 30, lambda step: (act_rng.uniform(-1, 1, (n, 6)) if step % 20 < 10 else
                                                                   np.clip(act_rng.normal(0, 0.3, (n, 6)), -1, 1)),
                mocap=mocap).arrays()
    ee_gap = np.linalg.norm(venv.obs[:, 6:9].cpu().numpy() - mocap[:, :3], axis=1)
    venv.close()
    # the marker box at the target (so_arm100_ee.xml:155) collides with the gripper (pairs 143..151 against the link
    # hulls, 200..208 against the cube and the pads): its contacts are in the lists the GPU and the oracle agree on
    from gym_so100.model import PAIR_MOCAPHULL0, PAIR_PAD0, PAIR_MOCAPBOX0
    marker = np.array([int((((p >= PAIR_MOCAPHULL0) & (p < PAIR_PAD0)) | (p >= PAIR_MOCAPBOX0)).sum()) for p in r.pairs])
    print(f"\nee-target gap after 30 steps: median {np.median(ee_gap):.3f} m; marker contacts in "
          f"{np.mean(marker > 0):.2f} of env-steps; " + r.summary(f"ee {solver}"))
    assert np.mean(marker > 0) > 0.2 and np.mean(r.same[marker > 0]) > 0.8
    assert np.median(r.qp) <= 1e-5 and np.median(r.qv) <= 1e-5
    assert np.quantile(r.qv, 0.9) <= 2 * r.floor("qv", 0.9) + 1e-4
    assert r.qv.max() <= 2 * r.floor("qv", 1.0) + 1e-3


@pytest.mark.parametrize("n", [4099, 12291])
def test_product_builds_bitwise(n):
    """The kernels the product launches give one result, bit for bit, on contact-rich states: the fused
    step's debug build (<true>), its product builds for 2 and 3 waves per SIMD (<false, 2>, <false, 3>) and
    the split path (4 env chunks on concurrent streams), with the heavy-first wave order and the issue
    priorities active (n / 4 > 256 groups), a ragged tail wave, auto-resets and a TimeLimit of 4 steps.
    The states mix folded arm poses (self / Base / pad-link contacts), cubes pressed into a bin corner (up
    to 12 contacts) and spawned cubes; every env's state must change in every step (no group lost or
    duplicated by the order)."""
    from gym_so100 import SO100VecEnv
    from gym_so100.model import PAIR_MPR0, PAIR_PAD0, build_model
    env = SO100VecEnv(n, device="cuda:0", seed=12, max_episode_steps=4, debug=True)
    env.reset(seed=100)
    model = build_model()
    rng = np.random.default_rng(n)
    lo_j = np.array([r[0] for r in model.jnt_range]); hi_j = np.array([r[1] for r in model.jnt_range])
    qpos = env.qpos.cpu().numpy()
    qpos[:, :6] = rng.uniform(lo_j, hi_j, (n, 6))
    corner = np.arange(n) % 4 == 1
    pen = rng.uniform(2e-4, 1e-3, (corner.sum(), 3))
    qpos[corner, 6] = -0.165 + pen[:, 0]
    qpos[corner, 7] = 0.735 + pen[:, 1]
    qpos[corner, 8] = 0.021 - pen[:, 2]
    qpos[corner, 9:13] = [1, 0, 0, 0]
    env.set_state(qpos, np.zeros((n, 12), np.float32), np.zeros((n, 12), np.float32))
    g = torch.Generator(device="cuda").manual_seed(3)
    ncon, mpr, resets = [], 0, 0
    for step in range(10):
        before = env.qpos.clone()
        a = torch.rand(n, 6, generator=g, device="cuda") * 2 - 1
        _, _, _, dbg, builds = _step_all_builds(env, a)
        assert builds == ["fused2", "fused3", "split"]
        assert (env.qpos != before).any(dim=1).all(), step        # every env stepped (and only once)
        nc = dbg[:, 0].astype(int)
        ncon.append(nc)
        pairs = dbg[:, 48:64]
        mpr += int(((pairs >= PAIR_MPR0) & (pairs < PAIR_PAD0)).sum())
        resets += int((env.elapsed == 0).sum())
    env.close()
    ncon = np.concatenate(ncon)
    print(f"\n{n} envs x 10 steps, all builds bitwise equal: contacts/env mean {ncon.mean():.2f}, max {ncon.max()}, "
          f"envs > 8 contacts {(ncon > 8).mean():.3f}, MPR contacts {mpr}, auto-resets {resets}")
    # (contact-rich: 2.2 contacts per env before round 5, 1.96 since the table's edges and side faces collide exactly:
    # a link hanging past the edge no longer takes a top-face contact)
    assert ncon.mean() > 1.5 and ncon.max() > 8 and mpr > 100 and resets >= n


@pytest.mark.parametrize("fused", [True, False])
def test_config2_benched_full_size(fused):
    """configs[2] as bench.py times it on one GPU: 65,536 envs in one process, the fused step (auto mode, the
    benched path) and the split step (4 env chunks on concurrent streams), with auto-reset; 40 steps of random
    actions keep the state finite and the contract: unit quaternions, obs layout, reward ladder, no divergence,
    TimeLimit counters, and every contact kept: MuJoCo keeps every box-box point (up to 8 per pair), and a jaw
    jammed into the bin walls collects 20-46 pad-bin contacts; the list holds them all (no per-env cap since
    round 4), so none is dropped, and the envs with more than the 16 held on chip are counted."""
    from gym_so100 import SO100VecEnv
    n = 65536
    env = SO100VecEnv(n, device="cuda:0", seed=0)
    assert env.fused                                            # auto mode at this size
    env.fused = fused
    assert env.chunk_info()[0] == (1 if fused else 4)
    env.reset(seed=1000)
    g = torch.Generator(device="cuda").manual_seed(0)
    drops, rewards, over16 = 0, set(), 0
    for k in range(40):
        obs, rew, term, trunc, info = env.step(torch.rand(n, 6, generator=g, device="cuda") * 2 - 1)
        drops += int(info["ncon_dropped"].sum())
        over16 += int((env.contact_counts() > 16).sum())
        if k % 10 == 9:
            rewards |= set(torch.unique(rew).tolist())
    torch.cuda.synchronize()
    assert torch.isfinite(env.qpos).all() and torch.isfinite(env.qvel).all()
    qn = env.qpos[:, 9:13].norm(dim=1)
    assert torch.allclose(qn, torch.ones_like(qn), atol=1e-5)
    # a cube below the table top has left the table's footprint (the scene has no floor: knocked off the
    # edge, it falls)
    from gym_so100.model import build_model
    m = build_model()
    x, y, z = env.qpos[:, 6], env.qpos[:, 7], env.qpos[:, 8]
    off = (x < m.table_lo[0] - 0.03) | (x > m.table_hi[0] + 0.03) | (y < m.table_lo[1] - 0.03) | (y > m.table_hi[1] + 0.03)
    assert ((z > -0.05) | off).all()
    print(f"\ncubes knocked off the table: {int((z < -0.05).sum())}")
    assert torch.equal(obs[:, 9:15], env.qpos[:, :6])
    assert torch.allclose(obs[:, 3:6], torch.tensor([-0.2, 0.7, 0.021], device="cuda").expand(n, 3))
    assert not info["diverged"].any()
    assert ((env.elapsed == 40) | (env.episode > 1)).all()         # TimeLimit 700 not reached (only successes reset)
    assert rewards <= {0.0, 1.0, 2.0, 2.5, 3.0, 4.0}
    print(f"\n65,536 envs x 40 steps: env steps ending with more than the 16 contacts held on chip: {over16} "
          f"({over16 / (40 * n):.2e} per env step); contacts dropped: {drops}")
    assert drops == 0
    env.close()


def test_config2_shard_equals_slice():
    """configs[2]'s 8-GPU shard (8,192 joint-space envs per GPU): the shard at env_offset 8,192 (fused step,
    the 2-wave build) runs the same trajectories, auto-resets included, as envs 8,192..16,383 of a 16,384-env
    run (fused, the 3-wave build), bit for bit."""
    from gym_so100 import SO100VecEnv
    full = SO100VecEnv(16384, device="cuda:0", seed=6, max_episode_steps=12)
    shard = SO100VecEnv(8192, device="cuda:0", seed=6, env_offset=8192, max_episode_steps=12)
    assert full.fused and shard.fused and full.fused_build == 3 and shard.fused_build == 2
    full.reset(seed=[1000 + i for i in range(16384)])
    shard.reset(seed=[1000 + 8192 + i for i in range(8192)])
    g = torch.Generator(device="cuda").manual_seed(2)
    for _ in range(30):
        a = torch.rand(16384, 6, generator=g, device="cuda") * 2 - 1
        rf = full.step(a)
        rs = shard.step(a[8192:].contiguous())
        torch.cuda.synchronize()
        assert torch.equal(rf[1][8192:], rs[1]) and torch.equal(rf[3][8192:], rs[3])
    for name in ("qpos", "qvel", "qacc_warmstart", "obs", "elapsed", "episode", "contact_bits"):
        assert torch.equal(getattr(full, name)[8192:], getattr(shard, name)), name
    assert (full.episode > 1).any()                       # auto-resets happened (TimeLimit 12)
    full.close()
    shard.close()
