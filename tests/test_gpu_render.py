"""GPU camera images (csrc/so100_render.hip through the C-ABI so100_render).

* the HIP rasteriser against its numpy restatement (tests/render_ref.py) on the oracle's float64 body
  frames of the GPU's own states: pixels may differ only on silhouette edges (fp32 vs fp64 frames);
* pixel-mode envs step bit-for-bit like state-mode envs, auto-reset included, and their terminal images
  show the terminal state;
* determinism, per-env independence, the reference's observation shapes (env.py:50-66, 218-224).
Parity with MuJoCo's OpenGL images is unpinned."""
import numpy as np
import pytest
import torch

import render_ref
from gym_so100 import SO100VecEnv, SO100Env, SO100GoalEnv
from gym_so100 import render as R

pytestmark = pytest.mark.gpu
NBODY = 9


def frames_of(o, m, qpos):
    d = o.new_data()
    o.reset(m, d, np.array(qpos[6:13], np.float64))
    for k in range(6):
        d.qpos[k] = float(qpos[k])
    o.call("so100o_fwd_position", m, d)
    return [(np.array(d.xmat[b][:]).reshape(3, 3), np.array(d.xpos[b][:])) for b in range(NBODY)]


def rollout(env, steps, seed=0):
    g = torch.Generator().manual_seed(seed)
    env.reset(seed=seed)
    for _ in range(steps):
        env.step(torch.rand(env.num_envs, 6, generator=g) * 2 - 1)
    torch.cuda.synchronize()


@pytest.mark.parametrize("W,H,N", [(96, 72, 8), (640, 480, 2)])
def test_render_matches_numpy_rasteriser(model, oracle64, W, H, N):
    env = SO100VecEnv(N, obs_type="so100_pixels_agent_pos", observation_width=W, observation_height=H,
                      autoreset=False, max_episode_steps=0)
    rollout(env, 25, seed=3)
    img = env.pixels.cpu().numpy()
    qpos = env.qpos.cpu().numpy().astype(np.float64)
    scene = R.load_scene()
    cam = render_ref.camera_dict(env.renderer.camera)
    worst = 0.0
    for i in range(N):
        ref = render_ref.render(scene["tri"], scene["body"], scene["rgb"], frames_of(oracle64, model, qpos[i]),
                                cam, W, H)
        diff = np.any(img[i] != ref, axis=-1)
        worst = max(worst, diff.mean())
        assert diff.mean() < 0.01, (i, diff.sum())
        assert (img[i, ..., 0] > 200).sum() > 0 or (ref[..., 0] > 200).sum() == 0
    print(f"worst share of differing pixels {worst:.4f}")


def test_cube_is_red_where_it_projects():
    W, H, N = 160, 120, 16
    env = SO100VecEnv(N, obs_type="so100_pixels_agent_pos", observation_width=W, observation_height=H)
    env.reset(seed=11)
    torch.cuda.synchronize()
    img = env.pixels.cpu().numpy()
    cube = env.qpos[:, 6:9].cpu().numpy()
    th = np.tan(np.radians(39.0))
    seen = 0
    for i in range(N):
        c = cube[i] + np.array([0, 0, 0.01]) - np.array([0, 0.6, 0.8])     # top face centre, camera frame
        u = (c[0] / -c[2] / (th * W / H) * 0.5 + 0.5) * W
        v = (0.5 - c[1] / -c[2] / th * 0.5) * H
        red = (img[i, ..., 0] > 200) & (img[i, ..., 1] < 40) & (img[i, ..., 2] < 40)
        if red.any():                    # the arm at its home pose hides spawns below the gripper
            seen += 1
            ys, xs = np.nonzero(red)
            assert abs(xs.mean() + 0.5 - u) < 3 and abs(ys.mean() + 0.5 - v) < 3, (i, xs.mean(), u, ys.mean(), v)
    assert seen >= N // 2


def test_pixel_mode_steps_like_state_mode():
    N, T = 32, 14
    kw = dict(max_episode_steps=5, seed=7)
    a = SO100VecEnv(N, **kw)
    b = SO100VecEnv(N, obs_type="so100_pixels_agent_pos", observation_width=48, observation_height=36, **kw)
    a.reset(seed=5)
    b.reset(seed=5)
    g = torch.Generator().manual_seed(0)
    saw_done = False
    for t in range(T):
        act = torch.rand(N, 6, generator=g) * 2 - 1
        oa, ra, ta, ua, ia = a.step(act)
        prev = b.pixels.clone()
        ob, rb, tb, ub, ib = b.step(act)
        torch.testing.assert_close(ob["agent_pos"], oa[:, 9:15], rtol=0, atol=0)
        torch.testing.assert_close(b.qpos, a.qpos, rtol=0, atol=0)
        torch.testing.assert_close(b.qvel, a.qvel, rtol=0, atol=0)
        torch.testing.assert_close(rb, ra, rtol=0, atol=0)
        assert torch.equal(ub, ua) and torch.equal(tb, ta)
        done = ua | ta
        if bool(done.any()):
            saw_done = True
            torch.testing.assert_close(ib["final_observation"]["agent_pos"][done],
                                       ia["final_observation"][done][:, 9:15], rtol=0, atol=0)
            # the terminal image shows the terminal state, the new image the new episode's spawn
            assert not torch.equal(ib["final_observation"]["pixels"][done], ob["pixels"][done])
        assert not torch.equal(prev, b.pixels)
    assert saw_done


def test_render_deterministic_and_per_env():
    W, H = 64, 48
    big = SO100VecEnv(64, obs_type="so100_pixels_agent_pos", observation_width=W, observation_height=H,
                      autoreset=False, max_episode_steps=0)
    small = SO100VecEnv(4, obs_type="so100_pixels_agent_pos", observation_width=W, observation_height=H,
                        autoreset=False, max_episode_steps=0)
    big.reset(seed=100)
    small.reset(seed=[100, 101, 102, 103])
    torch.cuda.synchronize()
    first = big.pixels.clone()
    big.renderer.render()
    torch.cuda.synchronize()
    assert torch.equal(first, big.pixels)
    assert torch.equal(small.pixels, big.pixels[:4])
    mask = torch.zeros(64, dtype=torch.bool, device=big.device)
    mask[::2] = True
    out = torch.zeros_like(big.pixels)
    big.renderer.render(out=out, mask=mask)
    torch.cuda.synchronize()
    assert torch.equal(out[::2], first[::2]) and int(out[1::2].sum()) == 0


def test_reference_observation_shapes():
    e = SO100Env("so100_cube_to_bin", obs_type="so100_pixels_agent_pos", observation_width=80,
                 observation_height=60, visualization_width=128, visualization_height=96)
    obs, info = e.reset(seed=1)
    assert obs["pixels"].shape == (60, 80, 3) and obs["pixels"].dtype == np.uint8
    assert obs["agent_pos"].shape == (6,) and obs["agent_pos"].dtype == np.float32
    obs, r, term, trunc, info = e.step(np.zeros(6, np.float32))
    assert obs["pixels"].shape == (60, 80, 3)
    assert e.render().shape == (96, 128, 3)
    g = SO100GoalEnv(observation_width=32, observation_height=24)
    obs, _ = g.reset(seed=2)
    assert obs["observation"].shape == (32 * 24 * 3 + 6,) and obs["observation"].dtype == np.float32
    assert 0.0 <= obs["observation"][:-6].min() and obs["observation"][:-6].max() <= 1.0
    assert obs["observation"][:-6].max() > 0
    obs, r, term, trunc, info = g.step(np.zeros(6, np.float32))
    assert obs["observation"].shape == (32 * 24 * 3 + 6,)
    assert g.observation_space["observation"].shape == (32 * 24 * 3 + 6,)


def test_demo_recorder_reference_layout(tmp_path):
    """Episodes recorded from 4 GPU envs in the reference's expert-demonstration layout
    (record_teleop.py:163-184): per step the observation the step returned, channel-first pixels."""
    from gym_so100.demos import DemoRecorder, load_demonstrations, lerobot_frames
    env = SO100VecEnv(4, obs_type="so100_pixels_agent_pos", observation_width=64, observation_height=48,
                      max_episode_steps=6)
    rec = DemoRecorder(env, env_ids=[0, 2], max_episodes=3)
    env.reset(seed=0)
    g = torch.Generator().manual_seed(0)
    for t in range(14):
        act = torch.rand(4, 6, generator=g) * 2 - 1
        obs, r, term, trunc, info = env.step(act)
        rec.add(act, obs, r, term, trunc, info)
    assert len(rec.demonstrations) == 3 and rec.done
    ep = rec.demonstrations[0]
    assert len(ep["observations"]) == len(ep["actions"]) == len(ep["rewards"]) == len(ep["infos"]) == 6
    o = ep["observations"][0]
    assert o["pixels"].shape == (1, 3, 48, 64) and o["pixels"].dtype == np.uint8
    assert o["agent_pos"].shape == (1, 6) and o["agent_pos"].dtype == np.float32
    assert ep["infos"][-1][0].get("TimeLimit.truncated") is True
    path = rec.save(str(tmp_path / "expert_demonstrations.pkl"))
    back = load_demonstrations(path)
    np.testing.assert_array_equal(back[1]["observations"][3]["pixels"], rec.demonstrations[1]["observations"][3]["pixels"])
    assert len(lerobot_frames(back[0])) == 6


def test_tracking_camera_matches_numpy_rasteriser(model, oracle64):
    """front_close: the camera frame follows each env's end effector (computed in the kernel)."""
    W, H, N = 96, 72, 4
    env = SO100VecEnv(N, obs_type="so100_pixels_agent_pos", observation_width=W, observation_height=H,
                      autoreset=False, max_episode_steps=0)
    rollout(env, 15, seed=9)
    cam_r = R.CameraRenderer(env, W, H, camera="front_close")
    img = cam_r.render().cpu().numpy()
    qpos = env.qpos.cpu().numpy().astype(np.float64)
    scene = R.load_scene()
    cam = render_ref.camera_dict(cam_r.camera)
    for i in range(N):
        fr = frames_of(oracle64, model, qpos[i])
        d = oracle64.new_data()
        oracle64.reset(model, d, np.array(qpos[i][6:13]))
        for k in range(6):
            d.qpos[k] = qpos[i][k]
        oracle64.call("so100o_fwd_position", model, d)
        ref = render_ref.render(scene["tri"], scene["body"], scene["rgb"], fr, cam, W, H, target=np.array(d.site_ee[:]))
        diff = np.any(img[i] != ref, axis=-1)
        assert diff.mean() < 0.01, (i, diff.sum())
