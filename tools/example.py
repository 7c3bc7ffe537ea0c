"""configs[0]: the reference's scripts/example.py (10-28) on this build.

TouchCube with pixel observations at 64x48, 1000 random-action steps, ``render()`` every step, reset when an
episode terminates or is truncated (the registered TimeLimit of 300), the observation frames kept.  The
reference writes them to outputs/example.mp4 with imageio; imageio is absent in this image, so the frames
go to outputs/example.npz (uint8 [1000, 48, 64, 3]) unless imageio is importable.

    python tools/example.py [--steps 1000] [--out outputs/example]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gym-so100-c_amd"))

import gym_so100  # noqa: E402


def run(steps=1000, seed=None, width=64, height=48):
    """The example's loop; returns the frames and per-step records for checks (tests/test_gpu_example.py)."""
    env = gym_so100.make("gym_so100/SO100TouchCube-v0", obs_type="so100_pixels_agent_pos",
                         observation_width=width, observation_height=height)
    observation, info = env.reset(seed=seed)
    env.action_space.seed(seed)
    frames, log = [], []
    for _ in range(steps):
        action = env.action_space.sample()
        observation, reward, terminated, truncated, info = env.step(action)
        image = env.render()
        frames.append(observation["pixels"])
        log.append(dict(action=action, reward=reward, terminated=terminated, truncated=truncated,
                        agent_pos=observation["agent_pos"], image_shape=image.shape, info=info,
                        cube=env.unwrapped._venv.qpos[0, 6:13].cpu().numpy()))
        if terminated or truncated:
            observation, info = env.reset()
    env.close()
    return np.stack(frames), log


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--out", default=os.path.join("outputs", "example"))
    args = ap.parse_args()
    t0 = time.time()
    frames, log = run(args.steps)
    dt = time.time() - t0
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    try:
        import imageio
        imageio.mimsave(args.out + ".mp4", frames, fps=25)
        path = args.out + ".mp4"
    except ImportError:
        np.savez_compressed(args.out + ".npz", frames=frames)
        path = args.out + ".npz"
    resets = sum(1 for r in log if r["terminated"] or r["truncated"])
    print(f"{len(log)} steps in {dt:.1f} s ({len(log) / dt:.0f} steps/s, render every step), {resets} episode ends, "
          f"frames {frames.shape} -> {path}")


if __name__ == "__main__":
    main()
