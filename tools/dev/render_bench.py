"""Render throughput: envs/s and images/s of so100_render at a few sizes (HIP events around launches)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "gym-so100-c_amd"))

from gym_so100 import SO100VecEnv

out = []
for n, w, h in [(4096, 64, 48), (16384, 64, 48), (4096, 96, 72), (1024, 160, 120), (256, 640, 480),
                (2048, 640, 480)]:
    env = SO100VecEnv(n, obs_type="so100_pixels_agent_pos", observation_width=w, observation_height=h)
    env.reset(seed=1)
    for _ in range(3):
        env.renderer.render()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 10
    e0.record()
    for _ in range(reps):
        env.renderer.render()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    # env steps with pixel observations (physics step + terminal/auto-reset images + render)
    act = torch.rand(n, 6, device=env.device) * 2 - 1
    env.step(act)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        env.step(act)
    e1.record()
    torch.cuda.synchronize()
    step_ms = e0.elapsed_time(e1) / reps
    r = {"n": n, "w": w, "h": h, "render_ms": round(ms, 4), "images_per_s": round(n / ms * 1e3),
         "Mpix_per_s": round(n * w * h / ms * 1e-3, 1), "ntri": env.renderer.ntri,
         "pixel_step_ms": round(step_ms, 4), "pixel_env_steps_per_s": round(n / step_ms * 1e3)}
    print(json.dumps(r), flush=True)
    out.append(r)
    env.close()
    del env
json.dump(out, open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/render_bench.json", "w"), indent=1)
