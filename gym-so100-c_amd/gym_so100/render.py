"""Batched camera images on the GPU: the reference's ``so100_pixels_agent_pos`` observation.

The reference renders the ``top`` camera with dm_control's ``physics.render`` on every observation
(gym_so100/tasks/single_arm.py:88-92, env.py:130-136).  ``CameraRenderer`` draws the same camera for
all N envs of an ``SO100VecEnv`` with one HIP launch (csrc/so100_render.hip, C-ABI ``so100_render``):
the scene's visible geoms (assets/so100_render.npz, built by tools/compile_render.py from the
reference MJCF), the camera pose of scene_so100.xml:26-29 (mode="targetbody" on the static table),
fovy 78 and the scene's headlight + three directional lights.  Output: uint8 [N, H, W, 3] on the device.

It is a rasteriser of its own, not MuJoCo's OpenGL pipeline: geometry and colours are the scene's, the
pixel values are not MuJoCo's (no specular, shadows, fog or anti-aliasing).
"""
import ctypes
import os

import numpy as np

from . import _native

ASSET = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets", "so100_render.npz")
CAMERAS = ("top", "angle", "left_pillar", "right_pillar", "front_close")
TRACKING = ("front_close",)              # mode="targetbody" on the ee body: frame per env
ZNEAR = 0.01


def _torch():
    import torch
    return torch


def load_scene(path=ASSET):
    with np.load(path, allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def make_camera(scene, name="top"):
    """so100_camera for one of the scene's cameras (scene_so100.xml:26-29)."""
    if name not in CAMERAS:
        raise ValueError(f"camera {name!r}: one of {CAMERAS}")
    cam = _native.SO100Camera()
    cam.pos[:] = [float(x) for x in scene[f"cam_{name}_pos"]]
    cam.mat[:] = [float(x) for x in scene[f"cam_{name}_mat"].reshape(-1)]
    cam.track = 1 if name in TRACKING else 0
    cam.fovy = float(scene["fovy"])
    cam.znear = ZNEAR
    cam.head_ambient, cam.head_diffuse = (float(x) for x in scene["head"])
    nl = len(scene["light_diffuse"])
    if nl > _native.SO100_MAX_LIGHTS:
        raise ValueError("too many lights")
    cam.nlight = nl
    for i in range(nl):
        cam.light_dir[i][:] = [float(x) for x in scene["light_dir"][i]]
        cam.light_diffuse[i] = float(scene["light_diffuse"][i])
    return cam


class CameraRenderer:
    """Renders every env of ``venv`` (an SO100VecEnv) from one camera into a persistent uint8 tensor."""

    def __init__(self, venv, width=640, height=480, camera="top"):
        torch = _torch()
        self.venv = venv
        self.width, self.height = int(width), int(height)
        if not (0 < self.width <= 4096 and 0 < self.height and self.width * self.height <= 1 << 22):
            raise ValueError(f"image {self.width}x{self.height}: width <= 4096 and width*height <= 2^22")
        scene = load_scene()
        tri = np.ascontiguousarray(scene["tri"], dtype=np.float32)
        body = np.ascontiguousarray(scene["body"], dtype=np.int32)
        rgb = np.ascontiguousarray(scene["rgb"], dtype=np.float32)
        _native.check(venv.lib.so100_render_mesh(venv._handle, tri.ctypes.data, body.ctypes.data, rgb.ctypes.data,
                                                 len(body)), "so100_render_mesh")
        self.camera_name = camera
        self.camera = make_camera(scene, camera)
        self.ntri = len(body)
        self.pixels = torch.zeros(venv.num_envs, self.height, self.width, 3, dtype=torch.uint8, device=venv.device)

    def render(self, qpos=None, out=None, mask=None):
        """Enqueue the render of qpos (default: the env's state) into out (default self.pixels); mask: [N]
        bool/uint8 device tensor of the envs to draw (the others keep their previous image)."""
        torch = _torch()
        v = self.venv
        q = v.qpos if qpos is None else qpos
        o = self.pixels if out is None else out
        if q.shape != (v.num_envs, v.qpos.shape[1]) or q.dtype != torch.float32 or not q.is_contiguous():
            raise ValueError("qpos must be a contiguous float32 [N, 13] device tensor")
        if o.shape != (v.num_envs, self.height, self.width, 3) or o.dtype != torch.uint8 or not o.is_contiguous():
            raise ValueError("out must be a contiguous uint8 [N, H, W, 3] device tensor")
        m = None
        if mask is not None:
            if mask.shape != (v.num_envs,) or mask.device != v.device:
                raise ValueError("mask must be an [N] tensor on the env's device")
            m = mask.to(torch.uint8).contiguous()
            self._mask_ref = m                    # keep alive until the launch has run
        _native.check(v.lib.so100_render(v._handle, _native.ptr(q), _native.ptr(m), ctypes.byref(self.camera),
                                         self.width, self.height, _native.ptr(o), v._stream()), "so100_render")
        return o
