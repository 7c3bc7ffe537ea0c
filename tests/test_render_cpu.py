"""Render scene asset + the numpy restatement of the rasteriser's rules (CPU).

The images are this framework's own rasterisation of the reference scene, so these tests pin scene
facts the reference MJCF fixes: the camera poses of scene_so100.xml:26-29 (mode="targetbody" on the
table), where the cube and the table land in the top camera's image, and the Lambert lighting sum of
the headlight (ambient .4, diffuse .4) and the three .3 directional lights on an upward face."""
import numpy as np
import pytest

import render_ref
from gym_so100 import render as R

NBODY = 9


@pytest.fixture(scope="module")
def scene():
    return R.load_scene()


def frames_of(o, m, qpos):
    d = o.new_data()
    o.reset(m, d, np.array(qpos[6:13], np.float64))
    for k in range(6):
        d.qpos[k] = float(qpos[k])
    o.call("so100o_fwd_position", m, d)
    return [(np.array(d.xmat[b][:]).reshape(3, 3), np.array(d.xpos[b][:])) for b in range(NBODY)]


def project(cam, p, width, height):
    c = (np.asarray(p, float) - cam["pos"]) @ cam["mat"]
    th = np.tan(0.5 * np.radians(cam["fovy"]))
    u = (c[0] / -c[2] / (th * width / height) * 0.5 + 0.5) * width
    v = (0.5 - c[1] / -c[2] / th * 0.5) * height
    return int(u), int(v)


def test_scene_asset(scene):
    tri, body, rgb = scene["tri"], scene["body"], scene["rgb"]
    assert tri.shape == (len(body), 3, 3) and rgb.shape == (len(body), 3)
    assert body.min() >= 0 and body.max() == NBODY - 1
    assert np.all(np.bincount(body, minlength=NBODY)[2:8] > 0)        # every arm link drawn
    assert np.all((rgb >= 0) & (rgb <= 1))
    assert np.sum(np.all(rgb == [1, 0, 0], axis=1)) == 12               # the red cube: 12 triangles
    assert np.all(body[np.all(rgb == [1, 0, 0], axis=1)] == 8)


@pytest.mark.parametrize("name", [c for c in R.CAMERAS if c not in R.TRACKING])
def test_targetbody_cameras(scene, name):
    pos, mat = scene[f"cam_{name}_pos"].astype(float), scene[f"cam_{name}_mat"].astype(float)
    np.testing.assert_allclose(mat.T @ mat, np.eye(3), atol=1e-6)
    assert np.linalg.det(mat) > 0
    z = pos - np.array([0.0, 0.6, 0.0])                                 # looks at the table body
    np.testing.assert_allclose(mat[:, 2], z / np.linalg.norm(z), atol=1e-6)
    assert abs(mat[2, 0]) < 1e-6                                        # camera x stays horizontal
    if name == "top":
        np.testing.assert_allclose(mat, np.eye(3), atol=1e-7)


def test_top_camera_known_pixels(scene, model, oracle64):
    W, H = 160, 120
    cube = (0.12, 0.72, 0.01)                                           # clear of the arm and bin
    fr = frames_of(oracle64, model, np.r_[np.zeros(6), cube, 1, 0, 0, 0])
    cam = render_ref.camera_dict(R.make_camera(scene, "top"))
    img = render_ref.render(scene["tri"], scene["body"], scene["rgb"], fr, cam, W, H)
    # the cube's top face: red saturates under 1.36 x light
    u, v = project(cam, (cube[0], cube[1], cube[2] + 0.01), W, H)
    np.testing.assert_array_equal(img[v, u], [255, 0, 0])
    # the table under the camera: 0.2 grey (51/255) x (0.4 + 0.4 + 0.3 (2/sqrt3 + 1/sqrt2)) = 69
    u, v = project(cam, (0.2, 0.45, 0.0), W, H)
    lum = 0.4 + 0.4 + 0.3 * (2 / np.sqrt(3) + 1 / np.sqrt(2))
    np.testing.assert_array_equal(img[v, u], [int(51 * lum + 0.5)] * 3)
    # outside the table: background
    np.testing.assert_array_equal(img[0, 0], [0, 0, 0])


def test_numpy_rasteriser_depth_order(scene, model, oracle64):
    """Moving the cube under the camera's line of sight through the bin floor changes the pixel from
    bin grey to red only when the cube is above the floor (nearest surface wins)."""
    W, H = 96, 72
    cam = render_ref.camera_dict(R.make_camera(scene, "top"))
    bin_body = [i for i in range(len(scene["body"])) if scene["body"][i] == 0 and
                np.allclose(scene["rgb"][i], 0.5)]
    c = scene["tri"][bin_body].reshape(-1, 3).mean(axis=0)              # bin centre (world)
    above = render_ref.render(scene["tri"], scene["body"], scene["rgb"],
                              frames_of(oracle64, model, np.r_[np.zeros(6), c[0], c[1], 0.02, 1, 0, 0, 0]),
                              cam, W, H)
    below = render_ref.render(scene["tri"], scene["body"], scene["rgb"],
                              frames_of(oracle64, model, np.r_[np.zeros(6), c[0], c[1], -0.05, 1, 0, 0, 0]),
                              cam, W, H)
    u, v = project(cam, (c[0], c[1], 0.0), W, H)
    np.testing.assert_array_equal(above[v, u], [255, 0, 0])
    assert below[v, u][0] == below[v, u][1] == below[v, u][2] > 0


def test_tracking_camera_looks_at_the_end_effector(scene, model, oracle64):
    """front_close (scene_so100.xml:30) targets vx300s_left/camera_focus, whose origin is ee_site: the
    end effector projects to the image centre whatever the arm pose."""
    cam = render_ref.camera_dict(R.make_camera(scene, "front_close"))
    assert cam["track"] == 1
    rng = np.random.default_rng(0)
    for _ in range(5):
        arm = rng.uniform(-0.8, 0.8, 6)
        d = oracle64.new_data()
        oracle64.reset(model, d, np.array([-0.2, 0.45, 0.01, 1, 0, 0, 0]))
        for k in range(6):
            d.qpos[k] = arm[k]
        oracle64.call("so100o_fwd_position", model, d)
        ee = np.array(d.site_ee[:])
        mat = render_ref.tracking_frame(cam["pos"], ee)
        np.testing.assert_allclose(mat.T @ mat, np.eye(3), atol=1e-12)
        u, v = project(dict(cam, mat=mat), ee, 64, 48)
        assert (u, v) == (32, 24)
