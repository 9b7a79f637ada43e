"""Shared test helpers: load one synthetic scene into both the oracle and the GPU context."""
import numpy as np

import oracle
import prt
from prt import scenes

RMSE_TOL = 1e-4  # BASELINE.json north star: per-channel RMSE <= 1e-4 vs the CPU reference


def rmse(a, b):
    d = np.asarray(a, np.float64)[:, :3] - np.asarray(b, np.float64)[:, :3]
    return float(np.sqrt(np.mean(d * d)))


def primary_dirs(pos, tl, tr, bl, W, H):
    """Camera::GetPrimaryRay directions (before the tinybvh ctor normalisation), numpy float32."""
    ys, xs = np.mgrid[0:H, 0:W]
    u = xs.astype(np.float32) * (np.float32(1) / np.float32(W))
    v = ys.astype(np.float32) * (np.float32(1) / np.float32(H))
    P = (tl[None, None, :] + u[..., None] * (tr - tl)[None, None, :]) + v[..., None] * (bl - tl)[None, None, :]
    d = (P - pos).astype(np.float32).reshape(-1, 3)
    dd = (d[:, 0] * d[:, 0] + d[:, 1] * d[:, 1]) + d[:, 2] * d[:, 2]
    return (d * (np.float32(1) / np.sqrt(dd))[:, None]).astype(np.float32)


def gpu_scene(ctx, sd, W, H):
    scene = prt.Scene.from_data(sd)
    cam = prt.Camera(sd.cam_pos, sd.cam_target, np.float32(W) / np.float32(H))
    ctx.set_scene(scene)
    ctx.set_camera(cam)
    ctx.reset_accumulation(full=True)
    return scene, cam


def random_rays(sd, n, seed=1):
    rng = np.random.default_rng(seed)
    O = rng.uniform(-4, 4, (n, 3)).astype(np.float32)
    O[:, 1] = rng.uniform(0.5, 4.0, n).astype(np.float32)
    tgt = rng.uniform(-5, 5, (n, 3)).astype(np.float32)
    tgt[:, 1] = rng.uniform(-0.5, 0.5, n).astype(np.float32)
    D = (tgt - O).astype(np.float32)
    return O, D
