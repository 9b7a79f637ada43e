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


def dump_scene(sd, W, H, path):
    """Binary scene file read by tests/cpp/render_scene.cpp (the C++ host mirror, include/prt_renderer.hpp).
    Little-endian: b"PRTS", int32 W, H; camera pos[3], target[3], aspect (f32); lights: 39 f32 in prt_lights
    order; sky: int32 w, h + w*h*3 f32; textures: int32 n + per texture int32 w, h + w*h u32; meshes:
    int32 n + per mesh int32 T, V, 4 texture ids + triangles 12T f32, normals 12T f32, uvs 6T f32,
    indices 3T i32, vertices 3V f32, face normals 3T f32; instances: int32 n + per instance 16 f32, u32 mesh;
    then the extensions (materials, area light) as written below."""
    import struct
    F = np.float32
    with open(path, "wb") as f:
        f.write(b"PRTS")
        f.write(struct.pack("<ii", W, H))
        f.write(np.asarray(sd.cam_pos, F).tobytes() + np.asarray(sd.cam_target, F).tobytes())
        f.write(np.array([np.float32(W) / np.float32(H)], F).tobytes())
        L = sd.lights
        f.write(np.concatenate([np.asarray(a, F).ravel() for a in (L.point_pos, L.point_col, L.dir_pos, L.dir_col,
                                                                     L.spot_pos, L.spot_col, L.spot_rot)]).tobytes())
        if sd.sky is None:
            f.write(struct.pack("<ii", 0, 0))
        else:
            f.write(struct.pack("<ii", sd.sky.shape[1], sd.sky.shape[0]) + np.ascontiguousarray(sd.sky, F).tobytes())
        f.write(struct.pack("<i", len(sd.textures)))
        for t in sd.textures:
            f.write(struct.pack("<ii", t.shape[1], t.shape[0]) + np.ascontiguousarray(t, np.uint32).tobytes())
        f.write(struct.pack("<i", len(sd.meshes)))
        for m in sd.meshes:
            f.write(struct.pack("<iiiiii", m.tri_count, m.vertices.size // 3, m.albedo, m.normal, m.metalness,
                                m.emission))
            for a, dt in ((m.triangles, F), (m.fixed_normals, F), (m.fixed_uvs, F), (m.indices, np.int32),
                          (m.vertices, F), (m.face_normals, F)):
                f.write(np.ascontiguousarray(a, dt).tobytes())
        f.write(struct.pack("<i", len(sd.instances)))
        for mi, xf in sd.instances:
            f.write(np.ascontiguousarray(xf, F).tobytes() + struct.pack("<I", mi))
        # extensions: int32 material per instance (all 0 when None); int32 area flag + 12 f32 + int32 two_sided
        mats = sd.materials if sd.materials is not None else [0] * len(sd.instances)
        f.write(np.asarray(mats, np.int32).tobytes())
        al = sd.area_light
        f.write(struct.pack("<i", 0 if al is None else 1))
        if al is not None:
            f.write(np.concatenate([np.asarray(al[k], F) for k in ("corner", "edge_u", "edge_v", "radiance")]).tobytes())
            f.write(struct.pack("<i", 1 if al.get("two_sided", False) else 0))
