#!/usr/bin/env python3
"""Generate the committed golden fixtures from the reference's own tinybvh (oracle/_ref).

oracle/_ref/libref_tinybvh.so is compiled by oracle/Makefile from /root/reference/Core/tiny_bvh.h
(v1.4.2, unmodified; BVH8_CPU::BuildHQ BLASes + TLAS, the structures Core/Scene.cpp:43,222 builds) and
is only available where /root/reference exists.  The fixtures it produces hold inputs and reference
outputs only, so the parity tests run anywhere (CPU here, GPU box) without the reference:

  c2_primary.npz   C2 torus (10k tris), primary rays at 160x90: O, D in; tinybvh t/u/v/prim/inst out
  multi_rays.npz   multi-instance heightfield (TLAS path), 8192 random rays: closest-hit records,
                   and IsOccluded for tmax = 0.999 t (every third ray tmax = 1e30)
  trace_64x48.npz  the oracle's Trace (Core/Renderer.cpp:150-406 restated) running on tinybvh's BVH8_CPU
                   traversal: avg RGBA, RGB8, segment / shadow-ray counts.  The traversal half is the
                   reference's; the shading half is the restatement (BRDF.cpp is unbuildable here).
  many_inst.npz    scenes.instance_field(300) (301 instances: tinybvh's TLAS over them), 8192 random rays:
                   closest-hit records and IsOccluded as multi_rays; plus a 96x64, 2 spp, depth 3 render
The headline configs, through the same reference traversal (`make_golden.py ref`):
  c4_ref_crop.npz      C4 1920x1080, 4 spp, depth 4: whole-frame ray counts + digests, a 480x270 window's pixels
  c3_ref_480x270.npz   C3 at 480x270, 4 spp, depth 4: the whole frame
  c2_ref_1280x720.npz  C2 primary rays at the full 1280x720: prim per pixel, digests of t / u / v
  c1_scene1.npz        C1 as data (the SciFiHelmet arrays the ingest reads from the reference's glTF, scene1's
                       instance / lights / camera, stand-in maps) + its 256x256 1 spp depth-1 renders
  spaceship.npz        the textured Spaceship (scenes.config_spaceship) as data -- indexed mesh arrays, the three
                       1024x1024 maps as decoded texels, two instances, lights, sky, camera -- plus its
                       reference-traversal renders at 160x160: shaded (4 spp, depth 3), albedo and shading-normal views
Every fixture records a digest of the scene arrays it was made from, so a change of scenes.py is caught.

usage: python tests/golden/make_golden.py [small] [inst] [ref] [ship]
"""
import hashlib
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "physically-based-ray-tracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import oracle  # noqa: E402
from helpers import primary_dirs, random_rays  # noqa: E402
from prt import scenes  # noqa: E402


def scene_digest(sd):
    h = hashlib.sha256()
    for m in sd.meshes:
        for a in (m.triangles, m.fixed_normals, m.fixed_uvs, m.indices, m.vertices, m.face_normals):
            h.update(np.ascontiguousarray(a).tobytes())
    for t in sd.textures:
        h.update(np.ascontiguousarray(t).tobytes())
    for mi, xf in sd.instances:
        h.update(np.int64(mi).tobytes())
        h.update(np.ascontiguousarray(xf, np.float32).tobytes())
    L = sd.lights
    for a in (L.point_pos, L.point_col, L.dir_pos, L.dir_col, L.spot_pos, L.spot_col, L.spot_rot):
        h.update(np.ascontiguousarray(a, np.float32).tobytes())
    if sd.sky is not None:
        h.update(np.ascontiguousarray(sd.sky).tobytes())
    h.update(np.ascontiguousarray(sd.cam_pos, np.float32).tobytes())
    h.update(np.ascontiguousarray(sd.cam_target, np.float32).tobytes())
    return h.hexdigest()


def c2_primary():
    sd = scenes.config_c2()
    W, H = 160, 90
    osc = oracle.OracleScene(sd, W, H)
    pos, tl, tr, bl = osc.camera_basis(W, H)
    D = primary_dirs(pos, tl, tr, bl, W, H)
    O = np.broadcast_to(pos, D.shape).astype(np.float32)
    t, u, v, p, i = oracle.RefScene(sd).intersect(O, D)
    np.savez_compressed(os.path.join(HERE, "c2_primary.npz"), W=W, H=H, O=O[:1], D=D, t=t, u=u, v=v, prim=p,
                        inst=i, digest=scene_digest(sd))
    return int((t < 1e30).sum())


def multi_rays():
    sd = scenes.multi_instance(scenes.config_small(60, 40))
    O, D = random_rays(sd, 8192, seed=11)
    ref = oracle.RefScene(sd)
    t, u, v, p, i = ref.intersect(O, D)
    tmax = np.where(t < 1e30, t * np.float32(0.999), np.float32(1e30)).astype(np.float32)
    tmax[::3] = np.float32(1e30)
    occ = ref.occluded(O, D, tmax)
    np.savez_compressed(os.path.join(HERE, "multi_rays.npz"), O=O, D=D, t=t, u=u, v=v, prim=p, inst=i, tmax=tmax,
                        occ=occ, digest=scene_digest(sd))
    return int((t < 1e30).sum())


def many_inst():
    sd = scenes.instance_field(300)
    O, D = random_rays(sd, 8192, seed=13)
    ref = oracle.RefScene(sd)
    t, u, v, p, i = ref.intersect(O, D)
    tmax = np.where(np.arange(len(t)) % 3 == 0, np.float32(1e30), t * np.float32(0.999)).astype(np.float32)
    occ = ref.occluded(O, D, tmax)
    W, H = 96, 64
    avg, rgb8, _, st = _ref_render(sd, W, H, 2, 3)
    np.savez_compressed(os.path.join(HERE, "many_inst.npz"), O=O, D=D, t=t, u=u, v=v, prim=p, inst=i, tmax=tmax, occ=occ,
                        W=W, H=H, avg=avg[:, :3].copy(), rgb8=rgb8, segments=int(st.segments),
                        shadow_rays=int(st.shadow_rays), digest=scene_digest(sd))
    return int((t < 1e30).sum()), int((i[t < 1e30] > 0).sum())


def trace_small():
    sd = scenes.multi_instance(scenes.config_small(50, 40))
    W, H = 64, 48
    osc = oracle.OracleScene(sd, W, H)
    osc.use_reference_traversal()
    avg, rgb8, _, st = osc.render(W, H, spp=4, bounces=4)
    np.savez_compressed(os.path.join(HERE, "trace_64x48.npz"), W=W, H=H, spp=4, bounces=4, flags=oracle.DEFAULT_FLAGS,
                        avg=avg, rgb8=rgb8, segments=int(st.segments), shadow_rays=int(st.shadow_rays),
                        digest=scene_digest(sd))
    return int(st.segments)


def _ref_render(sd, W, H, spp, bounces, flags=oracle.DEFAULT_FLAGS, mode=0):
    """The restated Trace on tinybvh's BVH8_CPU + TLAS traversal (the reference's hot path minus BRDF.cpp)."""
    osc = oracle.OracleScene(sd, W, H)
    osc.use_reference_traversal()
    return osc.render(W, H, spp=spp, bounces=bounces, flags=flags, mode=mode, nthreads=os.cpu_count() or 1)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# window of the C4 frame kept in c4_ref_crop.npz (x0, y0, w, h): the centre of the 1920x1080 frame
C4_CROP = (720, 405, 480, 270)


def c4_ref_crop():
    """C4 (1M tris, 1920x1080, 4 spp, depth 4, all reference features) through the reference traversal: the
    whole frame's ray counts and digests, and the avg RGB / RGB8 of a 480x270 window."""
    sd = scenes.config_c4()
    W, H = 1920, 1080
    avg, rgb8, _, st = _ref_render(sd, W, H, 4, 4)
    x0, y0, w, h = C4_CROP
    a = avg.reshape(H, W, 4)[y0:y0 + h, x0:x0 + w, :3]
    r = rgb8.reshape(H, W)[y0:y0 + h, x0:x0 + w]
    np.savez_compressed(os.path.join(HERE, "c4_ref_crop.npz"), W=W, H=H, spp=4, bounces=4, flags=oracle.DEFAULT_FLAGS,
                        crop=np.array(C4_CROP), avg=a, rgb8=r, segments=int(st.segments),
                        shadow_rays=int(st.shadow_rays), avg_sha=sha(avg), rgb8_sha=sha(rgb8), digest=scene_digest(sd))
    return int(st.segments), int(st.shadow_rays)


def c3_ref():
    """C3 (100k tris) at 480x270, 4 spp, depth 4 through the reference traversal: the whole frame."""
    sd = scenes.config_c3()
    W, H = 480, 270
    avg, rgb8, _, st = _ref_render(sd, W, H, 4, 4)
    np.savez_compressed(os.path.join(HERE, "c3_ref_480x270.npz"), W=W, H=H, spp=4, bounces=4,
                        flags=oracle.DEFAULT_FLAGS, avg=avg[:, :3].copy(), rgb8=rgb8, segments=int(st.segments),
                        shadow_rays=int(st.shadow_rays), digest=scene_digest(sd))
    return int(st.segments), int(st.shadow_rays)


def c2_ref_full():
    """C2 (10k-tri torus) primary rays at the full 1280x720 through tinybvh: the prim of every pixel, and
    digests of the t / u / v arrays (bit-identical records are expected; the 160x90 fixture keeps the values)."""
    sd = scenes.config_c2()
    W, H = 1280, 720
    osc = oracle.OracleScene(sd, W, H)
    pos, tl, tr, bl = osc.camera_basis(W, H)
    D = primary_dirs(pos, tl, tr, bl, W, H)
    O = np.broadcast_to(pos, D.shape).astype(np.float32)
    t, u, v, p, i = oracle.RefScene(sd).intersect(O, D)
    hit = t < 1e30
    prim = np.where(hit, p, np.uint32(0xFFFFFFFF)).astype(np.uint32)
    np.savez_compressed(os.path.join(HERE, "c2_ref_1280x720.npz"), W=W, H=H, prim=prim, t_sha=sha(np.where(hit, t, 0)),
                        u_sha=sha(np.where(hit, u, 0)), v_sha=sha(np.where(hit, v, 0)), digest=scene_digest(sd))
    return int(hit.sum())


def c1_lit(sd):
    """C1 with point light 0 at the camera (colour 3): scene1 as shipped renders its BRDF image black (the camera
    looks into the helmet's lower shell, which blocks the directional light; the point lights are zero and the
    spot's rot = 0 never lights), so this variant checks the shading on the helmet."""
    import dataclasses
    L = sd.lights
    pp, pc = np.array(L.point_pos, np.float32), np.array(L.point_col, np.float32)
    pp[0], pc[0] = sd.cam_pos, (3.0, 3.0, 3.0)
    return dataclasses.replace(sd, lights=dataclasses.replace(L, point_pos=pp, point_col=pc))


C1_RENDERS = (("shipped", 0), ("shipped", 1), ("shipped", 2), ("lit", 0))


def c1_scene1():
    """Config C1 as data: scene1's SciFiHelmet as the ingest reads it from the reference's glTF (indexed positions,
    normals, flipped UVs, corner indices), the XShip instance transform, scene1's lights, prefabs/camera.json and the
    1x1 stand-in maps; plus the reference-traversal renders at 256x256, 1 spp, depth 1 (SKYBOX and AA off)."""
    sd = scenes.config_c1()
    m = sd.meshes[0]
    P = m.vertices.reshape(-1, 3)
    tri = m.indices.reshape(-1, 3)
    N = np.zeros_like(P)
    UV = np.zeros((P.shape[0], 2), np.float32)
    N[m.indices] = m.fixed_normals.reshape(-1, 4)[:, :3]
    UV[m.indices] = m.fixed_uvs.reshape(-1, 2)
    from prt import ingest
    m2 = ingest.mesh_from_indexed(P, N, UV, tri)
    for f in ("triangles", "fixed_normals", "fixed_uvs", "indices", "vertices", "face_normals"):
        assert np.array_equal(getattr(m, f), getattr(m2, f)), f
    W = H = 256
    out = {}
    for variant, mode in C1_RENDERS:
        s = sd if variant == "shipped" else c1_lit(sd)
        avg, rgb8, _, st = _ref_render(s, W, H, 1, 1, flags=scenes.C1_FLAGS, mode=mode)
        out[f"{variant}{mode}_avg"] = avg[:, :3].copy()
        out[f"{variant}{mode}_counts"] = np.array([st.segments, st.shadow_rays], np.int64)
    L = sd.lights
    np.savez_compressed(os.path.join(HERE, "c1_scene1.npz"), P=P, N=N, UV=UV, tri=tri.astype(np.int32),
                        albedo=m.albedo, normal=m.normal, metalness=m.metalness, emission=m.emission,
                        textures=np.stack([t.reshape(-1)[:1] for t in sd.textures]).astype(np.uint32),
                        xf=np.stack([x for _, x in sd.instances]).astype(np.float32),
                        xf_mesh=np.array([mi for mi, _ in sd.instances], np.int32),
                        point_pos=L.point_pos, point_col=L.point_col, dir_pos=L.dir_pos, dir_col=L.dir_col,
                        spot_pos=L.spot_pos, spot_col=L.spot_col, spot_rot=L.spot_rot, cam_pos=sd.cam_pos,
                        cam_target=sd.cam_target, W=W, H=H, flags=scenes.C1_FLAGS, digest=scene_digest(sd), **out)
    return {k: v.tolist() for k, v in out.items() if k.endswith("counts")}


SHIP_RENDERS = (("shaded", 0, 4, 3), ("albedo", 1, 1, 1), ("normal", 3, 1, 1))
SHIP_WH = 160


def ship_flags(spp):
    """reference defaults; a 1-spp render has AA off (SURVEY 8d canonical estimator)"""
    return oracle.DEFAULT_FLAGS if spp > 1 else oracle.DEFAULT_FLAGS & ~1


def indexed(m):
    """(P, N, UV, tri) of a Mesh whose corners were expanded from an indexed model (ingest.mesh_from_indexed)."""
    P = m.vertices.reshape(-1, 3)
    tri = m.indices.reshape(-1, 3)
    N = np.zeros_like(P)
    UV = np.zeros((P.shape[0], 2), np.float32)
    N[m.indices] = m.fixed_normals.reshape(-1, 4)[:, :3]
    UV[m.indices] = m.fixed_uvs.reshape(-1, 2)
    return P, N, UV, tri


def spaceship():
    """The textured Spaceship scene as data, and its reference-traversal renders (SHIP_RENDERS)."""
    sd = scenes.config_spaceship()
    m = sd.meshes[0]
    P, N, UV, tri = indexed(m)
    from prt import ingest
    m2 = ingest.mesh_from_indexed(P, N, UV, tri)
    for f in ("triangles", "fixed_normals", "fixed_uvs", "indices", "vertices", "face_normals"):
        assert np.array_equal(getattr(m, f), getattr(m2, f)), f
    W = H = SHIP_WH
    out = {}
    for name, mode, spp, bounces in SHIP_RENDERS:
        avg, rgb8, _, st = _ref_render(sd, W, H, spp, bounces, flags=ship_flags(spp), mode=mode)
        out[f"{name}_avg"] = avg[:, :3].copy()
        out[f"{name}_rgb8"] = rgb8
        out[f"{name}_counts"] = np.array([st.segments, st.shadow_rays], np.int64)
    L = sd.lights
    np.savez_compressed(os.path.join(HERE, "spaceship.npz"), P=P, N=N, UV=UV, tri=tri.astype(np.int32),
                        albedo=m.albedo, normal=m.normal, metalness=m.metalness, emission=m.emission,
                        tex0=sd.textures[0], tex1=sd.textures[1], tex2=sd.textures[2],
                        xf=np.stack([x for _, x in sd.instances]).astype(np.float32),
                        xf_mesh=np.array([mi for mi, _ in sd.instances], np.int32),
                        point_pos=L.point_pos, point_col=L.point_col, dir_pos=L.dir_pos, dir_col=L.dir_col,
                        spot_pos=L.spot_pos, spot_col=L.spot_col, spot_rot=L.spot_rot, sky=sd.sky,
                        cam_pos=sd.cam_pos, cam_target=sd.cam_target, W=W, H=H, digest=scene_digest(sd), **out)
    return {k: v.tolist() for k, v in out.items() if k.endswith("counts")}


def main():
    if oracle.reflib() is None:
        sys.exit("oracle/_ref/libref_tinybvh.so is missing: run `make -C oracle ref` where /root/reference exists")
    which = sys.argv[1:] or ["small", "ref"]
    if "small" in which:
        print("c2_primary hits", c2_primary())
        print("multi_rays hits", multi_rays())
        print("trace segments", trace_small())
    if "small" in which or "inst" in which:
        print("many_inst hits (all, on tori)", many_inst())
    if "ref" in which:
        print("c4_ref_crop rays", c4_ref_crop())
        print("c3_ref rays", c3_ref())
        print("c2_ref_full hits", c2_ref_full())
        print("c1_scene1", c1_scene1())
    if "ship" in which or "ref" in which:
        print("spaceship", spaceship())


if __name__ == "__main__":
    main()
