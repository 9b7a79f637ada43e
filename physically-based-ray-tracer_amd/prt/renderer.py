"""Host-side mirror of the reference's Renderer / Scene / Camera API surface (Core/Renderer.h:12-112,
Core/Scene.h:12-80, Core/Camera.h:198-231), driving the MI355X hot path through the C ABI (include/prt.h).

The reference's hot loop (Renderer::Tick's OpenMP pixel loop + Renderer::Trace) becomes one
prt_render() call per Tick; everything Trace reads (models, BLAS instances, lights, sky, camera
basis) is handed over once and stays resident in HBM.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import check

F32 = np.float32


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


@dataclass
class LightTransform:
    """LightTransform (Core/LightTransform.cpp:4-23): position, color, rotation."""
    position: np.ndarray
    color: np.ndarray
    rotation: np.ndarray = field(default_factory=lambda: np.zeros(3, F32))


class Camera:
    """Camera (Core/Camera.cpp:6-37,113-139): screen plane at 2*ahead, height 2, width 2*aspect."""

    def __init__(self, camPos, camTarget, aspect):
        self.camPos = _f32(camPos)
        self.camTarget = _f32(camTarget)
        self.aspect = np.float32(aspect)
        # post-process members (Core/Camera.h:12,23,27), read when Renderer.isPostProcessed is set
        self.colorGrading = np.ones(4, F32)
        self.fov, self.distortion, self.vignetteIntensity, self.vignetteRadius = 40.0, 40.0, 20.0, 0.3
        self.abberationIntensity = 0
        self.update()

    def postfx(self, enabled=True):
        pf = _lib.PostFx()
        pf.enabled = 1 if enabled else 0
        pf.aberration = int(self.abberationIntensity)
        pf.fov, pf.distortion = float(self.fov), float(self.distortion)
        pf.vignette_intensity, pf.vignette_radius = float(self.vignetteIntensity), float(self.vignetteRadius)
        for i in range(4):
            pf.color_grading[i] = float(self.colorGrading[i])
        return pf

    def update(self):
        L = _lib.load()
        cd = _lib.CameraDesc()
        check(L.prt_camera_look_at(self.camPos.ctypes.data, self.camTarget.ctypes.data, C.c_float(self.aspect),
                                   C.byref(cd)))
        self.desc = cd
        self.topLeft = np.array(cd.top_left[:], F32)
        self.topRight = np.array(cd.top_right[:], F32)
        self.bottomLeft = np.array(cd.bottom_left[:], F32)
        self.right = np.array(cd.right[:], F32)
        self.up = np.array(cd.up[:], F32)
        self.ahead = np.array(cd.ahead[:], F32)


def postfx_preset(preset=0, **overrides):
    """prt_postfx with Renderer::isPostProcessed on: preset 0 = the Camera member defaults, 1 = the GAME
    preset P1 (Core/Camera.cpp:18-23); keyword overrides set single fields (color_grading: 4 floats)."""
    pf = _lib.PostFx()
    check(_lib.load().prt_postfx_preset(preset, C.byref(pf)))
    for k, v in overrides.items():
        if k == "color_grading":
            for i in range(4):
                pf.color_grading[i] = float(v[i])
        else:
            setattr(pf, k, v)
    return pf


class Scene:
    """Scene (Core/Scene.h): models, BLAS instances (gameobject -> modelIndex + transform), lights, sky."""

    def __init__(self):
        self.models = []          # scenes.Mesh (Model fat-triangle arrays)
        self.textures = []        # (h, w) uint32 0x00RRGGBB
        self.blases = []          # (modelIndex, 4x4 row-major transform)
        self.pointLights = [LightTransform(np.zeros(3, F32), np.zeros(3, F32)) for _ in range(4)]
        self.directionalLights = []
        self.spotlights = []
        self.sky = None           # (h, w, 3) float32
        self.materials = None     # per-blas material kind (_lib.MAT_*), None = all textured (Scene.cpp:193-205)
        self.areaLights = []      # at most one dict(corner, edge_u, edge_v, radiance, two_sided) (AreaLight.h)

    @classmethod
    def from_data(cls, sd):
        s = cls()
        s.models = list(sd.meshes)
        s.textures = list(sd.textures)
        s.blases = [(m, np.asarray(T, F32)) for m, T in sd.instances]
        lt = sd.lights
        s.pointLights = [LightTransform(_f32(lt.point_pos[i]), _f32(lt.point_col[i])) for i in range(4)]
        s.directionalLights = [LightTransform(_f32(lt.dir_pos), _f32(lt.dir_col))]
        s.spotlights = [LightTransform(_f32(lt.spot_pos), _f32(lt.spot_col), _f32(lt.spot_rot))]
        s.sky = sd.sky
        s.materials = list(sd.materials) if sd.materials is not None else None
        s.areaLights = [dict(sd.area_light)] if sd.area_light is not None else []
        return s

    @property
    def tri_count(self):
        return sum(self.models[m].tri_count for m, _ in self.blases)


class Context:
    """One prt_ctx on one HIP device (one process per GPU)."""

    def __init__(self, device: int = 0, group=None, tile: int = 32):
        """group: a list of device ordinals -> one context over several GPUs of this process
        (prt_create_group: pixel tiles rendered concurrently, gathered on the first device); a device may
        repeat, which runs several shards on one GPU."""
        L = _lib.load()
        n = C.c_int32(0)
        check(L.prt_device_count(C.byref(n)))
        if n.value <= 0:
            raise _lib.PrtError("no HIP device visible (the product path has no CPU fallback)")
        h = C.c_void_p()
        if group is None:
            check(L.prt_create(C.byref(_lib.DeviceDesc(device, 0)), C.byref(h)))
        else:
            devs = (_lib.DeviceDesc * len(group))(*[_lib.DeviceDesc(int(d), 0) for d in group])
            check(L.prt_create_group(devs, len(group), tile, C.byref(h)))
            device = int(group[0])
        self.L = L
        self.h = h
        self.device = device

    # -- multi-GPU inside the boundary (include/prt.h, prt_shard_*)
    @staticmethod
    def shard_unique_id() -> bytes:
        """A fresh RCCL id (rank 0 makes it, the caller carries the bytes to the other ranks)."""
        buf = (C.c_uint8 * _lib.SHARD_ID_BYTES)()
        check(_lib.load().prt_shard_unique_id(buf))
        return bytes(buf)

    def shard_rccl(self, uid: bytes, rank: int, world: int, tile: int = 32):
        """Join the RCCL communicator of `uid` as `rank` of `world`: prt_render then renders this rank's
        pixel tiles and gathers the frame on rank 0 (one ncclGather per frame, on the context stream)."""
        if len(uid) != _lib.SHARD_ID_BYTES:
            raise ValueError("RCCL id must be %d bytes" % _lib.SHARD_ID_BYTES)
        buf = (C.c_uint8 * _lib.SHARD_ID_BYTES).from_buffer_copy(uid)
        check(self.L.prt_shard_init_rccl(self.h, buf, rank, world, tile))

    def shard_info(self):
        si = _lib.ShardInfo()
        check(self.L.prt_get_shard_info(self.h, C.byref(si)))
        return si

    def close(self):
        if self.h:
            self.L.prt_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- scene upload
    def set_scene(self, scene: Scene):
        L = self.L
        keep = []
        texs = (_lib.Texture * max(1, len(scene.textures)))()
        for i, t in enumerate(scene.textures):
            t = np.ascontiguousarray(t, np.uint32)
            keep.append(t)
            texs[i] = _lib.Texture(t.shape[1], t.shape[0], t.ctypes.data)
        check(L.prt_set_textures(self.h, texs, len(scene.textures)))
        ms = (_lib.Mesh * len(scene.models))()
        for i, m in enumerate(scene.models):
            arrs = [_f32(m.triangles), _f32(m.fixed_normals), _f32(m.fixed_uvs),
                    np.ascontiguousarray(m.indices, np.int32), _f32(m.vertices), _f32(m.face_normals)]
            keep.extend(arrs)
            ms[i] = _lib.Mesh(m.tri_count, m.vertices.size // 3, *[a.ctypes.data for a in arrs], m.albedo, m.normal,
                              m.metalness, m.emission)
        check(L.prt_set_meshes(self.h, ms, len(scene.models)))
        xf = _f32(np.stack([T for _, T in scene.blases]).reshape(-1))
        mi = np.ascontiguousarray([m for m, _ in scene.blases], np.uint32)
        check(L.prt_set_instances(self.h, xf.ctypes.data, mi.ctypes.data, len(scene.blases)))
        self.set_materials(scene.materials)
        self.set_area_light(scene.areaLights[0] if scene.areaLights else None)
        lt = _lib.Lights()
        for i in range(4):
            lt.point_pos[i][:] = [float(v) for v in scene.pointLights[i].position]
            lt.point_color[i][:] = [float(v) for v in scene.pointLights[i].color]
        d, s = scene.directionalLights[0], scene.spotlights[0]
        lt.dir_pos[:] = [float(v) for v in d.position]
        lt.dir_color[:] = [float(v) for v in d.color]
        lt.spot_pos[:] = [float(v) for v in s.position]
        lt.spot_color[:] = [float(v) for v in s.color]
        lt.spot_rot[:] = [float(v) for v in s.rotation]
        check(L.prt_set_lights(self.h, C.byref(lt)))
        if scene.sky is not None:
            sky = _f32(scene.sky)
            check(L.prt_set_sky(self.h, sky.ctypes.data, sky.shape[1], sky.shape[0]))
        else:
            check(L.prt_set_sky(self.h, None, 0, 0))

    def set_instances(self, blases):
        """Per-frame instance update (physics moved the game objects, Core/Renderer.cpp:33-41): the transforms
        go to the device and are refit there in stream order, so frames already queued keep the old ones."""
        xf = _f32(np.stack([T for _, T in blases]).reshape(-1))
        mi = np.ascontiguousarray([m for m, _ in blases], np.uint32)
        check(self.L.prt_set_instances(self.h, xf.ctypes.data, mi.ctypes.data, len(blases)))

    def set_materials(self, kinds=None):
        """Per-instance material kinds (_lib.MAT_TEXTURED / MAT_DIELECTRIC / MAT_MIRROR), None = all textured."""
        if kinds is None:
            check(self.L.prt_set_instance_materials(self.h, None, 0))
            return
        k = np.ascontiguousarray(kinds, np.int32)
        check(self.L.prt_set_instance_materials(self.h, k.ctypes.data, len(k)))

    def set_area_light(self, al=None):
        """One area light (dict: corner, edge_u, edge_v, radiance, two_sided) or None."""
        if al is None:
            check(self.L.prt_set_area_lights(self.h, None, 0))
            return
        a = _lib.AreaLight()
        a.corner[:] = [float(v) for v in al["corner"]]
        a.edge_u[:] = [float(v) for v in al["edge_u"]]
        a.edge_v[:] = [float(v) for v in al["edge_v"]]
        a.radiance[:] = [float(v) for v in al["radiance"]]
        a.two_sided = 1 if al.get("two_sided", False) else 0
        check(self.L.prt_set_area_lights(self.h, C.byref(a), 1))

    def set_camera(self, cam: Camera):
        check(self.L.prt_set_camera(self.h, C.byref(cam.desc)))

    def set_postfx(self, pf=None):
        """Post-processing on (a prt_postfx, see postfx_preset) or off (None)."""
        if pf is None:
            pf = _lib.PostFx()
        check(self.L.prt_set_postfx(self.h, C.byref(pf)))

    def set_bvh_builder(self, builder):
        """BLAS builder for the next set_scene: _lib.BUILDER_HOST_SAH (default), _lib.BUILDER_GPU_LBVH,
        _lib.BUILDER_HOST_SBVH (spatial splits) or _lib.BUILDER_GPU_PLOC."""
        check(self.L.prt_set_bvh_builder(self.h, builder))

    def scene_info(self):
        si = _lib.SceneInfo()
        check(self.L.prt_get_scene_info(self.h, C.byref(si)))
        return si

    # -- rendering
    def render(self, width, height, spp, bounces, flags=_lib.FLAGS_DEFAULT, mode=0, frame_index=0, seed=0,
               avg=None, rgb8=None, device_out=False, stats=True):
        p = _lib.RenderParams(width, height, spp, bounces, flags, mode, frame_index, seed)
        st = _lib.Stats() if stats else None
        if not device_out:
            if avg is None:
                avg = np.zeros((height * width, 4), F32)
            if rgb8 is None:
                rgb8 = np.zeros(height * width, np.uint32)
            pa, pr = avg.ctypes.data, rgb8.ctypes.data
        else:
            pa, pr = avg, rgb8  # raw device pointers (ints) or None
        check(self.L.prt_render(self.h, C.byref(p), pa, pr, _lib.OUT_DEVICE if device_out else 0,
                                C.byref(st) if st is not None else None))
        return avg, rgb8, _checked(st)

    def reset_accumulation(self, full=True):
        check(self.L.prt_reset_accumulation(self.h, 1 if full else 0))

    def ray_totals(self, reset=False):
        """(segments, shadow_rays) of every render since creation or the last reset, counted on the device
        (prt_ray_totals): a frame loop can count rays without stats=True, which waits for each frame."""
        seg, sh = C.c_uint64(), C.c_uint64()
        check(self.L.prt_ray_totals(self.h, C.byref(seg), C.byref(sh), 1 if reset else 0))
        return int(seg.value), int(sh.value)

    def save_accumulation(self) -> bytes:
        """The accumulation state (accumulator, samplesPerPixel, distances) as an opaque blob
        (prt_save_accumulation); b"" before the first render."""
        n = C.c_uint64()
        check(self.L.prt_accumulation_bytes(self.h, C.byref(n)))
        if n.value == 0:
            return b""
        buf = (C.c_uint8 * n.value)()
        check(self.L.prt_save_accumulation(self.h, buf, n.value))
        return bytes(buf)

    def load_accumulation(self, blob: bytes):
        buf = (C.c_uint8 * len(blob)).from_buffer_copy(blob)
        check(self.L.prt_load_accumulation(self.h, buf, len(blob)))

    def trace_primary(self, width, height):
        hits = np.zeros(width * height, dtype=[("t", F32), ("u", F32), ("v", F32), ("prim", np.uint32),
                                               ("inst", np.uint32)])
        st = _lib.Stats()
        check(self.L.prt_trace_primary(self.h, width, height, hits.ctypes.data, 0, C.byref(st)))
        return hits, _checked(st)

    def intersect(self, O, D, tmax=None):
        O, D = _f32(O), _f32(D)
        n = O.shape[0]
        tm = _f32(tmax) if tmax is not None else None
        hits = np.zeros(n, dtype=[("t", F32), ("u", F32), ("v", F32), ("prim", np.uint32), ("inst", np.uint32)])
        check(self.L.prt_intersect(self.h, n, O.ctypes.data, D.ctypes.data,
                                   tm.ctypes.data if tm is not None else None, hits.ctypes.data))
        return hits

    def occluded(self, O, D, tmax):
        O, D, tm = _f32(O), _f32(D), _f32(tmax)
        occ = np.zeros(O.shape[0], np.int32)
        check(self.L.prt_occluded(self.h, O.shape[0], O.ctypes.data, D.ctypes.data, tm.ctypes.data, occ.ctypes.data))
        return occ

    def brdf_probe(self, op, records):
        """prt_brdf_probe: the device BRDF functions on n records (float32 [n, 24] in, [n, 8] out; include/prt.h)."""
        rec = np.ascontiguousarray(records, np.float32).reshape(-1, 24)
        out = np.zeros((rec.shape[0], 8), np.float32)
        check(self.L.prt_brdf_probe(self.h, int(op), rec.shape[0], rec.ctypes.data, out.ctypes.data))
        return out

    def tile_buffer_pixels(self, width, height, tile, world):
        n = C.c_int64(0)
        check(self.L.prt_tile_buffer_pixels(width, height, tile, world, C.byref(n)))
        return n.value

    def render_tiles(self, width, height, spp, bounces, tile, rank, world, tiles_dev_ptr, flags=_lib.FLAGS_DEFAULT,
                     mode=0, frame_index=0, seed=0, stats=False):
        p = _lib.RenderParams(width, height, spp, bounces, flags, mode, frame_index, seed)
        st = _lib.Stats() if stats else None
        check(self.L.prt_render_tiles(self.h, C.byref(p), tile, rank, world, tiles_dev_ptr,
                                      C.byref(st) if st is not None else None))
        return _checked(st)

    def untile(self, gathered_dev_ptr, width, height, tile, world, avg_dev_ptr, rgb8_dev_ptr):
        check(self.L.prt_untile(self.h, gathered_dev_ptr, width, height, tile, world, avg_dev_ptr, rgb8_dev_ptr))

    def set_stream(self, stream_ptr):
        check(self.L.prt_set_stream(self.h, stream_ptr))

    def set_frames_in_flight(self, n):
        """prt_set_frames_in_flight: with n = 2 a render with device outputs overlaps the previous one; its outputs
        are complete in the context stream's order once the next render is enqueued or finish() was called."""
        check(self.L.prt_set_frames_in_flight(self.h, int(n)))

    def finish(self):
        """prt_finish: the context stream waits for every frame in flight."""
        check(self.L.prt_finish(self.h))


def _checked(st):
    """Stats of a call whose context has dropped a traversal stack group (prt_stats.stack_overflows) raise:
    such a render may have lost hits, and the host sizes the stacks so that it cannot happen."""
    if st is not None and st.stack_overflows:
        raise _lib.PrtError(f"traversal stack overflow: {st.stack_overflows} node groups dropped")
    return st


class Renderer:
    """Renderer (Core/Renderer.h:12-112): public flags + Tick().  Tick() renders one reference frame
    (two camera paths per pixel with AA) and folds it into the progressive accumulator; screen holds
    the packed 0x00RRGGBB pixels, average the float average (Core/Renderer.cpp:22-148)."""

    RENDER_STATES = dict(BRDF=0, BASECOLOR=1, GEOMETRYNORMAL=2, SHADINGNORMAL=3, METAL=4, ROUGHNESS=5, EMMISIVE=6)

    def __init__(self, scene: Scene, camera: Camera, width: int, height: int, device: int = 0):
        self.accumulates = True
        self.bounces = 2
        self.renderingMode = 0
        self.LIGHTED = self.GAMMACORRECTED = self.NORMALMAPPED = self.SKYBOX = self.AA = self.isStochastic = True
        self.isPostProcessed = False
        self.width, self.height = width, height
        self.scene, self.camera = scene, camera
        self.ctx = Context(device)
        self.frame = 0
        self.seed = 0
        self.screen = np.zeros(width * height, np.uint32)
        self.average = np.zeros((width * height, 4), F32)
        self.last_stats = None
        self.Init()

    def Init(self):
        self.ctx.set_scene(self.scene)
        self.ctx.set_camera(self.camera)

    def flags(self):
        f = 0
        for bit, on in ((_lib.FLAG_AA, self.AA), (_lib.FLAG_ACCUMULATE, self.accumulates),
                        (_lib.FLAG_GAMMA, self.GAMMACORRECTED), (_lib.FLAG_NORMALMAP, self.NORMALMAPPED),
                        (_lib.FLAG_SKYBOX, self.SKYBOX), (_lib.FLAG_LIGHTED, self.LIGHTED),
                        (_lib.FLAG_STOCHASTIC, self.isStochastic)):
            if on:
                f |= bit
        return f

    def Tick(self, deltaTime: float = 0.0, frames: int = 1):
        spp = frames * (2 if self.AA else 1)
        self.ctx.set_postfx(self.camera.postfx(self.isPostProcessed))
        _, _, st = self.ctx.render(self.width, self.height, spp, self.bounces, self.flags(), self.renderingMode,
                                   self.frame, self.seed, avg=self.average, rgb8=self.screen)
        self.frame += frames
        self.last_stats = st
        return st

    def Capture(self, path):
        """Renderer::Capture (Core/Renderer.cpp:437-465): the screen as a PNG (the reference names it by time)."""
        from .ingest import capture_png
        capture_png(path, self.screen, self.width, self.height)

    def SaveCheckpoint(self, path):
        """Checkpoint of a long progressive render: the accumulation state plus the frame counter and
        seed the RNG stream continues from, as an .npz of plain arrays (load with allow_pickle=False)."""
        blob = np.frombuffer(self.ctx.save_accumulation(), np.uint8)
        # through a file handle: np.savez(<str>) would append ".npz" to a path without it, and LoadCheckpoint(path)
        # would then look for a file that does not exist
        with open(path, "wb") as f:
            np.savez(f, accumulation=blob, frame=np.int64(self.frame), seed=np.int64(self.seed),
                     size=np.array([self.width, self.height], np.int64))

    def LoadCheckpoint(self, path):
        """Resume from SaveCheckpoint: the next Tick continues the same frame sequence bit for bit."""
        with open(path, "rb") as f:
            z = dict(np.load(f, allow_pickle=False))
        if tuple(int(v) for v in z["size"]) != (self.width, self.height):
            raise ValueError("checkpoint of another image size")
        self.ctx.load_accumulation(z["accumulation"].tobytes())
        self.frame, self.seed = int(z["frame"]), int(z["seed"])

    def CameraMoved(self):
        """Camera::HandleInput returned true: memset of the accumulator only (Core/Renderer.cpp:147)."""
        self.ctx.set_camera(self.camera)
        self.ctx.reset_accumulation(full=False)
