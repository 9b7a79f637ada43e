"""oracle/oracle.py -- TEST INFRASTRUCTURE ONLY.

ctypes binding of the C restatement (oracle/liboracle.so) and of the reference's own
tinybvh compiled into oracle/_ref/libref_tinybvh.so.  Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg -- never by the product.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.environ.get("PRT_ORACLE_LIB") or os.path.join(HERE, "liboracle.so")  # override: sanitizer builds
REFLIB = os.path.join(HERE, "_ref", "libref_tinybvh.so")

AA, ACCUMULATE, GAMMA, NORMALMAP, SKYBOX, LIGHTED, STOCHASTIC = (1 << i for i in range(7))
DEFAULT_FLAGS = AA | ACCUMULATE | GAMMA | NORMALMAP | SKYBOX | LIGHTED | STOCHASTIC  # Core/Renderer.h:33,48


def build() -> None:
    """Compile liboracle.so (and oracle/_ref when /root/reference exists)."""
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)


class Params(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("spp", C.c_int32), ("bounces", C.c_int32),
                ("flags", C.c_uint32), ("render_mode", C.c_int32), ("frame_index", C.c_uint32), ("seed", C.c_uint32)]


class Stats(C.Structure):
    _fields_ = [("segments", C.c_uint64), ("shadow_rays", C.c_uint64), ("paths", C.c_uint64)]


class Backend(C.Structure):
    _fields_ = [("user", C.c_void_p), ("closest", C.c_void_p), ("anyhit", C.c_void_p)]


def _p(a, t=C.c_float):
    return a.ctypes.data_as(C.POINTER(t)) if a is not None else None


_lib = None
_ref = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        L.orc_scene_create.restype = C.c_void_p
        L.orc_scene_destroy.argtypes = [C.c_void_p]
        L.orc_add_texture.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p]
        L.orc_add_mesh.argtypes = [C.c_void_p, C.c_int32] + [C.c_void_p] * 5 + [C.c_int32, C.c_void_p] + [C.c_int32] * 4
        L.orc_add_instance.argtypes = [C.c_void_p, C.c_int32, C.c_void_p]
        L.orc_set_lights.argtypes = [C.c_void_p] + [C.c_void_p] * 7
        L.orc_set_instance_material.argtypes = [C.c_void_p, C.c_int32, C.c_int32]
        L.orc_set_area_light.argtypes = [C.c_void_p, C.c_int32] + [C.c_void_p] * 4 + [C.c_int32]
        L.orc_set_sky.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_void_p]
        L.orc_set_camera.argtypes = [C.c_void_p] + [C.c_void_p] * 4
        L.orc_build.argtypes = [C.c_void_p]
        L.orc_set_backend.argtypes = [C.c_void_p, C.c_void_p]
        L.orc_camera_lookat.argtypes = [C.c_void_p, C.c_void_p, C.c_float, C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_camera_basis.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_set_postfx.argtypes = [C.c_void_p, C.c_int32, C.c_int32] + [C.c_float] * 4 + [C.c_void_p] * 2
        L.orc_render.argtypes = [C.c_void_p, C.POINTER(Params), C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_void_p, C.c_int32, C.POINTER(Stats)]
        L.orc_render_frames.argtypes = [C.c_void_p, C.POINTER(Params), C.c_void_p, C.c_void_p, C.c_int32,
                                        C.POINTER(Stats)]
        L.orc_primary_hits.argtypes = [C.c_void_p, C.c_int32, C.c_int32] + [C.c_void_p] * 5 + [C.c_int32]
        L.orc_intersect.argtypes = [C.c_void_p, C.c_int32] + [C.c_void_p] * 8 + [C.c_int32]
        L.orc_occluded.argtypes = [C.c_void_p, C.c_int32] + [C.c_void_p] * 4 + [C.c_int32]
        L.orc_collect_rays.argtypes = [C.c_void_p, C.POINTER(Params), C.c_int32, C.c_void_p, C.c_int64, C.c_void_p,
                                       C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]
        L.orc_init_seed.argtypes = [C.c_uint32]
        L.orc_init_seed.restype = C.c_uint32
        L.orc_rng_floats.argtypes = [C.c_uint32, C.c_int32, C.c_void_p]
        L.orc_eval_combined_brdf.argtypes = [C.c_void_p] * 5
        L.orc_brdf_probe.argtypes = [C.c_int32, C.c_int32, C.c_void_p, C.c_void_p]
        L.orc_brdf_probability.argtypes = [C.c_void_p] * 3
        L.orc_brdf_probability.restype = C.c_float
        L.orc_eval_indirect.argtypes = [C.c_void_p] * 4 + [C.c_int32, C.c_void_p, C.c_void_p]
        L.orc_sample_sky.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_pack_rgb8.argtypes = [C.c_void_p]
        L.orc_pack_rgb8.restype = C.c_uint32
        _lib = L
    return _lib


def reflib():
    """The reference's own tinybvh (compiled from /root/reference into oracle/_ref), or None."""
    global _ref
    if _ref is None:
        if not os.path.exists(REFLIB):
            return None
        R = C.CDLL(REFLIB)
        R.ref_create.restype = C.c_void_p
        R.ref_destroy.argtypes = [C.c_void_p]
        R.ref_add_mesh.argtypes = [C.c_void_p, C.c_int32, C.c_void_p]
        R.ref_add_instance.argtypes = [C.c_void_p, C.c_int32, C.c_void_p]
        R.ref_build.argtypes = [C.c_void_p]
        R.ref_intersect.argtypes = [C.c_void_p, C.c_int32] + [C.c_void_p] * 8
        R.ref_occluded.argtypes = [C.c_void_p, C.c_int32] + [C.c_void_p] * 4
        R.ref_count_visits.argtypes = [C.c_void_p, C.c_int32] + [C.c_void_p] * 8
        R.ref_count_visits.restype = C.c_int32
        R.ref_count_visits_any.argtypes = [C.c_void_p, C.c_int32] + [C.c_void_p] * 7
        R.ref_count_visits_any.restype = C.c_int32
        _ref = R
    return _ref


def f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


class OracleScene:
    """The restated Scene/Camera/Renderer state, loaded from a scenes.SceneData."""

    def __init__(self, sd, width=None, height=None):
        L = lib()
        self.L = L
        self.sd = sd
        self.h = C.c_void_p(L.orc_scene_create())
        self._keep = []
        for t in sd.textures:
            t = np.ascontiguousarray(t, np.uint32)
            assert L.orc_add_texture(self.h, t.shape[1], t.shape[0], t.ctypes.data) >= 0
        for m in sd.meshes:
            arrs = [f32(m.triangles), f32(m.fixed_normals), f32(m.fixed_uvs),
                    np.ascontiguousarray(m.indices, np.int32), f32(m.vertices), f32(m.face_normals)]
            rc = L.orc_add_mesh(self.h, m.tri_count, arrs[0].ctypes.data, arrs[1].ctypes.data, arrs[2].ctypes.data,
                                arrs[3].ctypes.data, arrs[4].ctypes.data, m.vertices.size // 3, arrs[5].ctypes.data,
                                m.albedo, m.normal, m.metalness, m.emission)
            assert rc >= 0, rc
        for mi, T in sd.instances:
            T = f32(T)
            assert L.orc_add_instance(self.h, mi, T.ctypes.data) >= 0
        lt = sd.lights
        la = [f32(lt.point_pos), f32(lt.point_col), f32(lt.dir_pos), f32(lt.dir_col), f32(lt.spot_pos),
              f32(lt.spot_col), f32(lt.spot_rot)]
        L.orc_set_lights(self.h, *[a.ctypes.data for a in la])
        for i, k in enumerate(getattr(sd, "materials", None) or []):
            assert L.orc_set_instance_material(self.h, i, int(k)) == 0
        al = getattr(sd, "area_light", None)
        if al is not None:
            arr = [f32(al[k]) for k in ("corner", "edge_u", "edge_v", "radiance")]
            self._keep.extend(arr)
            L.orc_set_area_light(self.h, 1, *[a.ctypes.data for a in arr], 1 if al.get("two_sided", False) else 0)
        if sd.sky is not None:
            sky = f32(sd.sky)
            L.orc_set_sky(self.h, sky.shape[1], sky.shape[0], sky.ctypes.data)
        assert L.orc_build(self.h) == 0
        self.width = width
        self.height = height
        if width:
            self.set_camera(width, height)
        self.backend_scene = None

    def camera_basis(self, width, height):
        tl, tr, bl = (np.zeros(3, np.float32) for _ in range(3))
        pos, tgt = f32(self.sd.cam_pos), f32(self.sd.cam_target)
        aspect = np.float32(width) / np.float32(height)
        self.L.orc_camera_lookat(pos.ctypes.data, tgt.ctypes.data, C.c_float(aspect), tl.ctypes.data,
                                 tr.ctypes.data, bl.ctypes.data)
        return pos, tl, tr, bl

    def set_camera(self, width, height):
        pos, tl, tr, bl = self.camera_basis(width, height)
        self.L.orc_set_camera(self.h, pos.ctypes.data, tl.ctypes.data, tr.ctypes.data, bl.ctypes.data)
        self.width, self.height = width, height

    def set_postfx(self, enabled=True, aberration=0, fov=40.0, distortion=40.0, vignette_intensity=20.0,
                   vignette_radius=0.3, color_grading=(1, 1, 1, 1)):
        """Renderer::isPostProcessed + the Camera post-process members (defaults: Core/Camera.h:12,23,27)."""
        basis = np.zeros(9, np.float32)
        pos, tgt = f32(self.sd.cam_pos), f32(self.sd.cam_target)
        self.L.orc_camera_basis(pos.ctypes.data, tgt.ctypes.data, basis.ctypes.data)
        g = f32(color_grading)
        self.L.orc_set_postfx(self.h, int(enabled), int(aberration), fov, distortion, vignette_intensity,
                              vignette_radius, g.ctypes.data, basis.ctypes.data)

    def use_reference_traversal(self):
        """Route closest/any-hit through the reference's tinybvh BVH8_CPU + TLAS (oracle/_ref)."""
        R = reflib()
        if R is None:
            raise RuntimeError("oracle/_ref/libref_tinybvh.so not built")
        rs = RefScene(self.sd)
        self.backend_scene = rs
        be = Backend(C.c_void_p(rs.h.value), C.cast(R.ref_closest, C.c_void_p), C.cast(R.ref_anyhit, C.c_void_p))
        self._be = be
        self.L.orc_set_backend(self.h, C.byref(be))

    def use_builtin_traversal(self):
        self.L.orc_set_backend(self.h, None)

    def render(self, width, height, spp=4, bounces=4, flags=DEFAULT_FLAGS, mode=0, frame_index=0, seed=0,
               state=None, nthreads=0):
        """Renderer::Tick over the reference frames of one spp-sample image; returns (avg_rgba, rgb8, state, stats)."""
        if (width, height) != (self.width, self.height):
            self.set_camera(width, height)
        n = width * height
        if state is None:
            state = new_state(width, height)
        acc, ns, dist = state
        avg = np.zeros((n, 4), np.float32)
        rgb8 = np.zeros(n, np.uint32)
        p = Params(width, height, spp, bounces, flags, mode, frame_index, seed)
        st = Stats()
        rc = self.L.orc_render(self.h, C.byref(p), acc.ctypes.data, ns.ctypes.data, dist.ctypes.data, avg.ctypes.data,
                               rgb8.ctypes.data, nthreads, C.byref(st))
        assert rc == 0, rc
        return avg, rgb8, state, st

    def render_frames(self, width, height, spp=4, bounces=4, flags=DEFAULT_FLAGS, mode=0, frame_index=0, seed=0,
                      nthreads=0):
        if (width, height) != (self.width, self.height):
            self.set_camera(width, height)
        F = nframes(spp, flags)
        out = np.zeros((F, width * height, 4), np.float32)
        tp = np.zeros((F, width * height), np.float32)
        p = Params(width, height, spp, bounces, flags, mode, frame_index, seed)
        st = Stats()
        assert self.L.orc_render_frames(self.h, C.byref(p), out.ctypes.data, tp.ctypes.data, nthreads,
                                        C.byref(st)) == 0
        return out, tp, st

    def collect_rays(self, width, height, spp=4, bounces=4, flags=DEFAULT_FLAGS, stride=97, cap=4_000_000):
        """(O, D, tmax) of every closest-hit and shadow ray Trace fires for every stride-th pixel."""
        if (width, height) != (self.width, self.height):
            self.set_camera(width, height)
        cl = np.zeros((cap, 7), np.float32)
        an = np.zeros((cap, 7), np.float32)
        nc, na = C.c_int64(0), C.c_int64(0)
        p = Params(width, height, spp, bounces, flags, 0, 0, 0)
        assert self.L.orc_collect_rays(self.h, C.byref(p), stride, cl.ctypes.data, cap, an.ctypes.data, cap,
                                       C.byref(nc), C.byref(na)) == 0
        assert nc.value <= cap and na.value <= cap
        return cl[:nc.value], an[:na.value]

    def primary_hits(self, width, height, nthreads=0):
        if (width, height) != (self.width, self.height):
            self.set_camera(width, height)
        n = width * height
        t, u, v = (np.zeros(n, np.float32) for _ in range(3))
        prim, inst = np.zeros(n, np.uint32), np.zeros(n, np.uint32)
        assert self.L.orc_primary_hits(self.h, width, height, t.ctypes.data, u.ctypes.data, v.ctypes.data,
                                       prim.ctypes.data, inst.ctypes.data, nthreads) == 0
        return t, u, v, prim, inst

    def intersect(self, O, D, tmax=None, nthreads=0):
        O, D = f32(O), f32(D)
        n = O.shape[0]
        tm = f32(tmax) if tmax is not None else None
        t, u, v = (np.zeros(n, np.float32) for _ in range(3))
        prim, inst = np.zeros(n, np.uint32), np.zeros(n, np.uint32)
        assert self.L.orc_intersect(self.h, n, O.ctypes.data, D.ctypes.data, tm.ctypes.data if tm is not None else None,
                                    t.ctypes.data, u.ctypes.data, v.ctypes.data, prim.ctypes.data, inst.ctypes.data,
                                    nthreads) == 0
        return t, u, v, prim, inst

    def occluded(self, O, D, tmax, nthreads=0):
        O, D, tm = f32(O), f32(D), f32(tmax)
        occ = np.zeros(O.shape[0], np.int32)
        assert self.L.orc_occluded(self.h, O.shape[0], O.ctypes.data, D.ctypes.data, tm.ctypes.data, occ.ctypes.data,
                                   nthreads) == 0
        return occ

    def __del__(self):
        try:
            self.L.orc_scene_destroy(self.h)
        except Exception:
            pass


class RefScene:
    """The reference's tinybvh: BVH8_CPU::BuildHQ per mesh + TLAS over instances."""

    def __init__(self, sd):
        R = reflib()
        if R is None:
            raise RuntimeError("oracle/_ref/libref_tinybvh.so not built")
        self.R = R
        self.h = C.c_void_p(R.ref_create())
        self._keep = []
        for m in sd.meshes:
            tri = f32(m.triangles)
            self._keep.append(tri)
            assert R.ref_add_mesh(self.h, m.tri_count, tri.ctypes.data) >= 0
        for mi, T in sd.instances:
            assert R.ref_add_instance(self.h, mi, f32(T).ctypes.data) >= 0
        R.ref_build(self.h)

    def intersect(self, O, D, tmax=None):
        O, D = f32(O), f32(D)
        n = O.shape[0]
        tm = f32(tmax) if tmax is not None else None
        t, u, v = (np.zeros(n, np.float32) for _ in range(3))
        prim, inst = np.zeros(n, np.uint32), np.zeros(n, np.uint32)
        self.R.ref_intersect(self.h, n, O.ctypes.data, D.ctypes.data, tm.ctypes.data if tm is not None else None,
                             t.ctypes.data, u.ctypes.data, v.ctypes.data, prim.ctypes.data, inst.ctypes.data)
        return t, u, v, prim, inst

    def occluded(self, O, D, tmax):
        O, D, tm = f32(O), f32(D), f32(tmax)
        occ = np.zeros(O.shape[0], np.int32)
        self.R.ref_occluded(self.h, O.shape[0], O.ctypes.data, D.ctypes.data, tm.ctypes.data, occ.ctypes.data)
        return occ

    def count_visits(self, O, D, tmax=None):
        O, D = f32(O), f32(D)
        n = O.shape[0]
        tm = f32(tmax) if tmax is not None else None
        sw, sl = np.zeros(n, np.int32), np.zeros(n, np.int32)
        nint, nleaf = C.c_uint64(0), C.c_uint64(0)
        tw = np.zeros(n, np.float32)
        rc = self.R.ref_count_visits(self.h, n, O.ctypes.data, D.ctypes.data, tm.ctypes.data if tm is not None else None,
                                     sw.ctypes.data, sl.ctypes.data, C.byref(nint), C.byref(nleaf), tw.ctypes.data)
        assert rc == 0
        return sw, sl, nint.value, nleaf.value, tw

    def count_visits_any(self, O, D, tmax):
        O, D, tm = f32(O), f32(D), f32(tmax)
        n = O.shape[0]
        ow, ol = np.zeros(n, np.int32), np.zeros(n, np.int32)
        nint, nleaf = C.c_uint64(0), C.c_uint64(0)
        rc = self.R.ref_count_visits_any(self.h, n, O.ctypes.data, D.ctypes.data, tm.ctypes.data, ow.ctypes.data,
                                         ol.ctypes.data, C.byref(nint), C.byref(nleaf))
        assert rc == 0
        return ow, ol, nint.value, nleaf.value

    def __del__(self):
        try:
            self.R.ref_destroy(self.h)
        except Exception:
            pass


def nframes(spp, flags):
    if spp <= 0:
        return 0
    return max(spp // 2, 1) if flags & AA else spp


def new_state(width, height):
    """Renderer accumulation state: accumulator float4, samplesPerPixel, distances (Core/Renderer.h:61-63)."""
    n = width * height
    return (np.zeros((n, 4), np.float32), np.zeros(n, np.int32), np.full(n, -1.0, np.float32))


def init_seed(base):
    return lib().orc_init_seed(base)


def rng_floats(seed, n):
    out = np.zeros(n, np.float32)
    lib().orc_rng_floats(seed, n, out.ctypes.data)
    return out


def eval_combined_brdf(N, L, V, mat8):
    o = np.zeros(3, np.float32)
    lib().orc_eval_combined_brdf(f32(N).ctypes.data, f32(L).ctypes.data, f32(V).ctypes.data, f32(mat8).ctypes.data,
                                 o.ctypes.data)
    return o


def brdf_probe(op, records):
    """orc_brdf_probe: the restated BRDF functions on float32 [n, 24] records -> [n, 8] (include/prt.h PRT_PROBE_*)."""
    rec = np.ascontiguousarray(records, np.float32).reshape(-1, 24)
    out = np.zeros((rec.shape[0], 8), np.float32)
    if lib().orc_brdf_probe(int(op), rec.shape[0], rec.ctypes.data, out.ctypes.data) != 0:
        raise ValueError(f"bad probe op {op}")
    return out


def brdf_probability(mat8, V, N):
    return lib().orc_brdf_probability(f32(mat8).ctypes.data, f32(V).ctypes.data, f32(N).ctypes.data)


def eval_indirect(u2, N, V, mat8, typ):
    d = np.zeros(3, np.float32)
    w = np.ones(3, np.float32)
    ok = lib().orc_eval_indirect(f32(u2).ctypes.data, f32(N).ctypes.data, f32(V).ctypes.data, f32(mat8).ctypes.data,
                                 typ, d.ctypes.data, w.ctypes.data)
    return ok, d, w


def pack_rgb8(rgba):
    return lib().orc_pack_rgb8(f32(rgba).ctypes.data)
