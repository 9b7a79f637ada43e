"""ctypes binding of libprt.so (include/prt.h).  Loads the in-tree library and fails loudly when it is
missing: there is no CPU fallback for the product path."""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# PRT_LIBPATH: another build of the library (A/B runs of two builds in one session; scripts/ab_bench.sh)
LIBPATH = os.environ.get("PRT_LIBPATH") or os.path.join(HERE, "libprt.so")

PRT_OK = 0
ABI_VERSION = 10  # PRT_ABI_VERSION of the include/prt.h these structs mirror
FLAG_AA, FLAG_ACCUMULATE, FLAG_GAMMA, FLAG_NORMALMAP, FLAG_SKYBOX, FLAG_LIGHTED, FLAG_STOCHASTIC = (1 << i for i in range(7))
FLAGS_DEFAULT = 0x7F
OUT_DEVICE = 1
BUILDER_HOST_SAH, BUILDER_GPU_LBVH, BUILDER_HOST_SBVH, BUILDER_GPU_PLOC = 0, 1, 2, 3

# Renderer::RENDER_STATES (Core/Renderer.h:37-46)
MODE_BRDF, MODE_BASECOLOR, MODE_GEOMETRYNORMAL, MODE_SHADINGNORMAL, MODE_METAL, MODE_ROUGHNESS, MODE_EMISSIVE = range(7)

# every symbol include/prt.h declares (tests check the library exports all of them)
EXPORTS = [
    "prt_abi_version", "prt_last_error", "prt_device_count", "prt_create", "prt_destroy", "prt_set_stream",
    "prt_set_textures", "prt_set_meshes", "prt_set_instances", "prt_set_lights", "prt_set_sky", "prt_set_camera",
    "prt_camera_look_at", "prt_postfx_preset", "prt_set_postfx", "prt_render", "prt_reset_accumulation", "prt_tile_buffer_pixels", "prt_tile_pixel_map",
    "prt_render_tiles",
    "prt_untile", "prt_trace_primary", "prt_intersect", "prt_occluded", "prt_brdf_probe", "prt_get_scene_info", "prt_set_bvh_builder",
    "prt_set_instance_materials", "prt_set_area_lights", "prt_shard_unique_id", "prt_shard_init_rccl",
    "prt_shard_attach_rccl", "prt_create_group", "prt_get_shard_info", "prt_accumulation_bytes",
    "prt_save_accumulation", "prt_load_accumulation", "prt_ray_totals", "prt_set_frames_in_flight", "prt_finish",
]
SHARD_ID_BYTES = 128
SHARD_NONE, SHARD_RCCL, SHARD_GROUP = 0, 1, 2  # prt_shard_info.transport

# instance material kinds (prt_set_instance_materials; the reference's dead Scene.cpp:193-205 branches)
MAT_TEXTURED, MAT_DIELECTRIC, MAT_MIRROR = 0, 1, 2


class PrtError(RuntimeError):
    pass


class DeviceDesc(C.Structure):
    _fields_ = [("device", C.c_int32), ("flags", C.c_uint32)]


class Texture(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("pixels", C.c_void_p)]


class Mesh(C.Structure):
    _fields_ = [("tri_count", C.c_int32), ("vertex_count", C.c_int32), ("triangles", C.c_void_p),
                ("fixed_normals", C.c_void_p), ("fixed_uvs", C.c_void_p), ("indices", C.c_void_p),
                ("vertices", C.c_void_p), ("face_normals", C.c_void_p), ("albedo_tex", C.c_int32),
                ("normal_tex", C.c_int32), ("metalness_tex", C.c_int32), ("emission_tex", C.c_int32)]


class Lights(C.Structure):
    _fields_ = [("point_pos", (C.c_float * 3) * 4), ("point_color", (C.c_float * 3) * 4),
                ("dir_pos", C.c_float * 3), ("dir_color", C.c_float * 3),
                ("spot_pos", C.c_float * 3), ("spot_color", C.c_float * 3), ("spot_rot", C.c_float * 3)]


class AreaLight(C.Structure):
    _fields_ = [("corner", C.c_float * 3), ("edge_u", C.c_float * 3), ("edge_v", C.c_float * 3),
                ("radiance", C.c_float * 3), ("two_sided", C.c_int32)]


class CameraDesc(C.Structure):
    _fields_ = [("pos", C.c_float * 3), ("top_left", C.c_float * 3), ("top_right", C.c_float * 3),
                ("bottom_left", C.c_float * 3), ("right", C.c_float * 3), ("up", C.c_float * 3),
                ("ahead", C.c_float * 3)]


class PostFx(C.Structure):
    """prt_postfx: Renderer::isPostProcessed + the Camera post-process members (Core/Camera.h:11-31)."""
    _fields_ = [("enabled", C.c_int32), ("aberration", C.c_int32), ("fov", C.c_float), ("distortion", C.c_float),
                ("vignette_intensity", C.c_float), ("vignette_radius", C.c_float), ("color_grading", C.c_float * 4)]


class RenderParams(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("spp", C.c_int32), ("bounces", C.c_int32),
                ("flags", C.c_uint32), ("render_mode", C.c_int32), ("frame_index", C.c_uint32), ("seed", C.c_uint32)]


class Stats(C.Structure):
    _fields_ = [("segments", C.c_uint64), ("shadow_rays", C.c_uint64), ("paths", C.c_uint64), ("ms", C.c_double),
                ("ms_trace", C.c_double), ("ms_closest", C.c_double), ("ms_anyhit", C.c_double),
                ("pipeline", C.c_int32), ("iterations", C.c_int32),
                ("batches", C.c_int32), ("ranks", C.c_int32), ("stack_overflows", C.c_uint64)]


class Hit(C.Structure):
    _fields_ = [("t", C.c_float), ("u", C.c_float), ("v", C.c_float), ("prim", C.c_uint32), ("inst", C.c_uint32)]


class ShardInfo(C.Structure):
    _fields_ = [("rank", C.c_int32), ("world", C.c_int32), ("tile_size", C.c_int32), ("transport", C.c_int32)]


class SceneInfo(C.Structure):
    _fields_ = [("blas_nodes", C.c_int64), ("blas_leaves", C.c_int64), ("device_bytes", C.c_int64),
                ("max_depth", C.c_int32), ("triangles", C.c_int32), ("build_ms", C.c_double), ("builder", C.c_int32),
                ("tlas_depth", C.c_int32), ("tlas_rebuilds", C.c_int32), ("tlas_async", C.c_int32),
                ("tlas_median", C.c_int32), ("tlas_build_ms", C.c_float), ("tlas_build_cpu_ms", C.c_float)]


_lib = None


def load():
    """Load libprt.so (built in-tree by __graft_entry__.build())."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIBPATH):
        raise PrtError(f"{LIBPATH} is missing: run __graft_entry__.build() (no CPU fallback exists)")
    # One HIP runtime per process: torch ships its own libamdhip64.so.7 (same SONAME as /opt/rocm's).
    # Load torch's first so libprt.so binds to it and torch's device memory / streams stay valid.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIBPATH)
    vp, i32, u32 = C.c_void_p, C.c_int32, C.c_uint32
    sig = {
        "prt_abi_version": ([], C.c_int),
        "prt_last_error": ([], C.c_char_p),
        "prt_device_count": ([C.POINTER(i32)], C.c_int),
        "prt_create": ([C.POINTER(DeviceDesc), C.POINTER(vp)], C.c_int),
        "prt_destroy": ([vp], C.c_int),
        "prt_set_stream": ([vp, vp], C.c_int),
        "prt_set_frames_in_flight": ([vp, i32], C.c_int),
        "prt_finish": ([vp], C.c_int),
        "prt_set_textures": ([vp, C.POINTER(Texture), i32], C.c_int),
        "prt_set_meshes": ([vp, C.POINTER(Mesh), i32], C.c_int),
        "prt_set_instances": ([vp, vp, vp, i32], C.c_int),
        "prt_set_lights": ([vp, C.POINTER(Lights)], C.c_int),
        "prt_set_sky": ([vp, vp, i32, i32], C.c_int),
        "prt_set_camera": ([vp, C.POINTER(CameraDesc)], C.c_int),
        "prt_camera_look_at": ([vp, vp, C.c_float, C.POINTER(CameraDesc)], C.c_int),
        "prt_postfx_preset": ([i32, C.POINTER(PostFx)], C.c_int),
        "prt_set_postfx": ([vp, C.POINTER(PostFx)], C.c_int),
        "prt_render": ([vp, C.POINTER(RenderParams), vp, vp, u32, C.POINTER(Stats)], C.c_int),
        "prt_reset_accumulation": ([vp, i32], C.c_int),
        "prt_accumulation_bytes": ([vp, C.POINTER(C.c_uint64)], C.c_int),
        "prt_save_accumulation": ([vp, vp, C.c_uint64], C.c_int),
        "prt_load_accumulation": ([vp, vp, C.c_uint64], C.c_int),
        "prt_ray_totals": ([vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_int32], C.c_int),
        "prt_tile_buffer_pixels": ([i32, i32, i32, i32, C.POINTER(C.c_int64)], C.c_int),
        "prt_tile_pixel_map": ([i32, i32, i32, i32, i32, C.c_void_p], C.c_int),
        "prt_render_tiles": ([vp, C.POINTER(RenderParams), i32, i32, i32, vp, C.POINTER(Stats)], C.c_int),
        "prt_untile": ([vp, vp, i32, i32, i32, i32, vp, vp], C.c_int),
        "prt_trace_primary": ([vp, i32, i32, vp, u32, C.POINTER(Stats)], C.c_int),
        "prt_intersect": ([vp, i32, vp, vp, vp, vp], C.c_int),
        "prt_occluded": ([vp, i32, vp, vp, vp, vp], C.c_int),
        "prt_brdf_probe": ([vp, i32, i32, vp, vp], C.c_int),
        "prt_get_scene_info": ([vp, C.POINTER(SceneInfo)], C.c_int),
        "prt_set_bvh_builder": ([vp, i32], C.c_int),
        "prt_set_instance_materials": ([vp, vp, i32], C.c_int),
        "prt_set_area_lights": ([vp, C.POINTER(AreaLight), i32], C.c_int),
        "prt_shard_unique_id": ([vp], C.c_int),
        "prt_shard_init_rccl": ([vp, vp, i32, i32, i32], C.c_int),
        "prt_shard_attach_rccl": ([vp, vp, i32], C.c_int),
        "prt_create_group": ([C.POINTER(DeviceDesc), i32, i32, C.POINTER(vp)], C.c_int),
        "prt_get_shard_info": ([vp, C.POINTER(ShardInfo)], C.c_int),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    if L.prt_abi_version() != ABI_VERSION:
        raise PrtError(f"{LIBPATH}: ABI {L.prt_abi_version()} != {ABI_VERSION} (stale build: rerun __graft_entry__.build())")
    _lib = L
    return L


def check(rc: int) -> None:
    if rc != PRT_OK:
        msg = load().prt_last_error()
        raise PrtError(f"prt error {rc}: {msg.decode() if msg else ''}")
