"""Synthetic, seeded scene inputs for the configs of BASELINE.json.

Every array is produced in float64 by numpy and rounded once to float32, so the same
inputs come out on any host.  The layouts are exactly the reference's Model arrays
(Core/Model.cpp:25-119, Core/Model.h:36-44):

  triangles      float4 x 3T   fat triangles handed to tinybvh (w = 0)
  fixed_normals  float4 x 3T   per-corner vertex normals
  fixed_uvs      float2 x 3T   per-corner texture coordinates
  indices        int32  x 3T
  vertices       float3 x V
  face_normals   float3 x T    normalize(cross(v1-v0, v2-v0)) (Core/Model.cpp:100-110)

Textures are packed 0x00RRGGBB uint32 (template/surface.cpp:47-66).  The sky is a float RGB
equirect (Core/Camera.cpp:9,43-74).  Reference assets with missing blobs (textures, HDR
sky) are replaced by these procedural maps.
"""
from __future__ import annotations

import dataclasses
import os
import numpy as np

F32 = np.float32


@dataclasses.dataclass
class Mesh:
    triangles: np.ndarray
    fixed_normals: np.ndarray
    fixed_uvs: np.ndarray
    indices: np.ndarray
    vertices: np.ndarray
    face_normals: np.ndarray
    albedo: int = 0
    normal: int = -1
    metalness: int = -1
    emission: int = -1

    @property
    def tri_count(self) -> int:
        return self.indices.shape[0] // 3


@dataclasses.dataclass
class Lights:
    """4 SIMD point lights (Core/Renderer.h:80-88), directionalLights[0], spotlights[0]."""
    point_pos: np.ndarray   # (4,3)
    point_col: np.ndarray   # (4,3)
    dir_pos: np.ndarray     # (3,)
    dir_col: np.ndarray
    spot_pos: np.ndarray
    spot_col: np.ndarray
    spot_rot: np.ndarray


@dataclasses.dataclass
class SceneData:
    meshes: list
    textures: list          # list of (h, w) uint32 arrays
    instances: list         # list of (mesh_index, 4x4 float32 row-major)
    lights: Lights
    sky: np.ndarray | None  # (h, w, 3) float32
    cam_pos: np.ndarray
    cam_target: np.ndarray
    name: str = ""
    # extensions: per-instance material kinds (_lib.MAT_*; None = all textured) and one
    # area light {"corner", "edge_u", "edge_v", "radiance": (3,) float32, "two_sided": bool} (None = none)
    materials: list | None = None
    area_light: dict | None = None

    @property
    def tri_count(self) -> int:
        return sum(self.meshes[m].tri_count for m, _ in self.instances)


def _mesh_from_grid(P: np.ndarray, N: np.ndarray, UV: np.ndarray, tris: np.ndarray) -> Mesh:
    """P,N: (V,3) float64; UV (V,2) float64; tris (T,3) int -> reference Model arrays."""
    verts = P.astype(F32)
    nrm = N.astype(F32)
    uv = UV.astype(F32)
    idx = tris.astype(np.int32).reshape(-1)
    T = tris.shape[0]
    tri4 = np.zeros((T * 3, 4), F32)
    tri4[:, :3] = verts[idx]
    n4 = np.zeros((T * 3, 4), F32)
    n4[:, :3] = nrm[idx]
    uv2 = uv[idx]
    # face normal: normalize(cross(edge1, edge2)) in float32, tmpl8 normalize (Core/Model.cpp:100-110)
    v0, v1, v2 = verts[tris[:, 0]], verts[tris[:, 1]], verts[tris[:, 2]]
    e1 = (v1 - v0).astype(F32)
    e2 = (v2 - v0).astype(F32)
    c = np.stack([e1[:, 1] * e2[:, 2] - e1[:, 2] * e2[:, 1],
                  e1[:, 2] * e2[:, 0] - e1[:, 0] * e2[:, 2],
                  e1[:, 0] * e2[:, 1] - e1[:, 1] * e2[:, 0]], axis=1).astype(F32)
    d = (c[:, 0] * c[:, 0] + c[:, 1] * c[:, 1]) + c[:, 2] * c[:, 2]
    inv = (F32(1.0) / np.sqrt(d.astype(F32))).astype(F32)
    fn = (c * inv[:, None]).astype(F32)
    return Mesh(tri4.reshape(-1).copy(), n4.reshape(-1).copy(), uv2.reshape(-1).copy(), idx.copy(),
                verts.reshape(-1).copy(), fn.reshape(-1).copy())


def torus(nu: int = 100, nv: int = 50, R: float = 1.0, r: float = 0.4) -> Mesh:
    """C2: torus, nu*nv*2 triangles (100x50 -> 10,000)."""
    iu, iv = np.meshgrid(np.arange(nu + 1), np.arange(nv + 1), indexing="ij")
    th = iu / nu * 2.0 * np.pi
    ph = iv / nv * 2.0 * np.pi
    P = np.stack([(R + r * np.cos(ph)) * np.cos(th), r * np.sin(ph), (R + r * np.cos(ph)) * np.sin(th)], -1)
    N = np.stack([np.cos(ph) * np.cos(th), np.sin(ph), np.cos(ph) * np.sin(th)], -1)
    UV = np.stack([iu / nu * 0.999, iv / nv * 0.999], -1)
    P = P.reshape(-1, 3); N = N.reshape(-1, 3); UV = UV.reshape(-1, 2)
    vid = lambda a, b: a * (nv + 1) + b
    a, b = np.meshgrid(np.arange(nu), np.arange(nv), indexing="ij")
    a = a.reshape(-1); b = b.reshape(-1)
    t1 = np.stack([vid(a, b), vid(a, b + 1), vid(a + 1, b)], 1)
    t2 = np.stack([vid(a + 1, b), vid(a, b + 1), vid(a + 1, b + 1)], 1)
    tris = np.stack([t1, t2], 1).reshape(-1, 3)
    return _mesh_from_grid(P, N, UV, tris)


def heightfield(nx: int, nz: int, extent: float = 5.0) -> Mesh:
    """C3/C4: y = 0.3 sin(3x) cos(2z) + 0.1 sin(17x + 5z) over [-5,5]^2, nx*nz*2 triangles."""
    ix, iz = np.meshgrid(np.arange(nx + 1), np.arange(nz + 1), indexing="ij")
    x = -extent + 2.0 * extent * ix / nx
    z = -extent + 2.0 * extent * iz / nz
    y = 0.3 * np.sin(3 * x) * np.cos(2 * z) + 0.1 * np.sin(17 * x + 5 * z)
    dydx = 0.9 * np.cos(3 * x) * np.cos(2 * z) + 1.7 * np.cos(17 * x + 5 * z)
    dydz = -0.6 * np.sin(3 * x) * np.sin(2 * z) + 0.5 * np.cos(17 * x + 5 * z)
    N = np.stack([-dydx, np.ones_like(x), -dydz], -1)
    N /= np.linalg.norm(N, axis=-1, keepdims=True)
    P = np.stack([x, y, z], -1).reshape(-1, 3)
    UV = np.stack([ix / nx * 0.999, iz / nz * 0.999], -1).reshape(-1, 2)
    N = N.reshape(-1, 3)
    vid = lambda a, b: a * (nz + 1) + b
    a, b = np.meshgrid(np.arange(nx), np.arange(nz), indexing="ij")
    a = a.reshape(-1); b = b.reshape(-1)
    # winding (v00, v01, v10) gives +y face normals
    t1 = np.stack([vid(a, b), vid(a, b + 1), vid(a + 1, b)], 1)
    t2 = np.stack([vid(a + 1, b), vid(a, b + 1), vid(a + 1, b + 1)], 1)
    tris = np.stack([t1, t2], 1).reshape(-1, 3)
    return _mesh_from_grid(P, N, UV, tris)


def _pack(r, g, b) -> np.ndarray:
    return ((np.asarray(r, np.uint32) << 16) + (np.asarray(g, np.uint32) << 8) + np.asarray(b, np.uint32)).astype(np.uint32)


def procedural_textures(size: int = 256):
    """albedo checker, metalness map (G = roughness ramp, B = metal stripes), normal bumps, emission stripe."""
    j, i = np.meshgrid(np.arange(size), np.arange(size), indexing="ij")  # j = row (v), i = column (u)
    cell = size // 8
    chk = ((i // cell) + (j // cell)) % 2
    albedo = np.where(chk == 0, np.uint32(0xC08040), np.uint32(0x4080C0)).astype(np.uint32)
    rough = (i * 255 // (size - 1)).astype(np.uint32)
    metal = np.where(((j // (size // 4)) % 2) == 1, 255, 0).astype(np.uint32)
    metalness = _pack(np.zeros_like(rough), rough, metal)
    u = (i + 0.5) / size
    v = (j + 0.5) / size
    nx = -0.35 * np.cos(2 * np.pi * 4 * u) * np.sin(2 * np.pi * 3 * v)
    ny = -0.35 * np.sin(2 * np.pi * 4 * u) * np.cos(2 * np.pi * 3 * v)
    nz = np.ones_like(nx)
    L = np.sqrt(nx * nx + ny * ny + nz * nz)
    enc = lambda c: np.clip(np.floor((c / L + 1.0) * 0.5 * 255.0 + 0.5), 0, 255).astype(np.uint32)
    normal = _pack(enc(nx), enc(ny), enc(nz))
    emis = np.zeros((size, size), np.uint32)
    emis[:, size // 2 - 8: size // 2 + 8] = 0xFFC878
    return albedo, metalness, normal, emis


def procedural_sky(w: int = 64, h: int = 32) -> np.ndarray:
    """float RGB equirect: zenith (0.6,0.7,1.0) -> horizon (1,1,1) -> nadir (0.2,0.2,0.2), mild azimuth variation."""
    j, i = np.meshgrid(np.arange(h), np.arange(w), indexing="ij")
    theta = (j + 0.5) / h * np.pi
    yy = np.cos(theta)
    zen = np.array([0.6, 0.7, 1.0]); hor = np.array([1.0, 1.0, 1.0]); nad = np.array([0.2, 0.2, 0.2])
    up = yy[..., None]
    col = np.where(up > 0, hor + (zen - hor) * up, hor + (nad - hor) * (-up))
    col = col * (0.9 + 0.1 * np.cos(2 * np.pi * (i + 0.5) / w))[..., None]
    return col.astype(F32)


def scene1_lights() -> Lights:
    """assets/scene1 light JSONs; point lights 2-4 (at the origin in the asset) moved to (+-2, 3, +-2);
    spot at (0,4,0) pointing up-vector (0,1,0) so 'dot(L, rotation) > 0.9' holds under it."""
    pp = np.array([[-2.4000000953674316, 2.299999952316284, -0.30000001192092896],
                   [2.0, 3.0, 2.0], [-2.0, 3.0, 2.0], [2.0, 3.0, -2.0]], F32)
    pc = np.array([[2.9000000953674316, 3.5999999046325684, 4.599999904632568],
                   [1.0, 4.5, 0.8999999761581421], [2.0, 12.0, 1.899999976158142],
                   [5.099999904632568, 3.0, 3.0]], F32)
    return Lights(pp, pc,
                  np.array([149.5, 25.399999618530273, -44.400001525878906], F32), np.array([4.0, 4.0, 4.0], F32),
                  np.array([0.0, 4.0, 0.0], F32), np.array([1.0, 2.0, 4.0], F32), np.array([0.0, 1.0, 0.0], F32))


IDENTITY = np.eye(4, dtype=F32)


def config_c2() -> SceneData:
    """C2: single 10k-tri torus, primary rays only."""
    albedo, metalness, normal, emis = procedural_textures()
    m = torus(100, 50)
    m.albedo, m.metalness = 0, 1
    return SceneData([m], [albedo, metalness], [(0, IDENTITY.copy())], scene1_lights(), procedural_sky(),
                     np.array([0.3, 1.7, -3.2], F32), np.array([0.0, 0.0, 0.0], F32), "c2-torus10k")


def config_heightfield(nx: int, nz: int, name: str) -> SceneData:
    albedo, metalness, normal, emis = procedural_textures()
    m = heightfield(nx, nz)
    m.albedo, m.normal, m.metalness, m.emission = 0, 1, 2, 3
    return SceneData([m], [albedo, normal, metalness, emis], [(0, IDENTITY.copy())], scene1_lights(),
                     procedural_sky(), np.array([0.3, 3.0, -7.0], F32), np.array([0.0, 0.0, 0.0], F32), name)


def config_c3() -> SceneData:
    """C3: 250x200-quad heightfield = 100,000 triangles, full BRDF + shadow rays."""
    return config_heightfield(250, 200, "c3-heightfield100k")


def config_c4() -> SceneData:
    """C4: 1000x500-quad heightfield = 1,000,000 triangles."""
    return config_heightfield(1000, 500, "c4-heightfield1m")


def config_small(nx: int = 40, nz: int = 30) -> SceneData:
    """A small heightfield with every feature on, for fast parity tests."""
    return config_heightfield(nx, nz, f"hf{nx}x{nz}")


def multi_instance(base: SceneData) -> SceneData:
    """Two extra instances of mesh 0 with rotation+scale+translation (exercises the TLAS/instance path)."""
    def trs(t, ang, s):
        c, sn = np.cos(ang), np.sin(ang)
        M = np.array([[c * s, 0, sn * s, t[0]], [0, s, 0, t[1]], [-sn * s, 0, c * s, t[2]], [0, 0, 0, 1]], np.float64)
        return M.astype(F32)
    inst = list(base.instances) + [(0, trs((1.5, 0.6, 2.0), 0.7, 0.35)), (0, trs((-1.8, 0.9, 1.0), -0.4, 0.25))]
    return dataclasses.replace(base, instances=inst, name=base.name + "+inst")


def instance_field(n: int = 300, seed: int = 5) -> SceneData:
    """Many instances (the reference's TLAS over up to 2^32 BLASInstances, Core/tiny_bvh.h:103-104,1732-1770): the
    small heightfield as instance 0 plus `n` copies of a 576-triangle torus scattered over it with random
    rotation about Y, tilt and scale -- more than kLinearInstances, so the rays walk the instance BVH."""
    base = config_small(40, 30)
    albedo, metalness, normal, emis = procedural_textures()
    tor = torus(24, 12, 0.22, 0.08)
    tor.albedo, tor.metalness = 0, 2
    rng = np.random.default_rng(seed)
    inst = list(base.instances)
    for _ in range(n):
        a, b, sc = rng.uniform(0, 2 * np.pi), rng.uniform(-0.6, 0.6), rng.uniform(0.5, 1.6)
        ca, sa, cb, sb = np.cos(a), np.sin(a), np.cos(b), np.sin(b)
        Ry = np.array([[ca, 0, sa], [0, 1, 0], [-sa, 0, ca]])
        Rx = np.array([[1, 0, 0], [0, cb, -sb], [0, sb, cb]])
        M = np.eye(4)
        M[:3, :3] = (Ry @ Rx) * sc
        M[:3, 3] = (rng.uniform(-4.5, 4.5), rng.uniform(0.25, 1.2), rng.uniform(-4.5, 4.5))
        inst.append((1, M.astype(F32)))
    return dataclasses.replace(base, meshes=list(base.meshes) + [tor], instances=inst,
                               name=f"instance-field-{n}")


def deep_bvh(n: int = 1000, r: float = 1.04) -> SceneData:
    """A pathological mesh whose SAH tree is 23 levels deep (deeper than the LDS traversal stacks hold, so the
    HIP path spills to HBM, prt_traverse8.h LaneStack): n nested triangles in the planes z = 0.01 k, triangle k
    spanning r^k around the origin, so every box on the spine contains the rays and its siblings are stacked."""
    from . import ingest
    k = np.arange(n, dtype=np.float64)
    a, z = r ** k, 0.01 * k
    P = np.stack([np.stack([-a, -a, z], 1), np.stack([2 * a, -a, z], 1), np.stack([-a, 2 * a, z], 1)], 1)
    P = P.reshape(-1, 3).astype(F32)
    N = np.tile(np.array([0.0, 0.0, -1.0], F32), (3 * n, 1))
    UV = np.tile(np.array([[0.1, 0.1], [0.9, 0.1], [0.1, 0.9]], F32), (n, 1))
    # face normals stated exactly: every triangle lies in a z plane with counter-clockwise corners seen from -z,
    # so normalize(cross(e1, e2)) = (0, 0, 1); tmpl8's float normalize of the outer triangles' cross products
    # (|c|^2 ~ 1e70) would overflow to zero-length normals
    fn = np.tile(np.array([0.0, 0.0, 1.0], F32), (n, 1))
    m = ingest.mesh_from_indexed(P, N, UV, np.arange(3 * n).reshape(-1, 3), face_normals=fn)
    albedo, metalness, normal, emis = procedural_textures()
    m.albedo, m.metalness = 0, 1
    return SceneData([m], [albedo, metalness], [(0, IDENTITY.copy())], scene1_lights(), procedural_sky(),
                     np.array([0.4, 0.3, -3.0], F32), np.array([0.0, 0.0, 0.5], F32), f"deep-bvh-{n}")


def ceiling_light(corner=(-1.5, 4.0, -1.0), edge_u=(3.0, 0.0, 0.0), edge_v=(0.0, 0.0, 2.0), radiance=(8.0, 7.0, 6.0),
                  two_sided=False) -> dict:
    """One quad area light (extension; the reference's AreaLight is never sampled): by default a 3 x 2 panel
    4 units above the heightfield, emitting downwards (cross(edge_u, edge_v) points to -y)."""
    return {"corner": np.asarray(corner, F32), "edge_u": np.asarray(edge_u, F32), "edge_v": np.asarray(edge_v, F32),
            "radiance": np.asarray(radiance, F32), "two_sided": bool(two_sided)}


def with_extensions(base: SceneData, materials=None, area_light=None) -> SceneData:
    """base with per-instance material kinds (_lib.MAT_*) and/or an area light."""
    return dataclasses.replace(base, materials=list(materials) if materials is not None else None,
                               area_light=area_light, name=base.name + "+ext")


def config_c5() -> SceneData:
    """C5 (BASELINE configs[4]): the C4 scene plus one quad area light (3840x2160, 16 spp, depth 8)."""
    return dataclasses.replace(config_c4(), area_light=ceiling_light(), name="c5-heightfield1m-arealight")


REFERENCE_ROOT = os.environ.get("PRT_REFERENCE_ROOT", "/root/reference")


def config_c1(root: str = REFERENCE_ROOT) -> SceneData:
    """C1 (BASELINE configs[0]): scene1 as the reference ships it -- SciFiHelmet (23,358 triangles) as
    model 0, the XShip game object (~pi about Y), scene1's directional + spot light, zero point lights,
    prefabs/camera.json; render at 256x256, 1 spp (AA off), depth 1, SKYBOX off.  The helmet's maps are
    missing blobs in the reference tree, so 1x1 maps stand in (albedo 0xB0B0B0; G = roughness 128,
    B = metal 0).  Needs the reference's asset files (`root`, PRT_REFERENCE_ROOT); see prt/ingest.py."""
    from . import ingest
    model = os.path.join(root, "Core", "assets", "prefabs", "models", "SciFiHelmet", "SciFiHelmet.gltf")
    if not os.path.exists(model):
        raise FileNotFoundError(f"C1 needs the reference assets ({model})")
    return ingest.load_scene([model], os.path.join(root, "assets", "scene1"),
                             os.path.join(root, "Core", "assets", "prefabs", "camera.json"), name="c1-scene1-helmet")


C1_FLAGS = 0x7F & ~(1 << 4) & ~(1 << 0)  # reference defaults without SKYBOX (C1) and AA (1 spp)


def config_spaceship(root: str = REFERENCE_ROOT) -> SceneData:
    """The reference's textured Spaceship (Core/assets/prefabs/models/Spaceship: 12,490 triangles, 1024x1024
    albedo / normal / metalness PNGs, Core/Model.cpp:183-204) as scene1's model 0: the XShip game object
    (~pi about Y) plus a second, untransformed copy beside it (a two-instance TLAS), the C3/C4 lights and sky,
    a camera framing both ships.  Needs the reference's asset files (`root`); tests use the committed
    fixture tests/golden/spaceship.npz made from it."""
    from . import ingest
    model = os.path.join(root, "Core", "assets", "prefabs", "models", "Spaceship", "Spaceship.gltf")
    if not os.path.exists(model):
        raise FileNotFoundError(f"the Spaceship scene needs the reference assets ({model})")
    sd = ingest.load_scene([model], os.path.join(root, "assets", "scene1"),
                           os.path.join(root, "Core", "assets", "prefabs", "camera.json"), name="spaceship-textured")
    beside = IDENTITY.copy()
    beside[0, 3], beside[2, 3] = 0.6, 0.2
    return dataclasses.replace(sd, instances=sd.instances + [(0, beside)], lights=scene1_lights(),
                               sky=procedural_sky(), cam_pos=np.array([0.55, 0.3, -0.75], F32),
                               cam_target=np.array([0.3, -0.02, 0.0], F32))
