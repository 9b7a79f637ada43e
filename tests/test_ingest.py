"""Scene ingest (prt/ingest.py): PNG, glTF / GLB, the game-object transform chain, scene1.

Ingest parity is unpinned against the reference's binaries (assimp / Bullet are prebuilt Windows libraries);
the checks are self-contained round trips plus the counts and transform SURVEY.md recorded for scene1.
Tests that read the reference's asset files skip where the tree is absent (the GPU box)."""
import json
import os
import struct
import zlib

import numpy as np
import pytest

from prt import ingest, scenes

HAVE_REF = os.path.exists(os.path.join(scenes.REFERENCE_ROOT, "Core", "assets", "prefabs", "models", "SciFiHelmet"))


def _png(path, img, ctype, filters):
    """Minimal PNG encoder: one filter type per row from `filters` (cycled)."""
    h, w = img.shape[:2]
    n = {0: 1, 2: 3, 4: 2, 6: 4}[ctype]
    px = img.reshape(h, w * n).astype(np.int32)
    rows = []
    for y in range(h):
        ft = filters[y % len(filters)]
        cur = px[y]
        prev = px[y - 1] if y else np.zeros_like(cur)
        left = np.concatenate([np.zeros(n, np.int32), cur[:-n]])
        ul = np.concatenate([np.zeros(n, np.int32), prev[:-n]])
        if ft == 0:
            f = cur
        elif ft == 1:
            f = cur - left
        elif ft == 2:
            f = cur - prev
        elif ft == 3:
            f = cur - ((left + prev) >> 1)
        else:
            p = left + prev - ul
            pa, pb, pc = np.abs(p - left), np.abs(p - prev), np.abs(p - ul)
            pred = np.where((pa <= pb) & (pa <= pc), left, np.where(pb <= pc, prev, ul))
            f = cur - pred
        rows.append(bytes([ft]) + (f & 0xFF).astype(np.uint8).tobytes())

    def chunk(kind, body):
        return struct.pack(">I", len(body)) + kind + body + struct.pack(">I", zlib.crc32(kind + body) & 0xFFFFFFFF)
    data = (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, ctype, 0, 0, 0)) +
            chunk(b"IDAT", zlib.compress(b"".join(rows))) + chunk(b"IEND", b""))
    open(path, "wb").write(data)


@pytest.mark.parametrize("ctype", [0, 2, 4, 6])
def test_png_all_filters(tmp_path, ctype):
    rng = np.random.default_rng(ctype)
    n = {0: 1, 2: 3, 4: 2, 6: 4}[ctype]
    img = rng.integers(0, 256, (13, 17, n), dtype=np.uint8)
    f = str(tmp_path / "t.png")
    _png(f, img, ctype, [0, 1, 2, 3, 4])
    out = ingest.load_png(f)
    if n <= 2:
        g = img[..., 0].astype(np.uint32)
        exp = g + (g << 8) + (g << 16)
    else:
        exp = (img[..., 0].astype(np.uint32) << 16) + (img[..., 1].astype(np.uint32) << 8) + img[..., 2]
    assert np.array_equal(out, exp)  # Surface::LoadFromFile packing (template/surface.cpp:57-64)


def _write_gltf(tmp_path, P, N, UV, idx, mode=4, glb=False):
    blobs, views, acc = [], [], []

    def add(arr, ctype, typ):
        b = np.ascontiguousarray(arr).tobytes()
        off = sum(len(x) for x in blobs)
        blobs.append(b + b"\0" * ((-len(b)) % 4))
        views.append({"buffer": 0, "byteOffset": off, "byteLength": len(b)})
        acc.append({"bufferView": len(views) - 1, "componentType": ctype, "count": len(arr), "type": typ})
        return len(acc) - 1
    attrs = {"POSITION": add(P.astype(np.float32), 5126, "VEC3")}
    if N is not None:
        attrs["NORMAL"] = add(N.astype(np.float32), 5126, "VEC3")
    if UV is not None:
        attrs["TEXCOORD_0"] = add(UV.astype(np.float32), 5126, "VEC2")
    ii = add(idx.astype(np.uint16), 5123, "SCALAR")
    binary = b"".join(blobs)
    doc = {"asset": {"version": "2.0"}, "accessors": acc, "bufferViews": views,
           "meshes": [{"primitives": [{"attributes": attrs, "indices": ii, "mode": mode}]}],
           "buffers": [{"byteLength": len(binary)}]}
    if glb:
        js = json.dumps(doc).encode()
        js += b" " * ((-len(js)) % 4)
        body = struct.pack("<II", len(js), 0x4E4F534A) + js + struct.pack("<II", len(binary), 0x004E4942) + binary
        path = str(tmp_path / "m.glb")
        open(path, "wb").write(b"glTF" + struct.pack("<II", 2, 12 + len(body)) + body)
    else:
        doc["buffers"][0]["uri"] = "m.bin"
        open(str(tmp_path / "m.bin"), "wb").write(binary)
        path = str(tmp_path / "m.gltf")
        open(path, "w").write(json.dumps(doc))
    return path


@pytest.mark.parametrize("glb", [False, True])
def test_gltf_model_arrays(tmp_path, glb):
    P = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [1, 1, 0.5]], np.float32)
    N = np.array([[0, 0, 1], [0, 0, 1], [0, 0.6, 0.8], [0.6, 0, 0.8]], np.float32)
    UV = np.array([[0, 0], [1, 0], [0, 1], [0.25, 0.75]], np.float32)
    idx = np.array([0, 1, 2, 2, 1, 3])
    m = ingest.load_model(_write_gltf(tmp_path, P, N, UV, idx, glb=glb))
    assert m.tri_count == 2 and m.vertices.size == 12
    tri = m.triangles.reshape(-1, 4)
    assert np.array_equal(tri[:, :3], P[idx]) and np.all(tri[:, 3] == 0)         # Model::triangles, corner order
    assert np.array_equal(m.fixed_normals.reshape(-1, 4)[:, :3], N[idx])         # file normals kept
    uv = m.fixed_uvs.reshape(-1, 2)
    assert np.array_equal(uv[:, 0], UV[idx, 0]) and np.array_equal(uv[:, 1], np.float32(1) - UV[idx, 1])  # FlipUVs
    assert np.array_equal(m.indices, idx.astype(np.int32))
    fn = m.face_normals.reshape(-1, 3)
    assert np.allclose(fn[0], [0, 0, 1]) and np.allclose(np.linalg.norm(fn, axis=1), 1, atol=1e-6)


def test_gltf_strip_and_generated_normals(tmp_path):
    P = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [1, 1, 0]], np.float32)
    m = ingest.load_model(_write_gltf(tmp_path, P, None, None, np.arange(4), mode=5))
    assert m.tri_count == 2
    assert np.array_equal(m.indices, np.array([0, 1, 2, 2, 1, 3], np.int32))  # odd strip triangles flipped
    n = m.fixed_normals.reshape(-1, 4)[:, :3]
    assert np.allclose(np.abs(n[:, 2]), 1)  # GenSmoothNormals of a flat quad
    assert np.all(m.fixed_uvs == 0)


def test_instance_transform_chain():
    # GameObject::Synchronise hands glm's (x, y, z, w) to tmpl8 quat(w, x, y, z): a zero rotation becomes
    # w=0, z=1, i.e. pi about Z (Core/GameObject.cpp:60-62)
    assert np.allclose(ingest.instance_transform((0, 0, 0), (0, 0, 0)), np.diag([-1, -1, 1, 1]), atol=1e-7)
    M = ingest.instance_transform((1, 2, 3), (0, 0, 180))
    # scene1's XShip (rotationZ = 180) ends up as ~pi about Y through the Bullet / glm chain
    assert np.allclose(M[:3, :3], np.diag([-1, 1, -1]), atol=1e-6) and np.allclose(M[:3, 3], [1, 2, 3])
    for rot in ((30, 0, 0), (0, 45, 0), (10, 20, 30)):
        R = ingest.instance_transform((0, 0, 0), rot)[:3, :3].astype(np.float64)
        assert np.allclose(R @ R.T, np.eye(3), atol=1e-5) and abs(np.linalg.det(R) - 1) < 1e-5


@pytest.mark.skipif(not HAVE_REF, reason="reference asset tree absent")
def test_scene1_c1_ingest(oracle_mod):
    sd = scenes.config_c1()
    m = sd.meshes[0]
    assert m.tri_count == 23_358 and m.vertices.size // 3 == 70_074
    assert len(sd.instances) == 1 and sd.instances[0][0] == 0
    assert np.allclose(sd.instances[0][1][:3, :3], np.diag([-1, 1, -1]), atol=1e-6)
    assert np.all(sd.lights.point_col == 0) and np.array_equal(sd.lights.dir_col, np.float32([4, 4, 4]))
    W = H = 64
    osc = oracle_mod.OracleScene(sd, W, H)
    avg, rgb8, _, st = osc.render(W, H, spp=1, bounces=1, flags=scenes.C1_FLAGS)
    assert st.segments == W * H and np.isfinite(avg).all()
    # camera.json looks into the helmet's lower shell: every directional shadow ray is blocked by nearby
    # geometry, point lights are zero and the spot's rot = 0 never lights, so depth-1 BRDF is black; the
    # base-colour view shows the hits (0xB0B0B0 linearised)
    assert avg[:, :3].max() == 0
    base, _, _, _ = osc.render(W, H, spp=1, bounces=1, flags=scenes.C1_FLAGS, mode=1)
    t = osc.primary_hits(W, H)[0]
    assert (t < 1e30).sum() > 1000 and np.all(base[t < 1e30, :3] > 0)


def test_capture_png_round_trip(tmp_path):
    """Renderer::Capture's PNG (prt_capture_png) decodes back to the screen's 0x00RRGGBB pixels."""
    rng = np.random.default_rng(5)
    scr = rng.integers(0, 1 << 24, (37, 53), dtype=np.uint32)
    f = str(tmp_path / "capture.png")
    ingest.capture_png(f, scr, 53, 37)
    assert np.array_equal(ingest.load_png(f), scr)
