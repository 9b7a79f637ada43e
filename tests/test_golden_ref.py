"""The headline configs pinned to the reference's own traversal (tests/golden/make_golden.py `ref`): frames rendered
by the restated Trace on tinybvh v1.4.2's BVH8_CPU + TLAS (compiled unmodified from /root/reference into oracle/_ref),
committed as data.  C4 and C3 are the BASELINE workloads, C2 the primary-ray config, C1 scene1's SciFiHelmet, and
the textured Spaceship (1024x1024 albedo / normal / metalness maps) the real-asset case of the ingest row.

Bar (BASELINE.json north star): per-channel RMSE <= 1e-4 against the reference-traversal image, identical ray
counts.  The remaining differences are tinybvh's BVH-dependent choices (an exact-t tie across two leaves goes to
the first leaf visited; a 1-ulp-closer triangle behind a box its slab test culls), about 2 rays per million on C4;
each test reports the exact-pixel fraction.  CPU tests pin the oracle's own traversal; GPU tests pin libprt.so
through the C ABI.  On a box that holds oracle/_ref, the full C4 frame is also compared live."""
import os

import numpy as np
import pytest

import oracle
from golden.make_golden import C1_RENDERS, SHIP_RENDERS, c1_lit, scene_digest, ship_flags
from helpers import RMSE_TOL, gpu_scene, rmse
from prt import ingest, scenes
from prt.scenes import Lights, SceneData

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
THREADS = min(16, os.cpu_count() or 1)


def _load(name, sd):
    z = np.load(os.path.join(GOLDEN, name))  # allow_pickle=False (default): plain arrays only
    assert str(z["digest"]) == scene_digest(sd), f"{name}: scene generator changed; regenerate the fixture"
    return z


def _crop(img, W, H, crop):
    x0, y0, w, h = (int(v) for v in crop)
    return img.reshape(H, W, -1)[y0:y0 + h, x0:x0 + w]


def _report(tag, ref, got):
    err = rmse(ref.reshape(-1, 3), got.reshape(-1, 4)[:, :3] if got.shape[-1] == 4 else got.reshape(-1, 3))
    a = ref.reshape(-1, 3)
    b = got.reshape(-1, got.shape[-1])[:, :3]
    exact = float(np.mean(np.all(a == b, axis=1)))
    print(f"{tag}: rmse={err:.3e} exact_pixels={exact:.6f}")
    return err, exact


def c1_scene():
    """SceneData of config C1 rebuilt from the committed fixture (no reference tree needed)."""
    z = np.load(os.path.join(GOLDEN, "c1_scene1.npz"))
    m = ingest.mesh_from_indexed(z["P"], z["N"], z["UV"], z["tri"])
    m.albedo, m.normal, m.metalness, m.emission = (int(z[k]) for k in ("albedo", "normal", "metalness", "emission"))
    tex = [t.reshape(1, 1) for t in z["textures"]]
    L = Lights(z["point_pos"], z["point_col"], z["dir_pos"], z["dir_col"], z["spot_pos"], z["spot_col"], z["spot_rot"])
    inst = [(int(mi), x) for mi, x in zip(z["xf_mesh"], z["xf"])]
    sd = SceneData([m], tex, inst, L, None, z["cam_pos"], z["cam_target"], "c1-scene1-helmet")
    assert scene_digest(sd) == str(z["digest"])
    return sd, z


def ship_scene():
    """SceneData of the textured Spaceship rebuilt from the committed fixture (no reference tree needed)."""
    z = np.load(os.path.join(GOLDEN, "spaceship.npz"))
    m = ingest.mesh_from_indexed(z["P"], z["N"], z["UV"], z["tri"])
    m.albedo, m.normal, m.metalness, m.emission = (int(z[k]) for k in ("albedo", "normal", "metalness", "emission"))
    tex = [z[f"tex{i}"] for i in range(3)]
    L = Lights(z["point_pos"], z["point_col"], z["dir_pos"], z["dir_col"], z["spot_pos"], z["spot_col"], z["spot_rot"])
    inst = [(int(mi), x) for mi, x in zip(z["xf_mesh"], z["xf"])]
    sd = SceneData([m], tex, inst, L, z["sky"], z["cam_pos"], z["cam_target"], "spaceship-textured")
    assert scene_digest(sd) == str(z["digest"])
    return sd, z


# ---------------------------------------------------------------- fixtures vs the reference asset tree (CPU)

@pytest.mark.skipif(not os.path.exists(os.path.join(scenes.REFERENCE_ROOT, "Core", "assets")),
                    reason="reference asset tree absent")
def test_spaceship_fixture_is_the_ingested_scene():
    sd, _ = ship_scene()
    assert scene_digest(sd) == scene_digest(scenes.config_spaceship())
    assert all(t.shape == (1024, 1024) for t in sd.textures) and sd.meshes[0].tri_count == 12490

@pytest.mark.skipif(not os.path.exists(os.path.join(scenes.REFERENCE_ROOT, "Core", "assets")),
                    reason="reference asset tree absent")
def test_c1_fixture_is_the_ingested_scene():
    sd, _ = c1_scene()
    ref = scenes.config_c1()
    assert scene_digest(sd) == scene_digest(ref)


# ---------------------------------------------------------------- oracle (CPU)

def test_oracle_c1_matches_reference_traversal(oracle_mod):
    sd, z = c1_scene()
    W, H = int(z["W"]), int(z["H"])
    for variant, mode in C1_RENDERS:
        s = sd if variant == "shipped" else c1_lit(sd)
        osc = oracle_mod.OracleScene(s, W, H)
        avg, _, _, st = osc.render(W, H, spp=1, bounces=1, flags=int(z["flags"]), mode=mode)
        ref = z[f"{variant}{mode}_avg"]
        err, _ = _report(f"C1 {variant} mode {mode}", ref, avg)
        assert err <= RMSE_TOL
        assert [st.segments, st.shadow_rays] == z[f"{variant}{mode}_counts"].tolist()
    assert z["lit0_avg"].max() > 0 and z["shipped1_avg"].max() > 0  # non-black images are part of the pin


def test_oracle_spaceship_matches_reference_traversal(oracle_mod):
    sd, z = ship_scene()
    W, H = int(z["W"]), int(z["H"])
    for name, mode, spp, bounces in SHIP_RENDERS:
        osc = oracle_mod.OracleScene(sd, W, H)
        avg, rgb8, _, st = osc.render(W, H, spp=spp, bounces=bounces, flags=ship_flags(spp), mode=mode,
                                      nthreads=THREADS)
        err, _ = _report(f"Spaceship {name}", z[f"{name}_avg"], avg)
        assert err <= RMSE_TOL
        assert [st.segments, st.shadow_rays] == z[f"{name}_counts"].tolist()
    # the albedo view samples the ship's texture: many distinct colours, not a stand-in map
    assert len(np.unique(z["albedo_rgb8"])) > 1000


def test_oracle_c3_matches_reference_traversal(oracle_mod):
    sd = scenes.config_c3()
    z = _load("c3_ref_480x270.npz", sd)
    W, H = int(z["W"]), int(z["H"])
    avg, _, _, st = oracle_mod.OracleScene(sd, W, H).render(W, H, spp=4, bounces=4, nthreads=THREADS)
    err, _ = _report("C3 480x270", z["avg"], avg)
    assert err <= RMSE_TOL
    assert (st.segments, st.shadow_rays) == (int(z["segments"]), int(z["shadow_rays"]))


def test_oracle_c4_matches_reference_traversal(oracle_mod):
    sd = scenes.config_c4()
    z = _load("c4_ref_crop.npz", sd)
    W, H = int(z["W"]), int(z["H"])
    avg, rgb8, _, st = oracle_mod.OracleScene(sd, W, H).render(W, H, spp=4, bounces=4, nthreads=THREADS)
    err, _ = _report("C4 480x270 window", z["avg"], _crop(avg, W, H, z["crop"]))
    assert err <= RMSE_TOL
    assert (st.segments, st.shadow_rays) == (int(z["segments"]), int(z["shadow_rays"]))


def test_oracle_c2_full_matches_reference_traversal(oracle_mod):
    sd = scenes.config_c2()
    z = _load("c2_ref_1280x720.npz", sd)
    W, H = int(z["W"]), int(z["H"])
    t, u, v, p, _ = oracle_mod.OracleScene(sd, W, H).primary_hits(W, H, nthreads=THREADS)
    _assert_c2(z, t, u, v, p)


def _assert_c2(z, t, u, v, p):
    from golden.make_golden import sha
    hit = t < 1e30
    assert np.array_equal(np.where(hit, p, np.uint32(0xFFFFFFFF)), z["prim"])
    assert sha(np.where(hit, t, 0)) == str(z["t_sha"])
    assert sha(np.where(hit, u, 0)) == str(z["u_sha"]) and sha(np.where(hit, v, 0)) == str(z["v_sha"])


# ---------------------------------------------------------------- HIP path (GPU)

@pytest.mark.gpu
def test_gpu_c1_matches_reference_traversal(gpu_ctx):
    """C1 through libprt.so: scene1's helmet as shipped (BRDF black, base colour, geometry normal) and lit."""
    sd, z = c1_scene()
    W, H = int(z["W"]), int(z["H"])
    for variant, mode in C1_RENDERS:
        s = sd if variant == "shipped" else c1_lit(sd)
        gpu_scene(gpu_ctx, s, W, H)
        avg, _, st = gpu_ctx.render(W, H, 1, 1, int(z["flags"]), mode=mode)
        err, _ = _report(f"GPU C1 {variant} mode {mode}", z[f"{variant}{mode}_avg"], avg)
        assert err <= RMSE_TOL
        assert [st.segments, st.shadow_rays] == z[f"{variant}{mode}_counts"].tolist()


@pytest.mark.gpu
def test_gpu_spaceship_matches_reference_traversal(gpu_ctx):
    """The textured Spaceship (two instances, 1024x1024 maps) through libprt.so: shaded, albedo, shading normal."""
    sd, z = ship_scene()
    W, H = int(z["W"]), int(z["H"])
    gpu_scene(gpu_ctx, sd, W, H)
    for name, mode, spp, bounces in SHIP_RENDERS:
        gpu_ctx.reset_accumulation(full=True)
        avg, rgb8, st = gpu_ctx.render(W, H, spp, bounces, flags=ship_flags(spp), mode=mode)
        err, exact = _report(f"GPU Spaceship {name}", z[f"{name}_avg"], avg)
        assert err <= RMSE_TOL
        assert [st.segments, st.shadow_rays] == z[f"{name}_counts"].tolist()
        assert np.mean(rgb8 == z[f"{name}_rgb8"]) > 0.999


@pytest.mark.gpu
def test_gpu_c2_full_matches_reference_traversal(gpu_ctx):
    sd = scenes.config_c2()
    z = _load("c2_ref_1280x720.npz", sd)
    W, H = int(z["W"]), int(z["H"])
    gpu_scene(gpu_ctx, sd, W, H)
    h, _ = gpu_ctx.trace_primary(W, H)
    _assert_c2(z, h["t"], h["u"], h["v"], h["prim"])


@pytest.mark.gpu
def test_gpu_c3_matches_reference_traversal(gpu_ctx):
    sd = scenes.config_c3()
    z = _load("c3_ref_480x270.npz", sd)
    W, H = int(z["W"]), int(z["H"])
    gpu_scene(gpu_ctx, sd, W, H)
    avg, _, st = gpu_ctx.render(W, H, 4, 4)
    err, _ = _report("GPU C3 480x270", z["avg"], avg)
    assert err <= RMSE_TOL
    assert (st.segments, st.shadow_rays) == (int(z["segments"]), int(z["shadow_rays"]))


@pytest.mark.gpu
def test_gpu_c4_matches_reference_traversal(gpu_ctx):
    """The bench frame (C4, 1920x1080, 4 spp, depth 4): the 480x270 window against the reference-traversal pixels,
    the whole frame's ray counts against the reference's."""
    sd = scenes.config_c4()
    z = _load("c4_ref_crop.npz", sd)
    W, H = int(z["W"]), int(z["H"])
    gpu_scene(gpu_ctx, sd, W, H)
    avg, rgb8, st = gpu_ctx.render(W, H, 4, 4)
    err, _ = _report("GPU C4 480x270 window", z["avg"], _crop(avg, W, H, z["crop"]))
    assert err <= RMSE_TOL
    assert (st.segments, st.shadow_rays) == (int(z["segments"]), int(z["shadow_rays"]))
    r = _crop(rgb8, W, H, z["crop"]).reshape(-1)
    assert np.mean(r == z["rgb8"].reshape(-1)) >= 0.999


@pytest.mark.gpu
@pytest.mark.skipif(oracle.reflib() is None, reason="oracle/_ref not built on this machine")
def test_gpu_c4_full_frame_vs_live_reference_traversal(gpu_ctx):
    """The whole C4 bench frame against the restated Trace running on the reference's tinybvh, rendered here on the
    host cores (oracle/_ref travels with the tree; the reference source does not)."""
    sd = scenes.config_c4()
    W, H = 1920, 1080
    gpu_scene(gpu_ctx, sd, W, H)
    avg, _, st = gpu_ctx.render(W, H, 4, 4)
    osc = oracle.OracleScene(sd, W, H)
    osc.use_reference_traversal()
    a_r, _, _, s_r = osc.render(W, H, spp=4, bounces=4, nthreads=THREADS)
    err, exact = _report("GPU C4 full frame vs live tinybvh", a_r[:, :3], avg)
    assert err <= RMSE_TOL and exact >= 0.9999
    assert (st.segments, st.shadow_rays) == (s_r.segments, s_r.shadow_rays)
