"""Parity against the committed golden fixtures (tests/golden/make_golden.py, produced by the reference's own
tinybvh v1.4.2 BVH8_CPU + TLAS compiled from /root/reference).  No reference code is needed at test time.

CPU tests pin the oracle (its built-in BVH) to the fixtures; GPU tests pin the HIP path (both BLAS layouts)
through the C ABI to the same fixtures.  Bar: bit-exact hit records and occlusion, bit-exact images."""
import os

import numpy as np
import pytest

import oracle
from golden.make_golden import scene_digest
from helpers import gpu_scene
from prt import scenes

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _load(name, sd):
    z = np.load(os.path.join(GOLDEN, name))  # allow_pickle=False (default): plain arrays only
    assert str(z["digest"]) == scene_digest(sd), f"{name}: scene generator changed; regenerate the fixture"
    return z


def _c2():
    sd = scenes.config_c2()
    return sd, _load("c2_primary.npz", sd)


def _multi():
    sd = scenes.multi_instance(scenes.config_small(60, 40))
    return sd, _load("multi_rays.npz", sd)


def _trace():
    sd = scenes.multi_instance(scenes.config_small(50, 40))
    return sd, _load("trace_64x48.npz", sd)


def _many():
    sd = scenes.instance_field(300)
    return sd, _load("many_inst.npz", sd)


def _assert_hits(z, t, u, v, prim, inst):
    hit = z["t"] < 1e30
    assert hit.sum() > 1000
    assert np.array_equal(hit, t < 1e30)
    assert np.array_equal(prim[hit], z["prim"][hit]) and np.array_equal(inst[hit], z["inst"][hit])
    assert np.array_equal(t[hit], z["t"][hit])
    assert np.array_equal(u[hit], z["u"][hit]) and np.array_equal(v[hit], z["v"][hit])


# ---------------------------------------------------------------- oracle (CPU)

def test_oracle_c2_primary_matches_golden(oracle_mod):
    sd, z = _c2()
    W, H = int(z["W"]), int(z["H"])
    osc = oracle_mod.OracleScene(sd, W, H)
    pos, _, _, _ = osc.camera_basis(W, H)
    assert np.array_equal(pos, z["O"][0])
    _assert_hits(z, *osc.primary_hits(W, H))


def test_oracle_multi_rays_match_golden(oracle_mod):
    sd, z = _multi()
    osc = oracle_mod.OracleScene(sd)
    _assert_hits(z, *osc.intersect(z["O"], z["D"]))
    assert np.array_equal(osc.occluded(z["O"], z["D"], z["tmax"]), z["occ"])


def test_oracle_many_instances_match_golden(oracle_mod):
    """301 instances: tinybvh walks its TLAS, the oracle its linear list -- identical records and image."""
    sd, z = _many()
    osc = oracle_mod.OracleScene(sd)
    _assert_hits(z, *osc.intersect(z["O"], z["D"]))
    assert np.array_equal(osc.occluded(z["O"], z["D"], z["tmax"]), z["occ"])
    W, H = int(z["W"]), int(z["H"])
    avg, rgb8, _, st = oracle_mod.OracleScene(sd, W, H).render(W, H, spp=2, bounces=3)
    assert (st.segments, st.shadow_rays) == (int(z["segments"]), int(z["shadow_rays"]))
    assert np.array_equal(avg[:, :3], z["avg"]) and np.array_equal(rgb8, z["rgb8"])


def test_oracle_trace_matches_golden(oracle_mod):
    sd, z = _trace()
    W, H = int(z["W"]), int(z["H"])
    osc = oracle_mod.OracleScene(sd, W, H)
    avg, rgb8, _, st = osc.render(W, H, spp=int(z["spp"]), bounces=int(z["bounces"]), flags=int(z["flags"]))
    assert st.segments == int(z["segments"]) and st.shadow_rays == int(z["shadow_rays"])
    assert np.array_equal(avg, z["avg"]) and np.array_equal(rgb8, z["rgb8"])


# ---------------------------------------------------------------- HIP path (GPU)

@pytest.mark.gpu
def test_gpu_c2_primary_matches_golden(gpu_ctx):
    sd, z = _c2()
    W, H = int(z["W"]), int(z["H"])
    gpu_scene(gpu_ctx, sd, W, H)
    h, _ = gpu_ctx.trace_primary(W, H)
    _assert_hits(z, h["t"], h["u"], h["v"], h["prim"], h["inst"])


@pytest.mark.gpu
def test_gpu_multi_rays_match_golden(gpu_ctx):
    sd, z = _multi()
    gpu_scene(gpu_ctx, sd, 64, 64)
    g = gpu_ctx.intersect(z["O"], z["D"])
    _assert_hits(z, g["t"], g["u"], g["v"], g["prim"], g["inst"])
    assert np.array_equal(gpu_ctx.occluded(z["O"], z["D"], z["tmax"]).astype(bool), z["occ"].astype(bool))


@pytest.mark.gpu
def test_gpu_trace_matches_golden(gpu_ctx):
    sd, z = _trace()
    W, H = int(z["W"]), int(z["H"])
    gpu_scene(gpu_ctx, sd, W, H)
    avg, rgb8, st = gpu_ctx.render(W, H, int(z["spp"]), int(z["bounces"]), int(z["flags"]))
    assert st.segments == int(z["segments"]) and st.shadow_rays == int(z["shadow_rays"])
    assert np.array_equal(avg, z["avg"]) and np.array_equal(rgb8, z["rgb8"])


@pytest.mark.gpu
def test_gpu_many_instances_match_golden(gpu_ctx):
    """More instances than the linear list holds: the HIP path walks its instance BVH (query kernels and the
    persistent wavefront traversal) and must equal tinybvh's TLAS records and the reference-traversal image."""
    sd, z = _many()
    W, H = int(z["W"]), int(z["H"])
    gpu_scene(gpu_ctx, sd, W, H)
    assert gpu_ctx.scene_info().tlas_depth > 0
    g = gpu_ctx.intersect(z["O"], z["D"])
    _assert_hits(z, g["t"], g["u"], g["v"], g["prim"], g["inst"])
    assert np.array_equal(gpu_ctx.occluded(z["O"], z["D"], z["tmax"]).astype(bool), z["occ"].astype(bool))
    avg, rgb8, st = gpu_ctx.render(W, H, 2, 3)
    assert (st.segments, st.shadow_rays) == (int(z["segments"]), int(z["shadow_rays"]))
    assert np.array_equal(avg[:, :3], z["avg"]) and np.array_equal(rgb8, z["rgb8"])


@pytest.mark.gpu
def test_gpu_forced_tlas_matches_golden(gpu_ctx, monkeypatch):
    """PRT_TLAS=1: a 3-instance scene through the instance BVH instead of the linear list, bit-identical."""
    monkeypatch.setenv("PRT_TLAS", "1")
    sd, z = _multi()
    gpu_scene(gpu_ctx, sd, 64, 64)
    assert gpu_ctx.scene_info().tlas_depth > 0
    g = gpu_ctx.intersect(z["O"], z["D"])
    _assert_hits(z, g["t"], g["u"], g["v"], g["prim"], g["inst"])
    assert np.array_equal(gpu_ctx.occluded(z["O"], z["D"], z["tmax"]).astype(bool), z["occ"].astype(bool))
    sd, z = _trace()
    W, H = int(z["W"]), int(z["H"])
    gpu_scene(gpu_ctx, sd, W, H)
    avg, rgb8, st = gpu_ctx.render(W, H, int(z["spp"]), int(z["bounces"]), int(z["flags"]))
    assert st.segments == int(z["segments"]) and st.shadow_rays == int(z["shadow_rays"])
    assert np.array_equal(avg, z["avg"]) and np.array_equal(rgb8, z["rgb8"])
    monkeypatch.delenv("PRT_TLAS")
    gpu_scene(gpu_ctx, sd, W, H)  # instances re-packed without the instance BVH for later tests
    assert gpu_ctx.scene_info().tlas_depth == 0
