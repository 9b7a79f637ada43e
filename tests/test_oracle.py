"""CPU tests: pin the oracle against the reference's own tinybvh (oracle/_ref) and known answers."""
import math

import numpy as np
import pytest

from helpers import primary_dirs, random_rays
from prt import scenes


def _ref_or_skip(oracle_mod):
    if oracle_mod.reflib() is None:
        pytest.skip("oracle/_ref not built (needs /root/reference)")


def test_rng_sequence(oracle_mod):
    # template/tmpl8math.cpp:15-48 -- xorshift32 (13,17,5), float = u32 * 2^-32, seeded by WangHash
    seed = 0x12345678
    out = oracle_mod.rng_floats(seed, 5)
    s = seed
    for k in range(5):
        s ^= (s << 13) & 0xFFFFFFFF
        s ^= s >> 17
        s ^= (s << 5) & 0xFFFFFFFF
        assert out[k] == np.float32(np.float32(s) * np.float32(2.3283064365387e-10))

    def wang(s):
        s = (s ^ 61) ^ (s >> 16)
        s = (s * 9) & 0xFFFFFFFF
        s = s ^ (s >> 4)
        s = (s * 0x27D4EB2D) & 0xFFFFFFFF
        return s ^ (s >> 15)
    for b in (0, 1, 2, 12345, 0xFFFFFFF0):
        exp = wang(((b + 1) * 17) & 0xFFFFFFFF) or 0x12345678
        assert oracle_mod.init_seed(b) == exp


def test_pack_rgb8(oracle_mod):
    # template/precomp.h:310-315: (uint)(255 * min(1, x)), packed (r<<16)+(g<<8)+b
    assert oracle_mod.pack_rgb8([1.0, 0.5, 0.0, 0]) == (255 << 16) + (127 << 8)
    assert oracle_mod.pack_rgb8([2.0, float("nan"), 0.999, 0]) == (255 << 16) + (255 << 8) + 254


def test_brdf_known_answers(oracle_mod):
    # Lambert-only limit: metal 0, base 0 -> diffuse 0; F0 = 0.4 (MIN_DIELECTRICS_F0, BRDF.h:65)
    N = np.array([0, 0, 1], np.float32)
    L = np.array([0, 0, 1], np.float32)
    V = np.array([0, 0, 1], np.float32)
    mat = np.array([0.5, 0.5, 0.5, 0.0, 0, 0, 0, 1.0], np.float32)  # base .5, metal 0, rough 1
    out = oracle_mod.eval_combined_brdf(N, L, V, mat)
    # at normal incidence: F = F0 = 0.4 (pow(0,5)=0); alpha=1: D = 1/pi; G2 = 0.5/(1*1+1*1) = 0.25
    F = 0.4
    spec = F * (0.25 * (1 / math.pi) * 1.0)
    diff = (1 - F) * 0.5 * (1 / math.pi)
    assert np.allclose(out, spec + diff, rtol=1e-6)
    # backfacing light -> 0 (BRDF.cpp:445)
    assert np.all(oracle_mod.eval_combined_brdf(N, -L, V, mat) == 0)
    # lobe probability is clamped to [0.05, 0.7] (BRDF.cpp:525)
    for base in (0.0, 0.3, 1.0):
        for metal in (0.0, 1.0):
            p = oracle_mod.brdf_probability(np.array([base, base, base, metal, 0, 0, 0, 0.5], np.float32), V, N)
            assert 0.05 <= p <= 0.7
    # specular sampling keeps the caller's weight (sampleSpecularMicrofacet takes it by value)
    ok, d, w = oracle_mod.eval_indirect([0.3, 0.6], N, V, mat, 2)
    assert ok and np.all(w == 1.0)
    assert abs(np.linalg.norm(d) - 1) < 1e-6
    # diffuse sample: cosine hemisphere around N
    ok, d, w = oracle_mod.eval_indirect([0.25, 0.1], N, V, mat, 1)
    assert ok and d[2] > 0 and np.all(w > 0) and np.all(w < 0.5)


def test_oracle_primary_hits_match_tinybvh(oracle_mod):
    """C2 (10k-tri torus): the restated MT leaf test reproduces tinybvh BVH8_CPU hit records bit for bit."""
    _ref_or_skip(oracle_mod)
    sd = scenes.config_c2()
    W, H = 320, 180
    osc = oracle_mod.OracleScene(sd, W, H)
    t, u, v, prim, inst = osc.primary_hits(W, H)
    pos, tl, tr, bl = osc.camera_basis(W, H)
    D = primary_dirs(pos, tl, tr, bl, W, H)
    assert np.all(D != 0), "parity cameras must avoid exact-zero direction components (BVH8_CPU octant bug)"
    ref = oracle_mod.RefScene(sd)
    rt, ru, rv, rp, ri = ref.intersect(np.broadcast_to(pos, D.shape), D)
    hit = t < 1e30
    assert hit.sum() > 5000
    assert np.array_equal(hit, rt < 1e30)
    assert np.array_equal(prim[hit], rp[hit])
    assert np.array_equal(t[hit], rt[hit]) and np.array_equal(u[hit], ru[hit]) and np.array_equal(v[hit], rv[hit])


def test_oracle_random_rays_match_tinybvh(oracle_mod):
    """Closest-hit and any-hit over random rays into a multi-instance heightfield (TLAS path)."""
    _ref_or_skip(oracle_mod)
    sd = scenes.multi_instance(scenes.config_small(60, 40))
    osc = oracle_mod.OracleScene(sd)
    ref = oracle_mod.RefScene(sd)
    O, D = random_rays(sd, 20000)
    t, u, v, prim, inst = osc.intersect(O, D)
    rt, ru, rv, rp, ri = ref.intersect(O, D)
    hit = t < 1e30
    assert hit.mean() > 0.5
    assert np.array_equal(hit, rt < 1e30)
    same = (prim == rp) & (inst == ri)
    assert same[hit].mean() > 0.9999
    assert np.array_equal(t[hit & same], rt[hit & same])
    tmax = np.where(hit, t * np.float32(0.999), np.float32(1e30)).astype(np.float32)
    tmax[::3] = np.float32(1e30)
    occ = osc.occluded(O, D, tmax)
    rocc = ref.occluded(O, D, tmax)
    assert (occ == rocc).mean() > 0.9999


def test_oracle_full_trace_matches_tinybvh_backend(oracle_mod):
    """The restated Trace gives the same image on the built-in BVH and on tinybvh's BVH8_CPU + TLAS."""
    _ref_or_skip(oracle_mod)
    sd = scenes.multi_instance(scenes.config_small(50, 40))
    W, H = 64, 48
    osc = oracle_mod.OracleScene(sd, W, H)
    a1, r1, _, s1 = osc.render(W, H, spp=4, bounces=4)
    osc.use_reference_traversal()
    a2, r2, _, s2 = osc.render(W, H, spp=4, bounces=4)
    assert s1.segments == s2.segments and s1.shadow_rays == s2.shadow_rays
    assert np.array_equal(a1, a2) and np.array_equal(r1, r2)


def test_visit_counter_replicates_library(oracle_mod):
    """The N_int/N_leaf counter re-walks BVH8_CPU::Intersect exactly (same step count, same t)."""
    _ref_or_skip(oracle_mod)
    sd = scenes.config_small(80, 60)
    ref = oracle_mod.RefScene(sd)
    O, D = random_rays(sd, 4000, seed=3)
    sw, sl, nint, nleaf, tw = ref.count_visits(O, D)
    rt = ref.intersect(O, D)[0]
    assert np.array_equal(sw, sl)
    assert np.array_equal(tw, rt)
    assert nint + nleaf == int(sw.sum())


def test_accumulation_semantics(oracle_mod):
    """Renderer.cpp:81-104: two 1-frame calls == one 2-frame call (progressive mean keyed on r1.hit.t)."""
    sd = scenes.config_small(30, 20)
    W, H = 32, 24
    osc = oracle_mod.OracleScene(sd, W, H)
    a_once, r_once, st_once, _ = osc.render(W, H, spp=4, bounces=3)
    st = oracle_mod.new_state(W, H)
    osc.render(W, H, spp=2, bounces=3, frame_index=0, state=st)
    a_two, r_two, st, _ = osc.render(W, H, spp=2, bounces=3, frame_index=1, state=st)
    assert np.array_equal(a_once, a_two) and np.array_equal(r_once, r_two)
    assert np.all(st[1] == 2)
