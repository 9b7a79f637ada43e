"""Post-processing in the oracle: Panini primary rays (Core/Camera.cpp:81-139) and the
screen pass of Renderer::Tick (Core/Renderer.cpp:107-133).  The reference cannot run here (Windows/SDL
app), so the restatement is pinned by the properties its code implies: distortion 0 is a rectilinear
projection, a zero vignette exponent and unit grading leave the pixel alone, the aberration blends the
accumulators of the neighbours in the row-walk order.  Parity unpinned against reference binaries."""
import numpy as np
import pytest

import oracle
from prt import scenes

F = np.float32


def _pack(c):
    m = np.minimum(F(1), c.astype(F))
    q = np.where(m > 0, (F(255) * m).astype(np.uint32), 0).astype(np.uint32)
    return (q[..., 0] << 16) + (q[..., 1] << 8) + q[..., 2]


@pytest.fixture(scope="module")
def osc():
    sd = scenes.config_small(30, 20)
    return oracle.OracleScene(sd, 48, 32)


def test_panini_zero_distortion_is_rectilinear(osc):
    """distortion 0: b = f = 2 cot(pi/2 - fov/2) and the Panini direction is normalize(b*ndc.x, b*ndc.y, 1)
    (Camera.cpp:86-110 with d = 0); the primary rays must then follow the camera basis exactly so."""
    W, H = 48, 32
    osc.set_postfx(True, distortion=0.0, fov=1.2, vignette_radius=0.0)
    # primary hits from the post-processed camera vs rays built here from the same formula
    t, u, v, prim, inst = osc.primary_hits(W, H)
    sd = osc.sd
    basis = np.zeros(9, F)
    osc.L.orc_camera_basis(oracle.f32(sd.cam_pos).ctypes.data, oracle.f32(sd.cam_target).ctypes.data,
                           basis.ctypes.data)
    right, up, ahead = basis[:3].astype(np.float64), basis[3:6].astype(np.float64), basis[6:].astype(np.float64)
    f = 2.0 / np.tan(np.pi / 2 - 1.2 * 0.5)
    ys, xs = np.mgrid[0:H, 0:W]
    ndx, ndy = 2 * xs / W - 1, 1 - 2 * ys / H
    d = (f * ndx)[..., None] * right + (f * ndy)[..., None] * up + ahead
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    O, D = np.repeat(oracle.f32(sd.cam_pos)[None], W * H, 0), d.reshape(-1, 3).astype(F)
    t2, _, _, prim2, _ = osc.intersect(O, D)
    hit = t < 1e30
    agree = (hit == (t2 < 1e30)) & (~hit | (prim == prim2))
    assert agree.mean() > 0.995                       # float vs double directions: edge pixels may flip
    assert np.allclose(t[hit & agree], t2[hit & agree], rtol=1e-4)
    osc.set_postfx(False)


def test_screen_pass_identity_and_grading(osc):
    W, H = 48, 32
    base = osc.render(W, H, spp=2, bounces=2)
    # same Panini camera both times (post on): a zero vignette exponent gives vig = 1, unit grading nothing
    osc.set_postfx(True, vignette_radius=0.0)
    a1, r1, _, _ = osc.render(W, H, spp=2, bounces=2)
    assert np.array_equal(r1, _pack(a1[:, :3]))
    assert not np.array_equal(a1, base[0])                     # Panini changed the primary rays
    g = (0.5, 1.0, 2.0, 1.0)
    osc.set_postfx(True, vignette_radius=0.0, color_grading=g)
    a2, r2, _, _ = osc.render(W, H, spp=2, bounces=2)
    assert np.array_equal(a1, a2)                               # avg_rgba is never post-processed
    assert np.array_equal(r2, _pack(a2[:, :3] * F(g[:3])))
    # the vignette: pow(x(1-x)/W^2 .. * intensity, radius) darkens the border, centre brightest
    osc.set_postfx(True, vignette_intensity=20.0, vignette_radius=0.3)
    a3, r3, _, _ = osc.render(W, H, spp=2, bounces=2)
    ys, xs = np.mgrid[0:H, 0:W]
    ux, uy = (xs / F(W)).astype(F), (ys / F(H)).astype(F)
    vig = np.power(((ux * (1 - ux)) * (uy * (1 - uy)) * F(20)).astype(np.float64), np.float64(F(0.3))).astype(F)
    exp = _pack(a3[:, :3] * vig.reshape(-1, 1))
    assert np.mean(exp == r3) > 0.999
    osc.set_postfx(False)


@pytest.mark.parametrize("ab", [1, -1, 3])
def test_aberration_row_walk(osc, ab):
    """Fresh state, one frame: the neighbour left of x already holds this frame's accumulator, the one
    right of x still the previous (zero) one; both divided by x's own sample count (Renderer.cpp:111-120)."""
    W, H = 48, 32
    osc.set_postfx(True, aberration=ab, vignette_radius=0.0)
    a, r, _, _ = osc.render(W, H, spp=2, bounces=2)                 # AA: one reference frame, fresh state
    A = a.reshape(H, W, 4)
    xs = np.arange(W)
    xr, xb = np.clip(xs + ab, 0, W - 1), np.clip(xs - ab, 0, W - 1)
    R = np.where((xr <= xs)[None, :], A[:, xr, 0], F(0))
    B = np.where((xb <= xs)[None, :], A[:, xb, 2], F(0))        # count 1: accumulator == average
    red = (F(0.75) * A[..., 0] + F(0.25) * R).astype(F)
    blue = (F(0.75) * A[..., 2] + F(0.25) * B).astype(F)
    exp = _pack(np.stack([red, A[..., 1], blue], -1)).reshape(-1)
    assert np.array_equal(exp, r)
    osc.set_postfx(False)


def test_no_accumulate_leaves_zero_accumulator(osc):
    """!accumulates: the accumulator is cleared after every frame (Renderer.cpp:147), so a later
    accumulating frame at the same hit distance adds to zero (average = frame / samples)."""
    W, H = 48, 32
    st = oracle.new_state(W, H)
    a0, _, st, _ = osc.render(W, H, spp=2, bounces=2, state=st)
    acc, ns, dist = st
    assert np.all(ns == 1)
    a1, _, st, _ = osc.render(W, H, spp=2, bounces=2, flags=oracle.DEFAULT_FLAGS & ~oracle.ACCUMULATE, state=st)
    assert np.all(st[0] == 0) and np.all(st[1] == 1)
    a2, _, st, _ = osc.render(W, H, spp=2, bounces=2, frame_index=1, state=st)
    same = st[1] == 2
    assert same.mean() > 0.9
    fr = osc.render_frames(W, H, spp=2, bounces=2, frame_index=1)[0].reshape(-1, 4)
    assert np.array_equal(a2[same, :3], (fr[same, :3] * (F(1) / F(2))).astype(F))
