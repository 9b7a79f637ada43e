"""Checkpoint / resume of the progressive accumulation (include/prt.h prt_save_accumulation /
prt_load_accumulation): the reference keeps its accumulator (Core/Renderer.h:61-63) in memory only,
so a long 4K / 16 spp progressive run cannot resume.  Here the state leaves the device as one blob; a fresh
context that loads it and renders the next frame produces the bits the uninterrupted context produces."""
import numpy as np
import pytest

from helpers import gpu_scene
import prt
from prt import scenes

pytestmark = pytest.mark.gpu


def _frames(ctx, W, H, frames, post=None):
    ctx.set_postfx(post)
    out = []
    for f in frames:
        a, r, st = ctx.render(W, H, 2, 3, frame_index=f)
        out.append((a.copy(), r.copy(), st.segments))
    return out


@pytest.mark.parametrize("post", [False, True])
def test_resume_is_bit_identical(gpu_ctx, post):
    sd = scenes.multi_instance(scenes.config_small(40, 30))
    W, H = 96, 64
    pf = prt.postfx_preset(0, color_grading=(1.0, 0.9, 1.1, 1.0)) if post else None
    try:
        gpu_scene(gpu_ctx, sd, W, H)
        ref = _frames(gpu_ctx, W, H, [0, 1, 2, 3], pf)
        gpu_scene(gpu_ctx, sd, W, H)
        _frames(gpu_ctx, W, H, [0, 1], pf)
        blob = gpu_ctx.save_accumulation()
    finally:
        gpu_ctx.set_postfx(None)  # the session context's later users expect no screen pass (Panini moves rays)
    assert len(blob) == 48 + W * H * 24
    c2 = prt.Context(0)
    try:
        gpu_scene(c2, sd, W, H)
        c2.load_accumulation(blob)
        got = _frames(c2, W, H, [2, 3], pf)
    finally:
        c2.close()
    for (a, r, s), (ea, er, es) in zip(got, ref[2:]):
        assert np.array_equal(a, ea) and np.array_equal(r, er) and s == es


def test_renderer_checkpoint_files(tmp_path):
    """The Python Renderer mirror: SaveCheckpoint after two Ticks, LoadCheckpoint in a new Renderer, one more
    Tick each: identical screen and average."""
    sd = scenes.config_small(30, 20)
    W, H = 64, 48
    cam = prt.Camera(sd.cam_pos, sd.cam_target, np.float32(W) / np.float32(H))
    r1 = prt.Renderer(prt.Scene.from_data(sd), cam, W, H)
    r2 = None
    try:
        r1.Tick()
        r1.Tick()
        path = str(tmp_path / "ckpt")  # no .npz suffix: SaveCheckpoint / LoadCheckpoint use the path as given
        r1.SaveCheckpoint(path)
        r1.Tick()
        r2 = prt.Renderer(prt.Scene.from_data(sd), cam, W, H)
        r2.LoadCheckpoint(path)
        r2.Tick()
        assert r2.frame == r1.frame == 3
        assert np.array_equal(r2.average, r1.average) and np.array_equal(r2.screen, r1.screen)
    finally:
        r1.ctx.close()
        if r2 is not None:
            r2.ctx.close()


def test_checkpoint_refusals(gpu_ctx):
    sd = scenes.config_small(20, 20)
    W, H = 48, 32
    c = prt.Context(0)
    try:
        gpu_scene(c, sd, W, H)
        assert c.save_accumulation() == b""  # nothing rendered yet
        c.render(W, H, 2, 2)
        blob = c.save_accumulation()
        with pytest.raises(prt.PrtError):
            c.load_accumulation(blob[:-4])  # truncated
        bad = bytearray(blob)
        bad[0] ^= 0xFF
        with pytest.raises(prt.PrtError):
            c.load_accumulation(bytes(bad))  # not a blob
        hdr = np.frombuffer(blob[:48], np.int32).copy()
        hdr[6] += 1  # sh_rank (magic 8 B, version, header bytes, w, h, then the shard geometry)
        with pytest.raises(prt.PrtError):
            c.load_accumulation(hdr.tobytes() + blob[48:])
        c.load_accumulation(blob)  # the intact blob still loads
    finally:
        c.close()
    g = prt.Context(group=[0, 0], tile=16)
    try:
        gpu_scene(g, sd, W, H)
        g.render(W, H, 2, 2)
        with pytest.raises(prt.PrtError):
            g.save_accumulation()
    finally:
        g.close()
