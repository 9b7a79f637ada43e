"""AddressSanitizer + UndefinedBehaviorSanitizer over the native host code that runs on the CPU (SURVEY.md §5,
race detection / sanitizers): the host BVH builders (physically-based-ray-tracer_amd/csrc/bvh_build.cpp, through
tests/cpp/bvh_check.cpp), the PNG scanline / capture helpers (csrc/ingest_png.c) and the oracle's C restatement
(oracle/prt_oracle.c).  Each is rebuilt with -fsanitize=address,undefined -fno-sanitize-recover=all, so any
out-of-bounds access, use after free, signed overflow, misaligned access or invalid shift aborts the run.  The
sanitized oracle must also render the same bits as the regular build.  GPU code is not covered (no GPU ASan on
this pool); the device side has its own overflow counter (prt_stats.stack_overflows)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from prt import scenes

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "physically-based-ray-tracer_amd", "csrc")
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=all", "-fno-omit-frame-pointer", "-g", "-O1"]
ENV = dict(os.environ, ASAN_OPTIONS="abort_on_error=0:halt_on_error=1:detect_leaks=0",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


def _libasan():
    p = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


pytestmark = pytest.mark.skipif(_libasan() is None, reason="gcc's ASan runtime is not installed")


@pytest.fixture(scope="module")
def bvh_checker(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("asan") / "bvh_check_asan")
    subprocess.run(["g++", "-std=c++17", *SAN, "-I", CSRC, os.path.join(ROOT, "tests", "cpp", "bvh_check.cpp"),
                    os.path.join(CSRC, "bvh_build.cpp"), "-o", exe], check=True, capture_output=True, text=True)
    return exe


def _check(exe, *args):
    r = subprocess.run([exe, *args], capture_output=True, text=True, timeout=600, env=ENV)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["ok"], out
    return out


@pytest.mark.parametrize("mesh,spatial", [("heightfield", 0), ("heightfield", 1), ("torus", 1), ("deep", 0)])
def test_bvh_builders_clean(bvh_checker, tmp_path, mesh, spatial):
    m = {"heightfield": lambda: scenes.config_small(60, 40).meshes[0], "torus": lambda: scenes.torus(80, 40),
         "deep": lambda: scenes.deep_bvh().meshes[0]}[mesh]()
    path = str(tmp_path / "tris.bin")
    np.ascontiguousarray(m.triangles, np.float32).tofile(path)
    assert _check(bvh_checker, "blas", path, str(spatial))["tris"] == m.tri_count


def test_tlas_builder_clean(bvh_checker, tmp_path):
    rng = np.random.default_rng(5)
    lo = rng.uniform(-50, 50, (500, 3)).astype(np.float32)
    boxes = np.concatenate([lo, lo + rng.uniform(0.1, 4, (500, 3)).astype(np.float32)], 1)
    path = str(tmp_path / "boxes.bin")
    boxes.tofile(path)
    _check(bvh_checker, "tlas", path)


_SCRIPT = r"""
import sys, numpy as np
sys.path[:0] = [{oracle!r}, {pkg!r}]
import oracle
from prt import ingest, scenes
out = {{}}
for name, sd in (("small", scenes.config_small(24, 16)),
                 ("ext", scenes.with_extensions(scenes.multi_instance(scenes.config_small(20, 14)), materials=[1, 2, 0],
                                                area_light=scenes.ceiling_light()))):
    osc = oracle.OracleScene(sd, 40, 30)
    avg, rgb8, _, st = osc.render(40, 30, spp=2, bounces=3, nthreads=1)
    out[name] = avg
scr = (np.arange(53 * 37, dtype=np.uint32) * 2654435761) & 0xFFFFFF
ingest.capture_png({png!r}, scr, 53, 37)
assert np.array_equal(ingest.load_png({png!r}), scr.reshape(37, 53))
np.savez({npz!r}, **out)
"""


def test_oracle_and_ingest_clean(tmp_path):
    """The oracle's Trace (plain and extension scenes) and the PNG helpers, sanitized, loaded into a child Python
    with the ASan runtime preloaded; the sanitized oracle renders the regular oracle's bits."""
    lib_o = str(tmp_path / "liboracle_asan.so")
    lib_i = str(tmp_path / "libprt_ingest_asan.so")
    subprocess.run(["gcc", "-std=c11", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math", *SAN, "-o", lib_o,
                    os.path.join(ROOT, "oracle", "prt_oracle.c"), "-lm"], check=True, capture_output=True, text=True)
    subprocess.run(["gcc", "-fPIC", "-shared", *SAN, "-o", lib_i, os.path.join(CSRC, "ingest_png.c"), "-lz"],
                   check=True, capture_output=True, text=True)
    npz, png = str(tmp_path / "out.npz"), str(tmp_path / "cap.png")
    script = _SCRIPT.format(oracle=os.path.join(ROOT, "oracle"), pkg=os.path.join(ROOT, "physically-based-ray-tracer_amd"),
                            png=png, npz=npz)
    env = dict(ENV, LD_PRELOAD=_libasan(), PRT_ORACLE_LIB=lib_o, PRT_INGEST_LIB=lib_i, OMP_NUM_THREADS="1")
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    got = np.load(npz)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    for name, sd in (("small", scenes.config_small(24, 16)),
                     ("ext", scenes.with_extensions(scenes.multi_instance(scenes.config_small(20, 14)),
                                                    materials=[1, 2, 0], area_light=scenes.ceiling_light()))):
        avg = oracle.OracleScene(sd, 40, 30).render(40, 30, spp=2, bounces=3)[0]
        assert np.array_equal(got[name], avg), name
