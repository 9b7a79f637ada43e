"""The bench line's roofline counters are tied to the timed library by a code-object hash (prt/codeobj.py):
CPU tests of the ELF / offload-bundle parsing and of bench.py's staleness rule (no GPU needed)."""
import json
import os

import pytest

from prt import _lib, codeobj

LIB = _lib.LIBPATH
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.skipif(not os.path.exists(LIB), reason="libprt.so not built")


def test_every_wavefront_kernel_is_hashed():
    h = codeobj.base_hashes(LIB)
    for k in ("k_trace2", "k_shade2", "k_resmiss2", "k_miss2", "k_wave_init", "k_accumulate", "k_refit"):
        assert k in h and len(h[k]) == 64


def test_instantiations_and_demangling():
    inst = codeobj.kernel_hash(LIB, "k_trace2")
    assert len(inst) >= 2  # the trace kernel is a template: occupancy / TLAS / spill forms
    assert all(codeobj.demangled_base(k) == "k_trace2" for k in inst)
    assert codeobj.profile_kernel_base("prt::k_trace2<32, 9, 7, 64, false, false>") == "k_trace2"
    assert codeobj.profile_kernel_base("void prt::k_accumulate(prt::TileMap, int)") == "k_accumulate"


def test_hash_is_stable_and_content_addressed(tmp_path):
    a = codeobj.base_hashes(LIB)
    assert a == codeobj.base_hashes(LIB)
    # flip one byte inside k_trace2's machine code: only k_trace2's hash may change
    lib = bytearray(open(LIB, "rb").read())
    secs = codeobj._sections(bytes(lib))
    fat_off = secs[".hip_fatbin"][0]
    cos = codeobj._code_objects(bytes(lib), "gfx950")
    for co in cos:
        csecs = codeobj._sections(co)
        syms = {n: (v, s) for n, v, s in codeobj._symbols(co, csecs)}
        names = [n for n in syms if codeobj.demangled_base(n) == "k_trace2" and n + ".kd" in syms]
        if names:
            v, _ = syms[names[0]]
            at = bytes(lib).find(co, fat_off) + codeobj._vaddr_to_off(csecs, v) + 16
            lib[at] ^= 0xFF
            break
    else:
        pytest.fail("k_trace2 not found in any code object")
    p = tmp_path / "libprt_mod.so"
    p.write_bytes(bytes(lib))
    b = codeobj.base_hashes(str(p))
    assert b["k_trace2"] != a["k_trace2"]
    assert {k: v for k, v in a.items() if k != "k_trace2"} == {k: v for k, v in b.items() if k != "k_trace2"}


def test_bench_withholds_frac_on_a_stale_profile():
    import bench
    live = bench.current_code_hash("k_trace2")
    assert live == codeobj.base_hashes(LIB)["k_trace2"]
    assert bench.fresh({"code_hash": live}, live)
    assert not bench.fresh({"code_hash": "0" * 64}, live)
    assert not bench.fresh({}, live)  # unstamped summaries never count
    assert not bench.fresh({"code_hash": live}, None)


def test_committed_profiles_are_stamped():
    for f in ("current_c4.json", "current_c5.json"):  # what bench.py prices (scripts/summarize_session.py)
        d = json.load(open(os.path.join(ROOT, "profiles", f)))
        rec = [v for k, v in d["kernels"].items() if codeobj.profile_kernel_base(k) == "k_trace2"]
        assert rec and len(rec[0].get("code_hash", "")) == 64, f
