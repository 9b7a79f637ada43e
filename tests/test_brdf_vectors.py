"""Known-answer vectors for the BRDF restatement (Core/BRDF.cpp:16-526, Core/BRDF.h:42-80), VERDICT r5 item 5.

Every expected value is computed HERE, in float64, from the closed forms the reference's BRDF.cpp spells out
(GGX D, height-correlated Smith G2 divided by the denominator, Schlick F with shadowedF90, getBrdfProbability,
Heitz's VNDF sampling, the hemisphere sample and evalIndirectCombinedBRDF's reuse of u) -- not by calling the
oracle.  The same records then go through
  - the oracle's C restatement (oracle/prt_oracle.c orc_brdf_probe, CPU test), and
  - the device functions the shading kernels inline (prt_shade.h, through prt_brdf_probe, GPU test),
each within a float32 tolerance of the closed form, and the device bit-identical to the oracle.
A transcription slip shared by both restatements would fail the closed forms."""
import math

import numpy as np
import pytest

import prt

PI = float(np.float32(3.141592653589))  # BRDF.h:27 PI (float macro), not common.h's double
F0_MIN = 0.4                             # MIN_DIELECTRICS_F0 (BRDF.h:65)
EVAL, PROB, INDIRECT, GGX_D, SMITH_G2, FRESNEL, SHADOWED_F90, VNDF = range(8)


# ---------------------------------------------------------------------------------------- closed forms (float64)
def lum(c):
    return 0.2126 * c[0] + 0.7152 * c[1] + 0.0722 * c[2]                                    # :16-19


def f0_of(base, metal):
    return [F0_MIN + (b - F0_MIN) * metal for b in base]                                   # :21-30 lerp


def f90_of(F0):
    return min(1.0, lum(F0) / F0_MIN)                                                      # :100-104


def schlick(f0, f90, x):
    return [f + (f90 - f) * (1.0 - x) ** 5 for f in f0]                                    # :84-87


def ggx(a2, nh):
    b = (a2 - 1.0) * nh * nh + 1.0                                                         # :218-222
    return a2 / (PI * b * b)


def g2(a2, nl, nv):                                                                        # :189-208
    a = nv * math.sqrt(a2 + nl * (nl - a2 * nl))
    b = nl * math.sqrt(a2 + nv * (nv - a2 * nv))
    return 0.5 / (a + b)


def nrm(v):
    v = np.asarray(v, np.float64)
    return v / np.linalg.norm(v)


def eval_brdf(N, L, V, base, metal, rough):                                               # :398-452
    N, L, V = (np.asarray(x, np.float64) for x in (N, L, V))
    H = nrm(L + V)
    nl, nv = float(N @ L), float(N @ V)
    if nl <= 0 or nv <= 0:
        return [0.0, 0.0, 0.0]
    nl, nv = min(max(1e-5, nl), 1.0), min(max(1e-5, nv), 1.0)
    lh, nh = min(max(float(L @ H), 0.0), 1.0), min(max(float(N @ H), 0.0), 1.0)
    F0 = f0_of(base, metal)
    F = schlick(F0, f90_of(F0), lh)
    a2 = (rough * rough) ** 2
    D, G = ggx(max(1e-5, a2), nh), g2(a2, nl, nv)
    diff = [b * (1.0 - metal) * nl / PI for b in base]
    return [(1.0 - F[k]) * diff[k] + F[k] * (G * D * nl) for k in range(3)]


def probability(N, V, base, metal):                                                        # :504-526
    sF0 = lum(f0_of(base, metal))
    dR = lum([b * (1.0 - metal) for b in base])
    ff = max(0.0, float(np.dot(V, N)))
    fr = min(max(lum(schlick([sF0] * 3, f90_of([sF0] * 3), ff)), 0.0), 1.0)
    spec = 0.5 * fr
    diff = dR * (1.0 - 0.5 * fr) * 1.5
    return min(max(spec / max(1e-4, spec + diff), 0.05), 0.7)


def vndf(Ve, ax, ay, u):                                                                   # :224-269 (Heitz 2018)
    Vh = nrm([ax * Ve[0], ay * Ve[1], Ve[2]])
    lensq = Vh[0] ** 2 + Vh[1] ** 2
    T1 = np.array([-Vh[1], Vh[0], 0.0]) / math.sqrt(lensq) if lensq > 0 else np.array([1.0, 0.0, 0.0])
    T2 = np.cross(Vh, T1)
    r, phi = math.sqrt(u[0]), 2.0 * PI * u[1]
    t1, t2 = r * math.cos(phi), r * math.sin(phi)
    s = 0.5 * (1.0 + Vh[2])
    t2 = (1.0 - s) * math.sqrt(1.0 - t1 * t1) + s * t2
    Nh = t1 * T1 + t2 * T2 + math.sqrt(max(0.0, 1.0 - t1 * t1 - t2 * t2)) * Vh
    return nrm([ax * Nh[0], ay * Nh[1], max(0.0, Nh[2])])


def to_local(N):                                                                           # :43-60
    N = np.asarray(N, np.float64)
    if N[2] < -0.99999:
        q = np.array([1.0, 0.0, 0.0, 0.0])
    else:
        q = np.array([N[1], -N[0], 0.0, 1.0 + N[2]])
        q = q / np.linalg.norm(q)

    def rot(qq, v):
        a, w = qq[:3], qq[3]
        return 2.0 * (a @ v) * a + (w * w - a @ a) * v + 2.0 * w * np.cross(a, v)
    return q, rot


def indirect(u, N, V, base, metal, rough, typ):                                            # :454-502
    q, rot = to_local(N)
    Vl = rot(q, np.asarray(V, np.float64))
    alpha = rough * rough
    w = np.ones(3)
    if typ == 1:  # diffuse: cosine hemisphere from u, then the VNDF half-vector of the SAME u for the Fresnel
        a, b = math.sqrt(u[0]), 2.0 * PI * u[1]
        rl = np.array([a * math.cos(b), a * math.sin(b), math.sqrt(1.0 - u[0])])
        F0 = f0_of(base, metal)
        Hs = vndf(Vl, alpha, alpha, u)
        vh = max(1e-5, min(1.0, float(Vl @ Hs)))
        F = schlick(F0, f90_of(F0), vh)
        w = np.array([base[k] * (1.0 - metal) * (1.0 - F[k]) for k in range(3)])
    else:  # specular: the caller's weight stays (1,1,1) (sampleSpecularMicrofacet takes it by value, :351)
        H = np.array([0.0, 0.0, 1.0]) if alpha == 0 else vndf(Vl, alpha, alpha, u)
        rl = -Vl - 2.0 * float(-Vl @ H) * H
    if lum(w) == 0:
        return 0.0, np.zeros(3), w
    qi = np.array([-q[0], -q[1], -q[2], q[3]])
    return 1.0, nrm(rot(qi, rl)), w


# ---------------------------------------------------------------------------------------- the vectors
def rec(**kw):
    r = np.zeros(24, np.float64)
    for k, (lo, v) in {"N": (0, None), "L": (3, None), "V": (6, None), "base": (9, None), "u": (17, None)}.items():
        if k in kw:
            r[lo:lo + len(kw[k])] = kw[k]
    for k, i in (("metal", 12), ("rough", 16), ("typ", 19)):
        if k in kw:
            r[i] = kw[k]
    if "raw" in kw:
        r[:len(kw["raw"])] = kw["raw"]
    return r


def vectors():
    """(op, record, expected[8], tolerance) tuples: >= 40 vectors over every probe op."""
    out = []
    for alpha in (0.05, 0.3, 1.0):
        a2 = alpha * alpha
        for nh in (1.0, 0.95, 0.7, 0.2):
            out.append((GGX_D, rec(raw=[a2, nh]), [ggx(a2, nh)], 2e-6))
        for nl, nv in ((1.0, 1.0), (0.05, 0.9), (0.9, 0.02), (0.01, 0.01)):   # grazing NdotL / NdotV
            out.append((SMITH_G2, rec(raw=[a2, nl, nv]), [g2(a2, nl, nv)], 2e-6))
    for f0 in ((0.4, 0.4, 0.4), (0.9, 0.6, 0.2)):
        for x in (1.0, 0.5, 0.1, 0.0):
            f90 = f90_of(f0)
            out.append((FRESNEL, rec(raw=[*f0, f90, x]), schlick(f0, f90, x), 2e-6))
    for f0 in ((0.4, 0.4, 0.4), (0.1, 0.1, 0.1), (0.9, 0.6, 0.2), (0.04, 0.04, 0.04), (0.0, 0.3, 0.0)):
        out.append((SHADOWED_F90, rec(raw=list(f0)), [f90_of(f0)], 2e-6))
    Nz, Vz = [0.0, 0.0, 1.0], [0.0, 0.0, 1.0]
    Vg = list(nrm([0.8, 0.1, 0.25]))
    for base, metal in (((0.0, 0.0, 0.0), 0.0), ((1.0, 1.0, 1.0), 0.0), ((0.02, 0.02, 0.02), 0.0),  # clamp edges
                        ((1.0, 1.0, 1.0), 1.0), ((0.5, 0.5, 0.5), 0.5), ((0.9, 0.3, 0.1), 0.0)):
        for V in (Vz, Vg):
            out.append((PROB, rec(N=Nz, V=V, base=base, metal=metal), [probability(Nz, V, base, metal)], 2e-6))
    for Ve, a, u in ((Vz, 0.3, (0.25, 0.6)), (Vg, 0.5, (0.7, 0.1)), (list(nrm([0.1, -0.3, 0.9])), 0.05, (0.5, 0.5)),
                     (list(nrm([-0.6, 0.2, 0.1])), 1.0, (0.9, 0.95))):
        out.append((VNDF, rec(raw=[*Ve, a, a, *u]), list(vndf(Ve, a, a, u)), 1e-5))
    N1 = list(nrm([0.2, 0.9, 0.3]))
    for L, V, base, metal, rough in ((Nz, Vz, (0.5, 0.5, 0.5), 0.0, 1.0), (Nz, Vz, (0.8, 0.2, 0.1), 1.0, 0.3),
                                     (list(nrm([0.3, 0.1, 0.9])), Vg, (0.5, 0.7, 0.9), 0.0, 0.5),
                                     (list(nrm([-0.5, 0.0, 0.1])), list(nrm([0.6, 0.2, 0.2])), (0.9, 0.9, 0.9), 0.2, 0.8),
                                     (list(nrm([0.1, 0.2, -0.5])), Vz, (0.5, 0.5, 0.5), 0.0, 0.5)):  # backfacing L
        out.append((EVAL, rec(N=Nz, L=L, V=V, base=base, metal=metal, rough=rough),
                    eval_brdf(Nz, L, V, base, metal, rough), 2e-5))
    out.append((EVAL, rec(N=N1, L=list(nrm([0.0, 1.0, 0.2])), V=list(nrm([0.3, 0.8, 0.0])), base=(0.3, 0.6, 0.9),
                          metal=0.5, rough=0.4),
                eval_brdf(N1, nrm([0.0, 1.0, 0.2]), nrm([0.3, 0.8, 0.0]), (0.3, 0.6, 0.9), 0.5, 0.4), 2e-5))
    for u, N, V, base, metal, rough, typ in (((0.25, 0.1), Nz, Vz, (0.5, 0.5, 0.5), 0.0, 1.0, 1),
                                             ((0.7, 0.4), N1, list(nrm([0.2, 0.7, 0.6])), (0.8, 0.4, 0.2), 0.3, 0.6, 1),
                                             ((0.05, 0.9), Nz, Vg, (0.9, 0.9, 0.9), 0.0, 0.2, 1),
                                             ((0.3, 0.6), Nz, Vz, (0.5, 0.5, 0.5), 0.0, 1.0, 2),
                                             ((0.6, 0.2), N1, list(nrm([0.2, 0.7, 0.6])), (0.8, 0.4, 0.2), 1.0, 0.5, 2)):
        ok, d, w = indirect(u, N, V, base, metal, rough, typ)
        out.append((INDIRECT, rec(N=N, V=V, base=base, metal=metal, rough=rough, u=u, typ=typ),
                    [ok, *d, *w], 3e-5))
    return out


def _check(results, vecs):
    bad = []
    for (op, _, exp, tol), got in zip(vecs, results):
        e = np.asarray(exp, np.float64)
        g = got[:len(e)].astype(np.float64)
        if not np.allclose(g, e, rtol=tol, atol=tol):
            bad.append((op, e.tolist(), g.tolist()))
    assert not bad, bad[:5]


def _run(probe, vecs):
    res = [None] * len(vecs)
    for op in sorted({v[0] for v in vecs}):
        idx = [i for i, v in enumerate(vecs) if v[0] == op]
        out = probe(op, np.stack([vecs[i][1] for i in idx]).astype(np.float32))
        for k, i in enumerate(idx):
            res[i] = out[k]
    return res


def test_vector_count():
    vecs = vectors()
    assert len(vecs) >= 40
    assert {v[0] for v in vecs} == set(range(8))


def test_oracle_brdf_known_answers(oracle_mod):
    vecs = vectors()
    _check(_run(oracle_mod.brdf_probe, vecs), vecs)


@pytest.mark.gpu
def test_device_brdf_known_answers(oracle_mod):
    """prt_brdf_probe (the device functions the shading kernels inline) against the closed forms, and bit for bit
    against the oracle's restatement."""
    vecs = vectors()
    ctx = prt.Context(0)
    try:
        dev = _run(ctx.brdf_probe, vecs)
    finally:
        ctx.close()
    _check(dev, vecs)
    orc = _run(oracle_mod.brdf_probe, vecs)
    for (op, _, _, _), a, b in zip(vecs, dev, orc):
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), (op, a, b)
