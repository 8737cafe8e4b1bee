"""The shared sin / tan / acos of the pose arithmetic (dynosam_amd/csrc/trig.h).

The kernels (se3.hpp) and the CPU oracle (oracle.c) both evaluate GTSAM's
Rot3/Pose3 Expmap and Logmap (SO3.cpp, Pose3.cpp of GTSAM 4.2.0) through
trig.h instead of the device / glibc libm, so the Between and Prior rows
round identically on both sides (tests/test_gpu_parity.py checks the bits
on the GPU). Here, on the CPU, through the oracle's build of the header:
- every coefficient is the nearest double of its exact series term;
- sin, tan and acos are within 1, 2 and 1 ulp of mpmath;
- Pose3 Logmap / Expmap built on them agree with a 200-bit mpmath
  evaluation of the same GTSAM formulas to a few ulp of the inputs' scale,
  including the cancelling small-rotation range of 1 - theta/(2 tan(theta/2))
  and the acos argument near 1.
"""
import ctypes as C
import math
import os
import re
from fractions import Fraction

import mpmath as mp
import numpy as np
import pytest

from oracle_binding import dptr, lib, pose_expmap, pose_logmap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "dynosam_amd", "csrc", "trig.h")


def trig(which, x):
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.zeros_like(x)
    L = lib()
    L.oracle_trig.argtypes = [C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_size_t]
    L.oracle_trig(which, dptr(x), dptr(y), x.size)
    return y


def ulp_err(got, exact):
    """|got - exact| in units of the last place of the double nearest exact"""
    e = float(exact)
    u = math.ulp(e) if e != 0.0 else math.ulp(0.0)
    return abs(mp.mpf(got) - exact) / u


def test_coefficients_are_the_series_terms():
    text = open(HEADER).read()
    consts = dict(re.findall(r"#define (DHT_[A-Z0-9_]+) (-?0x1\.[0-9a-f]+p[-+]\d+)", text))
    f = lambda k: float.fromhex(consts[k])
    for k in range(1, 9):
        assert f(f"DHT_S{k}") == float(Fraction((-1) ** k, math.factorial(2 * k + 1)))
        assert f(f"DHT_C{k}") == float(Fraction((-1) ** (k + 1), math.factorial(2 * k + 2)))
    asin = re.findall(r"p = (0x1\.[0-9a-f]+p[-+]\d+)", text[text.index("dht_asin_p"):])
    terms = [float(Fraction(math.factorial(2 * n), 4 ** n * math.factorial(n) ** 2 * (2 * n + 1)))
             for n in range(1, 27)]
    assert [float.fromhex(a) for a in reversed(asin)] == terms
    with mp.workprec(300):
        pio2 = mp.pi / 2
        assert mp.mpf(f("DHT_PIO2_1")) + f("DHT_PIO2_2") + f("DHT_PIO2_3") - pio2 < mp.mpf(2) ** -120
        assert f("DHT_PIO2_HI") == float(pio2) and f("DHT_PIO2_LO") == float(pio2 - f("DHT_PIO2_HI"))
        assert f("DHT_PI_HI") == float(mp.pi) and f("DHT_INV_PIO2") == float(1 / pio2)
    for k in ("DHT_PIO2_1", "DHT_PIO2_2"):   # 33 significant bits: n * part exact for |n| < 2^20
        m, _ = math.frexp(f(k))
        assert (m * 2 ** 33).is_integer()


def _samples(rng):
    return np.concatenate([
        rng.uniform(-np.pi, np.pi, 4000),
        rng.uniform(-1e-3, 1e-3, 1000),
        10.0 ** rng.uniform(-300, -5, 500),
        rng.uniform(-200.0, 200.0, 1000),
        np.arange(-8, 9) * np.pi / 4,            # octant edges of the reduction
        np.nextafter(np.pi / 4, [0.0, 4.0]),
        [0.0, -0.0, 1e-320, np.pi, np.pi / 2, 355.0, 1e5],
    ])


@pytest.mark.parametrize("which,fn,bound", [(0, mp.sin, 1.0), (1, mp.tan, 2.0)])
def test_sin_tan_ulp(which, fn, bound):
    xs = _samples(np.random.default_rng(7 + which))
    ys = trig(which, xs)
    worst = 0.0
    with mp.workprec(200):
        for x, y in zip(xs, ys):
            worst = max(worst, ulp_err(y, fn(mp.mpf(float(x)))))
    assert worst <= bound, worst


def test_acos_ulp():
    rng = np.random.default_rng(11)
    xs = np.concatenate([
        rng.uniform(-1.0, 1.0, 4000),
        1.0 - 10.0 ** rng.uniform(-16, -1, 2000),     # near 1: small rotations
        -1.0 + 10.0 ** rng.uniform(-16, -1, 500),
        [0.5, -0.5, np.nextafter(0.5, 1.0), np.nextafter(-0.5, -1.0), 1.0, -1.0, 0.0],
    ])
    ys = trig(2, xs)
    worst = 0.0
    with mp.workprec(200):
        for x, y in zip(xs, ys):
            worst = max(worst, ulp_err(y, mp.acos(mp.mpf(float(x)))))
    assert worst <= 1.0, worst


def test_special_values():
    y = trig(0, np.array([np.nan, np.inf, -np.inf]))
    assert np.all(np.isnan(y))
    y = trig(2, np.array([np.nan, 1.0 + 2 ** -52, -2.0]))
    assert np.all(np.isnan(y))
    assert trig(2, np.array([1.0]))[0] == 0.0
    assert trig(0, np.array([-0.0]))[0] == 0.0


def _mp_pose_logmap(T):
    """GTSAM 4.2.0 Pose3::Logmap / SO3::Logmap (normal branch) at 200 bits"""
    R = [mp.mpf(float(v)) for v in T[:9]]
    t = [mp.mpf(float(v)) for v in T[9:]]
    tr = R[0] + R[4] + R[8]
    if tr - 3 < -1e-6:
        theta = mp.acos((tr - 1) / 2)
        mag = theta / (2 * mp.sin(theta))
    else:                      # GTSAM's series branch near the identity
        mag = mp.mpf(0.5) - (tr - 3) / 12 + (tr - 3) ** 2 / 60
    w = [mag * (R[7] - R[5]), mag * (R[2] - R[6]), mag * (R[3] - R[1])]
    th = mp.sqrt(w[0] ** 2 + w[1] ** 2 + w[2] ** 2)
    if th < 1e-10:
        return w + t
    wn = [wi / th for wi in w]
    W = [[0, -wn[2], wn[1]], [wn[2], 0, -wn[0]], [-wn[1], wn[0], 0]]
    WT = [sum(W[i][j] * t[j] for j in range(3)) for i in range(3)]
    WWT = [sum(W[i][j] * WT[j] for j in range(3)) for i in range(3)]
    c = 1 - th / (2 * mp.tan(th / 2))
    return w + [t[i] - (th / 2) * WT[i] + c * WWT[i] for i in range(3)]


def _mp_pose_expmap(xi):
    w = [mp.mpf(float(v)) for v in xi[:3]]
    v = [mp.mpf(float(x)) for x in xi[3:]]
    th2 = w[0] ** 2 + w[1] ** 2 + w[2] ** 2
    if th2 <= np.finfo(np.float64).eps:   # GTSAM's first-order branch
        return [1, -w[2], w[1], w[2], 1, -w[0], -w[1], w[0], 1] + v
    th = mp.sqrt(th2)
    K = [[0, -w[2] / th, w[1] / th], [w[2] / th, 0, -w[0] / th], [-w[1] / th, w[0] / th, 0]]
    KK = [[sum(K[i][k] * K[k][j] for k in range(3)) for j in range(3)] for i in range(3)]
    R = [[(1 if i == j else 0) + mp.sin(th) * K[i][j] + (1 - mp.cos(th)) * KK[i][j] for j in range(3)]
         for i in range(3)]
    wv = sum(w[i] * v[i] for i in range(3))
    wxv = [w[1] * v[2] - w[2] * v[1], w[2] * v[0] - w[0] * v[2], w[0] * v[1] - w[1] * v[0]]
    Rwxv = [sum(R[i][j] * wxv[j] for j in range(3)) for i in range(3)]
    t = [(wxv[i] - Rwxv[i] + w[i] * wv) / th2 for i in range(3)]
    return [R[i][j] for i in range(3) for j in range(3)] + t


def test_pose_logmap_expmap_against_mpmath():
    """The Between/Prior residual is Logmap of a pose near identity (near
    convergence) or far from it (initial values); its Jacobian uses Expmap
    only through the retraction. Rotation angles from 1e-9 to 3 rad."""
    rng = np.random.default_rng(3)
    worst_log = worst_exp = 0.0
    eps = np.finfo(np.float64).eps
    with mp.workprec(200):
        for ang in 10.0 ** rng.uniform(-9, 0.45, 300):
            ax = rng.normal(size=3)
            xi = np.concatenate([ax / np.linalg.norm(ax) * ang, rng.normal(size=3) * rng.choice([1e-6, 1e-2, 1.0, 30.0])])
            T = pose_expmap(xi)
            e = _mp_pose_expmap(xi)
            # GTSAM's translation (w x v - R (w x v) + w w.v) / theta^2 cancels
            # for small theta: eps |v| / theta is the formula's own conditioning
            scale = 1.0 + np.linalg.norm(xi[3:]) * (1.0 + 1.0 / ang)
            worst_exp = max(worst_exp, max(abs(float(a) - float(b)) for a, b in zip(T, e)) / (eps * scale))
            got = pose_logmap(T)
            ref = _mp_pose_logmap(T)
            scale = np.linalg.norm(T[9:]) + ang
            err = max(abs(mp.mpf(float(g)) - r) for g, r in zip(got, ref))
            worst_log = max(worst_log, float(err) / (eps * scale))
    print(f"expmap worst {worst_exp:.2f}, logmap worst {worst_log:.2f} (eps x scale)")
    assert worst_exp < 8.0, worst_exp
    assert worst_log < 16.0, worst_log


def _domain(rng):
    """the arguments the pose arithmetic passes: sin(theta), sin(theta / 2)
    and tan(theta / 2) of rotation angles in [0, pi] (down to the 1e-10 of
    near-converged Between / Prior residuals), acos of (tr - 1) / 2 in
    [-1, 1], crowded near 1 (small rotations)"""
    th = np.concatenate([rng.uniform(0.0, np.pi, 3000), 10.0 ** rng.uniform(-10, 0, 2000)])
    c = np.concatenate([rng.uniform(-1.0, 1.0, 2000), 1.0 - 10.0 ** rng.uniform(-16, -1, 2000)])
    return th, c


@pytest.mark.parametrize("which", [0, 1, 2])
def test_trig_h_against_glibc(which):
    """trig.h against glibc's sin / tan / acos (what GTSAM calls: the oracle's
    libm build, liboracle_libm.so, and Python's math module) over the
    domain the formulations use: within 2 ulp everywhere, and equal on most
    arguments, so sharing trig.h between the kernels and the oracle removes
    no more than a 1-2 ulp gap from the parity tests."""
    th, c = _domain(np.random.default_rng(21 + which))
    xs = {0: np.concatenate([th, th / 2]), 1: th / 2, 2: c}[which]
    ours = trig(which, xs)
    glibc = np.zeros_like(xs)
    lib(libm=True).oracle_trig.argtypes = [C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_size_t]
    lib(libm=True).oracle_trig(which, dptr(np.ascontiguousarray(xs)), dptr(glibc), xs.size)
    pyf = (math.sin, math.tan, math.acos)[which]
    assert np.array_equal(glibc, np.array([pyf(float(x)) for x in xs]))   # the libm build calls glibc
    ulps = np.abs(ours - glibc) / np.array([math.ulp(float(g)) if g != 0 else math.ulp(0.0) for g in glibc])
    same = float(np.mean(ours == glibc))
    print(("sin", "tan", "acos")[which], f"max {ulps.max():.1f} ulp from glibc, {100 * same:.1f} % identical")
    assert ulps.max() <= 2.0
    assert same >= (0.9, 0.6, 0.9)[which]
