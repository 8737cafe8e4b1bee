"""Cycles per pivot of the in-wave 16x16 factorisation (f16wave.h) on the
GPU, and the accuracy of W = U^-1 against numpy; and the issue rate of
v_mfma_f64_16x16x4f64 on one wave (registers / LDS operands, four chains /
one): tools/pivot_probe.hip.
Usage: python tools/pivot_probe.py [reps]"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "tools", "build", "libpivot_probe.so")


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    src = os.path.join(ROOT, "tools", "pivot_probe.hip")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
                           "-o", SO, src])


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    if not os.path.exists(SO):
        build()
    L = C.CDLL(SO)
    P = C.POINTER(C.c_double)
    L.probe_run.argtypes = [C.c_int, P, P, C.POINTER(C.c_ulonglong), C.c_int]
    rng = np.random.default_rng(5)
    # the hardware reciprocal estimate's accuracy (v_rcp_f64): ulps from 1/x
    L.probe_rcp.argtypes = [P, P, C.c_int]
    x = np.concatenate([10.0 ** rng.uniform(-30, 30, 200000), rng.uniform(0.5, 2.0, 200000)])
    y = np.zeros_like(x)
    assert L.probe_rcp(x.ctypes.data_as(P), y.ctypes.data_as(P), x.size) == 0
    ex = 1.0 / x
    ulp = np.abs(y - ex) / np.spacing(ex)
    print(f"v_rcp_f64: max {ulp.max():.3g} ulp, mean {ulp.mean():.3g}, exact {np.mean(y == ex) * 100:.1f} %")
    L.probe_mfma.argtypes = [C.c_int, P, C.POINTER(C.c_ulonglong), C.c_int]
    xin = rng.normal(size=256)
    for v, what in ((0, "4 chains, registers"), (1, "4 chains, LDS operands (stride 68)"), (2, "1 chain, registers"),
                      (3, "4 chains, LDS operands, 16-byte reads"), (4, "1 chain, LDS operands, 16-byte reads"),
                      (5, "2 chains, LDS operands, 16-byte reads")):
        cyc = (C.c_ulonglong * 1)()
        assert L.probe_mfma(v, xin.ctypes.data_as(P), cyc, 200) == 0
        print(f"v_mfma_f64_16x16x4f64 {what}: {cyc[0] / (200 * 16):.1f} cycles each")
    for cond in (1e2, 1e8, 1e14):
        Q, _ = np.linalg.qr(rng.normal(size=(16, 16)))
        B = (Q * np.logspace(0, -np.log10(cond), 16)) @ Q.T
        B = 0.5 * (B + B.T)
        U = np.linalg.cholesky(B).T
        Wref = np.linalg.inv(U)
        Ws = {}
        for v in (0, 1, 2, 3, 4, 5, 6):
            W = np.zeros(256)
            cyc = (C.c_ulonglong * 2)()
            rc = L.probe_run(v, np.ascontiguousarray(B.ravel()).ctypes.data_as(P), W.ctypes.data_as(P), cyc, reps)
            assert rc == 0, rc
            W = W.reshape(16, 16)
            Ws[v] = W.copy()
            res = np.linalg.norm(W.T @ B @ W - np.eye(16))
            dev = np.linalg.norm(W - Wref) / np.linalg.norm(Wref)
            print(f"cond {cond:.0e} variant {v}: {cyc[0] / ((reps - 1) * 16):7.1f} cycles/pivot (s_memtime), ok={cyc[1]}, "
                  f"|W^T B W - I| {res:.2e}, W vs numpy {dev:.2e}")
        print(f"cond {cond:.0e}: variant 6 W bit-identical to variant 1: {np.array_equal(Ws[1], Ws[6])}")


if __name__ == "__main__":
    main()
