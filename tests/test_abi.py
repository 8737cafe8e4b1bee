"""The C-ABI library loads and exports every symbol include/*.h declares
(no compute calls: this runs without a GPU)."""
import ctypes as C
import os
import re

from dynosam_amd import _abi, _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header, prefix):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(" + prefix + r"\w+)\s*\(", src)))


def test_dynohip_exports_every_declared_symbol():
    lib = C.CDLL(_native.lib_path("libdynohip.so"))
    names = declared("dynohip.h", "dynohip_")
    assert len(names) > 30
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_dynosynth_exports_every_declared_symbol():
    lib = C.CDLL(_native.lib_path("libdynosynth.so"))
    names = declared("dynosynth.h", "dynosynth_")
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_abi_version_and_defaults():
    lib = _native.load("libdynohip.so")
    assert lib.dynohip_abi_version() == 3
    p = _abi.LMParams()
    lib.dynohip_lm_params_default(C.byref(p))
    d = _abi.LMParams.gtsam_default()
    for f, _ in p._fields_:
        assert getattr(p, f) == getattr(d, f), f


def test_struct_sizes_match_header():
    # field counts / sizes the C side expects
    assert C.sizeof(_abi.FactorBlock) == 40
    assert C.sizeof(_abi.GraphView) == 6 * 40
    assert C.sizeof(_abi.LMParams) == 8 * 8 + 4 * 4
    assert C.sizeof(_abi.LMSummary) == 4 + 4 + 3 * 8 + 4 + 4
    assert C.sizeof(_abi.TraceEntry) == 4 * 4 + 6 * 8


def test_no_device_create_fails_cleanly():
    import torch
    if torch.cuda.is_available():
        return
    lib = _native.load("libdynohip.so")
    h = C.c_void_p()
    assert lib.dynohip_create(0, C.byref(h)) != 0


def test_dynobackend_exports_every_declared_symbol():
    lib = C.CDLL(_native.lib_path("libdynohip.so"))
    names = declared("dynobackend.h", "dynob_")
    assert len(names) > 30
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_backend_struct_sizes():
    assert C.sizeof(_abi.Measurement) == 8 + 4 + 4 + 8 + 24
    assert C.sizeof(_abi.BackendParams) == 6 * 4 + 4 * 8 + 12 * 8 + 8
    assert C.sizeof(_abi.InputPacket) == 8 + 8 + 96 + 8 * 7
    assert C.sizeof(_abi.ModuleParams) == 4 + 4 + 8 + 4 * 6 + C.sizeof(_abi.LMParams)
    assert C.sizeof(_abi.SpinResult) == 4 * 4 + 8 * 6


def test_dynorefine_exports_every_declared_symbol():
    lib = C.CDLL(_native.lib_path("libdynohip.so"))
    names = declared("dynorefine.h", "dynorefine_")
    assert len(names) >= 9
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert C.sizeof(_abi.RefineBatch) == 8 + 12 * 8
    assert C.sizeof(_abi.RefineResult) == 4 * 4 + 2 * 8
