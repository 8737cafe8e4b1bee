"""A compiled C99 consumer of include/dynohip.h (tests/c_abi/abi_consumer.c),
built with gcc and linked against libdynohip.so directly: pins the C-ABI the
reference-side adapter would bind, without ctypes in
between. The GPU leg runs T2 through create/set_graph/set_values/optimize
and compares with the CPU oracle (liboracle.so, test infrastructure)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "dynosam_amd", "lib")
OLIB = os.path.join(ROOT, "oracle", "build")


@pytest.fixture(scope="module")
def consumer(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("cabi") / "abi_consumer")
    cmd = ["gcc", "-std=c99", "-O1", "-Wall", "-Wextra", "-Werror",
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "oracle"),
           os.path.join(ROOT, "tests", "c_abi", "abi_consumer.c"), "-o", exe,
           "-L", LIB, "-L", OLIB, "-ldynohip", "-ldynosynth", "-loracle", "-lm",
           f"-Wl,-rpath,{LIB}", f"-Wl,-rpath,{OLIB}"]
    subprocess.run(cmd, check=True, capture_output=True, text=True)
    return exe


def test_c_consumer_host_entry_points(consumer):
    env = dict(os.environ)
    try:
        import torch
        no_dev = not torch.cuda.is_available()
    except Exception:
        no_dev = True
    if no_dev:
        env["ABI_EXPECT_NO_DEVICE"] = "1"
    r = subprocess.run([consumer, "host"], capture_output=True, text=True, env=env, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK host" in r.stdout


@pytest.mark.gpu
def test_c_consumer_t2_matches_oracle(consumer):
    r = subprocess.run([consumer, "gpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("OK gpu"), r.stdout
