"""The C++ host layer (include/mgenx.hpp) over the C ABI: it compiles with plain g++ (CPU)
and its round-trip program passes on the GPU."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "host_roundtrip")


def test_header_compiles_with_gxx():
    src = os.path.join(ROOT, "tests", "cpp", "host_roundtrip.cpp")
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-Werror",
                        "-D__HIP_PLATFORM_AMD__", "-I" + os.path.join(ROOT, "include"),
                        "-I/opt/rocm/include", src], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.gpu
def test_host_roundtrip_program():
    if not os.path.exists(BIN):
        subprocess.run(["make", "-s", "-C", ROOT, "tests/cpp/host_roundtrip"], check=True)
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host_roundtrip ok" in r.stdout
