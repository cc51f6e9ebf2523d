"""The reference's Rust unit tests, ported to C++ against include/iris_hip.hpp (the C++
mirror of the crate's API over the C ABI) and run here: host-side cases on the CPU,
engine / arch cases on the GPU (tests/cpp/test_port.cpp)."""
import pathlib
import subprocess

import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]
CPP = ROOT / "tests" / "cpp"


def _binary():
    subprocess.run(["make", "-s", "-C", str(CPP)], check=True, capture_output=True, text=True, timeout=300)
    return CPP / "test_port"


def _run(which):
    r = subprocess.run([str(_binary()), which], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 failures" in r.stdout


def test_cpp_port_host_cases():
    _run("cpu")


@pytest.mark.gpu
def test_cpp_port_gpu_cases():
    _run("gpu")
