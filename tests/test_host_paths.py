"""CPU: the library's host-side copy-out paths without a GPU (tests/cpp/test_host_paths.cpp): the
expansion of packed MasksEngine rows -- escaped rows, every alignment of the caller's array, the
non-temporal 32-record blocks -- against a scalar restatement, and the helper pool's parallel
copies and expansions from concurrent callers."""
import pathlib
import subprocess

ROOT = pathlib.Path(__file__).resolve().parents[1]
CPP = ROOT / "tests" / "cpp"


def test_host_paths():
    subprocess.run(["make", "-s", "-C", str(CPP), "test_host_paths"], check=True, capture_output=True, text=True,
                   timeout=300)
    r = subprocess.run([str(CPP / "test_host_paths")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
