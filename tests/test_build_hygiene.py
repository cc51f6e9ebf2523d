"""CPU: the shipped library never carries a diagnostic compile knob.  Diagnostic knobs
(IRIS_*_DIAG, IRIS_STORE_DIAG) build kernels that drop work on purpose;
the Makefile refuses them for libiris_hip.so (variants go through tools/build_variant.sh
under their own names), the sources refuse them under IRIS_SHIPPED_BUILD, and
iris_version() names every -DIRIS_* knob a build was given."""
import pathlib
import subprocess

import iris_hip as ih

ROOT = pathlib.Path(__file__).resolve().parents[1]
PKG = ROOT / "mpc-iris-code_amd"


def _make(*args):
    return subprocess.run(["make", "-C", str(PKG), *args], capture_output=True, text=True, timeout=120)


def test_shipped_target_refuses_diag_knobs(tmp_path):
    for knob in ("-DIRIS_MFMA_DIAG=1", "-DIRIS_STORE_DIAG", "-DIRIS_BATCH2_DIAG=5", "-DIRIS_PREP_DIAG=2"):
        r = _make("-n", f"BUILD={tmp_path}/b", f"HIPFLAGS=-O3 --offload-arch=gfx950 {knob}")
        assert r.returncode != 0 and "refusing to build the shipped libiris_hip.so" in r.stderr, (knob, r.stderr)


def test_variant_and_zero_knobs_are_allowed(tmp_path):
    # a variant library may carry a diagnostic knob; a knob set to 0 is the default
    r = _make("-n", f"BUILD={tmp_path}/v", "LIB=libiris_variant_test.so", "HIPFLAGS=-O3 -DIRIS_MFMA_DIAG=1")
    assert r.returncode == 0, r.stderr
    assert "IRIS_SHIPPED_BUILD" not in r.stdout and "-DIRIS_BUILD_KNOBS='\"-DIRIS_MFMA_DIAG=1\"'" in r.stdout
    r = _make("-n", f"BUILD={tmp_path}/z", "HIPFLAGS=-O3 -DIRIS_MFMA_DIAG=0")
    assert r.returncode == 0 and "-DIRIS_SHIPPED_BUILD=1" in r.stdout, r.stderr


def test_source_guard_refuses_diag_knob_in_shipped_build(tmp_path):
    """Even past the Makefile, a shipped-build compile with a diagnostic knob stops at #error."""
    r = subprocess.run(["/opt/rocm/bin/hipcc", "-std=c++17", "-fsyntax-only", "-x", "c++", "--offload-arch=gfx950",
                        "-DIRIS_SHIPPED_BUILD=1", "-DIRIS_BATCH_DIAG=3", "-I", str(PKG / "csrc"),
                        str(PKG / "csrc" / "iris_internal.hpp")], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "diagnostic knob in the shipped" in r.stderr, r.stderr[-2000:]


def test_shipped_library_reports_no_knobs():
    v = ih.load_library().iris_version().decode()
    assert "gfx950" in v and "knobs" not in v, v
