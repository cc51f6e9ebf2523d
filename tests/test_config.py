"""CPU: runtime knob hygiene (iris_config, csrc/iris_host.cpp read_hooks).  The library reads
its IRIS_* environment once, when a device opens, into that device's configuration; the
test-only hooks (kernel-variant pins, injected delays and faults) take effect only with
IRIS_TEST_HOOKS=1 and are otherwise ignored and reported.  iris_config(NULL) shows what a
device opened now would get, so this runs without a GPU."""
import pytest

import iris_hip as ih

TEST_HOOKS = ["IRIS_TILES_PER_WAVE", "IRIS_FUSED_REDUCE", "IRIS_BATCH_KERNEL", "IRIS_SCHEDULE",
              "IRIS_LOAD_PREAD", "IRIS_GROUP_DELAY_US", "IRIS_GROUP_STALL", "IRIS_GROUP_UNORDERED", "IRIS_UPLOAD",
              "IRIS_LOAD_WINDOWS", "IRIS_READAHEAD_WINDOW", "IRIS_RESIDENT_BUDGET_MB",
              "IRIS_READAHEAD_PACKED", "IRIS_READAHEAD_WINDOW_MAX"]


@pytest.fixture(autouse=True)
def clean_env(monkeypatch):
    for k in TEST_HOOKS + ["IRIS_TEST_HOOKS", "IRIS_READAHEAD", "IRIS_AUTO_RESIDENT", "IRIS_GROUP_TIMEOUT_MS",
                           "IRIS_COPY_HELPERS", "IRIS_RESIDENT_MAX_MB"]:
        monkeypatch.delenv(k, raising=False)


def test_defaults():
    c = ih.config()
    assert c == {"readahead": "1", "auto_resident": "1", "group_timeout_ms": "auto", "group_init_timeout_ms": "120000",
                 "resident_max_mb": "auto", "copy_helpers": "3", "test_hooks": "0"}


def test_resident_cap_is_a_production_knob(monkeypatch):
    monkeypatch.setenv("IRIS_RESIDENT_MAX_MB", "4096")
    c = ih.config()
    assert c["resident_max_mb"] == "4096" and "ignored" not in c


def test_group_timeout_sets_the_formation_bound(monkeypatch):
    monkeypatch.setenv("IRIS_GROUP_TIMEOUT_MS", "6000")
    c = ih.config()
    assert c["group_timeout_ms"] == "6000" and c["group_init_timeout_ms"] == "6000"


def test_test_hooks_ignored_without_opt_in(monkeypatch):
    monkeypatch.setenv("IRIS_TILES_PER_WAVE", "1")
    monkeypatch.setenv("IRIS_FUSED_REDUCE", "0")
    monkeypatch.setenv("IRIS_GROUP_STALL", "1")
    monkeypatch.setenv("IRIS_TEST_HOOKS", "0")
    c = ih.config()
    assert c["test_hooks"] == "0"
    assert "tiles_per_wave" not in c and "group_stall" not in c  # not in effect
    assert c["ignored"] == ["IRIS_TILES_PER_WAVE", "IRIS_FUSED_REDUCE", "IRIS_GROUP_STALL"]


def test_test_hooks_with_opt_in(monkeypatch):
    monkeypatch.setenv("IRIS_TEST_HOOKS", "1")
    monkeypatch.setenv("IRIS_TILES_PER_WAVE", "1")
    monkeypatch.setenv("IRIS_BATCH_KERNEL", "2")
    monkeypatch.setenv("IRIS_SCHEDULE", "spin")
    monkeypatch.setenv("IRIS_GROUP_DELAY_US", "1500")
    monkeypatch.setenv("IRIS_UPLOAD", "pinned")
    c = ih.config()
    assert "ignored" not in c
    assert (c["test_hooks"], c["tiles_per_wave"], c["batch_kernel"], c["schedule"], c["group_delay_us"]) == \
        ("1", "1", "2", "spin", "1500")
    assert (c["fused_reduce"], c["group_stall"], c["load_pread"], c["upload"]) == ("1", "0", "0", "pinned")
    assert c["load_windows"] == "0"
    monkeypatch.setenv("IRIS_RESIDENT_BUDGET_MB", "700")
    assert ih.config()["resident_budget_mb"] == "700"


def test_production_knobs_need_no_opt_in(monkeypatch):
    monkeypatch.setenv("IRIS_READAHEAD", "0")
    monkeypatch.setenv("IRIS_AUTO_RESIDENT", "0")
    monkeypatch.setenv("IRIS_GROUP_TIMEOUT_MS", "45000")
    monkeypatch.setenv("IRIS_COPY_HELPERS", "5")
    c = ih.config()
    assert (c["readahead"], c["auto_resident"], c["group_timeout_ms"], c["copy_helpers"], c["test_hooks"]) == \
        ("0", "0", "45000", "5", "0")
    assert "ignored" not in c


def test_config_buffer_truncation():
    import ctypes

    lib = ih.load_library()
    need = ctypes.c_size_t()
    small = ctypes.create_string_buffer(8)
    assert lib.iris_config(None, small, 8, ctypes.byref(need)) == 0
    assert len(small.value) == 7 and need.value > 7
    assert lib.iris_config(None, None, 0, None) == 0
