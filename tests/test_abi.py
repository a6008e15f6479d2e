"""CPU: the C-ABI library loads and exports every entry point of include/mox.h."""
import ctypes
import os
import re

import pytest

from conftest import ROOT
import mox


def header_functions():
    src = open(os.path.join(ROOT, "include", "mox.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mox_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_drop_in_surface():
    fns = header_functions()
    for f in ["mox_engine_create", "mox_count", "mox_count_file", "mox_get_stats", "mox_table_free",
              "mox_engine_destroy", "mox_last_error", "mox_run_device", "mox_run_range", "mox_exchange",
              "mox_write_final_result", "mox_print_top_words"]:
        assert f in fns


def test_library_exports_every_declared_symbol():
    L = ctypes.CDLL(mox.LIB_PATH)
    missing = [f for f in header_functions() if not hasattr(L, f)]
    assert not missing, missing


def test_abi_version():
    assert mox.lib().mox_abi_version() == 4


def test_no_cpu_fallback_without_gpu():
    # In a container without a GPU the engine must refuse, not silently compute on the CPU.
    if os.path.exists("/dev/kfd") and os.environ.get("HIP_VISIBLE_DEVICES", "0") != "":
        pytest.skip("a GPU may be present")
    with pytest.raises(mox.MoxError):
        mox.Engine()


def test_cli_built():
    assert os.access(os.path.join(ROOT, "map-oxidize_amd", "mox", "meduce-gpu"), os.X_OK)
