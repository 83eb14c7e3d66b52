"""The C-ABI library loads (no GPU needed) and exports every entry point
include/nstl.h declares; the ctypes binding list matches the header."""
import ctypes
import os
import re

from tests.conftest import REPO

HEADER = os.path.join(REPO, "include", "nstl.h")


def declared():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(nstl_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_header_symbols():
    from neurosync_trainer_lite_amd import _hip
    lib = _hip.lib()
    names = declared()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert sorted(_hip.EXPORTS) == names


def test_version_and_error_string():
    from neurosync_trainer_lite_amd import _hip
    lib = _hip.lib()
    assert lib.nstl_version() >= 1
    # an argument error is reported without touching the device
    a = _hip.GemmArgs()
    a.dtype = 7
    rc = lib.nstl_gemm(ctypes.byref(a), None)
    assert rc != 0
    assert b"dtype" in lib.nstl_last_error_string()


def test_features_sizes_without_device():
    from neurosync_trainer_lite_amd import _hip
    # 1 s at 88.2 kHz: F120 = 1 + 88200 // 735 = 121 -> F60 = 61
    assert _hip.features_frames(88200, 88200) == 61
    assert _hip.features_workspace_bytes(88200, 88200) > 121 * 1472 * 4 * 2


def test_kernel_counters_without_device():
    """The launch counters exist, reset, and match the bindings' family list."""
    from neurosync_trainer_lite_amd import _hip
    _hip.kernel_counts_reset()
    c = _hip.kernel_counts()
    assert set(c) == set(_hip.KERNEL_COUNT_NAMES) and not any(c.values())
