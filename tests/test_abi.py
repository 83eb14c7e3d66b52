"""The C-ABI library loads (no GPU needed) and exports every entry point
include/nstl.h declares; the ctypes binding list matches the header.

Each check runs in a child Python process.  Loading the library brings /opt/rocm's
HIP runtime into the process beside torch's own; on a machine without a GPU that
left the pytest process unstable for later tests (torch.optim's triton import
segfaulted, numpy later raised a bus error), so the library is never loaded into
the CPU suite's own process."""
import os
import re
import subprocess
import sys
import textwrap

from tests.conftest import REPO

HEADER = os.path.join(REPO, "include", "nstl.h")


def declared():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(nstl_[a-z0-9_]+)\s*\(", text)))


def run_child(body, *args):
    """Run `body` (Python source; argv[1:] = args) in a child process at the repo root."""
    code = "import sys\nsys.path.insert(0, %r)\n" % REPO + textwrap.dedent(body)
    r = subprocess.run([sys.executable, "-c", code, *args], cwd=REPO, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, "child failed (%d):\n%s\n%s" % (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    return r.stdout


def test_library_exports_header_symbols():
    names = declared()
    assert len(names) >= 20
    run_child("""
        from neurosync_trainer_lite_amd import _hip
        lib = _hip.lib()
        names = sys.argv[1:]
        missing = [n for n in names if not hasattr(lib, n)]
        assert not missing, missing
        assert sorted(_hip.EXPORTS) == names, (sorted(_hip.EXPORTS), names)
    """, *names)


def test_version_and_error_string():
    run_child("""
        import ctypes
        from neurosync_trainer_lite_amd import _hip
        lib = _hip.lib()
        assert lib.nstl_version() >= 1
        # an argument error is reported without touching the device
        a = _hip.GemmArgs()
        a.dtype = 7
        rc = lib.nstl_gemm(ctypes.byref(a), None)
        assert rc != 0
        assert b"dtype" in lib.nstl_last_error_string()
    """)


def test_features_sizes_without_device():
    run_child("""
        from neurosync_trainer_lite_amd import _hip
        # 1 s at 88.2 kHz: F120 = 1 + 88200 // 735 = 121 -> F60 = 61
        assert _hip.features_frames(88200, 88200) == 61
        assert _hip.features_workspace_bytes(88200, 88200) > 121 * 1472 * 4 * 2
    """)


def test_kernel_counters_without_device():
    """The launch counters exist, reset, and match the bindings' family list."""
    run_child("""
        from neurosync_trainer_lite_amd import _hip
        _hip.kernel_counts_reset()
        c = _hip.kernel_counts()
        assert set(c) == set(_hip.KERNEL_COUNT_NAMES) and not any(c.values())
    """)
