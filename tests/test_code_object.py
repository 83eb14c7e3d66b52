"""The built library's gfx950 code objects (CPU: no GPU needed).

Register spills are a correctness hazard here, not only a cost: the GEMM and
attention kernels read LDS with inline asm and order those reads with explicit
lgkmcnt waits, and a spilled operand's reload can run before the read it
depends on has landed.  Every kernel of the library must be
spill-free, except the f32 (parity-mode) split attention backward, whose reads are
plain compiler-tracked loads.  The metadata come from the library's .hip_fatbin
section: one offload bundle per source file, each unbundled to its gfx950 code
object, whose notes carry .vgpr_spill_count per kernel."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "neurosync_trainer_lite_amd", "libnstl_hip.so")
LLVM = "/opt/rocm/lib/llvm/bin"
BUNDLER = os.path.join(LLVM, "clang-offload-bundler")
READELF = os.path.join(LLVM, "llvm-readelf")
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
# plain (compiler-tracked) LDS reads: a spill costs time, not correctness
ALLOWED = re.compile(r"attn_bwd_dq_kernelIf")


def _kernel_notes(tmp_path):
    if not os.path.exists(LIB):
        pytest.skip("libnstl_hip.so not built")
    if not (shutil.which("objcopy") and os.path.exists(BUNDLER) and os.path.exists(READELF)):
        pytest.skip("objcopy / clang-offload-bundler / llvm-readelf not available")
    fat = tmp_path / "fatbin.bin"
    subprocess.run(["objcopy", "--dump-section", ".hip_fatbin=%s" % fat, LIB], check=True, capture_output=True)
    data = fat.read_bytes()
    offs = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    assert offs, "no offload bundle in .hip_fatbin"
    kernels = {}
    for i, o in enumerate(offs):
        part = tmp_path / ("b%d.bin" % i)
        part.write_bytes(data[o:offs[i + 1] if i + 1 < len(offs) else len(data)])
        co = tmp_path / ("c%d.o" % i)
        subprocess.run([BUNDLER, "--type=o", "--unbundle", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        "--input=%s" % part, "--output=%s" % co], check=True, capture_output=True)
        notes = subprocess.run([READELF, "--notes", str(co)], check=True, capture_output=True, text=True).stdout
        # one metadata map per kernel: split at each map's first key
        for block in notes.split("  - .agpr_count:")[1:]:
            name = re.search(r"\.name:\s+(\S+)", block).group(1)
            spill = int(re.search(r"\.vgpr_spill_count:\s+(\d+)", block).group(1))
            kernels[name] = spill
    return kernels


def test_every_kernel_is_gfx950_and_spill_free(tmp_path):
    kernels = _kernel_notes(tmp_path)
    # the production kernels are all there (4-wave GEMM, its fp8 form, attention)
    for must in ("gemm4_kernel", "gemm4f8_kernel", "attn_fwd_persist_kernel", "attn_bwd_fused_kernel",
                 "ln_bwd_kernel_il", "adam_gcoef_kernel"):
        assert any(must in k for k in kernels), must
    spilling = {k: v for k, v in kernels.items() if v and not ALLOWED.search(k)}
    assert not spilling, "kernels with VGPR spills: %s" % spilling


OBJDUMP = os.path.join(LLVM, "llvm-objdump")


def test_gemm4_epilogues_have_no_compiler_vmcnt0_before_lds_reads(tmp_path):
    """The 4-wave GEMM reads its LDS with inline asm wherever an LDS-DMA may be in
    flight (stage pieces, epilogue side data, RoPE tables: DESIGN.md section 4,
    "Epilogue inputs off the vmcnt queue").  A plain LDS load there makes the
    compiler emit `s_waitcnt vmcnt(0)` in front of it: a wait for the next tile's
    stage pieces and every store before it.  Guard: no gemm4 kernel outside the
    stream-K tail form has a vmcnt(0) directly ahead of a ds_read."""
    if not os.path.exists(LIB):
        pytest.skip("libnstl_hip.so not built")
    if not (shutil.which("objcopy") and os.path.exists(BUNDLER) and os.path.exists(OBJDUMP)):
        pytest.skip("objcopy / clang-offload-bundler / llvm-objdump not available")
    fat = tmp_path / "fatbin.bin"
    subprocess.run(["objcopy", "--dump-section", ".hip_fatbin=%s" % fat, LIB], check=True, capture_output=True)
    data = fat.read_bytes()
    offs = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    checked, bad = 0, {}
    for i, o in enumerate(offs):
        part, co = tmp_path / ("d%d.bin" % i), tmp_path / ("d%d.o" % i)
        part.write_bytes(data[o:offs[i + 1] if i + 1 < len(offs) else len(data)])
        subprocess.run([BUNDLER, "--type=o", "--unbundle", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        "--input=%s" % part, "--output=%s" % co], check=True, capture_output=True)
        text = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", str(co)], check=True, capture_output=True,
                              text=True).stdout
        for block in re.split(r"\n(?=[0-9a-f]+ <)", text):
            m = re.match(r"[0-9a-f]+ <(.*)>:", block)
            # gemm4_kernel<AK, BKM, EM, GROUPED, DBG, SK, R3>: skip SK = true (..ELb1ELi<R3>E)
            if not m or "gemm4_kernel" not in m.group(1) or re.search(r"ELb1ELi[0-9]EEEv", m.group(1)):
                continue
            ins = [ln.split("//")[0].strip() for ln in block.split("\n")[1:]]
            ins = [x for x in ins if x and not x.startswith(";")]
            n = sum(1 for k in range(len(ins) - 1) if ins[k].startswith("s_waitcnt") and "vmcnt(0)" in ins[k]
                    and any(x.startswith("ds_read") for x in ins[k + 1:k + 3]))
            checked += 1
            if n:
                bad[m.group(1)] = n
    assert checked >= 10, checked
    assert not bad, bad
