"""Kernels of the built library where the compiler put `s_waitcnt vmcnt(0)` right
in front of an LDS access (CPU: no GPU needed).  With an LDS-DMA in flight the
compiler cannot separate a plain LDS load from it, so it waits for every VMEM
operation issued before: the stage pieces and the stores (DESIGN.md section 4,
"Epilogue inputs off the vmcnt queue").  Reads that may run with a DMA in flight
belong in inline asm with explicit lgkmcnt waits.
  python tools/scan_lds_waits.py [substring ...]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "neurosync_trainer_lite_amd", "libnstl_hip.so")
LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def kernels(tmp):
    fat = os.path.join(tmp, "fat.bin")
    subprocess.run(["objcopy", "--dump-section", ".hip_fatbin=%s" % fat, LIB], check=True, capture_output=True)
    data = open(fat, "rb").read()
    offs = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
    for i, o in enumerate(offs):
        part, co = os.path.join(tmp, "b%d" % i), os.path.join(tmp, "c%d.o" % i)
        open(part, "wb").write(data[o:offs[i + 1] if i + 1 < len(offs) else len(data)])
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--type=o", "--unbundle",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--input=" + part, "--output=" + co],
                       check=True, capture_output=True)
        text = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", co],
                              check=True, capture_output=True, text=True).stdout
        name, ins = None, []
        for line in text.split("\n") + ["0 <end>:"]:
            m = re.match(r"^[0-9a-f]+ <(.*)>:", line)
            if m:
                if name:
                    yield name, ins
                name, ins = m.group(1), []
                continue
            line = line.strip()
            if line and not line.startswith(";"):
                ins.append(line.split("//")[0].strip())


def main():
    want = sys.argv[1:]
    with tempfile.TemporaryDirectory() as tmp:
        found = []
        for name, ins in kernels(tmp):
            if want and not any(w in name for w in want):
                continue
            n = sum(1 for k in range(len(ins) - 1)
                    if ins[k].startswith("s_waitcnt") and "vmcnt(0)" in ins[k]
                    and any(x.startswith("ds_") for x in ins[k + 1:k + 3]))
            if n:
                found.append((n, name))
        for n, name in sorted(found, reverse=True):
            print("%3d  %s" % (n, name))


if __name__ == "__main__":
    main()
