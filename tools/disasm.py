"""Disassemble kernels of the built libdpi_hip.so, or of one hipcc object (gfx950).
usage: python tools/disasm.py <mangled-substring> [out] [--lib path.so|path.o]"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = "/opt/rocm/lib/llvm/bin"
args = sys.argv[1:]
lib = Path(__file__).resolve().parents[1] / "deeppicarditeration_amd" / "libdpi_hip.so"
if "--lib" in args:
    i = args.index("--lib")
    lib = Path(args[i + 1])
    del args[i:i + 2]
pat = args[0]
with tempfile.TemporaryDirectory() as d:
    fb = f"{d}/fb.bin"
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", str(lib), fb], check=True)
    data = Path(fb).read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"  # a multi-TU library carries one bundle per TU
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    out = []
    for k, st in enumerate(starts):
        part, co = f"{d}/p{k}.bin", f"{d}/c{k}.co"
        Path(part).write_bytes(data[st:starts[k + 1] if k + 1 < len(starts) else len(data)])
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
        if r.returncode:
            continue
        txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], capture_output=True,
                             text=True).stdout
        cur = None
        for line in txt.splitlines():
            if line.endswith(">:"):
                cur = pat in line
            if cur:
                out.append(line)
text = "\n".join(out)
if len(args) > 1:
    Path(args[1]).write_text(text)
else:
    print(text)
