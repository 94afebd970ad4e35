"""Disassemble one kernel of the built libdpi_hip.so (gfx950).  usage: python tools/disasm.py <mangled-substring> [out]"""
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = "/opt/rocm/lib/llvm/bin"
lib = Path(__file__).resolve().parents[1] / "deeppicarditeration_amd" / "libdpi_hip.so"
pat = sys.argv[1]
with tempfile.TemporaryDirectory() as d:
    fb, co = f"{d}/fb.bin", f"{d}/gfx950.co"
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", str(lib), fb], check=True)
    # a multi-TU library carries one bundle per TU: unbundle each
    data = Path(fb).read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [i for i in range(len(data)) if data.startswith(magic, i)]
    out = []
    for k, st in enumerate(starts):
        end = starts[k + 1] if k + 1 < len(starts) else len(data)
        part = f"{d}/p{k}.bin"
        Path(part).write_bytes(data[st:end])
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}.{k}"], capture_output=True)
        if r.returncode:
            continue
        txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", f"{co}.{k}"],
                             capture_output=True, text=True).stdout
        cur = None
        for line in txt.splitlines():
            if line.endswith(">:"):
                cur = pat in line
            if cur:
                out.append(line)
text = "\n".join(out)
if len(sys.argv) > 2:
    Path(sys.argv[2]).write_text(text)
else:
    print(text)
