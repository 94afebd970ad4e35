"""Per-kernel VGPR/AGPR/spill/LDS of the built libdpi_hip.so (gfx950 code object metadata).
usage: python tools/kernel_resources.py [name-substring ...]"""
import re
import subprocess
import sys
import tempfile
from pathlib import Path

LLVM = "/opt/rocm/lib/llvm/bin"
lib = Path(sys.argv.pop(1)) if len(sys.argv) > 2 and sys.argv[1].endswith(".so") else Path(__file__).resolve().parents[1] / "deeppicarditeration_amd" / "libdpi_hip.so"
with tempfile.TemporaryDirectory() as d:
    fb, co = f"{d}/fb.bin", f"{d}/gfx950.co"
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", str(lib), fb], check=True)
    # a multi-TU library carries one offload bundle per translation unit: unbundle each
    data = Path(fb).read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [i for i in range(len(data)) if data.startswith(magic, i)]
    notes = ""
    for k, st in enumerate(starts):
        part = f"{d}/p{k}.bin"
        Path(part).write_bytes(data[st:starts[k + 1] if k + 1 < len(starts) else len(data)])
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}.{k}"], capture_output=True)
        if r.returncode == 0:
            notes += subprocess.run([f"{LLVM}/llvm-readelf", "--notes", f"{co}.{k}"], check=True, capture_output=True,
                                    text=True).stdout
# kernel entries in amdhsa.kernels are YAML list items starting with "  - .agpr_count"
for item in re.split(r"\n\s+- \.agpr_count:", notes)[1:]:
    item = ".agpr_count:" + item
    def g(k):
        m = re.search(r"\." + k + r":\s+(\S+)", item)
        return m.group(1) if m else "?"
    name = g("name")
    if len(sys.argv) > 1 and not any(s in name for s in sys.argv[1:]):
        continue
    dem = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    print(f"vgpr {g('vgpr_count'):>4} agpr {g('agpr_count'):>4} spill {g('vgpr_spill_count'):>3} "
          f"lds {g('group_segment_fixed_size'):>6}  {dem[:110]}")
