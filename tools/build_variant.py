"""Build a variant libdpi_hip.so for same-box A/B runs: dpi_kernels.hip (or the translation units
named by --units a.hip,b.hip) recompiled with extra defines, linked with the product's other
objects.  usage: python tools/build_variant.py NAME [--units U,..] -DX=Y ...
-> tools/variants/libdpi_NAME.so (select it with DPI_HIP_LIB=...)."""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
from deeppicarditeration_amd import build as B  # noqa: E402

name, defs = sys.argv[1], sys.argv[2:]
units = ["dpi_kernels.hip"]
if defs and defs[0] == "--units":
    units, defs = defs[1].split(","), defs[2:]
B.build()
out_dir = ROOT / "tools" / "variants"
out_dir.mkdir(exist_ok=True)
objs = []
for u in units:
    obj = out_dir / f"{Path(u).stem}_{name}.o"
    subprocess.run([B.HIPCC, *B.FLAGS, *defs, "-c", "-o", str(obj), str(B.CSRC / u)], check=True)
    objs.append(obj)
objs += [B.OBJ / (Path(u).stem + ".o") for u in B.UNITS if u not in units] + [B.OBJ / "dpi_build_id.o"]
so = out_dir / f"libdpi_{name}.so"
subprocess.run([B.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(so), *map(str, objs)], check=True)
print(so)
