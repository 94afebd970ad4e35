"""Build libdpi_hip.so in-tree for gfx950 (hipcc cross-compiles without a GPU)."""
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent
REPO = ROOT.parent
SRC = ROOT / "csrc" / "dpi_kernels.hip"
OUT = ROOT / "libdpi_hip.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def sources():
    return [SRC] + sorted((ROOT / "csrc").glob("*.h")) + [REPO / "include" / "dpi.h"]


def needs_build():
    if not OUT.exists():
        return True
    t = OUT.stat().st_mtime
    return any(p.stat().st_mtime > t for p in sources())


def build(force=False, verbose=True):
    if not force and not needs_build():
        return OUT
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", f"-I{REPO / 'include'}",
           "-o", str(OUT), str(SRC)]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
