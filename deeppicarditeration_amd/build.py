"""Build libdpi_hip.so in-tree for gfx950 (hipcc cross-compiles without a GPU).

Thirteen translation units (the C-ABI / PIS / reduce TU, and per equation the k_paths family, its
TD-estimator family and the Tanh-activation twins of both) compile in parallel to objects, then link into one
shared library together with a generated one-function unit, `dpi_build_id()`, that returns the
SHA-256 of the sources and flags (`source_hash`).  A build is current when the library itself
embeds the tree's hash (not by mtime, and not by a side file that a checkout could leave behind
next to a stale library), and `_lib.load()` refuses a library whose embedded identity differs from
the tree it is loaded from.  `libdpi_hip.so.buildid` beside the library is an untracked copy of
the hash for humans."""
import hashlib
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parent
REPO = ROOT.parent
CSRC = ROOT / "csrc"
UNITS = ["dpi_kernels.hip", "dpi_paths_cha.hip", "dpi_paths_ou.hip", "dpi_paths_gbm.hip", "dpi_paths_td_cha.hip",
         "dpi_paths_td_ou.hip", "dpi_paths_td_gbm.hip", "dpi_paths_cha_tanh.hip", "dpi_paths_ou_tanh.hip",
         "dpi_paths_gbm_tanh.hip", "dpi_paths_td_cha_tanh.hip", "dpi_paths_td_ou_tanh.hip", "dpi_paths_td_gbm_tanh.hip",
         "dpi_paths_fb_cha.hip", "dpi_paths_fb_ou.hip", "dpi_paths_wide_cha.hip", "dpi_paths_wide_ou.hip",
         "dpi_paths_wide_cha_tanh.hip", "dpi_paths_wide_ou_tanh.hip", "dpi_paths_wide_gbm.hip",
         "dpi_paths_wide_gbm_tanh.hip"]
OBJ = ROOT / "build"
OUT = ROOT / "libdpi_hip.so"
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", f"-I{REPO / 'include'}"]


def sources():
    return [CSRC / u for u in UNITS] + sorted(CSRC.glob("*.h")) + [REPO / "include" / "dpi.h"]


BUILD_ID_FILE = OUT.with_name(OUT.name + ".buildid")


def source_hash():
    """SHA-256 (hex) of everything the library is compiled from: every csrc/*.hip and *.h, the
    C-ABI header, the unit list and the compiler flags."""
    h = hashlib.sha256()
    h.update(repr((UNITS, FLAGS[:-1])).encode())  # the -I path differs between checkouts
    files = sorted(CSRC.glob("*.hip")) + sorted(CSRC.glob("*.h")) + [REPO / "include" / "dpi.h"]
    for f in files:
        h.update(f.relative_to(REPO).as_posix().encode() + b"\0")
        h.update(f.read_bytes())
        h.update(b"\0")
    return h.hexdigest()


def embedded_id(lib=OUT):
    """The build id compiled into `lib` (the 64-hex string of dpi_build_id), read from the file's
    bytes without loading it; None if absent."""
    import re
    try:
        data = Path(lib).read_bytes()
    except OSError:
        return None
    hit = re.search(rb"(?<![0-9a-f])[0-9a-f]{64}(?![0-9a-f])", data)
    return hit.group(0).decode() if hit else None


def needs_build():
    if not OUT.exists():
        return True
    return source_hash().encode() not in OUT.read_bytes()


def includes(path, seen=None):
    """`path` and every file it #includes with quotes, transitively (the object's dependencies)."""
    import re
    seen = set() if seen is None else seen
    path = Path(path).resolve()
    if path in seen or not path.exists():
        return seen
    seen.add(path)
    for inc in re.findall(r'^\s*#\s*include\s+"([^"]+)"', path.read_text(), flags=re.M):
        includes(path.parent / inc, seen)
    return seen


def build(force=False, verbose=True):
    if not force and not needs_build():
        return OUT
    OBJ.mkdir(exist_ok=True)

    def compile_unit(u):
        obj = OBJ / (Path(u).stem + ".o")
        cmd = [HIPCC, *FLAGS, "-c", "-o", str(obj), str(CSRC / u)]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        return obj

    def stale(u):  # an object is rebuilt when its unit or a header it includes (transitively) is newer
        obj = OBJ / (Path(u).stem + ".o")
        newest = max(f.stat().st_mtime for f in includes(CSRC / u))
        return force or not obj.exists() or obj.stat().st_mtime < newest

    bid = source_hash()  # before compiling: a source edited during the build leaves the result stale
    todo = [u for u in UNITS if stale(u)]
    with ThreadPoolExecutor(max_workers=max(1, len(todo))) as ex:
        list(ex.map(compile_unit, todo))
    objs = [OBJ / (Path(u).stem + ".o") for u in UNITS]
    objs.append(build_id_object(bid))
    tmp = OUT.with_name(OUT.name + ".tmp")
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, OUT)  # a new inode: a process that has the old library mapped keeps it intact
    BUILD_ID_FILE.write_text(bid + "\n")
    return OUT


def build_id_object(bid, out_dir=OBJ):
    """The generated unit exporting dpi_build_id() (include/dpi.h) for hash `bid`, compiled."""
    src = out_dir / "dpi_build_id.c"
    obj = out_dir / "dpi_build_id.o"
    src.write_text('#include <stddef.h>\n#include <string.h>\n'
                   f'static const char k_id[] = "{bid}";\n'
                   'int dpi_build_id(char* buf, size_t len) {\n'
                   '  if (buf && len) { strncpy(buf, k_id, len - 1); buf[len - 1] = 0; }\n'
                   '  return (int)(sizeof(k_id) - 1);\n}\n')
    subprocess.run(["gcc", "-O2", "-fPIC", "-c", "-o", str(obj), str(src)], check=True)
    return obj


def kernel_resources(lib=OUT):
    """Per-kernel resources of the built library's gfx950 code objects (amdhsa.kernels metadata):
    a list of dicts with the demangled `name` and vgpr_count (VGPR + AGPR), agpr_count,
    vgpr_spill_count, sgpr_spill_count, private_segment_fixed_size (scratch bytes per lane),
    group_segment_fixed_size (LDS bytes), uses_dynamic_stack.  Host tools only (objcopy, the ROCm
    LLVM bundler and readelf, c++filt); no GPU."""
    import re
    import tempfile
    llvm = "/opt/rocm/lib/llvm/bin"
    notes = ""
    with tempfile.TemporaryDirectory() as d:
        fb = f"{d}/fb.bin"
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", str(lib), fb], check=True)
        data = Path(fb).read_bytes()
        magic = b"__CLANG_OFFLOAD_BUNDLE__"  # one offload bundle per translation unit
        starts = [m.start() for m in re.finditer(re.escape(magic), data)]
        for k, st in enumerate(starts):
            part, co = f"{d}/p{k}.bin", f"{d}/c{k}.co"
            Path(part).write_bytes(data[st:starts[k + 1] if k + 1 < len(starts) else len(data)])
            r = subprocess.run([f"{llvm}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                                "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], capture_output=True)
            if r.returncode == 0:
                notes += subprocess.run([f"{llvm}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                                        text=True).stdout
    out = []
    ints = ("vgpr_count", "agpr_count", "vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size",
            "group_segment_fixed_size")
    for item in re.split(r"\n\s+- \.agpr_count:", notes)[1:]:
        item = ".agpr_count:" + item
        meta = {k: re.search(r"\." + k + r":\s+(\S+)", item) for k in ints + ("name", "uses_dynamic_stack")}
        rec = {k: (int(m.group(1)) if k in ints else m.group(1)) for k, m in meta.items() if m}
        rec["mangled"] = rec["name"]
        rec["name"] = subprocess.run(["c++filt", rec["name"]], capture_output=True, text=True).stdout.strip()
        out.append(rec)
    return out


if __name__ == "__main__":
    build(force="--force" in sys.argv)
