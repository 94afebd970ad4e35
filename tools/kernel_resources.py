"""Per-kernel VGPR/AGPR/spill/scratch/LDS of the built libdpi_hip.so (gfx950 code object metadata).
usage: python tools/kernel_resources.py [lib.so] [name-substring ...]"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from deeppicarditeration_amd.build import OUT, kernel_resources  # noqa: E402

lib = Path(sys.argv.pop(1)) if len(sys.argv) > 1 and sys.argv[1].endswith((".so", ".o")) else OUT
for k in kernel_resources(lib):
    if len(sys.argv) > 1 and not any(s in k["name"] for s in sys.argv[1:]):
        continue
    print(f"vgpr {k['vgpr_count']:>4} agpr {k['agpr_count']:>4} spill {k['vgpr_spill_count']:>3} "
          f"scratch {k['private_segment_fixed_size']:>4} lds {k['group_segment_fixed_size']:>6}  {k['name'][:110]}")
