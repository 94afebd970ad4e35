#!/bin/bash
# Register / spill / LDS of ONE k_paths instantiation, device code only (fast iteration).
# usage: tools/unit_resources.sh "<KIND>, <H>, <L>, <ZERO>, <SPLIT>, <HESS>, <TD>"   e.g. "3, 64, 3, false, true, false, false"
set -e
args=$1
src=/tmp/unitres_$$.hip; out=/tmp/unitres_$$.co
cat > $src <<EOS
#include "$PWD/deeppicarditeration_amd/csrc/dpi_dispatch.h"
template __global__ void dpi::k_paths<$args>(dpi::EqDev, dpi::NetDev, dpi::PathArgs);
EOS
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I include --offload-device-only --no-gpu-bundle-output \
  -c $src -o $out ${EXTRA:-}
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $out | python3 -c "
import re,sys
notes=sys.stdin.read()
for item in re.split(r'\n\s+- \.agpr_count:', notes)[1:]:
    item='.agpr_count:'+item
    g=lambda k:(re.search(r'\.'+k+r':\s+(\S+)', item) or [None,'?'])[1]
    print(f\"vgpr {g('vgpr_count'):>4} agpr {g('agpr_count'):>4} spill {g('vgpr_spill_count'):>3} lds {g('group_segment_fixed_size'):>6} sgpr {g('sgpr_count')}\")
"
rm -f $src $out
