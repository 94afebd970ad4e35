#!/bin/bash
# A/B of the small-magnitude probe: the round-5 package (tools/variants/r05pkg, built from git HEAD of
# round 5, untracked) against this tree.  Usage: tools/ab_probe_small.sh <out-prefix> [case] [hows]
set -o pipefail
out=$1; case_=${2:-}; hows=${3:-homog,all}
mkdir -p gpurun_out
PYTHONPATH=tools/variants/r05pkg timeout -k 10 400 python -u -c "
import sys; sys.path.insert(0, 'tools/variants/r05pkg'); sys.argv = ['probe', '$case_', '$hows']
import deeppicarditeration_amd, oracle; assert 'r05pkg' in deeppicarditeration_amd.__file__, deeppicarditeration_amd.__file__
exec(open('tools/probe_small.py').read().replace('sys.path.insert(0, str(Path(__file__).resolve().parents[1]))', ''))
" > gpurun_out/${out}_r05.jsonl 2>&1 && \
timeout -k 10 400 python -u tools/probe_small.py "$case_" "$hows" > gpurun_out/${out}_r06.jsonl 2>&1
