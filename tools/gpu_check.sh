#!/bin/bash
# Run one GPU step under a time limit; stop the whole call on a fault / abort / timeout.
# usage: tools/gpu_check.sh <seconds> <logfile> <cmd...>
secs=$1; log=$2; shift 2
mkdir -p "$(dirname "$log")"
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
echo "[gpu_check] rc=$rc : $*" | tee -a "$log"
case $rc in
  0|1) exit 0 ;;   # success or ordinary test failure: keep going
  *) echo "[gpu_check] stopping: rc=$rc" ; exit $rc ;;
esac
