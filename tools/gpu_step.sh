#!/bin/bash
# Run one GPU step under its own time limit; stop the whole call on a crash/timeout.
# usage: tools/gpu_step.sh SECONDS LOGFILE cmd...   (exit 0/1 pass through; others abort)
secs=$1; log=$2; shift 2
mkdir -p "$(dirname "$log")"
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
echo "[gpu_step] rc=$rc : $*" | tee -a "$log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
  echo "[gpu_step] aborting call after rc=$rc" ; exit 99
fi
exit 0
