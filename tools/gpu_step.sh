#!/usr/bin/env bash
# Run one GPU step under a time limit; stop the whole call on crash/timeout
# (exit codes other than 0/1 = abort, segfault, fault or timeout).
# usage: tools/gpu_step.sh SECONDS LOGFILE cmd...
secs=$1; log=$2; shift 2
mkdir -p "$(dirname "$log")"
timeout -k 10 "$secs" "$@" > "$log" 2>&1
rc=$?
echo "[gpu_step] rc=$rc cmd=$*" >> "$log"
tail -5 "$log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "[gpu_step] fatal rc=$rc, stopping"; exit $rc; fi
exit 0
