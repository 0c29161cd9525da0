#!/bin/bash
# guard.sh SECONDS LOGFILE CMD... -- run one GPU step under its own time limit; on a fault-like
# exit (timeout 124/137, abort 134, segfault 139) stop the whole GPU call (exit 99) so nothing
# else touches the GPU after a fault.  Ordinary failures (e.g. a failing test, rc 1) continue.
T=$1; LOG=$2; shift 2
mkdir -p "$(dirname "$LOG")"
timeout -k 10 "$T" "$@" > "$LOG" 2>&1
rc=$?
echo "[guard] rc=$rc: $*" | tee -a "$LOG"
case $rc in 124|134|137|139) echo "[guard] fault-like exit, stopping"; exit 99;; esac
exit 0
