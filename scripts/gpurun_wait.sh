#!/bin/bash
# usage: scripts/gpurun_wait.sh OUTFILE TIMEOUT 'command'
# Waits for a GPU slot: re-issues the call only while gpurun reports that nothing ran (exit 3: no box / slot free, or
# a "transient" verdict with no run time: the pool could not create a box; nothing charged).  Any other outcome --
# success, a failing command, a refusal -- ends it.
out=$1; tl=$2; cmd=$3
for i in $(seq 1 60); do
  /usr/local/graft/bin/gpurun --timeout "$tl" -- "$cmd" > "$out" 2>&1; rc=$?
  if [ $rc -ne 3 ]; then
    python3 - "$(dirname "$0")/../gpurun_out/.last_call.json" << 'PY' || break
import json, sys
d = json.load(open(sys.argv[1]))
sys.exit(0 if d.get("status") == "transient" and not d.get("run_s") else 1)
PY
  fi
  sleep 60
done
echo "__done rc=$rc tries=$i" >> "$out"
