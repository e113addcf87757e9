#!/bin/bash
# usage: scripts/gpurun_wait.sh OUTFILE TIMEOUT 'command'
# Waits for a GPU slot: re-issues the call only while gpurun answers 3 (no box / slot free: nothing ran, nothing
# charged).  Any other outcome -- success, a failing command, a refusal -- ends it.
out=$1; tl=$2; cmd=$3
for i in $(seq 1 60); do
  /usr/local/graft/bin/gpurun --timeout "$tl" -- "$cmd" > "$out" 2>&1; rc=$?
  [ $rc -eq 3 ] || break
  sleep 60
done
echo "__done rc=$rc tries=$i" >> "$out"
