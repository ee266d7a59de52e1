#!/bin/bash
# run_hb.sh <seconds> <cmd...>: run a command under its own time limit,
# printing a heartbeat line every 30 s (gpurun takes 180 s of silence for a
# hang); exits with the command's status.
LIM=$1; shift
timeout -k 10 "$LIM" "$@" &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 30; kill -0 $pid 2>/dev/null && echo "  ... $(date +%T) running"; done
wait $pid
