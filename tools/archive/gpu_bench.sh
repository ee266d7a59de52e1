#!/bin/bash
# the default bench on the box -> gpurun_out/<tag>/bench.json (+ stderr), with a heartbeat
set -o pipefail
TAG=${1:-r04}
shift || true
mkdir -p gpurun_out/$TAG
timeout -k 10 1000 python3 -u bench.py "$@" > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err &
pid=$!
while kill -0 $pid 2>/dev/null; do sleep 30; kill -0 $pid 2>/dev/null && echo "  ... $(date +%T) bench running"; done
wait $pid
