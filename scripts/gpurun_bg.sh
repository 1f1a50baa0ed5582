#!/bin/bash
# Local helper: rebuild the in-tree extensions (so the snapshot ships fresh .so files), then run
# the given command on a GPU box via gpurun in the background, logging to $LOG.
# usage: LOG=/tmp/x.log TIMEOUT=1500 scripts/gpurun_bg.sh '<command>'
set -e
cd /root/repo
timeout 900 python -m smdt_amd._build > /tmp/_build.log 2>&1 || { echo "build failed"; tail -20 /tmp/_build.log; exit 1; }
LOG=${LOG:-/tmp/gpurun.log}
(/usr/local/graft/bin/gpurun --timeout ${TIMEOUT:-1500} -- "$1" > "$LOG" 2>&1 &)
echo "launched -> $LOG"
