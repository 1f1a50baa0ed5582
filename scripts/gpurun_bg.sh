#!/bin/bash
# Local helper: rebuild the in-tree extensions (so the snapshot ships fresh .so files), then run
# the given command on a GPU box via gpurun in the background, logging to $LOG. A call that got no
# box (gpurun exit 3: nothing ran, nothing charged) is re-submitted every 2 minutes, up to 30
# times; any other outcome ends the loop.
# usage: LOG=/tmp/x.log TIMEOUT=1500 scripts/gpurun_bg.sh '<command>'
set -e
cd /root/repo
timeout 900 python -m smdt_amd._build > /tmp/_build.log 2>&1 || { echo "build failed"; tail -20 /tmp/_build.log; exit 1; }
LOG=${LOG:-/tmp/gpurun.log}
(
  set +e
  for i in $(seq 1 30); do
    /usr/local/graft/bin/gpurun --timeout ${TIMEOUT:-1500} -- "$1" > "$LOG" 2>&1
    rc=$?
    echo "[gpurun_bg] attempt $i rc=$rc" >> "$LOG"
    [ $rc -ne 3 ] && break
    sleep 120
  done
) &
echo "launched -> $LOG"
