#!/bin/bash
# gpurun with a wait when no GPU slot is free (exit 3: nothing ran, nothing charged).  Any other exit --
# success, a failed or killed GPU step, a refusal -- ends it at once: a GPU step is never re-run.
# usage: tools/gpurun_retry.sh <timeout-seconds> <script> [args...]   (output: the last attempt's)
t=$1; shift
for attempt in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun --timeout "$t" -- bash "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[retry] no GPU slot (attempt $attempt), waiting 240 s"
  sleep 240
done
exit 3
