#!/bin/bash
# gpurun with a wait when no GPU slot or box is free (gpurun's own "status=transient": nothing ran,
# nothing charged).  Anything else -- success, a failed or killed GPU step, the command's own exit code,
# a refusal -- ends it at once: a GPU step is never re-run.
# usage: tools/gpurun_retry.sh <timeout-seconds> <script> [args...]
t=$1; shift
log=$(mktemp /tmp/gpurun_retry.XXXXXX)
for attempt in $(seq 1 ${GPURUN_ATTEMPTS:-20}); do
  /usr/local/graft/bin/gpurun --timeout "$t" -- bash "$@" 2>&1 | tee "$log"
  rc=${PIPESTATUS[0]}
  if [ $rc -eq 3 ] && grep -q "status=transient" "$log"; then
    echo "[retry] no GPU slot (attempt $attempt), waiting 240 s"
    sleep 240
    continue
  fi
  rm -f "$log"
  exit $rc
done
rm -f "$log"
exit 3
