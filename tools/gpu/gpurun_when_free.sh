#!/bin/bash
# Runs one gpurun command, retrying only while the pool reports no free slot / box (exit code 3, nothing charged),
# at most N times, a few minutes apart. Any other outcome (success, refusal, a failure of the command) ends it.
# usage: tools/gpu/gpurun_when_free.sh <log> <timeout-s> <command...>
log=$1; to=$2; shift 2
for i in $(seq ${TRIES:-20}); do
  /usr/local/graft/bin/gpurun --timeout $to -- "$@" > $log 2>&1
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  # (exit 3 is always "no box or slot right now, nothing charged")
  sleep ${WAIT:-200}
done
exit 3
