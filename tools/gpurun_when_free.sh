#!/usr/bin/env bash
# Submit one gpurun call, re-submitting ONLY while the pool reports that no box /
# slot was available (nothing ran, nothing charged).  A call that ran -- pass or
# fail -- is never repeated.  Usage: tools/gpurun_when_free.sh LOG TIMEOUT 'CMD'
LOG=$1; TMO=$2; CMD=$3
for i in $(seq 1 ${TRIES:-12}); do
  timeout $((TMO + 900)) /usr/local/graft/bin/gpurun --timeout "$TMO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if grep -qE "no free box|slot\(s\) on this pod are busy|backing off|stopped responding while being prepared" "$LOG" \
     && grep -qE "run 0\.0s|run Nones" "$LOG"; then
    echo "attempt $i: no box (rc $rc), waiting" >> "$LOG.tries"
    sleep ${WAIT:-180}
    continue
  fi
  exit $rc
done
exit 3
