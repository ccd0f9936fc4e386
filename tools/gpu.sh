#!/bin/bash
# Run a command on the MI355X box via gpurun; re-submit only on infrastructure events
# (box lost while being prepared / taken away), never on a failure of the command itself.
out=${GPU_OUT:-gpurun_out/last_call.txt}
for attempt in 1 2 3; do
  /usr/local/graft/bin/gpurun --timeout ${GPU_TIMEOUT:-900} -- "$@" > "$out" 2>&1
  rc=$?
  if grep -q "infrastructure event\|stopped responding while being prepared\|status=transient" "$out"; then
    sleep 20; continue
  fi
  break
done
tail -3 "$out"
exit $rc
