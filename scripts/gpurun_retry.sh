#!/bin/bash
# Submit one gpurun call; when the pool refuses it before anything ran
# (status=transient: no box free / backoff), wait as told and submit again,
# at most MAX_TRIES times.  A call that ran (any rc) is never repeated.
# usage: scripts/gpurun_retry.sh OUTFILE TIMEOUT 'command'
out=$1; lim=$2; cmd=$3; tries=${MAX_TRIES:-8}
for ((a = 1; a <= tries; a++)); do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$out" 2>&1
  rc=$?
  if ! grep -q "status=transient" "$out"; then exit $rc; fi
  wait_s=$(grep -o "retry in [0-9]*s" "$out" | grep -o "[0-9]*" | tail -1)
  [ -z "$wait_s" ] && wait_s=240
  echo "[retry] attempt $a transient; sleeping $((wait_s + 20))s" >> "$out.retries"
  sleep $((wait_s + 20))
done
exit $rc
