#!/bin/bash
# Submit one gpurun call; while the pool has no box (exit 3: nothing ran,
# nothing charged) wait and submit again, at most $TRIES times.  Any other
# outcome -- success, a failed command, a refusal -- ends it at once.
# usage: tools/gpurun_wait.sh OUTFILE TIMEOUT 'command'
out=$1 lim=$2 cmd=$3 tries=${TRIES:-8}
for ((t = 1; t <= tries; t++)); do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$out" 2>&1
  rc=$?
  if [ $rc -ne 3 ] && ! grep -q "no free box\|backing off\|stopped responding while being prepared" "$out"; then break; fi
  sleep 150
done
echo "gpurun_wait rc=$rc tries=$t" >> "$out"
