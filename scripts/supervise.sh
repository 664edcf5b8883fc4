#!/bin/bash
# Process supervision for the three roles -- the equivalent of the reference's systemd units with
# Restart=always (terraform/user_data.sh:35-80, written but never enabled there).
#   supervise.sh <pidfile-of-child> <command...>
# Restarts the command whenever it exits non-zero (or is killed), with exponential backoff
# (1 s .. 30 s) and at most MAX_RESTARTS (default 20) restarts; a clean exit (0) or SIGTERM to the
# supervisor ends supervision (SIGTERM is forwarded to the child). A restarted parameter server
# should run with --resume-latest so it comes back with its last checkpoint.
CHILD_PID_FILE=$1; shift
MAX_RESTARTS=${MAX_RESTARTS:-20}
restarts=0
backoff=1
stop=0
child=0
trap 'stop=1; [ $child -gt 0 ] && kill -TERM $child 2>/dev/null' TERM INT
while :; do
  "$@" &
  child=$!
  echo $child > "$CHILD_PID_FILE"
  wait $child
  rc=$?
  [ $stop -eq 1 ] && exit 0
  if [ $rc -eq 0 ]; then
    echo "supervise: '$1' exited cleanly" >&2
    exit 0
  fi
  restarts=$((restarts + 1))
  if [ $restarts -gt "$MAX_RESTARTS" ]; then
    echo "supervise: '$1' failed $restarts times, giving up (rc=$rc)" >&2
    exit $rc
  fi
  echo "supervise: '$1' exited with rc=$rc; restart $restarts in ${backoff}s" >&2
  sleep $backoff
  backoff=$((backoff * 2 > 30 ? 30 : backoff * 2))
done
