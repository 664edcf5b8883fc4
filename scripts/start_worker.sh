#!/bin/bash
# Start one worker (env vars of the reference's start_worker.sh). WORKER_GPU pins it to one GPU
# (HIP_VISIBLE_DEVICES) and runs the model there; WORKER_FLAGS passes extra flags.
set -e
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
WORKER_ID=${WORKER_ID:-0}
COORDINATOR_ADDR=${COORDINATOR_ADDR:-""}
ITERATIONS=${ITERATIONS:-100}
WORKER_ADDR=${WORKER_ADDR:-""}
WORKER_PORT=${WORKER_PORT:-0}
CHECKPOINT_PATH=${CHECKPOINT_PATH:-""}
BINARY_PATH=${BINARY_PATH:-$HERE/bin/worker_main}
LOG_FILE=${LOG_FILE:-/tmp/worker_${WORKER_ID}.log}
PID_FILE=${PID_FILE:-/tmp/worker_${WORKER_ID}.pid}
if [ -z "$COORDINATOR_ADDR" ]; then
  echo "error: COORDINATOR_ADDR not set"
  exit 1
fi
if [ -n "$WORKER_GPU" ]; then
  export HIP_VISIBLE_DEVICES=$WORKER_GPU
  WORKER_FLAGS="--device cuda $WORKER_FLAGS"
fi
echo "starting worker $WORKER_ID connecting to coordinator $COORDINATOR_ADDR" | tee -a "$LOG_FILE"
ARGS=("$COORDINATOR_ADDR" "$WORKER_ID" "$ITERATIONS" "$WORKER_ADDR" "$WORKER_PORT")
[ -n "$CHECKPOINT_PATH" ] && ARGS+=("$CHECKPOINT_PATH")
if [ "${SUPERVISE:-0}" = "1" ]; then  # restart on crash (the reference's systemd Restart=always)
  nohup "$HERE/scripts/supervise.sh" "$PID_FILE.child" "$BINARY_PATH" "${ARGS[@]}" $WORKER_FLAGS >> "$LOG_FILE" 2>&1 &
else
  nohup "$BINARY_PATH" "${ARGS[@]}" $WORKER_FLAGS >> "$LOG_FILE" 2>&1 &
fi
echo $! > "$PID_FILE"
echo "worker $WORKER_ID started with PID $(cat "$PID_FILE")"
