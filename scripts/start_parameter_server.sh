#!/bin/bash
# Start a parameter-server shard (env vars of the reference's start_parameter_server.sh).
# PS_DEVICE=cuda:i keeps the shard in HBM; PS_FLAGS passes extra flags (--mode async --staleness 2 ...).
set -e
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
PS_PORT=${PS_PORT:-50051}
TOTAL_WORKERS=${TOTAL_WORKERS:-3}
CHECKPOINT_INTERVAL=${CHECKPOINT_INTERVAL:-10}
PS_DEVICE=${PS_DEVICE:-cpu}
BINARY_PATH=${BINARY_PATH:-$HERE/bin/parameter_server}
LOG_FILE=${LOG_FILE:-/tmp/parameter_server.log}
PID_FILE=${PID_FILE:-/tmp/parameter_server.pid}
echo "starting parameter server on port $PS_PORT with $TOTAL_WORKERS workers" | tee -a "$LOG_FILE"
if [ "${SUPERVISE:-0}" = "1" ]; then  # restart on crash (the reference's systemd Restart=always)
  nohup "$HERE/scripts/supervise.sh" "$PID_FILE.child" "$BINARY_PATH" "0.0.0.0:$PS_PORT" "$TOTAL_WORKERS" "$CHECKPOINT_INTERVAL" --device "$PS_DEVICE" $PS_FLAGS \
  --resume-latest >> "$LOG_FILE" 2>&1 &
else
  nohup "$BINARY_PATH" "0.0.0.0:$PS_PORT" "$TOTAL_WORKERS" "$CHECKPOINT_INTERVAL" --device "$PS_DEVICE" $PS_FLAGS \
  >> "$LOG_FILE" 2>&1 &
fi
echo $! > "$PID_FILE"
echo "parameter server started with PID $(cat "$PID_FILE")"
