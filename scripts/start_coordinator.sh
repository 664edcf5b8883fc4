#!/bin/bash
# Start the coordinator (same env vars as the reference's scripts/start_coordinator.sh, plus
# PS_ADDRESS, which the reference's script forgot to pass -- its defect D2).
set -e
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
COORDINATOR_PORT=${COORDINATOR_PORT:-50052}
PS_ADDRESS=${PS_ADDRESS:-${PS_ADDR:-localhost:50051}}
BINARY_PATH=${BINARY_PATH:-$HERE/bin/coordinator}
LOG_FILE=${LOG_FILE:-/tmp/coordinator.log}
PID_FILE=${PID_FILE:-/tmp/coordinator.pid}
echo "starting coordinator on port $COORDINATOR_PORT (parameter server $PS_ADDRESS)" | tee -a "$LOG_FILE"
if [ "${SUPERVISE:-0}" = "1" ]; then  # restart on crash (the reference's systemd Restart=always)
  nohup "$HERE/scripts/supervise.sh" "$PID_FILE.child" "$BINARY_PATH" "0.0.0.0:$COORDINATOR_PORT" "$PS_ADDRESS" $COORDINATOR_FLAGS >> "$LOG_FILE" 2>&1 &
else
  nohup "$BINARY_PATH" "0.0.0.0:$COORDINATOR_PORT" "$PS_ADDRESS" $COORDINATOR_FLAGS >> "$LOG_FILE" 2>&1 &
fi
echo $! > "$PID_FILE"
echo "coordinator started with PID $(cat "$PID_FILE")"
