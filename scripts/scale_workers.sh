#!/bin/bash
# Elastic scaling: scale_workers.sh up N | down N   (reference: scripts/scale_workers.sh)
# The reference resized the Terraform worker pool and then *restarted the parameter server* with
# the new TOTAL_WORKERS, losing its in-memory state. Here the PS follows the coordinator's live
# membership (it was started with --coordinator), so nothing restarts:
#   up N   starts workers CURRENT..N-1; they register, the barrier grows, and each joiner starts at
#          the oldest iteration the PS has not aggregated (no duplicate or lost updates)
#   down N sends SIGTERM to workers N..CURRENT-1; they deregister and the barrier shrinks at once
#          (a killed worker is dropped after the heartbeat expiry instead)
# Env: CLUSTER_DIR (/tmp/psd_cluster) ITERATIONS (100) WORKER_FLAGS NUM_GPUS
set -e
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
CLUSTER_DIR=${CLUSTER_DIR:-/tmp/psd_cluster}
ITERATIONS=${ITERATIONS:-100}
CMD=$1
N=$2
if [ -z "$CMD" ] || [ -z "$N" ]; then
  echo "usage: $0 up|down N"
  exit 1
fi
CUR=$(cat "$CLUSTER_DIR/worker_count" 2>/dev/null || echo 0)
COORD=$(cat "$CLUSTER_DIR/coordinator_address")
# collective (MODE=collective deploy): joiners run with the deploy's elastic flags; the running world
# absorbs them at its next membership check, and leavers hand their PS shards over before exiting
[ -f "$CLUSTER_DIR/worker_flags" ] && WORKER_FLAGS="$(cat "$CLUSTER_DIR/worker_flags" | sed 's/--min-workers [0-9]*//') $WORKER_FLAGS"
NUM_GPUS=${NUM_GPUS:-$(python3 -c "import torch;print(torch.cuda.device_count())" 2>/dev/null || echo 0)}
case "$CMD" in
  up)
    [ "$N" -le "$CUR" ] && { echo "already $CUR workers"; exit 0; }
    for ((i = CUR; i < N; i++)); do
      GPU=""
      [ "$NUM_GPUS" -gt 0 ] 2>/dev/null && GPU=$((i % NUM_GPUS))
      WORKER_ID=$i COORDINATOR_ADDR=$COORD ITERATIONS=$ITERATIONS WORKER_GPU=$GPU WORKER_FLAGS="$WORKER_FLAGS" \
        LOG_FILE=$CLUSTER_DIR/worker_$i.log PID_FILE=$CLUSTER_DIR/worker_$i.pid bash "$HERE/scripts/start_worker.sh"
    done
    ;;
  down)
    if [ "$N" -lt 1 ]; then echo "minimum 1 worker"; exit 1; fi
    [ "$N" -ge "$CUR" ] && { echo "already $CUR workers"; exit 0; }
    for ((i = N; i < CUR; i++)); do
      P=$(cat "$CLUSTER_DIR/worker_$i.pid" 2>/dev/null || true)
      if [ -n "$P" ] && kill -0 "$P" 2>/dev/null; then
        kill -TERM "$P"
        echo "stopped worker $i (pid $P)"
      fi
    done
    ;;
  *)
    echo "usage: $0 up|down N"
    exit 1
    ;;
esac
echo "$N" > "$CLUSTER_DIR/worker_count"
echo "scaled $CMD from $CUR to $N workers"
