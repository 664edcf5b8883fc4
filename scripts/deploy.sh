#!/bin/bash
# Bring up a cluster: coordinator + parameter server + N workers, then print the addresses.
# The reference provisioned AWS EC2 with Terraform and copied binaries over ssh
# (scripts/deploy.sh, terraform/); on an MI355X node the "provision" step is GPU pinning:
#   HOSTFILE unset  -> everything on localhost, worker i pinned to GPU (i % NUM_GPUS) when GPUs exist
#   HOSTFILE=path   -> lines "host [gpu_count]"; the first host runs coordinator + PS, workers are
#                      spread round-robin over the hosts with ssh (REMOTE_DIR must hold this repo)
#   MODE=collective -> no PS process: workers run with --elastic, the PS shards live in their GPUs
#                      (RCCL data plane) and scale_workers.sh up|down resizes the world mid-run
# Env: WORKER_COUNT (3) ITERATIONS (100) COORDINATOR_PORT (50052) PS_PORT (50051)
#      CHECKPOINT_INTERVAL (10) PS_FLAGS WORKER_FLAGS CLUSTER_DIR (/tmp/psd_cluster) SSH_USER KEY_FILE
set -e
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
WORKER_COUNT=${WORKER_COUNT:-3}
ITERATIONS=${ITERATIONS:-100}
COORDINATOR_PORT=${COORDINATOR_PORT:-50052}
PS_PORT=${PS_PORT:-50051}
CHECKPOINT_INTERVAL=${CHECKPOINT_INTERVAL:-10}
CLUSTER_DIR=${CLUSTER_DIR:-/tmp/psd_cluster}
REMOTE_DIR=${REMOTE_DIR:-$HERE}
mkdir -p "$CLUSTER_DIR"

if [ -n "$HOSTFILE" ]; then
  mapfile -t HOSTS < <(grep -v '^\s*#' "$HOSTFILE" | awk 'NF{print $1}')
else
  HOSTS=(localhost)
fi
HEAD=${HOSTS[0]}
NUM_GPUS=${NUM_GPUS:-$(python3 -c "import torch;print(torch.cuda.device_count())" 2>/dev/null || echo 0)}
SSH="ssh -o StrictHostKeyChecking=no ${KEY_FILE:+-i $KEY_FILE} ${SSH_USER:+-l $SSH_USER}"

run_on() {  # host, command
  if [ "$1" = "localhost" ] || [ "$1" = "127.0.0.1" ]; then bash -c "$2"; else $SSH "$1" "cd $REMOTE_DIR && $2"; fi
}

COORD_HOST=$([ "$HEAD" = "localhost" ] && echo 127.0.0.1 || echo "$HEAD")
echo "coordinator: $COORD_HOST:$COORDINATOR_PORT  parameter server: $COORD_HOST:$PS_PORT  workers: $WORKER_COUNT"
run_on "$HEAD" "COORDINATOR_PORT=$COORDINATOR_PORT PS_ADDRESS=$COORD_HOST:$PS_PORT LOG_FILE=$CLUSTER_DIR/coordinator.log \
  PID_FILE=$CLUSTER_DIR/coordinator.pid bash scripts/start_coordinator.sh"
sleep 2
if [ "$MODE" = "collective" ]; then
  WORKER_FLAGS="--elastic --min-workers $WORKER_COUNT $WORKER_FLAGS"
  echo "$WORKER_FLAGS" > "$CLUSTER_DIR/worker_flags"
else
rm -f "$CLUSTER_DIR/worker_flags"
run_on "$HEAD" "PS_PORT=$PS_PORT TOTAL_WORKERS=$WORKER_COUNT CHECKPOINT_INTERVAL=$CHECKPOINT_INTERVAL \
  PS_FLAGS='--coordinator $COORD_HOST:$COORDINATOR_PORT --ckpt-dir $CLUSTER_DIR $PS_FLAGS' \
  LOG_FILE=$CLUSTER_DIR/parameter_server.log PID_FILE=$CLUSTER_DIR/parameter_server.pid \
  bash scripts/start_parameter_server.sh"
sleep 2
fi
for ((i = 0; i < WORKER_COUNT; i++)); do
  H=${HOSTS[$((i % ${#HOSTS[@]}))]}
  GPU=""
  [ "$NUM_GPUS" -gt 0 ] 2>/dev/null && GPU=$((i % NUM_GPUS))
  run_on "$H" "WORKER_ID=$i COORDINATOR_ADDR=$COORD_HOST:$COORDINATOR_PORT ITERATIONS=$ITERATIONS WORKER_GPU=$GPU \
    WORKER_FLAGS='$WORKER_FLAGS' LOG_FILE=$CLUSTER_DIR/worker_$i.log PID_FILE=$CLUSTER_DIR/worker_$i.pid \
    bash scripts/start_worker.sh"
done
echo "$WORKER_COUNT" > "$CLUSTER_DIR/worker_count"
echo "$COORD_HOST:$COORDINATOR_PORT" > "$CLUSTER_DIR/coordinator_address"
echo "cluster up; logs and pid files in $CLUSTER_DIR"
