#!/bin/bash
# Localhost integration test: 1 coordinator + 1 parameter server + N workers as separate processes
# talking gRPC over loopback (the reference's scripts/test_local.sh topology), WITH assertions
# (the reference's script only printed logs). Exit status 0 = every check passed.
#   TOTAL_WORKERS (2) ITERATIONS (5) PS_FLAGS WORKER_FLAGS COORD_PORT PS_PORT KEEP_LOGS
set -u
HERE="$(cd "$(dirname "${BASH_SOURCE[0]}")/.." && pwd)"
TOTAL_WORKERS=${TOTAL_WORKERS:-2}
ITERATIONS=${ITERATIONS:-5}
COORD_PORT=${COORD_PORT:-50052}
PS_PORT=${PS_PORT:-50051}
CKPT_INTERVAL=${CKPT_INTERVAL:-2}
PS_FLAGS=${PS_FLAGS:-"--optimizer momentum --lr 0.05"}
WORKER_FLAGS=${WORKER_FLAGS:-"--heartbeat-s 1"}
WORK=$(mktemp -d /tmp/psd_local.XXXXXX)
PIDS=()
cleanup() {
  for p in "${PIDS[@]}"; do kill "$p" 2>/dev/null; done
  wait 2>/dev/null
  [ -z "${KEEP_LOGS:-}" ] && rm -rf "$WORK"
}
trap cleanup EXIT
fail() { echo "FAIL: $*"; for f in "$WORK"/*.log; do echo "--- $f"; tail -20 "$f"; done; exit 1; }

cd "$WORK"
"$HERE/bin/coordinator" "127.0.0.1:$COORD_PORT" "127.0.0.1:$PS_PORT" > coordinator.log 2>&1 &
PIDS+=($!)
"$HERE/bin/parameter_server" "127.0.0.1:$PS_PORT" "$TOTAL_WORKERS" "$CKPT_INTERVAL" --ckpt-dir "$WORK" \
  --coordinator "127.0.0.1:$COORD_PORT" $PS_FLAGS > ps.log 2>&1 &
PIDS+=($!)
WPIDS=()
for ((w = 0; w < TOTAL_WORKERS; w++)); do
  "$HERE/bin/worker_main" "127.0.0.1:$COORD_PORT" "$w" "$ITERATIONS" --stats-json "stats$w.json" $WORKER_FLAGS \
    > "worker$w.log" 2>&1 &
  WPIDS+=($!)
done
for p in "${WPIDS[@]}"; do wait "$p" || fail "worker pid $p exited with $?"; done

for ((w = 0; w < TOTAL_WORKERS; w++)); do
  n=$(grep -c "done=true" "worker$w.log")
  [ "$n" = "$ITERATIONS" ] || fail "worker $w: $n/$ITERATIONS iterations done"
done
python3 - "$WORK" "$TOTAL_WORKERS" "$ITERATIONS" <<'PY' || fail "stats check"
import json, sys
work, W, I = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
for w in range(W):
    s = json.load(open(f"{work}/stats{w}.json"))
    l = s["losses"]
    assert l[-1] < l[0], f"worker {w}: loss did not decrease {l}"
    assert s["version"] >= I, f"PS version {s['version']} < {I}"
print("losses decrease, PS version", s["version"], "counters", s["counters"])
PY
sleep "$((CKPT_INTERVAL > 0 ? 6 : 0))"
if [ "$CKPT_INTERVAL" -gt 0 ]; then
  ls "$WORK"/checkpoint_epoch_*.ckpt > /dev/null 2>&1 || fail "no periodic checkpoint written"
fi
echo "PASS: $TOTAL_WORKERS workers x $ITERATIONS iterations"
