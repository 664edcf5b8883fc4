"""Elastic join/leave through the ops scripts (reference: scripts/deploy.sh + scripts/scale_workers.sh):
deploy 2 workers, scale up to 3 mid-run (the joiner starts at the PS's current iteration), scale
down to 1 (leavers deregister; the barrier shrinks) -- the parameter server is never restarted."""
import os
import re
import signal
import socket
import subprocess
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.slow


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _read(p):
    try:
        with open(p) as f:
            return f.read()
    except FileNotFoundError:
        return ""


def _done(txt):
    return [int(m) for m in re.findall(r"iter (\d+) done=true", txt)]


def test_deploy_scale_up_down(tmp_path):
    cd = str(tmp_path / "cluster")
    env = dict(os.environ, CLUSTER_DIR=cd, WORKER_COUNT="2", ITERATIONS="80", NUM_GPUS="0",
               COORDINATOR_PORT=str(_port()), PS_PORT=str(_port()), CHECKPOINT_INTERVAL="0",
               PS_FLAGS="--optimizer momentum --lr 0.05", WORKER_FLAGS="--heartbeat-s 0.5 --batch 32",
               PSD_FAULT="push_delay_ms=40", PYTHONPATH=ROOT)
    try:
        subprocess.run(["bash", f"{ROOT}/scripts/deploy.sh"], env=env, check=True, timeout=60, capture_output=True)
        t0 = time.time()
        while max(_done(_read(f"{cd}/worker_0.log")) or [0]) < 5 and time.time() - t0 < 60:
            time.sleep(0.2)
        r = subprocess.run(["bash", f"{ROOT}/scripts/scale_workers.sh", "up", "3"], env=env, capture_output=True,
                           text=True, timeout=60)
        assert r.returncode == 0, r.stdout + r.stderr
        t0 = time.time()
        while not _done(_read(f"{cd}/worker_2.log")) and time.time() - t0 < 60:
            time.sleep(0.2)
        joined = _read(f"{cd}/worker_2.log")
        m = re.search(r"starting at iteration (\d+)", joined)
        assert m and int(m.group(1)) > 0, joined
        t0 = time.time()  # the PS polls membership every second: wait for the barrier to grow to 3
        while "3 live workers" not in _read(f"{cd}/parameter_server.log") and time.time() - t0 < 30:
            time.sleep(0.2)
        assert "3 live workers" in _read(f"{cd}/parameter_server.log")
        r = subprocess.run(["bash", f"{ROOT}/scripts/scale_workers.sh", "down", "1"], env=env, capture_output=True,
                           text=True, timeout=60)
        assert r.returncode == 0, r.stdout + r.stderr
        # worker 0 runs to completion on its own once the others have left
        pid0 = int(_read(f"{cd}/worker_0.pid"))
        t0 = time.time()
        while time.time() - t0 < 120:
            try:
                os.kill(pid0, 0)
            except ProcessLookupError:
                break
            time.sleep(0.3)
        w0 = _read(f"{cd}/worker_0.log")
        assert "finished 80 iterations" in w0, w0[-2000:]
        assert "done=false" not in w0, w0[-2000:]
        ps = _read(f"{cd}/parameter_server.log")
        assert ps.count("live workers -> barrier size") >= 2, ps
        assert "leaving (signal 15)" in _read(f"{cd}/worker_1.log")
    finally:
        for name in ("worker_0", "worker_1", "worker_2", "parameter_server", "coordinator"):
            p = _read(f"{cd}/{name}.pid").strip()
            if p:
                try:
                    os.kill(int(p), signal.SIGKILL)
                except (ProcessLookupError, ValueError):
                    pass
