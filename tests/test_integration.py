"""Localhost multi-process integration (the reference's scripts/test_local.sh topology, with
assertions): coordinator + parameter server + workers as separate processes over gRPC; sync and
async SGD, worker failure with heartbeat expiry, checkpoint + resume."""
import os
import socket
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin")
pytestmark = pytest.mark.slow


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env(**kw):
    e = dict(os.environ)
    e["PYTHONPATH"] = ROOT + os.pathsep + e.get("PYTHONPATH", "")
    e.update({k: str(v) for k, v in kw.items()})
    return e


class Cluster:
    def __init__(self, tmp, workers, ps_args=(), coord_args=(), ckpt_interval=0):
        self.tmp = str(tmp)
        self.cp, self.pp = free_port(), free_port()
        self.procs = []
        self.coord = self._spawn("coordinator.log", [f"{BIN}/coordinator", f"127.0.0.1:{self.cp}",
                                                     f"127.0.0.1:{self.pp}", *coord_args])
        self.start_ps(workers, ps_args, ckpt_interval)

    def start_ps(self, workers, ps_args=(), ckpt_interval=0):
        self.ps = self._spawn("ps.log", [f"{BIN}/parameter_server", f"127.0.0.1:{self.pp}", str(workers),
                                         str(ckpt_interval), "--ckpt-dir", self.tmp,
                                         "--coordinator", f"127.0.0.1:{self.cp}", *ps_args])

    def _spawn(self, log, argv, env=None):
        f = open(os.path.join(self.tmp, log), "w")
        p = subprocess.Popen(argv, stdout=f, stderr=subprocess.STDOUT, env=env or _env(), cwd=self.tmp)
        self.procs.append(p)
        return p

    def worker(self, wid, iters, *args, env=None, log=None):
        return self._spawn(log or f"worker{wid}.log", [f"{BIN}/worker_main", f"127.0.0.1:{self.cp}", str(wid), str(iters),
                                                "--heartbeat-s", "0.5", *args], env)

    def log(self, name):
        with open(os.path.join(self.tmp, name)) as f:
            return f.read()

    def stop(self):
        for p in self.procs:
            if p.poll() is None:
                p.kill()
        for p in self.procs:
            p.wait(timeout=10)


@pytest.fixture
def cluster_factory(tmp_path):
    made = []

    def make(*a, **kw):
        c = Cluster(tmp_path, *a, **kw)
        made.append(c)
        return c

    yield make
    for c in made:
        c.stop()


def _done_lines(text):
    return [ln for ln in text.splitlines() if " iter " in ln and "done=" in ln]


@pytest.mark.parametrize("mode", ["sync", "async"])
def test_test_local_script(mode):
    env = _env(COORD_PORT=free_port(), PS_PORT=free_port(), TOTAL_WORKERS=2, ITERATIONS=4)
    if mode == "async":
        env["PS_FLAGS"] = "--mode async --staleness 1 --optimizer momentum --lr 0.05"
        env["WORKER_FLAGS"] = "--mode async --heartbeat-s 1"
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "test_local.sh")], env=env, capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS" in r.stdout


def test_worker_death_shrinks_barrier(cluster_factory):
    c = cluster_factory(3, coord_args=("--expiry-s", "2", "--sweep-s", "0.5"),
                        ps_args=("--optimizer", "momentum", "--lr", "0.05"))
    w0 = c.worker(0, 6)
    w1 = c.worker(1, 6)
    w2 = c.worker(2, 6, env=_env(PSD_FAULT="exit_after_push=2"))
    assert w2.wait(timeout=60) == 3  # fault injection exit code
    assert w0.wait(timeout=120) == 0, c.log("worker0.log")
    assert w1.wait(timeout=120) == 0, c.log("worker1.log")
    for log in ("worker0.log", "worker1.log"):
        lines = _done_lines(c.log(log))
        assert len(lines) == 6 and all("done=true" in ln for ln in lines), c.log(log)
    assert "expired workers [2]" in c.log("coordinator.log") or "worker 2 left" in c.log("coordinator.log")
    assert "live workers -> barrier size" in c.log("ps.log")


def test_checkpoint_and_resume(cluster_factory):
    c = cluster_factory(1, ckpt_interval=2, ps_args=("--optimizer", "momentum", "--lr", "0.05"))
    w = c.worker(0, 5)
    assert w.wait(timeout=90) == 0, c.log("worker0.log")
    deadline = time.time() + 15
    ck = os.path.join(c.tmp, "checkpoint_epoch_2.ckpt")
    while not (os.path.exists(ck) and os.path.exists(ck + ".state")) and time.time() < deadline:
        time.sleep(0.2)
    assert os.path.exists(ck) and os.path.exists(ck + ".state"), os.listdir(c.tmp)
    first = _done_lines(c.log("worker0.log"))
    # restart the PS from scratch and resume a worker from the checkpoint
    c.ps.kill()
    c.ps.wait()
    c.start_ps(1, ("--optimizer", "momentum", "--lr", "0.05"))
    w = c.worker(0, 2, "", "0", ck, log="resumed.log")  # argv: ... worker_addr worker_port checkpoint_path
    assert w.wait(timeout=90) == 0, c.log("resumed.log")
    txt = c.log("resumed.log")
    assert "resuming at iteration" in txt
    resumed = _done_lines(txt)
    it0 = int(resumed[0].split(" iter ")[1].split()[0])
    assert it0 >= 4, txt  # continues after the checkpointed iteration, not from 0 (reference D11)
    loss_first = float(first[0].split("loss=")[1].split()[0])
    loss_resumed = float(resumed[0].split("loss=")[1].split()[0])
    assert loss_resumed < loss_first


if __name__ == "__main__":
    sys.exit(pytest.main([__file__, "-q"]))


def test_supervise_restarts_until_clean_exit(tmp_path):
    """scripts/supervise.sh (Restart=always equivalent): a command that crashes twice is restarted
    with backoff and supervision ends at its first clean exit."""
    cnt = tmp_path / "count"
    cmd = (f"n=$(cat {cnt} 2>/dev/null || echo 0); echo $((n+1)) > {cnt}; "
           f"[ $n -ge 2 ] && exit 0 || kill -9 $$")
    r = subprocess.run([os.path.join(ROOT, "scripts", "supervise.sh"), str(tmp_path / "child.pid"), "bash", "-c", cmd],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert cnt.read_text().strip() == "3"
    assert r.stderr.count("restart") == 2 and "exited cleanly" in r.stderr


def test_supervised_parameter_server_resumes_after_sigkill(tmp_path):
    """SIGKILL the supervised PS after it checkpointed: the supervisor restarts it with
    --resume-latest and it serves the checkpointed iteration again (the reference's restart lost
    its in-memory parameters, scripts/scale_workers.sh:137-144)."""
    from parameter_server_distributed_amd.rpc import schema, service

    pp = free_port()
    env = _env(PS_PORT=pp, TOTAL_WORKERS=1, CHECKPOINT_INTERVAL=2, SUPERVISE=1,
               PS_FLAGS=f"--ckpt-dir {tmp_path} --optimizer momentum --lr 0.05",
               LOG_FILE=str(tmp_path / "ps.log"), PID_FILE=str(tmp_path / "ps.pid"))
    subprocess.run(["bash", os.path.join(ROOT, "scripts", "start_parameter_server.sh")], env=env, check=True, timeout=30)
    sup = int((tmp_path / "ps.pid").read_text())
    try:
        cp = free_port()
        coord = subprocess.Popen([f"{BIN}/coordinator", f"127.0.0.1:{cp}", f"127.0.0.1:{pp}"], env=_env(),
                                 stdout=open(tmp_path / "coord.log", "w"), stderr=subprocess.STDOUT)
        w = subprocess.Popen([f"{BIN}/worker_main", f"127.0.0.1:{cp}", "0", "6", "--heartbeat-s", "0.5"], env=_env(),
                             stdout=open(tmp_path / "w.log", "w"), stderr=subprocess.STDOUT, cwd=str(tmp_path))
        assert w.wait(timeout=120) == 0, (tmp_path / "w.log").read_text()[-2000:]
        ck = tmp_path / "checkpoint_epoch_2.ckpt"
        t0 = time.time()
        while not (ck.exists() and (tmp_path / "checkpoint_epoch_2.ckpt.state").exists()) and time.time() - t0 < 20:
            time.sleep(0.2)
        assert ck.exists(), os.listdir(tmp_path)
        child = int((tmp_path / "ps.pid.child").read_text())
        os.kill(child, 9)
        t0 = time.time()
        while "resumed from" not in (tmp_path / "ps.log").read_text() and time.time() - t0 < 60:
            time.sleep(0.3)
        assert "resumed from" in (tmp_path / "ps.log").read_text(), (tmp_path / "ps.log").read_text()[-3000:]
        stub = service.Stub(f"127.0.0.1:{pp}", schema.parameter_server, timeout=10.0)
        t0 = time.time()
        while True:
            try:
                st = stub.GetStats(schema.parameter_server.SyncStatusRequest())
                break
            except Exception:  # noqa: BLE001 -- the restarted server may still be binding
                if time.time() - t0 > 30:
                    raise
                time.sleep(0.3)
        assert st.current_iteration >= 3, st
        coord.kill()
    finally:
        os.kill(sup, 15)
