"""Elastic join/leave for the collective (RCCL/xGMI) data plane, mid-run, without a restart.

BASELINE.json config 5 ("... 8 PS shards + 8 workers, scale_workers.sh elastic join/leave
mid-epoch") on the GPU data plane. The reference's only elasticity was an ops-level restart of the
parameter server with a new TOTAL_WORKERS (scripts/scale_workers.sh:137-144,180-186), which lost
its in-memory parameters; membership lived in the coordinator (src/coordinator.cpp:7-67) and was
never told to the PS.

Here every worker process is one rank of a collective world built per *generation*:

* Membership is the coordinator's live set (RegisterWorker / Deregister / heartbeat expiry bump
  its membership epoch; each rank's heartbeat thread sees the epoch).
* Rendezvous is a TCPStore hosted by the coordinator process (``--store-port``), so it outlives
  any worker. Generation g's plan (members in rank order, global step, shard count) is a JSON key;
  its process group is built on ``PrefixStore("psd/elastic/g<g>")``.
* Every ``check_every`` steps all ranks all-reduce one small vector (a "leaving" flag per rank +
  "membership changed" from rank 0) -- the same step on every rank, so they agree.
* On a change, at that step boundary: in-flight bounded-staleness gradients are applied
  (``CollectivePS.drain``), the fp32 masters + optimizer state of all PS shards are gathered to the
  leader (lowest surviving rank) in a layout-independent order (``canonical_state``), the leader
  publishes the next plan, the old group is destroyed and leavers exit; survivors and joiners build
  the new group, re-shard the state for the new world (``load_canonical_state``: new owners keep
  their slices, every rank publishes the weights) and continue at the same global step. No update
  is lost or applied twice.

A joiner registers with the coordinator (which bumps the epoch) and waits for the first plan that
lists it. A graceful leaver (SIGTERM from ``scale_workers.sh down``) keeps training until the next
check, hands its shards over and exits 0.

Crash recovery (a rank dies without handing over -- SIGKILL, OOM, a lost node): its PS shards are
gone, so the job restarts from the last *canonical checkpoint* (every ``checkpoint_every`` steps
rank 0 writes the drained, layout-independent fp32 masters + optimizer state with the global step,
atomically, CRC-checked: csrc/checkpoint.cpp). Survivors notice the failure in one of two ways:
the collective they are blocked in fails (gloo sees the peer's socket close; the per-generation
process-group timeout bounds any other wait), or the watchdog thread sees the coordinator expire a
member of the current plan (missed heartbeats) and aborts the RCCL communicator so the blocked
collective returns. They then tear the group down, one survivor (store election) waits until the
coordinator's live set no longer lists the dead member and publishes the next plan (survivors +
joiners, step = checkpoint step, ``restore``), and everyone rebuilds the world, reloads the
checkpoint re-sharded for the new world and continues. Steps after the checkpoint are recomputed;
the parameter state is exactly the checkpoint's (reference: the coordinator's expiry,
src/coordinator.cpp:52-67, and the ops-level PS restart, scripts/scale_workers.sh:137-144, which
lost all in-memory state).
"""
from __future__ import annotations

import datetime
import json
import os
import signal
import socket
import threading
import time
from dataclasses import dataclass

import torch
import torch.distributed as dist

from ..rpc import schema, service
from ..utils.log import get_logger
from .coordinator import STORE_KEY, split_host_port

cpb = schema.coordinator
PREFIX = "psd/elastic"


@dataclass
class Plan:
    gen: int
    members: list  # worker ids in rank order (rank 0 first: it holds the handed-over state)
    step: int  # global step the generation starts at
    epoch: int  # coordinator membership epoch the plan was made from
    done: bool = False
    restore: bool = False  # start from the canonical checkpoint (crash recovery)

    def dumps(self) -> str:
        return json.dumps(self.__dict__)

    @staticmethod
    def loads(s) -> "Plan":
        return Plan(**json.loads(s))


class ElasticAgent:
    """Coordinator client + rendezvous store of one elastic worker."""

    def __init__(self, coordinator: str, worker_id: int, heartbeat_s: float = 1.0, timeout_s: float = 300.0):
        self.log = get_logger(f"elastic{worker_id}")
        self.worker_id = int(worker_id)
        self.coord = service.Stub(coordinator, cpb, timeout=30.0)
        self.timeout = datetime.timedelta(seconds=timeout_s)
        host, _ = split_host_port(coordinator, 50052)
        r = self.coord.KvGet(cpb.KvRequest(key=STORE_KEY, timeout_ms=int(timeout_s * 1000)))
        if not r.found:
            raise RuntimeError(f"coordinator {coordinator} hosts no rendezvous store (start it with --store-port)")
        self.store = dist.TCPStore(host if host not in ("0.0.0.0", "") else "127.0.0.1", int(r.value),
                                   is_master=False, timeout=self.timeout)
        self.epoch = -1
        self._stop = threading.Event()
        self.heartbeat_s = heartbeat_s
        self.status = cpb.IDLE
        self._register()
        self._hb = threading.Thread(target=self._heartbeat_loop, name="elastic-hb", daemon=True)
        self._hb.start()

    def _register(self):
        info = cpb.WorkerInfo(worker_id=self.worker_id, address="localhost", port=0,
                              hostname=f"worker-{self.worker_id}@{socket.gethostname()}")
        r = self.coord.RegisterWorker(info)
        self.epoch = r.membership_epoch

    def _heartbeat_loop(self):
        while not self._stop.wait(self.heartbeat_s):
            try:
                r = self.coord.Heartbeat(cpb.HeartbeatRequest(worker_id=self.worker_id, status=self.status),
                                         timeout=5.0, wait_for_ready=False)
                self.epoch = r.membership_epoch
                if not r.success:  # expired while busy (e.g. a long rebuild): come back
                    self._register()
            except Exception as e:  # noqa: BLE001
                self.log.debug("heartbeat failed: %s", e)

    def live(self) -> tuple[int, list[int]]:
        r = self.coord.ListWorkers(cpb.ListWorkersRequest())
        return r.membership_epoch, sorted(w.worker_id for w in r.workers)

    def leave(self):
        self._stop.set()
        try:
            self.coord.Deregister(cpb.WorkerInfo(worker_id=self.worker_id), timeout=5.0, wait_for_ready=False)
        except Exception:  # noqa: BLE001
            pass

    # ---- plans
    def publish(self, plan: Plan):
        self.store.set(f"{PREFIX}/plan/{plan.gen}", plan.dumps())
        self.store.set(f"{PREFIX}/latest", str(plan.gen))

    def read_plan(self, gen: int) -> Plan:
        self.store.wait([f"{PREFIX}/plan/{gen}"], self.timeout)
        return Plan.loads(self.store.get(f"{PREFIX}/plan/{gen}"))

    def first_plan(self, min_workers: int) -> Plan:
        """Generation 0 (the first rank to win the create lock writes it once ``min_workers`` are
        live), or -- for a late joiner -- the first later plan that lists this worker."""
        if self.store.add(f"{PREFIX}/create0", 1) == 1:
            t0 = time.time()
            while True:
                ep, ids = self.live()
                if len(ids) >= min_workers or time.time() - t0 > self.timeout.total_seconds():
                    break
                time.sleep(0.1)
            self.publish(Plan(0, ids, 0, ep))
        gen = 0
        while True:
            p = self.read_plan(gen)
            if p.done or self.worker_id in p.members:
                return p
            gen += 1

    def next_plan(self, gen: int) -> Plan:
        return self.read_plan(gen + 1)


def _init_group(agent: ElasticAgent, plan: Plan, backend: str, device) -> None:
    rank = plan.members.index(agent.worker_id)
    store = dist.PrefixStore(f"{PREFIX}/g{plan.gen}", agent.store)
    kw = {}
    if backend == "nccl":
        kw["device_id"] = device
    dist.init_process_group(backend, store=store, rank=rank, world_size=len(plan.members),
                            timeout=agent.timeout, **kw)


def _destroy_group():
    try:
        if dist.is_initialized():
            dist.destroy_process_group()
    except Exception:  # noqa: BLE001 -- the group of a failed generation may be half torn down
        pass


class _Watchdog:
    """Per-generation failure detector: when the coordinator expires a member of the current plan
    (missed heartbeats), abort the native RCCL communicator so a collective blocked on the dead
    peer returns, and flag the generation as failed."""

    def __init__(self, agent: ElasticAgent, plan: Plan, ps, period_s: float = 0.5):
        self.agent, self.plan, self.ps = agent, plan, ps
        self.fired = False
        self.dead: list[int] = []
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, args=(period_s,), name="elastic-watchdog", daemon=True)
        self._t.start()

    def _run(self, period_s):
        seen = self.agent.epoch
        while not self._stop.wait(period_s):
            if self.agent.epoch == seen:
                continue
            seen = self.agent.epoch
            try:
                _, live = self.agent.live()
            except Exception:  # noqa: BLE001
                continue
            dead = sorted(set(self.plan.members) - set(live))
            if dead:
                self.dead, self.fired = dead, True
                abort = getattr(getattr(self.ps, "t", None), "abort", None)
                if abort is not None:
                    try:
                        abort()
                    except Exception:  # noqa: BLE001
                        pass
                return

    def stop(self):
        self._stop.set()


class ElasticTrainer:
    """Runs ``steps`` global training steps across membership changes.

    ``make_ps(model, transport) -> CollectivePS`` builds the data plane for the current world;
    ``make_trainer(ps) -> Trainer`` wraps it. ``on_step(global_step, loss, plan)`` is a progress
    callback.
    """

    def __init__(self, agent: ElasticAgent, model, make_ps, make_trainer, steps: int, device,
                 check_every: int = 10, min_workers: int = 1, backend: str | None = None, on_step=None,
                 checkpoint_dir: str | None = None, checkpoint_every: int = 0, collective_timeout_s: float = 0.0):
        self.agent = agent
        self.model = model
        self.make_ps, self.make_trainer = make_ps, make_trainer
        self.steps = int(steps)
        self.device = torch.device(device)
        self.check_every = max(1, int(check_every))
        self.min_workers = min_workers
        self.backend = backend or ("nccl" if self.device.type == "cuda" else "gloo")
        self.on_step = on_step
        self.leaving = False
        self.history = []  # (gen, members, start step)
        self.resizes = 0
        self.recoveries = 0
        self.log = agent.log
        self.checkpoint_dir = checkpoint_dir
        self.checkpoint_every = int(checkpoint_every) if checkpoint_dir else 0
        # bounds every collective of a generation (a dead peer must not block survivors forever)
        if collective_timeout_s > 0:
            self.agent.timeout = datetime.timedelta(seconds=collective_timeout_s)

    def request_leave(self, *_):
        """SIGTERM handler (scale_workers.sh down): hand over at the next check, then exit."""
        self.leaving = True

    def install_signal_handler(self):
        signal.signal(signal.SIGTERM, self.request_leave)

    # ------------------------------------------------------------------ main loop
    def run(self) -> dict:
        from ..parallel.transport import make_transport

        plan = self.agent.first_plan(self.min_workers)
        state = None
        step = plan.step
        losses = []
        result = {"history": self.history}
        while not plan.done:
            _init_group(self.agent, plan, self.backend, self.device)
            rank, world = dist.get_rank(), dist.get_world_size()
            self.history.append((plan.gen, list(plan.members), plan.step))
            self.log.info("generation %d: rank %d of %d (members %s) from step %d%s", plan.gen, rank, world,
                          plan.members, plan.step, " (restored from checkpoint)" if plan.restore else "")
            ps = self.make_ps(self.model, make_transport("auto", self.device))
            if plan.restore:
                ps.load_canonical_state(self._load_checkpoint(ps))
                step = plan.step
                # the steps after the checkpoint are recomputed: their first losses are void
                losses = [(s_, l_) for (s_, l_) in losses if s_ <= step]
            elif plan.gen > 0:  # state handed over by the previous generation's leader (new rank 0)
                ps.load_canonical_state(self._broadcast_state(ps, state))
            state = None
            tr = self.make_trainer(ps)
            self.agent.status = cpb.TRAINING
            leavers = None
            watchdog = _Watchdog(self.agent, plan, ps)
            try:
                while step < self.steps and leavers is None:
                    loss = tr.step()
                    step += 1
                    losses.append((step, loss.detach().clone()))
                    if self.on_step is not None:
                        self.on_step(step, loss, plan)
                    if self.checkpoint_every and step % self.checkpoint_every == 0 and step < self.steps:
                        self._save_checkpoint(ps, step)
                    if step % self.check_every == 0 and step < self.steps:
                        leavers = self._check(plan, world, rank)
                    if watchdog.fired:
                        raise RuntimeError(f"member(s) {watchdog.dead} of generation {plan.gen} died")
            except Exception as e:  # noqa: BLE001 -- a peer died mid-collective: recover
                watchdog.stop()
                if not self.checkpoint_every:
                    raise
                self.log.warning("generation %d failed at step %d (%s): recovering from the last checkpoint",
                                 plan.gen, step, str(e).splitlines()[0][:200])
                try:
                    ps.close()
                except Exception:  # noqa: BLE001
                    pass
                del tr, ps
                _destroy_group()
                plan = self._recover(plan)
                self.recoveries += 1
                result["recovered_at"] = result.get("recovered_at", []) + [step]
                if self.agent.worker_id not in plan.members:
                    result["losses"] = [float(x) for _, x in losses]
                    self.agent.leave()
                    return result
                continue
            watchdog.stop()
            if hasattr(tr, "wait_checkpoint"):
                tr.wait_checkpoint()
            if leavers is None:  # all steps done
                if rank == 0:
                    self.agent.publish(Plan(plan.gen + 1, [], step, self.agent.epoch, done=True))
                if hasattr(ps, "refresh_weights"):  # async plane: workers hold their last pull
                    ps.drain()
                    ps.refresh_weights()
                result["params"] = {n: p.detach().float().cpu() for n, p in self.model.named_parameters()}
                result["staleness_hist"] = ps.staleness_histogram()
                ps.close()
                dist.destroy_process_group()
                break
            # ---- membership change at this step boundary: hand the PS state to the next world
            ps.drain()
            survivors = [m for i, m in enumerate(plan.members) if i not in leavers]
            leader = min(i for i in range(world) if i not in leavers) if survivors else 0
            state = ps.canonical_state(root=leader)
            if rank == leader:
                ep, live = self.agent.live()
                gone = {plan.members[i] for i in leavers}
                lead_id = plan.members[leader]
                rest = sorted((set(live) | set(survivors)) - gone - {lead_id})
                self.agent.publish(Plan(plan.gen + 1, [lead_id] + rest if survivors else [], step, ep,
                                        done=not survivors))
            plan = self.agent.next_plan(plan.gen)
            ps.close()
            del tr, ps
            dist.destroy_process_group()
            self.resizes += 1
            if self.agent.worker_id not in plan.members:
                self.log.info("left the job at step %d (handed over to %s)", step, plan.members)
                result["left_at"] = step
                result["losses"] = [float(x) for _, x in losses]
                self.agent.leave()
                return result
        result["finished_at"] = step
        result["resizes"] = self.resizes
        result["recoveries"] = self.recoveries
        result["losses"] = [float(x) for _, x in losses]
        result["loss_steps"] = [s_ for s_, _ in losses]
        self.agent.leave()
        return result

    # ------------------------------------------------------------------ crash recovery
    def _ckpt_path(self) -> str:
        return os.path.join(self.checkpoint_dir, "elastic_canonical.psd")

    def _save_checkpoint(self, ps, step: int):
        """Collective: drain, gather the canonical state to rank 0, write it atomically."""
        from .. import native

        ps.drain()
        sd = ps.canonical_state(root=0)
        if dist.get_rank() == 0:
            keys = [k for k in ("master", "state1", "state2", "dyn") if k in sd]
            man = json.dumps({"step": step, "keys": keys, "format": "psd-elastic-canonical-v1"})
            os.makedirs(self.checkpoint_dir, exist_ok=True)
            native().save_native_ckpt(self._ckpt_path(), man, [sd[k].detach().cpu() for k in keys])
        self.last_checkpoint = step

    def _load_checkpoint(self, ps) -> dict:
        from .. import native

        man, ts = native().load_native_ckpt(self._ckpt_path())
        m = json.loads(man)
        return {k: t for k, t in zip(m["keys"], ts)}

    def _checkpoint_step(self) -> int:
        from .. import native

        if not self.checkpoint_dir or not os.path.exists(self._ckpt_path()):
            raise RuntimeError("a member died and no canonical checkpoint exists to recover from")
        man, _ = native().load_native_ckpt(self._ckpt_path())
        return int(json.loads(man)["step"])

    def _recover(self, plan: Plan) -> Plan:
        """After a failed generation: one survivor (store election) waits for the coordinator to
        drop the dead member(s), then publishes the restore plan; everyone reads it."""
        if self.agent.store.add(f"{PREFIX}/recover/{plan.gen}", 1) == 1:
            t0 = time.time()
            while True:
                ep, live = self.agent.live()
                if set(plan.members) - set(live) or time.time() - t0 > self.agent.timeout.total_seconds():
                    break
                time.sleep(0.2)
            members = sorted(set(live))
            self.agent.publish(Plan(plan.gen + 1, members, self._checkpoint_step(), ep, done=not members,
                                    restore=True))
        return self.agent.next_plan(plan.gen)

    def _check(self, plan: Plan, world: int, rank: int):
        """Collective (same step on every rank): the set of ranks leaving if the membership changes,
        else None. Rank 0 compares the coordinator's live set with the plan when its heartbeat saw
        the membership epoch move; any rank asked to leave (SIGTERM) raises its flag."""
        v = torch.zeros(world + 1, dtype=torch.float32, device=self.device)
        if self.leaving:
            v[rank] = 1.0
        if rank == 0 and self.agent.epoch != plan.epoch:
            ep, live = self.agent.live()
            plan.epoch = ep
            if sorted(live) != sorted(plan.members):
                v[world] = 1.0
        dist.all_reduce(v)
        f = v.tolist()
        leavers = {i for i in range(world) if f[i] > 0}
        if not leavers and f[world] == 0:
            return None
        return leavers

    def _broadcast_state(self, ps, state):
        """New rank 0 holds the canonical state; give every rank a copy."""
        idx, n = ps._canon_index()
        if hasattr(ps, "canonical_keys"):  # AsyncPS: optimizer states from its config
            keys = ps.canonical_keys()
        else:
            keys = ["master"] + [k for k, t in (("state1", ps.state1), ("state2", ps.state2)) if t is not None]
        out = {}
        for k in keys:
            t = state[k].to(self.device) if dist.get_rank() == 0 else torch.empty(n, dtype=torch.float32,
                                                                                  device=self.device)
            dist.broadcast(t, 0)
            out[k] = t
        dyn = ps.dyn_template() if hasattr(ps, "dyn_template") else ps.dyn.t
        d = state["dyn"].to(dyn.device) if dist.get_rank() == 0 else torch.empty_like(dyn)
        dist.broadcast(d, 0)
        out["dyn"] = d
        return out

