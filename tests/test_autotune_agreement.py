"""Cross-rank agreement of the per-shape kernel choice (ops/autotune.py): at N > 1 the first rank
to reach a key times it and every other rank takes that decision through the store. Two gloo
ranks whose candidates time in opposite orders (each alone would pick a different one) must run
the same candidate; and a saved decision file pins choices with no timing."""
import os
import socket
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from parameter_server_distributed_amd.ops import autotune as at

    picks = []
    for i in range(3):
        slow_a = (rank + i) % 2 == 0  # rank-dependent: local timing would disagree across ranks

        def a():
            time.sleep(0.02 if slow_a else 0.0)
            return torch.ones(4)

        def b():
            time.sleep(0.0 if slow_a else 0.02)
            return torch.ones(4)

        picks.append(at.choose(("test", i), {"a": a, "b": b}, "a"))
    with open(os.path.join(out_dir, f"r{rank}.txt"), "w") as f:
        f.write(repr((picks, at.source())))
    if rank == 0:
        at.save_decisions(os.path.join(out_dir, "dec.json"))
    dist.barrier()
    dist.destroy_process_group()


def test_autotune_ranks_agree_and_file_roundtrip(tmp_path):
    mp.spawn(_rank, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    (p0, s0), (p1, s1) = (eval(open(tmp_path / f"r{r}.txt").read()) for r in range(2))
    assert p0 == p1, (p0, p1)
    assert s0["claimed"] + s1["claimed"] == 3 and s0["peer"] + s1["peer"] == 3, (s0, s1)
    from parameter_server_distributed_amd.ops import autotune as at

    n = at.load_decisions(str(tmp_path / "dec.json"))
    assert n == 3
    for i in range(3):
        assert at.choose(("test", i), {"a": None, "b": None}, "a") == p0[i]
        at.set_decision(("test", i), None)


def _rank_declined(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), PSD_AUTOTUNE_WAIT_S="60")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from parameter_server_distributed_amd.ops import autotune as at

    def nope():
        raise at.Declined("shape not taken")

    def boom():
        raise MemoryError("simulated OOM")

    res = []
    for rep in range(2):  # the second pass must neither re-claim nor wait on the key
        t0 = time.time()
        try:
            at.choose(("all_declined",), {"a": nope, "b": nope}, "a")
            res.append("chosen")
        except at.Declined:
            res.append("declined")
        res.append(time.time() - t0 < 30)
    dist.barrier()
    # a claiming rank that fails with a real error publishes it; the peer raises instead of hanging
    if rank == 0:
        try:
            at.choose(("fails",), {"a": boom}, "a")
        except MemoryError:
            res.append("error")
        dist.barrier()
    else:
        dist.barrier()  # rank 0 claims first
        try:
            at.choose(("fails",), {"a": boom}, "a")
        except RuntimeError as e:
            res.append("error" if "failed" in str(e) else repr(e))
    with open(os.path.join(out_dir, f"d{rank}.txt"), "w") as f:
        f.write(repr(res))
    dist.barrier()
    dist.destroy_process_group()


def test_autotune_all_declined_publishes_to_peers(tmp_path):
    """a claimed key whose candidates all decline (or whose timing raises) must be
    published, so peers raise at once instead of waiting PSD_AUTOTUNE_WAIT_S on it."""
    mp.spawn(_rank_declined, args=(2, _port(), str(tmp_path)), nprocs=2, join=True)
    for r in range(2):
        res = eval(open(tmp_path / f"d{r}.txt").read())
        assert res == ["declined", True, "declined", True, "error"], (r, res)


def test_prefer_own_within_margin(monkeypatch):
    """A library candidate ("miopen" / "gemm" / "blas") that wins by less than OWN_MARGIN yields to
    the fastest of our kernels; a clear library win stands; the feature off restores the plain min."""
    from parameter_server_distributed_amd.ops import autotune as at
    from parameter_server_distributed_amd.utils.config import set_feature

    out = torch.ones(4)
    times = {}
    monkeypatch.setattr(at, "_time_ms", lambda fn, probe=None: (times[fn()], [out, out]))
    cands = {n: (lambda n=n: n) for n in ("miopen", "psdw0", "igemm")}

    def pick(t, key):
        times.clear()
        times.update(t)
        return at._time_and_pick(key, cands, "miopen", None)

    try:
        assert pick({"miopen": 1.00, "psdw0": 1.015, "igemm": 1.3}, ("t", 1)) == "psdw0"
        assert pick({"miopen": 1.00, "psdw0": 1.05, "igemm": 1.3}, ("t", 2)) == "miopen"
        assert pick({"miopen": 1.2, "psdw0": 1.05, "igemm": 1.0}, ("t", 3)) == "igemm"
        set_feature("prefer_own", False)
        assert pick({"miopen": 1.00, "psdw0": 1.015, "igemm": 1.3}, ("t", 4)) == "miopen"
    finally:
        set_feature("prefer_own", None)
        for k in [("t", i) for i in range(1, 5)]:
            at._DECISIONS.pop(k, None)
            at._TIMES.pop(k, None)


def test_guard_rejects_zeros_on_small_magnitude_output():
    """with an absolute 1e-2 floor a candidate returning zeros passed wherever the
    reference's entries were all below 0.01 (a small weight gradient). The guard is now relative only."""
    from parameter_server_distributed_amd.ops import autotune as at

    g = torch.Generator().manual_seed(0)
    ref = torch.randn(64, 32, generator=g) * 1e-3  # |entries| < 0.01
    assert not at._agrees([torch.zeros_like(ref)], [ref])
    assert not at._agrees([ref * 0.9], [ref])  # a 10 % scale error is wrong, whatever the magnitude
    # bf16 rounding of the same values and a changed fp32 summation order are accepted
    assert at._agrees([ref.to(torch.bfloat16).float()], [ref])
    assert at._agrees([ref + 1e-4 * ref.abs().max() * torch.randn(64, 32, generator=g)], [ref])
    # an all-zero reference takes only zeros; non-finite reference entries are skipped
    z = torch.zeros(8)
    assert at._agrees([z.clone()], [z]) and not at._agrees([z + 1e-12], [z])
    r = torch.tensor([1.0, float("nan"), 2.0])
    assert at._agrees([torch.tensor([1.0, 5.0, 2.0])], [r])
    assert not at._agrees([torch.tensor([1.0, 5.0, float("inf")])], [r])


def test_zeros_candidate_never_chosen(monkeypatch):
    """End to end through _time_and_pick: the fastest candidate returns zeros on a small-magnitude
    weight gradient and must be rejected, not chosen."""
    from parameter_server_distributed_amd.ops import autotune as at

    ref = torch.full((16, 16), 3e-3)
    outs = {"mfma": ref, "fast_zero": torch.zeros(16, 16)}
    times = {"mfma": 1.0, "fast_zero": 0.5}
    monkeypatch.setattr(at, "_time_ms", lambda fn, probe=None: (times[fn()], [outs[fn()], outs[fn()]]))
    key = ("t", "zeros")
    try:
        assert at._time_and_pick(key, {"mfma": lambda: "mfma", "fast_zero": lambda: "fast_zero"}, "mfma", None) == "mfma"
        assert "fast_zero" in at.rejected()[key]
    finally:
        at._DECISIONS.pop(key, None)
        at._TIMES.pop(key, None)
        at._REJECTED.pop(key, None)


def test_decision_file_schema(tmp_path):
    """a decision file of another schema (older variant numbering) is refused."""
    import json

    import pytest

    from parameter_server_distributed_amd.ops import autotune as at

    old = tmp_path / "old.json"
    old.write_text(json.dumps({"('conv1x1', 'wgrad', 1, 2, 3)": "psdw1"}))  # pre-schema format
    with pytest.raises(ValueError, match="schema"):
        at.load_decisions(str(old))
    assert ("conv1x1", "wgrad", 1, 2, 3) not in at.decisions()
    at.set_decision(("t", "schema"), "a")
    try:
        at.save_decisions(str(tmp_path / "new.json"))
        assert json.loads((tmp_path / "new.json").read_text())["schema"] == at.SCHEMA
        assert at.load_decisions(str(tmp_path / "new.json")) >= 1
    finally:
        at.set_decision(("t", "schema"), None)


def test_library_candidates_off_keeps_only_own_kernels(monkeypatch):
    """feature library_candidates off: MIOpen / hipBLASLt leave every candidate set in which one of
    our kernels takes the shape (even when faster, and even as the default); they stay the fallback
    where nothing of ours does."""
    from parameter_server_distributed_amd.ops import autotune as at
    from parameter_server_distributed_amd.utils.config import set_feature

    out = torch.ones(4)
    times = {"miopen": 0.5, "blas": 0.4, "psdw0": 1.0, "mfma": 0.9}
    monkeypatch.setattr(at, "_time_ms", lambda fn, probe=None: (times[fn()], [out, out]))
    set_feature("library_candidates", False)
    keys = [("lib", 1), ("lib", 2), ("lib", 3)]
    try:
        assert at.choose(keys[0], {n: (lambda n=n: n) for n in ("miopen", "psdw0")}, "miopen") == "psdw0"
        assert at.choose(keys[1], {n: (lambda n=n: n) for n in ("mfma", "blas", "psdw0")}, "mfma") == "mfma"
        assert at.choose(keys[2], {"miopen": lambda: "miopen"}, "miopen") == "miopen"  # the only candidate
    finally:
        set_feature("library_candidates", None)
        for k in keys:
            at._DECISIONS.pop(k, None)
            at._TIMES.pop(k, None)


def test_groups_validate_within_family(monkeypatch):
    """Candidate families returning different tensors (a fused bwd-data epilogue's BN-masked gradient
    vs the plain kernels' dX) are each validated against their own family's reference: a correct
    fused candidate is not rejected for differing from dX, and a wrong one still is."""
    from parameter_server_distributed_amd.ops import autotune as at

    dx = torch.linspace(-1, 1, 64)
    g = dx * (dx > 0)  # the "masked" family
    outs = {"plain0": dx, "plain1": dx * (1 + 1e-4), "psdnb0": g, "psdnb1": g * (1 - 1e-4), "psdnb2": torch.zeros(64)}
    times = {"plain0": 1.0, "plain1": 0.9, "psdnb0": 0.8, "psdnb1": 0.7, "psdnb2": 0.1}
    monkeypatch.setattr(at, "_time_ms", lambda fn, probe=None: (times[fn()], [outs[fn()], outs[fn()]]))
    key = ("t", "groups")
    try:
        got = at._time_and_pick(key, {n: (lambda n=n: n) for n in outs}, "plain0", None,
                                group=lambda n: n.startswith("psdnb"))
        assert got == "psdnb1", got
        assert at.rejected()[key] == ["psdnb2"], at.rejected()[key]
    finally:
        at._DECISIONS.pop(key, None)
        at._TIMES.pop(key, None)
        at._REJECTED.pop(key, None)


def test_library_fallback_when_every_own_kernel_declines(monkeypatch):
    """library_candidates off, but every one of our candidates declines the shape at run time (a
    conv our implicit-GEMM kernels do not take): the library candidate is timed and chosen after
    all -- never an 'every candidate declined' error -- and the decision is cached."""
    from parameter_server_distributed_amd.ops import autotune as at
    from parameter_server_distributed_amd.utils.config import set_feature

    def nope():
        raise at.Declined("shape not taken")

    calls = []

    def lib():
        calls.append(1)
        return torch.ones(4)

    set_feature("library_candidates", False)
    key = ("lib", "fallback")
    try:
        assert at.choose(key, {"igemm": nope, "psds_igemm": nope, "miopen": lib}, "miopen") == "miopen"
        n = len(calls)
        assert at.choose(key, {"igemm": nope, "psds_igemm": nope, "miopen": lib}, "miopen") == "miopen"
        assert len(calls) == n  # cached: not re-timed
    finally:
        set_feature("library_candidates", None)
        at._DECISIONS.pop(key, None)
        at._TIMES.pop(key, None)
        at._REJECTED.pop(key, None)
