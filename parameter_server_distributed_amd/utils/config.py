"""Run-config files (YAML or JSON) for the bench and the role CLIs.

``--config run.yaml`` supplies defaults for any long option of the command (keys use either
``ps-shards`` or ``ps_shards`` spelling); explicit command-line flags still win. Files are read
with ``yaml.safe_load`` / ``json.load`` only. The reference configures everything through
positional argv and shell-script env vars (scripts/*.sh); this is additive.
"""
from __future__ import annotations

import argparse
import json
import os


def load_config(path: str) -> dict:
    with open(path) as f:
        text = f.read()
    if path.endswith(".json"):
        cfg = json.loads(text)
    else:
        import yaml

        cfg = yaml.safe_load(text) or {}
    if not isinstance(cfg, dict):
        raise ValueError(f"{path}: a run config must be a mapping of option -> value")
    return {str(k).replace("-", "_"): v for k, v in cfg.items()}


def apply_config(ap: argparse.ArgumentParser, argv: list[str] | None = None) -> None:
    """Pre-parse ``--config`` from ``argv`` and install the file's values as parser defaults."""
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--config", default=os.environ.get("PSD_CONFIG", ""))
    known, _ = pre.parse_known_args(argv)
    if not any(a.dest == "config" for a in ap._actions):
        ap.add_argument("--config", default="", help="YAML/JSON run config (flags override it)")
    if not known.config:
        return
    cfg = load_config(known.config)
    dests = {a.dest for a in ap._actions}
    unknown = sorted(set(cfg) - dests)
    if unknown:
        raise SystemExit(f"{known.config}: unknown option(s) {unknown}")
    ap.set_defaults(**cfg)


# ---------------------------------------------------------------------------------------------
# Kernel-path features: one documented default each, one override variable.
#
# Every fused / hand-written path that has a library or unfused fallback is gated by a feature
# here, so a test can pin the fallback as its reference and an A/B run can switch one path off
# without a code change. Override with PSD_FEATURES="name=0,other=1" (the variable is re-read when
# it changes: tests set it per case) or programmatically with set_feature(). The defaults are the
# production paths; the switches are not separate environment variables.
FEATURES: dict[str, tuple[bool, str]] = {
    # convolutions (ops/conv.py, kernels/convn.hip, convw.hip, gemm.hip)
    "conv1x1": (True, "per-shape routing of 1x1 convolutions (MIOpen / hipBLASLt / MFMA); off: MIOpen only"),
    "conv1x1_mfma": (True, "the 8-phase MFMA GEMM as a 1x1-convolution candidate"),
    "conv_igemm": (True, "implicit-GEMM MFMA convolution (gemm.hip) as a forward / bwd-data candidate"),
    "conv_wgrad": (True, "implicit-GEMM MFMA weight gradient as a candidate"),
    "convn": (True, "narrow implicit-GEMM convolution kernels (convn.hip) as candidates"),
    "convn_stats": (True, "consumer-BN statistics in the narrow convolution's epilogue"),
    "convn_persist": (True, "persistent layer-1 3x3 kernel (convh)"),
    "convn_p1": (True, "persistent 1x1 kernels (convp / convpr)"),
    "convn_p2": (True, "the persistent 1x1 kernel at two workgroups per CU (two-slot ring) as a candidate"),
    "convn_bwd": (True, "producing BN's backward reduction in the bwd-data epilogue (modes 1/2)"),
    "convn_bwd3": (True, "the dual-BN tail's reduction in the bwd-data epilogue (mode 3)"),
    "convn_bwd5": (True, "stride-2 downsample gradient added on the quarter grid (mode 5)"),
    "dgrad_s2_phase": (True, "stride-2 3x3 bwd-data as four output-parity phase launches of the narrow kernel "
                              "(with the producing BN's backward reduction in the epilogue) vs MIOpen"),
    "convw": (True, "narrow weight-gradient kernel (convw.hip) as a candidate"),
    "convw_persist": (True, "persistent layer-1 3x3 weight gradient (convhw)"),
    "convw_twostage": (True, "narrow weight-gradient tiles also on a two-stage ring at two workgroups per CU"),
    "convw_fold2": (True, "the BN-fold and Gram weight-gradient launches on the two-stage ring (two workgroups per CU)"),
    "gemm_stats": (True, "consumer-BN statistics in the 8-phase GEMM epilogue"),
    "library_candidates": (False, "convolutions: autotune also times MIOpen / hipBLASLt candidates wherever one of "
                                  "our kernels takes the shape; off (default): our kernels only there, the library "
                                  "only as the fallback -- same-box ResNet-50 15,681 / 15,695 vs 15,557 / 15,591 "
                                  "img/s with them (profiles/r6/ab_library_candidates.md)"),
    "library_linear": (True, "Linear layers: hipBLASLt stays an autotune candidate (BERT-base same-box 9,576 / 9,505 "
                             "vs 9,297 / 9,362 seq/s without it: it wins the QKV forward, the attention-output "
                             "bwd-data and the MLM-head weight gradient in the step, profiles/r6/ab_library_candidates.md)"),
    "prefer_own": (True, "autotune: our kernel takes a pick a library candidate wins by < 2 % (ops/autotune.py OWN_MARGIN)"),
    "wprep": (True, "every convolution's bwd-data weight operand (transpose / tap flip / stride-2 phases) in one batched launch per step (ops/wprep.py)"),
    # batch norm / bottleneck tail (ops/bn.py, ops/tail.py)
    "bn_fold": (True, "bn3's backward folded into conv3's bwd-data / weight-gradient GEMMs"),
    "bn_fold_ds": (True, "the stride-1 downsample BN folded into its convolution's backward"),
    "dual_nobx": (True, "downsample blocks' dual tail without the BN inputs in the consumer epilogue"),
    "tail_recompute": (True, "identity blocks' conv3 output recomputed instead of stored"),
    "tail_gram": (True, "the recomputing tail's statistics from the Gram matrix of conv3's input"),
    "dual_recompute": (True, "stride-1 downsample blocks: neither conv3's nor the downsample conv's output stored"),
    # fp8 (Wide-ResNet-101-2)
    "fp8_compute": (True, "fp8 convolutions where the model asks for them"),
    "fp8_mx": (True, "MX block scales for every fp8 operand; off: per-tensor scales"),
    "fp8_mx_handover": (True, "BN passes write the consumer's MX e4m3 input / producer's MX e5m2 dY"),
    "fp8_delayed": (True, "per-tensor fp8: delayed (previous-call amax) scaling"),
    "fp8_dgrad": (True, "fp8 e5m2-dY bwd-data of the fp8 convolutions"),
    "async_cached_local": (True, "async PS at world 1: inbox / publish buffers in plain (cached) device memory "
                                 "instead of uncached IPC memory (read by the native engine)"),
    "async_apply_background": (True, "async PS with SSP bound >= 1: the owner's apply on a normal-priority stream "
                                     "with at most 512 workgroups, beside the compute stream (read by the native "
                                     "engine); off: high priority, full grid (the S = 0 setting)"),
    "async_direct_pull": (True, "async PS at world 1: each step pulls straight into the model's working weights "
                                "on the compute stream (one local copy) instead of prefetching into a second "
                                "buffer and copying that into the working weights"),
    "tail_fp8": (False, "fp8 models' identity blocks: conv3 + bn3 as the bf16 recomputing tail (bn3 folded "
                       "into conv3's bf16 backward, conv3's output never stored); read at model build. Off: same-box "
                       "WRN-101-2 4,136 vs 4,170 img/s (profiles/r6/ab_tail_fp8.md)"),
    # BERT (ops/linear.py, ops/attention.py)
    "linear_tune": (True, "per-shape MFMA / hipBLASLt choice for Linear layers; off: MFMA only"),
    "gelu_fuse": (True, "GELU backward in the consumer Linear's bwd-data GEMM epilogue"),
    "attn_bias": (True, "QKV bias gradient handed over by the attention backward"),
}

_FEAT_ENV: str | None = None
_FEAT_OVR: dict[str, bool] = {}
_FEAT_SET: dict[str, bool] = {}


def _feature_env() -> dict[str, bool]:
    global _FEAT_ENV, _FEAT_OVR
    raw = os.environ.get("PSD_FEATURES", "")
    if raw != _FEAT_ENV:
        ovr = {}
        for item in filter(None, (t.strip() for t in raw.split(","))):
            name, _, val = item.partition("=")
            name = name.strip()
            if name not in FEATURES:
                raise ValueError(f"PSD_FEATURES: unknown feature {name!r} (known: {sorted(FEATURES)})")
            ovr[name] = val.strip() not in ("0", "false", "off", "no")
        _FEAT_ENV, _FEAT_OVR = raw, ovr
    return _FEAT_OVR


def feature(name: str) -> bool:
    """Whether kernel-path feature ``name`` (FEATURES) is on: set_feature > PSD_FEATURES > default."""
    if name in _FEAT_SET:
        return _FEAT_SET[name]
    ovr = _feature_env()
    if name in ovr:
        return ovr[name]
    return FEATURES[name][0]


def set_feature(name: str, on: bool | None) -> None:
    """Pin feature ``name`` for this process (None: back to PSD_FEATURES / the default)."""
    if name not in FEATURES:
        raise ValueError(f"unknown feature {name!r}")
    if on is None:
        _FEAT_SET.pop(name, None)
    else:
        _FEAT_SET[name] = bool(on)


def features() -> dict[str, bool]:
    """Every feature's current value (bench JSON / logs)."""
    return {n: feature(n) for n in FEATURES}


# Fault injection (tests, chaos runs): PSD_FAULT="key=value,..." with the keys below; -1 / 0 = off.
FAULTS: dict[str, tuple[int, str]] = {
    "stop_heartbeat_after": (-1, "worker: stop sending coordinator heartbeats after n of them"),
    "push_delay_ms": (0, "worker: sleep this long before every gradient push"),
    "exit_after_push": (-1, "worker: exit the process right after its k-th push"),
    "selftest_fail_rank": (-1, "async PS: this rank reports a failed start-up self-test"),
    "selftest_fail_kernel": (-1, "async PS: this rank fails the kernel-transport self-test attempt only"),
}


def fault(name: str) -> int:
    """Integer value of fault-injection key ``name`` from PSD_FAULT (FAULTS default when unset)."""
    if name not in FAULTS:
        raise ValueError(f"unknown fault key {name!r}")
    for item in filter(None, (t.strip() for t in os.environ.get("PSD_FAULT", "").split(","))):
        k, _, v = item.partition("=")
        if k.strip() == name:
            return int(v)
    return FAULTS[name][0]
