#!/usr/bin/env python3
"""Probe the library GEMMs behind ResNet-50's 1x1 convolutions (b1024 shapes) for non-finite or
wrong outputs: each forward ([M, cin] x [cout, cin]^T) and bwd-data ([M, cout] x [cout, cin]) GEMM
runs ``--reps`` times through torch.mm under the selected TunableOp mode; outputs are checked for
NaN/Inf and against an fp32 reference on a row subset. Also the MIOpen path (F.conv2d).

  python tools/gemm_nan_probe.py --tunableop use|off [--reps 10] [--miopen 1]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from parameter_server_distributed_amd.utils import miopen as _miopen  # noqa: E402

_miopen.install()
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from parameter_server_distributed_amd.utils import tunableop as _tunableop  # noqa: E402

SHAPES = [(3211264, 64, 64), (3211264, 256, 64), (3211264, 64, 256), (3211264, 256, 128), (802816, 128, 512),
          (802816, 512, 128), (802816, 512, 256), (200704, 256, 1024), (200704, 1024, 256), (200704, 1024, 512),
          (50176, 512, 2048), (50176, 2048, 512)]


def check(out, ref_rows, rows):
    nf = int((~torch.isfinite(out)).sum().item())
    got = out[rows].float()
    err = float(((got - ref_rows).abs().max() / (ref_rows.abs().max() + 1e-6)).item())
    return nf, err


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tunableop", default="auto")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--miopen", type=int, default=0)
    ap.add_argument("--shapes", default="")
    a = ap.parse_args()
    mode = _tunableop.install(a.tunableop)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    shapes = SHAPES if not a.shapes else [tuple(int(v) for v in s.split("x")) for s in a.shapes.split(",")]
    res = []
    for (M, cin, cout) in shapes:
        x = torch.randn(M, cin, generator=g).to(dev, torch.bfloat16)
        w = (torch.randn(cout, cin, generator=g) / cin ** 0.5).to(dev, torch.bfloat16)
        dy = torch.randn(M, cout, generator=g).to(dev, torch.bfloat16)
        rows = torch.cat([torch.arange(0, 2048), torch.arange(M - 2048, M)]).to(dev)
        ref_f = x[rows].float() @ w.float().t()
        ref_d = dy[rows].float() @ w.float()
        bad = {"fwd_nf": 0, "dgrad_nf": 0, "fwd_err": 0.0, "dgrad_err": 0.0}
        for _ in range(a.reps):
            nf, e = check(torch.mm(x, w.t()), ref_f, rows)
            bad["fwd_nf"] += nf
            bad["fwd_err"] = max(bad["fwd_err"], e)
            nf, e = check(torch.mm(dy, w), ref_d, rows)
            bad["dgrad_nf"] += nf
            bad["dgrad_err"] = max(bad["dgrad_err"], e)
            if a.miopen:
                n = M // 3136 if M % 3136 == 0 else M // 784
                hw = int((M // n) ** 0.5)
                x4 = x.view(n, hw, hw, cin).permute(0, 3, 1, 2)
                w4 = w.view(cout, cin, 1, 1).contiguous(memory_format=torch.channels_last)
                y4 = F.conv2d(x4, w4)
                y2 = y4.permute(0, 2, 3, 1).reshape(M, cout)
                nf, e = check(y2, ref_f, rows)
                bad["miopen_fwd_nf"] = bad.get("miopen_fwd_nf", 0) + nf
                bad["miopen_fwd_err"] = max(bad.get("miopen_fwd_err", 0.0), e)
        torch.cuda.synchronize()
        rec = {"M": M, "cin": cin, "cout": cout, "tunableop": mode, **bad}
        print(json.dumps(rec), flush=True)
        res.append(rec)
        del x, w, dy
        torch.cuda.empty_cache()
    print(json.dumps({"any_nonfinite": any(r["fwd_nf"] or r["dgrad_nf"] or r.get("miopen_fwd_nf", 0) for r in res),
                      "max_err": max(max(r["fwd_err"], r["dgrad_err"]) for r in res)}))


if __name__ == "__main__":
    main()
