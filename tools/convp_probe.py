#!/usr/bin/env python3
"""Run one narrow-conv 1x1 pass repeatedly (for rocprofv3 PMC passes): layer1 tail shapes
(M = 1024 x 56 x 56, 64 -> 256), the persistent 1x1 variant by default.
  python tools/convp_probe.py [--pass stats|apply|fwd] [--variant -1 (= persistent)] [--reps 5]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from parameter_server_distributed_amd import native  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--pass", dest="ps", default="stats")
ap.add_argument("--variant", type=int, default=-1)
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--cin", type=int, default=64)
ap.add_argument("--cout", type=int, default=256)
ap.add_argument("--hw", type=int, default=56)
a = ap.parse_args()
C = native()
dev = torch.device("cuda")
B, hw, cin, cout = 1024, a.hw, a.cin, a.cout
M = B * hw * hw
v = a.variant if a.variant >= 0 else [u for u in range(C.convn_variants(cout)) if C.convn_variant_kind(cout, u) == 3][0]
x = torch.randn(B, cin, hw, hw, device=dev).relu().bfloat16().contiguous(memory_format=torch.channels_last)
w = (torch.randn(cout, cin, device=dev) * 0.05).bfloat16()
part = torch.empty(max(C.convn_stats_rows(M), C.convn_part_rows(M, cout, v, hw, hw, 1)), 2, cout, device=dev)
shift = torch.zeros(cout, device=dev)
out = torch.empty(M, cout, device=dev, dtype=torch.bfloat16)
res = torch.randn(M, cout, device=dev).bfloat16()
mb = torch.empty(M * cout // 8, device=dev, dtype=torch.uint8)
ss = torch.randn(2 * cout, device=dev)
for _ in range(a.reps):
    if a.ps == "stats":
        C.convn_(x, w, part, 1, 1, 1, 0, part=part, shift=shift, variant=v, no_store=True)
    elif a.ps == "apply":
        C.convn_(x, w, out, 1, 1, 1, 0, variant=v, apply_ss=ss, apply_res=res, apply_mask=mb)
    else:
        C.convn_(x, w, out, 1, 1, 1, 0, part=part, shift=shift, variant=v)
torch.cuda.synchronize()
print("ok", a.ps, v)
