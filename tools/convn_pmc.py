#!/usr/bin/env python3
"""Launch the narrow implicit-GEMM convolution (kernels/convn.hip) on the ResNet-50 b1024 layer1
shapes a few times per variant, for rocprofv3 --pmc passes (one counter group per run):

  rocprofv3 --pmc SQ_WAVE_CYCLES ... --output-format csv -d out -- python3 tools/convn_pmc.py

Shapes: layer1 3x3 64->64 (every plain variant; the kernel name carries the tile template, so the
rows of the counter table separate them) and layer1 conv3 1x1 64->256 with / without the statistics
epilogue. PMC_BATCH overrides the batch (default 1024).
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from parameter_server_distributed_amd import native  # noqa: E402


def main():
    C_ = native()
    dev = torch.device("cuda")
    cl = dict(memory_format=torch.channels_last)
    N = int(os.environ.get("PMC_BATCH", "1024"))
    reps = int(os.environ.get("PMC_REPS", "3"))
    only = os.environ.get("PMC_VARIANTS")
    torch.manual_seed(0)
    for (cin, cout, R) in ((64, 64, 3), (64, 256, 1)):
        x = torch.randn(N, cin, 56, 56, device=dev).to(torch.bfloat16).contiguous(**cl)
        w = (torch.randn(cout, cin, R, R, device=dev) * 0.05).to(torch.bfloat16)
        w2 = w.permute(0, 2, 3, 1).reshape(cout, -1).contiguous()
        M = N * 56 * 56
        out = torch.empty(M, cout, device=dev, dtype=torch.bfloat16)
        shift = torch.zeros(cout, device=dev)
        for v in range(C_.convn_variants(cout)):
            if only and str(v) not in only.split(","):
                continue
            if not C_.convn_variant_ok(cout, v, R, R, 1, R // 2, 56):
                continue
            part = torch.empty(max(C_.convn_stats_rows(M), C_.convn_part_rows(M, cout, v, 56, 56, R)), 2, cout,
                               device=dev)
            for _ in range(reps):
                C_.convn_(x, w2, out, R, R, 1, R // 2, variant=v)
            if R == 1:
                for _ in range(reps):
                    C_.convn_(x, w2, out, R, R, 1, 0, part=part, shift=shift, variant=v)
        del x, w, w2, out
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
