#!/usr/bin/env python3
"""Launch the hand-written ResNet-50 b1024 hot kernels a few times each, for rocprofv3 --pmc passes:
stem conv fwd (+BN finalize, fused BN/ReLU/pool), stem wgrad, pool-fused BN backward, and a
layer1-sized residual BN forward / backward (csrc/kernels/stem.hip, bn.hip).

  rocprofv3 --pmc SQ_WAVE_CYCLES ... --output-format csv -d out -- python3 tools/kernel_pmc.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from parameter_server_distributed_amd import native  # noqa: E402


def main():
    C = native()
    dev = torch.device("cuda")
    cl = dict(memory_format=torch.channels_last)
    N = int(os.environ.get("PMC_BATCH", "1024"))
    torch.manual_seed(0)
    x = torch.randn(N, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(**cl)
    w = (torch.randn(64, 3, 7, 7, device=dev) * 0.1).to(torch.bfloat16).contiguous(**cl)
    g = torch.ones(64, device=dev, dtype=torch.bfloat16)
    b = torch.zeros(64, device=dev, dtype=torch.bfloat16)
    rm, rv = torch.zeros(64, device=dev), torch.ones(64, device=dev)
    for _ in range(3):
        y, arg, mean, invstd, ss, conv = C.stem_fwd(x, w, g, b, rm, rv, 0.1, 1e-5)
        gy = torch.randn_like(y)
        dconv, dg, db = C.bn_pool_bwd(gy, None, arg, conv, g, mean, invstd, ss)
        C.stem_wgrad(x, dconv)
    del x, y, arg, conv, gy, dconv
    M, Ch = N * 3136, 256
    xb = torch.randn(M, Ch, device=dev, dtype=torch.bfloat16)
    r = torch.randn_like(xb)
    g2 = torch.ones(Ch, device=dev, dtype=torch.bfloat16)
    b2 = torch.zeros(Ch, device=dev, dtype=torch.bfloat16)
    rm2, rv2 = torch.zeros(Ch, device=dev), torch.ones(Ch, device=dev)
    dgb, dbb = torch.empty_like(g2), torch.empty_like(g2)
    for _ in range(3):
        yb, mb, ib, ssb, bits = C.bn_fwd(xb, g2, b2, rm2, rv2, r, True, True, 0.1, 1e-5, None, None, mask_out=True)
        C.bn_bwd(r, xb, None, g2, mb, ib, True, True, dgb, dbb, yb, None, bits)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
