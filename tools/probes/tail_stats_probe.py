#!/usr/bin/env python3
"""Where does the recomputing tail's loss deviation come from?

ResNet-50, 64x64 images, batch 8, non-zero bn3 scales (the setting of
tests/test_tail.py::test_resnet_tail_matches_unfused). For every identity-block tail:
  * the conv3 input a2 and weight are captured, and the batch mean / biased variance of
    y = a2 W^T are computed in fp64 from the bf16 operands (exact up to fp64 rounding), and of
    bf16(y) (what the apply pass normalises);
  * both statistics routes of ops/tail.py run on the captured a2: "gram" (convw_gram_ + bnfold_gram_stats:
    sum y = W s, sum y^2 = W^T G W) and "pass" (the narrow kernel's statistics-only pass);
  * their mean / variance errors against fp64 are printed per layer.
Then the end-to-end loss: fp32 composite, unfused, tail (gram), tail (pass), each 3x, with the
autotune decisions of the first unfused run kept for every shared key.
"""
import copy
import sys

import torch
import torch.nn as nn

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__)))))

from parameter_server_distributed_amd import models, native  # noqa: E402
from parameter_server_distributed_amd.models import resnet as R  # noqa: E402
from parameter_server_distributed_amd.models.resnet import Bottleneck  # noqa: E402
from parameter_server_distributed_amd.ops import autotune, tail  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    C = native()
    torch.manual_seed(0)
    spec = models.build("resnet50", dev, torch.bfloat16, image_size=64, num_classes=10)
    for mod in spec.model.modules():
        if isinstance(mod, Bottleneck):
            nn.init.uniform_(mod.bn3.weight, 0.5, 1.5)
    for p in spec.model.parameters():
        p.data = p.data.to(torch.bfloat16)
    init = copy.deepcopy(spec.model.state_dict())
    m32 = copy.deepcopy(spec.model).float()  # before any forward leaves non-leaf tensors on modules
    x, y = spec.make_batch(8, dev, seed=3)

    caps = []
    orig = R.conv_bn_tail

    def cap(conv, bn, a2, idt, resid_to=None):
        caps.append((a2.detach().clone(), conv.weight.detach().clone(), bn))
        return orig(conv, bn, a2, idt, resid_to)

    R.conv_bn_tail = cap
    import os
    os.environ["PSD_FEATURES"] = "tail_recompute=1"
    spec.model.load_state_dict(init)
    spec.loss(spec.model(x), y).backward()
    R.conv_bn_tail = orig
    print(f"{len(caps)} tails captured")
    print("layer  M     cin cout | mean/std(fp64)  | gram: dmean/std dvar/var | pass: dmean/std dvar/var | bf16(y) vs y: dvar/var")
    worst = {"gram": 0.0, "pass": 0.0}
    for li, (a2, w, bn) in enumerate(caps):
        n, cin, h, wd = a2.shape
        cout = w.shape[0]
        M = n * h * wd
        w2 = w.reshape(cout, cin).contiguous()
        A = a2.permute(0, 2, 3, 1).reshape(M, cin)
        y64 = A.double() @ w2.double().t()
        mu, var = y64.mean(0), y64.var(0, unbiased=False)
        yb = y64.float().bfloat16().double()
        var_b = yb.var(0, unbiased=False)
        shift = torch.zeros(cout, device=dev)
        res = {}
        P = torch.empty(C.convw_gram_rows(cin), cin, device=dev, dtype=torch.float32)
        if C.convw_gram_(a2, P):
            row = torch.empty(2, cout, device=dev, dtype=torch.float32)
            C.bnfold_gram_stats(P, w2, shift, M, row)
            res["gram"] = row.double()
        v = 0
        rows = 0
        part = None
        for v in range(C.convn_variants(cout)):
            if C.convn_variant_kind(cout, v) in (0, 3) and C.convn_variant_ok(cout, v, 1, 1, 1, 0, wd):
                part = torch.empty(tail._part_rows(M, cout, v, h, wd, 1), 2, cout, device=dev, dtype=torch.float32)
                rows = C.convn_(a2, w2, part, 1, 1, 1, 0, part=part, shift=shift, variant=v, no_store=True)
                if rows:
                    break
        if rows:
            res["pass"] = part[:rows].double().sum(0)
        line = f"{li:5d} {M:5d} {cin:4d} {cout:4d} | {float((mu.abs() / var.sqrt().clamp_min(1e-30)).mean()):14.3f} |"
        for k in ("gram", "pass"):
            if k not in res:
                line += "   n/a                      |"
                continue
            s1, s2 = res[k][0], res[k][1]
            m_k = s1 / M
            v_k = s2 / M - m_k * m_k
            dm = float(((m_k - mu).abs() / var.sqrt().clamp_min(1e-30)).max())
            dv = float(((v_k - var).abs() / var.clamp_min(1e-30)).max())
            worst[k] = max(worst[k], dv)
            line += f" {dm:.2e} {dv:.2e}       |"
        line += f" {float(((var_b - var).abs() / var.clamp_min(1e-30)).max()):.2e}"
        print(line)
    print("worst relative variance error:", worst)

    def run(tail_on, fp32=False, stats=None):
        os.environ["PSD_FEATURES"] = f"tail_recompute={int(tail_on)}"
        for key in list(autotune._DECISIONS):
            if key[:2] == ("tail", "stats"):
                del autotune._DECISIONS[key]
        if stats is not None:
            os.environ["PSD_AUTOTUNE_FORCE"] = stats
        m = m32 if fp32 else spec.model
        m.load_state_dict(init)
        m.zero_grad(set_to_none=True)
        loss = spec.loss(m(x.float() if fp32 else x), y)
        loss.backward()
        loss = float(loss)
        os.environ.pop("PSD_AUTOTUNE_FORCE", None)
        return loss

    ref = run(False, fp32=True)
    out = {"fp32": [ref]}
    for name, kw in (("unfused", dict(tail_on=False)), ("tail_auto", dict(tail_on=True)),
                     ("tail_gram", dict(tail_on=True, stats="gram")),
                     ("tail_pass", dict(tail_on=True, stats="pass")), ("unfused_again", dict(tail_on=False))):
        out[name] = [run(**kw) for _ in range(3)]
    for k, v in out.items():
        print(f"loss {k:14s} " + " ".join(f"{l:.5f}" for l in v) + f"   (vs fp32 {max(abs(l - ref) for l in v) / ref:.2%})")

    # how chaotic is this setting? the fp32 model's loss under bf16-rounding-sized perturbations
    # (relative noise 2^-9 on the input / on every weight)
    def fp32_loss(xin, noise_w=0.0, seed=0):
        m32.load_state_dict(init)
        if noise_w:
            g = torch.Generator(device=dev).manual_seed(seed)
            with torch.no_grad():
                for p_ in m32.parameters():
                    p_.mul_(1 + noise_w * torch.randn(p_.shape, device=dev, generator=g))
        with torch.no_grad():
            return float(spec.loss(m32(xin), y))
    g = torch.Generator(device=dev).manual_seed(7)
    xs = [x.float() * (1 + 2 ** -9 * torch.randn(x.shape, device=dev, generator=g)) for _ in range(3)]
    print("fp32 loss, input x (1 + 2^-9 noise):", " ".join(f"{fp32_loss(xi):.5f}" for xi in xs))
    print("fp32 loss, weights x (1 + 2^-9 noise):", " ".join(f"{fp32_loss(x.float(), 2 ** -9, s):.5f}" for s in range(3)))
    print("fp32 loss, x rounded to bf16 only:", f"{fp32_loss(x.float()):.5f}", "(x is bf16 already)")


if __name__ == "__main__":
    main()
