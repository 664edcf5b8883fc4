"""Shipped TunableOp results (utils/tunableop.py): the file parses, carries the validators of this
image, and merge() keeps the validators of the first file and the last row per (op, params)."""
import os

import pytest

from parameter_server_distributed_amd.utils import tunableop as t


def test_shipped_file_has_validators_and_rows():
    assert os.path.isfile(t.SHIPPED)
    lines = [line.rstrip("\n") for line in open(t.SHIPPED) if line.strip()]
    vals = dict(line.split(",", 2)[1:] for line in lines if line.startswith("Validator,"))
    assert vals.get("GCN_ARCH_NAME", "").startswith("gfx950")
    assert "PT_VERSION" in vals and "HIPBLASLT_VERSION" in vals
    rows = [line.split(",") for line in lines if not line.startswith("Validator,")]
    assert rows and all(len(r) == 4 and r[0].startswith("Gemm") for r in rows)
    assert all(float(r[3]) > 0 for r in rows)


def test_merge(tmp_path):
    a, b, out = tmp_path / "a.csv", tmp_path / "b.csv", tmp_path / "m.csv"
    a.write_text("Validator,PT_VERSION,1\nGemmX,nt_1_2_3,Gemm_Hipblaslt_1,0.5\nGemmX,nt_4_5_6,Gemm_Rocblas_2,0.7\n")
    b.write_text("Validator,PT_VERSION,2\nGemmX,nt_1_2_3,Gemm_Hipblaslt_9,0.4\n")
    assert t.merge([str(a), str(b)], str(out)) == 2
    text = out.read_text()
    assert "Validator,PT_VERSION,1" in text and "PT_VERSION,2" not in text
    assert "Gemm_Hipblaslt_9" in text and "Gemm_Hipblaslt_1" not in text and "Gemm_Rocblas_2" in text


def _operands(layout: str, m: int, n: int, k: int, dev):
    """torch.mm operands reproducing a TunableOp (column-major BLAS) GEMM row: returns (P, Q) with
    torch.mm(P, Q) issuing op(A)[m,k] . op(B)[k,n] = C[m,n] col-major == row-major [n, m]."""
    import torch

    g = torch.Generator(device=dev).manual_seed(m * 31 + n * 7 + k)
    r = lambda *s: torch.randn(*s, generator=g, device=dev, dtype=torch.bfloat16)  # noqa: E731
    ta, tb = layout[0], layout[1]
    # row-major C^T[n, m] = op(B)^T[n, k] . op(A)^T[k, m]
    bt = r(n, k) if tb == "n" else r(k, n).t()   # B col-major k x n == row-major [n][k]
    at = r(m, k).t() if ta == "t" else r(k, m)   # A col-major m x k == row-major [k][m]
    return bt, at


@pytest.mark.gpu
def test_shipped_tunableop_rows_agree_with_library_default(gpu):
    """Every GEMM solution in the shipped TunableOp file must compute the same product as the
    library's default heuristic (a recorded hipBLASLt solution once returned NaN rows for ResNet-50's
    layer1 conv3 at b1024; README 'Round-2 fix')."""
    import torch
    import torch.cuda.tunable as tn

    assert t.install("use") == "use"
    rows = [line.strip().split(",") for line in open(t.SHIPPED) if line.strip() and not line.startswith("Validator")]
    bad = []
    for op, params, kernel, _ in rows:
        if not op.startswith("GemmTunableOp_BFloat16_"):
            continue
        f = params.split("_")
        layout, m, n, k = f[0], int(f[1]), int(f[2]), int(f[3])
        P, Q = _operands(layout, m, n, k, gpu)
        tn.enable(True)
        outs = [torch.mm(P, Q) for _ in range(3)]
        tn.enable(False)
        ref = torch.mm(P, Q).float()
        for o in outs:
            o = o.float()
            err = float((o - ref).abs().max() / (ref.abs().max() + 1e-6))
            if not bool(torch.isfinite(o).all()) or err > 2e-2:
                bad.append((params, kernel, err))
                break
    tn.enable(True)
    assert not bad, bad
