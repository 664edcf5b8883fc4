"""Shipped TunableOp results (utils/tunableop.py): the file parses, carries the validators of this
image, and merge() keeps the validators of the first file and the last row per (op, params)."""
import os

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
