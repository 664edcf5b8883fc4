"""Ship tuned hipBLASLt / rocBLAS GEMM solution choices (PyTorch TunableOp) with the repo.

Every library GEMM this framework issues (the hipBLASLt side of ``ops/linear.py`` and the 1x1
convolutions of ``ops/conv.py``) goes through ``torch.mm`` / ``torch.addmm``. hipBLASLt's default
heuristic picks one solution per shape; TunableOp times every hipBLASLt and rocBLAS solution for
the shape instead and keeps the fastest. ``tuning/tunableop/gfx950.csv`` holds the choices made on
an MI355X for the bench shapes (``bench.py --tunableop tune``); ``install("use")`` loads it with
tuning off, so no timing runs during a bench or inside a hipGraph capture. Shapes that are not in
the file keep the library heuristic. The file carries TunableOp's validators (torch, ROCm,
hipBLASLt, rocBLAS versions and the gfx arch); on a mismatch TunableOp ignores it.
"""
from __future__ import annotations

import os


ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SHIPPED = os.path.join(ROOT, "tuning", "tunableop", "gfx950.csv")


def install(mode: str = "auto", path: str | None = None) -> str:
    """``auto``: use the shipped file when present; ``use``: load ``path`` (or the shipped file);
    ``tune``: time every solution for each new shape (results exported by ``dump``); ``off``."""
    import torch.cuda.tunable as tn

    if mode == "auto":
        mode = "use" if os.path.isfile(path or SHIPPED) else "off"
    if mode == "off":
        tn.enable(False)
        return "off"
    tn.enable(True)
    if mode == "tune":
        tn.tuning_enable(True)
        tn.set_max_tuning_duration(30)  # ms per GEMM shape
        tn.set_max_tuning_iterations(20)
        return "tune"
    tn.tuning_enable(False)
    tn.record_untuned_enable(False)
    try:
        ok = tn.read_file(path or SHIPPED)
    except Exception:  # unreadable / other library versions: keep the library heuristic
        ok = False
    if ok is False:
        tn.enable(False)
        return "off"
    return "use"


def dump(path: str) -> int:
    """Write TunableOp's in-memory results (validators + one line per tuned GEMM) to ``path``."""
    import torch.cuda.tunable as tn

    res = tn.get_results()
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        for k, v in tn.get_validators():
            f.write(f"Validator,{k},{v}\n")
        for op, params, kernel, ms in res:
            f.write(f"{op},{params},{kernel},{ms}\n")
    return len(res)


def merge(paths: list[str], out: str) -> int:
    """Union of several result files (the later file wins per (op, params)); validators from the first."""
    vals: list[str] = []
    rows: dict[tuple, str] = {}
    for i, p in enumerate(paths):
        for line in open(p):
            line = line.rstrip("\n")
            if not line:
                continue
            if line.startswith("Validator,"):
                if i == 0:
                    vals.append(line)
                continue
            parts = line.split(",")
            rows[(parts[0], parts[1])] = line
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    with open(out, "w") as f:
        f.write("\n".join(vals + list(rows.values())) + "\n")
    return len(rows)

