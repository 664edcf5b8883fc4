"""In-tree native build: gfx950 HIP kernels + C++ runtime cores -> ``parameter_server_distributed_amd/_C.so``.

Why a hand-rolled builder instead of ``torch.utils.cpp_extension.CUDAExtension``: on ROCm that
path runs hipify over the sources; ours are written in HIP for CDNA4 directly and must be compiled
as-is. Device code (``csrc/kernels/*.hip``) goes through ``hipcc --offload-arch=gfx950``; the host
runtime (``csrc/*.cpp``) through the host C++ compiler against the torch headers; everything is
linked against the *torch-bundled* ROCm runtime (libamdhip64 / librccl in ``torch/lib``) so that
the process only ever holds one HIP runtime.

Rebuilds are incremental: each object records a hash of its source, the headers it may include
and the flags.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
BUILD = PKG.parent / "build" / "native"
OUT = PKG / "_C.so"
ARCH = os.environ.get("PSD_OFFLOAD_ARCH", "gfx950")


def _rocm() -> Path:
    return Path(os.environ.get("ROCM_PATH", "/opt/rocm"))


def _torch_paths():
    import torch  # noqa: F401  (import first: its HIP runtime must be the one we link)
    import torch.utils.cpp_extension as ce

    inc = ce.include_paths()
    lib = Path(ce.library_paths()[0])
    return inc, lib


def _headers() -> list[Path]:
    return sorted(list(CSRC.rglob("*.h")))


def _digest(src: Path, flags: list[str]) -> str:
    h = hashlib.sha256()
    h.update(src.read_bytes())
    for hd in _headers():
        h.update(hd.read_bytes())
    h.update(" ".join(flags).encode())
    return h.hexdigest()


def _compile(cmd: list[str], src: Path, obj: Path, flags_for_hash: list[str], verbose: bool) -> str:
    stamp = obj.with_suffix(obj.suffix + ".sha")
    dg = _digest(src, flags_for_hash)
    if obj.exists() and stamp.exists() and stamp.read_text() == dg:
        return f"up-to-date {src.name}"
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {src}\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    stamp.write_text(dg)
    return f"built {src.name}"


def build(verbose: bool = False, jobs: int | None = None, force: bool = False) -> Path:
    inc, torch_lib = _torch_paths()
    BUILD.mkdir(parents=True, exist_ok=True)
    if force:
        for p in BUILD.glob("*"):
            p.unlink()
    rocm = _rocm()
    hipcc = str(rocm / "bin" / "hipcc")
    cxx = shutil.which("g++") or "c++"
    py_inc = sysconfig.get_paths()["include"]

    hip_flags = [
        f"--offload-arch={ARCH}", "-O3", "-fPIC", "-std=c++17", "-I", str(CSRC), "-I", str(CSRC / "kernels"),
        "-munsafe-fp-atomics", "-Wno-unused-result",
    ]
    import torch

    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    cxx_flags = [
        "-O2", "-fPIC", "-std=c++17", "-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1",
        "-DTORCH_EXTENSION_NAME=_C", "-DTORCH_API_INCLUDE_EXTENSION_H", f"-D_GLIBCXX_USE_CXX11_ABI={abi}",
        "-I", str(CSRC), "-I", py_inc, "-isystem", str(rocm / "include"), "-Wno-deprecated-declarations",
        "-fvisibility=hidden",
    ]
    for p in inc:
        cxx_flags += ["-isystem", p]

    jobs_list = []
    for src in sorted(CSRC.rglob("*.hip")):
        obj = BUILD / (src.stem + ".hip.o")
        jobs_list.append(([hipcc, *hip_flags, "-c", str(src), "-o", str(obj)], src, obj, hip_flags))
    for src in sorted(CSRC.glob("*.cpp")):
        obj = BUILD / (src.stem + ".o")
        jobs_list.append(([cxx, *cxx_flags, "-c", str(src), "-o", str(obj)], src, obj, cxx_flags))

    n = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(max_workers=n) as ex:
        futs = [ex.submit(_compile, c, s, o, f, verbose) for (c, s, o, f) in jobs_list]
        for f in futs:
            msg = f.result()
            if verbose:
                print(msg, flush=True)

    objs = [str(o) for (_, _, o, _) in jobs_list]
    link_stamp = BUILD / "link.sha"
    h = hashlib.sha256()
    for o in objs:
        h.update(Path(o).read_bytes())
    dg = h.hexdigest()
    if OUT.exists() and link_stamp.exists() and link_stamp.read_text() == dg:
        return OUT
    tmp = OUT.with_name(f"_C.so.{os.getpid()}.tmp")
    cmd = [
        cxx, "-shared", "-o", str(tmp), *objs,
        f"-L{torch_lib}", "-lc10", "-ltorch", "-ltorch_cpu", "-ltorch_python", "-lc10_hip", "-ltorch_hip",
        "-lamdhip64", "-lrccl", f"-Wl,-rpath,{torch_lib}", "-Wl,--no-as-needed",
    ]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, OUT)
    link_stamp.write_text(dg)
    return OUT


if __name__ == "__main__":
    out = build(verbose="-v" in sys.argv, force="--force" in sys.argv)
    print(out)
