"""Race detection / memory safety for the host-side C++ cores under
ThreadSanitizer and Address+UndefinedBehaviorSanitizer:

* the std-only Registry + StalenessTracker (csrc/tests/host_stress.cpp);
* PSCore -- mutex + condition variable + slot pool + SSP clocks + checkpoint writer, the C1
  ParameterServerCore counterpart -- on CPU tensors, linked against libtorch
  (csrc/tests/ps_core_stress.cpp; the gfx950 launchers are stubs, only CPU tensors reach them);
* the asynchronous apply-on-arrival engine on host shared memory (csrc/tests/async_stress.cpp).

Host code only (GPU sanitizers are not available on the MI355X pool)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "parameter_server_distributed_amd", "csrc")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_host_cores_under_sanitizer(tmp_path, san):
    exe = str(tmp_path / "stress")
    cmd = ["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer",
           os.path.join(CSRC, "tests", "host_stress.cpp"), os.path.join(CSRC, "registry.cpp"), "-o", exe, "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="halt_on_error=1 detect_leaks=1", UBSAN_OPTIONS="halt_on_error=1 print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok epochs=" in r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr


def _torch_flags():
    import torch
    import torch.utils.cpp_extension as ce

    tl = os.path.dirname(torch.__file__)
    inc = []
    for p in ce.include_paths():
        inc += ["-isystem", p]
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return (["-D__HIP_PLATFORM_AMD__=1", "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-I", CSRC,
             "-isystem", "/opt/rocm/include"] + inc,
            [f"-L{tl}/lib", "-lc10", "-ltorch_cpu", "-lc10_hip", "-lamdhip64", "-L/opt/rocm/lib",
             f"-Wl,-rpath,{tl}/lib", "-Wl,-rpath,/opt/rocm/lib", "-lpthread"])


TARGETS = {
    # PSCore: sync barrier + async SSP push/pull from 4 threads, concurrent status / checkpoint /
    # membership calls (PSCore was never run under TSAN)
    "pscore": (["ps_core_stress.cpp", "ps_core.cpp", "checkpoint.cpp"],
               ["sync ok version=40 failures=0", "async ok version=160 failures=0"]),
    # AsyncEngine on host memory: worker thread pull/push/commit vs the engine's apply thread
    # (shared-memory rings, reader pins, version/clock atomics) vs a monitor thread
    "async": (["async_stress.cpp", "async_ps.cpp"], ["ok async applies=600 v0=300 v1=300 err=''"]),
}


@pytest.mark.slow
@pytest.mark.parametrize("target", list(TARGETS))
@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_torch_cores_under_sanitizer(tmp_path, san, target):
    cflags, ldflags = _torch_flags()
    exe = str(tmp_path / "stress")
    files, want = TARGETS[target]
    srcs = [os.path.join(CSRC, "tests", files[0]), os.path.join(CSRC, "tests", "launcher_stubs.cpp"),
            os.path.join(CSRC, "ops.cpp")] + [os.path.join(CSRC, f) for f in files[1:]]
    cmd = ["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer", "-w", *cflags, *srcs,
           "-o", exe, *ldflags]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="halt_on_error=1 detect_leaks=0", UBSAN_OPTIONS="halt_on_error=1 print_stacktrace=1",
               OMP_NUM_THREADS="1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr[-6000:]
    for w in want:
        assert w in r.stdout, r.stdout
    assert "WARNING: ThreadSanitizer" not in r.stderr and "ERROR: AddressSanitizer" not in r.stderr
