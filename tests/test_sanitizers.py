"""Race detection / memory safety for the host-side C++ cores: the std-only
Registry + StalenessTracker under ThreadSanitizer and Address+UndefinedBehaviorSanitizer, driven by a
multi-threaded stress program (csrc/tests/host_stress.cpp). Host code only (GPU sanitizers are not
available on the MI355X pool)."""
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
