"""Host-side AddressSanitizer run of the library's C++ (SURVEY §5 sanitizers row): every .hip file's
host half built with -fsanitize=address (tools/asan_host.py: --cuda-host-only, no device code),
then the C-ABI's planning entry points and every launch entry's argument validation exercised with
valid and refused arguments in a child process with the ASan runtime preloaded.  CPU only."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))


def test_host_code_is_asan_clean():
    import asan_host
    if asan_host.asan_runtime() is None:
        pytest.skip("no ASan runtime in this ROCm image")
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "asan_host.py")], capture_output=True, text=True,
                       timeout=900)
    out = r.stdout + r.stderr
    assert "ERROR: AddressSanitizer" not in out, out[-4000:]
    assert r.returncode == 0, out[-4000:]
    assert "asan host checks:" in r.stdout and "clean" in r.stdout
