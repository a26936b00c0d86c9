"""The native C++ self-test, plain and under AddressSanitizer/UBSan (host code)."""
import subprocess

import pytest

from parallel_heat_amd import _native


@pytest.mark.parametrize("target", ["selftest", "selftest-asan"])
def test_native_selftest(target):
    p = subprocess.run(["make", "-s", "-C", str(_native.REPO_DIR), target], capture_output=True,
                       text=True, timeout=600)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "selftest: ok" in p.stdout
