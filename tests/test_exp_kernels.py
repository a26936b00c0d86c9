"""The experiment kernels' library (csrc/kernels/tb_exp.hpp, `make exp`):
the measured-slower TB builds live in libheat_exp.so, not in the product
library, and register with it when loaded.  CPU only (no launch)."""
import os
import subprocess
import sys

import pytest

from parallel_heat_amd import _native

SYMS = ("tbp", "tbn", "tbxm", "tbxnp", "tbc")



def test_product_library_carries_no_experiment_kernels():
    sys.path.insert(0, os.path.join(str(_native.REPO_DIR), "tools"))
    try:
        names = [k["name"] for k in __import__("kernel_resources").kernels(str(_native.LIB_PATH))]
        exp = [k["name"] for k in __import__("kernel_resources").kernels(str(_native.EXP_PATH))]
    except Exception as e:  # noqa: BLE001 - toolchain missing
        pytest.skip(f"cannot read code objects: {e}")
    for ns in SYMS:
        tag = f"_ZN4heat3gpu{len(ns)}{ns}"
        assert not any(n.startswith(tag) for n in names), ns
        assert any(n.startswith(tag) for n in exp), ns


def test_exp_library_registers_when_loaded():
    # A fresh interpreter: nothing registered until load_exp().
    code = ("from parallel_heat_amd import _native as n; a = n.lib().heat_tb_exp_loaded(); "
            "n.load_exp(); b = n.lib().heat_tb_exp_loaded(); n.unload_exp(); "
            "c = n.lib().heat_tb_exp_loaded(); n.load_exp(); "
            "print(a, b, c, n.lib().heat_tb_exp_loaded())")
    env = dict(os.environ, PYTHONPATH=str(_native.REPO_DIR))
    env.pop("HEAT_EXP", None)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env,
                         timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.split() == ["0", "1", "0", "1"]
    out = subprocess.run([sys.executable, "-c", "from parallel_heat_amd import _native as n; "
                          "print(n.lib().heat_tb_exp_loaded())"], capture_output=True, text=True,
                         env=dict(env, HEAT_EXP="1"), timeout=300)
    assert out.stdout.split() == ["1"], out.stderr[-2000:]
