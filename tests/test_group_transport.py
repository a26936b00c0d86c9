"""Single-process multi-rank runs (`heat --gpus N`, parallel.group.run_group):
which transport the shared native rule picks (heat::choose_group_transport,
SURVEY R10 / §2.4: one process owning N GPUs over RCCL, the ncclCommInitAll
model that replaces mpi/mpi_heat_improved_persistent_stat.c:48-69).  CPU
only: the rule needs no device."""
import pytest

from parallel_heat_amd import _native
from parallel_heat_amd.models.config import HeatConfig
from parallel_heat_amd.parallel import comm as pcomm
from parallel_heat_amd.parallel.group import default_devices


@pytest.mark.parametrize("devices,want", [
    ([0, 1], "rccl"),                      # a GPU per rank
    (list(range(8)), "rccl"),              # one node, 8 ranks
    ([3, 0, 5], "rccl"),                   # any distinct devices
    ([0, 0], "loopback"),                  # ranks sharing one GPU
    ([0, 1, 0, 1], "loopback"),            # 4 ranks on 2 GPUs
    ([0], "loopback"),                     # one rank: no communicator needed
])
def test_auto_choice(devices, want):
    assert pcomm.group_transport("auto", devices) == want


def test_forced_choices():
    assert pcomm.group_transport("loopback", [0, 1]) == "loopback"
    assert pcomm.group_transport("rccl", [0, 1, 2]) == "rccl"
    with pytest.raises(_native.NativeError, match="one GPU per rank"):
        pcomm.group_transport("rccl", [0, 0])
    with pytest.raises(_native.NativeError, match="unknown group transport"):
        pcomm.group_transport("tcp", [0, 1])
    with pytest.raises(_native.NativeError, match="no device"):
        pcomm.group_transport("auto", [0, -1])


def test_default_devices(monkeypatch):
    monkeypatch.setattr(_native, "device_count", lambda: 8)
    assert default_devices(HeatConfig(backend="hip"), 4) == [0, 1, 2, 3]
    assert default_devices(HeatConfig(backend="hip"), 10) == [0, 1, 2, 3, 4, 5, 6, 7, 0, 1]
    assert default_devices(HeatConfig(backend="hip", device=2), 3) == [2, 2, 2]
    monkeypatch.setattr(_native, "device_count", lambda: 1)
    devs = default_devices(HeatConfig(backend="hip"), 3)
    assert devs == [0, 0, 0] and pcomm.group_transport("auto", devs) == "loopback"
    monkeypatch.setattr(_native, "device_count", lambda: 8)
    assert pcomm.group_transport("auto", default_devices(HeatConfig(backend="hip"), 8)) == "rccl"


def test_cli_gpus_reports_transport_rule():
    # The native CLI refuses --transport rccl when ranks would share devices
    # (here: no GPU at all, so the rule itself is not reached; the flag parses).
    import subprocess
    p = subprocess.run([str(_native.CLI_PATH), "--help"], capture_output=True, text=True)
    assert "--watchdog" in p.stdout and "RCCL (one rank per" in p.stdout
