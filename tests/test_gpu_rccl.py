"""The RCCL transport on the real library, one rank: grouped self
send/recv eagerly and inside a captured hipGraph (the way the solver's
passes are replayed), plus the all-reduce.  Multi-rank RCCL on one GPU (one
RCCL host id per rank, socket transport) is test_gpu_rccl_multirank.py."""
import ctypes

import pytest

from parallel_heat_amd import _native

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("graph", [0, 1])
@pytest.mark.parametrize("nbytes", [4, 272 * 1024, 4 << 20])
def test_rccl_self_sendrecv(gpu, graph, nbytes):
    g = ctypes.c_double()
    _native.call("heat_rccl_self_test", 0, nbytes, graph, 20, ctypes.byref(g))
    assert g.value > 0
