"""Multi-rank RCCL on ONE MI355X: 2-3 processes share cuda:0, each claiming
its own RCCL host id (``NCCL_HOSTID``), so RCCL's duplicate-device check
passes and the ranks talk over its socket transport on loopback.  The engine
code is the multi-GPU path exactly: its own communicator from a broadcast
unique id, grouped ncclSend/ncclRecv of device halo buffers and
ncclAllReduce(max) for the residual, captured into the segment hipGraphs
(or eager), deep halos, all three schedules.  Results must equal the
single-rank run bit for bit.  Only the wire differs from an 8-GPU node
(sockets instead of xGMI)."""
import numpy as np
import pytest

from parallel_heat_amd import HeatConfig, HeatSolver

from .dist_worker import run_tune, run_world

pytestmark = pytest.mark.gpu

BASE = dict(nx=150, ny=300, steps=0, init="random", seed=5, backend="hip", tb_depth=8)


def single(base, steps):
    with HeatSolver(HeatConfig(**{**base, "decomp": "auto", "px": 0, "py": 0})) as s:
        r = s.run(steps)
        return s.gather(), r, s.checksum()["hash"]


@pytest.mark.parametrize("world,kw", [
    (2, dict(decomp="rows", schedule="sync")),
    (2, dict(px=1, py=2, schedule="overlap")),
    (3, dict(decomp="rows", schedule="pipeline")),
    (4, dict(px=2, py=2, schedule="sync")),  # ghost corners from the diagonal ranks
    (2, dict(decomp="rows", schedule="sync", use_graph=False)),
])
def test_rccl_ranks_one_device(gpu, tmp_path, world, kw):
    base = {**BASE, **kw}
    res = run_world(world, base, 0, tmp_path, transport="rccl", chunks=[45, 7, 30])
    ref, _, h = single(base, 82)
    assert int(res["done"]) == 82
    assert np.array_equal(res["grid"], ref)
    assert str(res["hash"]) == h


def test_rccl_convergence_allreduce(gpu, tmp_path):
    kw = dict(nx=40, ny=26, steps=40000, converge=True, check_interval=20, eps=1e-3,
              backend="hip", tb_depth=8, decomp="rows")
    res = run_world(2, kw, 40000, tmp_path, transport="rccl")
    ref, r, _ = single(kw, 40000)
    assert bool(res["conv"]) == r.converged
    assert int(res["conv_at"]) == r.converged_at and int(res["done"]) == r.steps_done
    assert np.array_equal(res["grid"], ref)


def test_rccl_bench_shape(gpu, tmp_path):
    # bench.py in miniature: rows slabs, auto depth/halo, repeated runs of
    # one "step" replayed from cached graphs with the residual all-reduce.
    base = dict(nx=1024, ny=768, steps=0, init="random", seed=1234, backend="hip",
                decomp="rows", converge=True, check_interval=50, eps=1e-12)
    res = run_world(2, base, 0, tmp_path, transport="rccl", chunks=[200] * 4)
    with HeatSolver(HeatConfig(**{**base, "decomp": "auto"})) as s:
        for _ in range(4):
            s.run(200)
        ref, h = s.gather(), s.checksum()["hash"]
    assert int(res["done"]) == 800
    assert np.array_equal(res["grid"], ref)
    assert str(res["hash"]) == h


def test_rccl_autotune(gpu, tmp_path):
    res = run_tune(2, dict(nx=256, ny=512, steps=0, init="random", seed=3, backend="hip"),
                   tmp_path, transport="rccl")
    assert res["choices"][0] == res["choices"][1]
    assert all("ms_per_1000_iters" in r for r in res["table"])


@pytest.mark.parametrize("schedule", ["pipeline", "overlap"])
def test_rccl_schedule_convergence_graph(gpu, tmp_path, schedule):
    # The overlap schedules under graph capture with the residual all-reduce
    # and the device-judged gate (mpi/...c:235-262): under capture the
    # interior launch runs on the forked comm stream and is joined before the
    # all-reduce reads the residual word (Solver::enqueue_pass).
    kw = dict(nx=64, ny=48, steps=40000, converge=True, check_interval=20, eps=1e-3,
              init="ref-wrap", backend="hip", tb_depth=8, decomp="rows", schedule=schedule,
              use_graph=True)
    res = run_world(2, kw, 40000, tmp_path, transport="rccl")
    ref, r, _ = single(kw, 40000)
    assert str(res["schedule"]) == schedule
    assert r.converged and bool(res["conv"])
    assert int(res["conv_at"]) == r.converged_at and int(res["done"]) == r.steps_done
    assert np.array_equal(res["grid"], ref)


def test_rccl_dead_peer_fails_fast(gpu, tmp_path):
    # Rank 1 dies at its 4th transport call (HEAT_TEST_FAIL_AFTER=3: the
    # warm-up exchange and all-reduce pass, the first captured segment does
    # not).  Rank 0 has launched that segment and waits on the device for
    # halo rows that never come; its watchdog (HEAT_WATCHDOG_S) aborts the
    # communicator and the process exits non-zero instead of hanging like
    # the reference's MPI_Allreduce (mpi/...c:255) would.
    import os
    import subprocess
    import time

    from parallel_heat_amd import _native

    from .dist_worker import free_port

    env0 = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()),
                WORLD_SIZE="2", HEAT_WATCHDOG_S="10", NCCL_SOCKET_IFNAME="lo",
                NCCL_IB_DISABLE="1")
    cmd = [str(_native.CLI_PATH), "--backend", "hip", "--nx", "512", "--ny", "256",
           "--steps", "2000000", "--converge", "--check-interval", "50", "--eps", "0",
           "--decomp", "rows", "--out", "none", "--json"]
    procs = []
    for r in range(2):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r), NCCL_HOSTID=f"heat-rank-{r}")
        if r == 1:
            env["HEAT_TEST_FAIL_AFTER"] = "3"
        procs.append(subprocess.Popen(cmd, env=env, cwd=tmp_path, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    t0 = time.time()
    outs = [None, None]
    try:
        outs[1] = procs[1].communicate(timeout=60)
        outs[0] = procs[0].communicate(timeout=60)
    except subprocess.TimeoutExpired:
        for p in procs:
            if p.poll() is None:
                p.kill()
        tails = [p.communicate()[1][-1500:] for p in procs]
        pytest.fail(f"rank(s) still running after 60 s; rank 0 stderr: {tails[0]!r}; "
                    f"rank 1 stderr: {tails[1]!r}")
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    (out0, err0), (out1, err1) = outs
    elapsed = time.time() - t0
    assert procs[1].returncode != 0 and "injected transport failure" in err1, err1[-2000:]
    assert procs[0].returncode != 0, (out0[-500:], err0[-2000:])
    assert "no progress" in err0 or "RCCL" in err0 or "aborted" in err0, err0[-2000:]
    assert elapsed < 60


def test_rccl_abort_while_calls_run(gpu):
    # RcclTransport::abort() freed the communicator while
    # another thread could be between its liveness check and its next RCCL
    # call.  Calls now announce themselves and re-check the abort flag; an
    # abort waits for calls already inside RCCL.  20 rounds of a thread
    # issuing send/recv + all-reduce back to back while this thread aborts:
    # every round ends with the worker's calls refused, nothing crashes.
    import ctypes

    from parallel_heat_amd import _native
    calls = ctypes.c_int()
    _native.call("heat_rccl_abort_race_test", 0, 20, ctypes.byref(calls))
    assert calls.value > 0


@pytest.mark.parametrize("world,kw", [
    (2, dict(decomp="rows")),
    (4, dict(px=2, py=2)),  # ghost corners, 2-D span boxes
])
def test_rccl_resident_spans_converge_inside(gpu, tmp_path, world, kw):
    # The sequence a real multi-GPU run executes: resident-tile launches (m
    # passes each, tiles kept in VGPRs) with grouped RCCL exchanges between
    # them, captured in the segment graphs, checks every 20 steps inside the
    # spans, one all-reduce + device judge per span.  Separate processes, one
    # RCCL host id each (socket transport on one GPU); HEAT_TB_RESIDENT=2
    # lets the ranks' small resident grids share the device (they all fit
    # one dispatch round together).  Convergence lands at step 440 = 6 spans
    # of 64 steps + 7 passes of 8: inside a span, replayed bit-exactly from
    # the span's source.  Bitwise against one rank.
    base = dict(nx=600, ny=1024, steps=20000, init="random", seed=11, backend="hip",
                converge=True, check_interval=20, eps=1e-2, **kw)
    res = run_world(world, base, 20000, tmp_path, transport="rccl",
                    env={"HEAT_TB_RESIDENT": "2"})
    ref, r, h = single(base, 20000)
    assert r.converged and r.converged_at == 440
    assert bool(res["conv"]) and int(res["conv_at"]) == 440 and int(res["done"]) == 440
    assert (res["resident_passes"] > 0).all(), res["resident_passes"]
    assert (res["resident_giveups"] == 0).all()
    assert (res["halo"] == 64).all()  # m = 8 passes of depth 8 per exchange
    assert np.array_equal(res["grid"], ref)
    assert str(res["hash"]) == h


def test_rccl_resident_spans_across_runs(gpu, tmp_path):
    # Unchecked resident spans with exchanges, runs of odd lengths (spans cut
    # by run ends, remainder passes), graphs replayed across runs.
    base = dict(nx=700, ny=900, steps=0, init="random", seed=3, backend="hip", decomp="rows")
    res = run_world(2, base, 0, tmp_path, transport="rccl", chunks=[45, 300, 129, 200],
                    env={"HEAT_TB_RESIDENT": "2"})
    ref, _, h = single(base, 674)
    assert int(res["done"]) == 674
    assert (res["resident_passes"] > 0).all() and (res["resident_giveups"] == 0).all()
    assert np.array_equal(res["grid"], ref)
    assert str(res["hash"]) == h
