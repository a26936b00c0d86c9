"""The `heat` CLI (native binary) and `python -m parallel_heat_amd`: reference
output names and lines, multi-process TCP runs, checkpoint/resume."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from parallel_heat_amd import HeatConfig, HeatSolver, _native
from parallel_heat_amd.utils import io as hio

from .dist_worker import free_port

HEAT = str(_native.CLI_PATH)
ROOT = str(_native.REPO_DIR)


def heat(args, cwd, env=None, check=True):
    e = dict(os.environ)
    e.update(env or {})
    return subprocess.run([HEAT] + args, cwd=cwd, env=e, capture_output=True, text=True,
                          check=check, timeout=300)


def reference_grid(nx, ny, steps, **kw):
    with HeatSolver(HeatConfig(nx=nx, ny=ny, steps=steps, backend="cpu", **kw)) as s:
        s.run()
        return s.gather()


def test_cli_mpi_naming_and_lines(tmp_path):
    p = heat(["--backend", "cpu", "--nx", "20", "--ny", "20", "--steps", "100", "--naming", "mpi"],
             tmp_path)
    lines = p.stdout.splitlines()
    assert lines[0] == "Starting mpi_heat2D with 1 worker tasks."
    assert lines[1] == "Grid size: X= 20  Y= 20  Time steps= 100"
    assert lines[2].startswith("Elapsed time ") and lines[2].endswith(" secs")
    assert (tmp_path / "initial_im.dat").exists()
    # compat=mpi -> STEPS+1 updates
    g = reference_grid(20, 20, 100, compat="mpi")
    ref = tmp_path / "ref.dat"
    hio.write_dat(str(ref), g)
    assert (tmp_path / "final_im.dat").read_bytes() == ref.read_bytes()


def test_cli_cuda_naming_and_convergence(tmp_path):
    p = heat(["--backend", "cpu", "--nx", "24", "--ny", "30", "--steps", "10000", "--converge",
              "--naming", "cuda"], tmp_path)
    # NB for 24x30 with T=32: ceil(22/32)*ceil(28/32) = 1 block
    assert (tmp_path / "out_cuda_1024_1_10000.dat").exists()
    first = p.stdout.splitlines()[0]
    assert first.startswith("Converged at ") and first.endswith(" steps")
    k = int(first.split()[2])
    assert k % 20 == 0  # CUDA prints i with i % CHECK_INTERVAL == 0
    assert p.stdout.splitlines()[1].startswith("Elapsed time: ")


def test_cli_json_and_checksum(tmp_path):
    p = heat(["--backend", "cpu", "--nx", "64", "--ny", "48", "--steps", "30", "--init", "random",
              "--out-format", "checksum", "--out", "cs.json", "--json"], tmp_path)
    m = json.loads(p.stdout.splitlines()[-1])
    assert m["steps_done"] == 30 and m["backend"] == "cpu" and m["mcells_per_s"] > 0
    cs = json.loads((tmp_path / "cs.json").read_text())
    with HeatSolver(HeatConfig(nx=64, ny=48, steps=30, init="random", backend="cpu")) as s:
        s.run()
        assert cs["hash"] == s.checksum()["hash"]


@pytest.mark.parametrize("world,extra", [(2, []), (4, []), (4, ["--decomp", "rows", "--tb-depth", "3"]),
                                         (3, ["--px", "1", "--py", "3"])])
def test_cli_tcp_multiprocess_invariance(tmp_path, world, extra):
    port = free_port()
    base = ["--backend", "cpu", "--nx", "41", "--ny", "39", "--steps", "57", "--init", "random",
            "--seed", "3", "--out", "g.bin", "--out-format", "bin", "--transport", "tcp",
            "--port", str(port)] + extra
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1")
        procs.append(subprocess.Popen([HEAT] + base, cwd=tmp_path, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e
    g, h = hio.read_bin(str(tmp_path / "g.bin"))
    assert h["step"] == 57
    ref = reference_grid(41, 39, 57, init="random", seed=3)
    assert np.array_equal(np.asarray(g), ref)


def test_cli_checkpoint_resume(tmp_path):
    heat(["--backend", "cpu", "--nx", "30", "--ny", "30", "--steps", "40", "--init", "random",
          "--checkpoint", "ck.bin", "--checkpoint-every", "25", "--out", "full.bin",
          "--out-format", "bin"], tmp_path)
    # ck.bin holds the state after the last chunk (40); resume a 25-step checkpoint instead
    heat(["--backend", "cpu", "--nx", "30", "--ny", "30", "--steps", "25", "--init", "random",
          "--out", "c25.bin", "--out-format", "bin"], tmp_path)
    heat(["--backend", "cpu", "--nx", "30", "--ny", "30", "--steps", "40", "--init", "random",
          "--resume", "c25.bin", "--out", "resumed.bin", "--out-format", "bin"], tmp_path)
    a, _ = hio.read_bin(str(tmp_path / "full.bin"))
    b, hb = hio.read_bin(str(tmp_path / "resumed.bin"))
    c, hc = hio.read_bin(str(tmp_path / "ck.bin"))
    assert hb["step"] == 40 and hc["step"] == 40
    assert np.array_equal(np.asarray(a), np.asarray(b))
    assert np.array_equal(np.asarray(a), np.asarray(c))
    # written as ck.bin.tmp and renamed: no temporary left behind
    assert not (tmp_path / "ck.bin.tmp").exists()


def test_cli_resume_warns_on_other_physics(tmp_path):
    heat(["--backend", "cpu", "--nx", "16", "--ny", "16", "--steps", "5", "--init", "random",
          "--out", "s5.bin", "--out-format", "bin"], tmp_path)
    p = subprocess.run([HEAT, "--backend", "cpu", "--nx", "16", "--ny", "16", "--steps", "8",
                        "--cx", "0.2", "--resume", "s5.bin", "--out", "none"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr
    assert "warning" in p.stderr and "cx=0.1" in p.stderr


def test_python_cli(tmp_path):
    p = subprocess.run([sys.executable, "-m", "parallel_heat_amd", "--backend", "cpu", "--nx", "20",
                        "--ny", "20", "--steps", "100", "--naming", "mpi", "--json"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, PYTHONPATH=ROOT))
    assert p.returncode == 0, p.stderr
    lines = p.stdout.splitlines()
    assert lines[0] == "Starting mpi_heat2D with 1 worker tasks."
    m = json.loads(lines[-1])
    assert m["steps_done"] == 101
    native = tmp_path / "native"
    native.mkdir()
    heat(["--backend", "cpu", "--nx", "20", "--ny", "20", "--steps", "100", "--naming", "mpi"],
         native)
    assert (tmp_path / "final_im.dat").read_bytes() == (native / "final_im.dat").read_bytes()


def test_python_cli_torchrun_gloo(tmp_path):
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "-m", "parallel_heat_amd",
           "--backend", "cpu", "--nx", "33", "--ny", "21", "--steps", "40", "--init", "random",
           "--out", "g.dat", "--json"]
    p = subprocess.run(cmd, cwd=tmp_path, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1"))
    assert p.returncode == 0, p.stderr[-3000:]
    m = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert m["ranks"] == 2 and m["transport"] == "torch"
    g = hio.read_dat(str(tmp_path / "g.dat"))
    ref = reference_grid(33, 21, 40, init="random")
    assert np.allclose(g, np.round(ref, 1), atol=0.051)


def test_make_ref_variants_wrappers(tmp_path):
    """R21: `make ref-variants` writes the reference's mpi/Makefile program names
    (mpi/Makefile:12-22) as wrappers over `heat`; NP=1 and NP=2 (torchrun
    ranks over TCP, 127.0.0.1) give byte-identical final_im.dat."""
    subprocess.run(["make", "-s", "-C", ROOT, "ref-variants", "SIZE=40", "STEPS=60", "STEP=10",
                    "THREADS=2"], check=True, capture_output=True, timeout=600)
    ref_dir = os.path.join(os.path.dirname(HEAT), "ref")
    for name in ("heat_40", "heat_omp_40", "heat_con_40", "heat_con_omp_40", "cuda_heat"):
        assert os.access(os.path.join(ref_dir, name), os.X_OK), name
    outs = {}
    for np_ in ("1", "2"):
        d = tmp_path / f"np{np_}"
        d.mkdir()
        p = subprocess.run([os.path.join(ref_dir, "heat_omp_40")], cwd=d, capture_output=True,
                           text=True, timeout=300, env=dict(os.environ, NP=np_))
        assert p.returncode == 0, p.stderr[-3000:]
        assert f"Starting mpi_heat2D with {np_} worker tasks." in p.stdout
        outs[np_] = (d / "final_im.dat").read_bytes()
    assert outs["1"] == outs["2"]
    p = subprocess.run([os.path.join(ref_dir, "heat_con_omp_40")], cwd=tmp_path,
                       capture_output=True, text=True, timeout=300, env=dict(os.environ, NP="2"))
    assert p.returncode == 0, p.stderr[-3000:]
    assert "converged" in p.stdout


def test_cli_memory_plan(tmp_path):
    # --plan: per-GPU bytes of the worst rank without allocating anything
    # (131072^2 = two 68.7 GB fields: one MI355X or 1/8 of it per GPU).
    one = json.loads(heat(["--nx", "131072", "--ny", "131072", "--plan"], tmp_path).stdout)
    eight = json.loads(heat(["--nx", "131072", "--ny", "131072", "--gpus", "8", "--plan"],
                            tmp_path).stdout)
    assert one["process_grid"] == "1x1" and one["fits_288gb"]
    assert 2 * 131072 ** 2 * 4 < one["bytes_per_gpu"] < 1.01 * 2 * 131072 ** 2 * 4
    assert eight["process_grid"] == "4x2" and eight["ranks"] == 8
    assert eight["bytes_per_gpu"] < one["bytes_per_gpu"] / 7.5
    huge = json.loads(heat(["--nx", "600000", "--ny", "600000", "--gpus", "8", "--plan"],
                           tmp_path).stdout)
    assert not huge["fits_288gb"]


def test_cli_plan_resident_aware_halo(tmp_path):
    # Passes per exchange follow resident fit (plan.hpp resident_halo_passes,
    # the same rule as the solver and parallel/model.py): 8192^2 on 2 x 2
    # ranks takes m = 5 (4144-cell span boxes, 20 x 16 resident tiles) instead
    # of m = 8 (4180: no one-round plan); 8 ranks take m = 7 (m = 8 boxes fall
    # to another tile shape); slabs whose only fitting m is below
    # kResMinPasses keep m = 8; --halo-passes overrides.
    from parallel_heat_amd.parallel.model import resident_halo_passes
    want = {("auto", 4): (5, True), ("rows", 4): (8, False), ("auto", 8): (7, True),
            ("rows", 8): (7, True), ("auto", 2): (8, False)}
    for (decomp, g), (m, res) in want.items():
        p = json.loads(heat(["--nx", "8192", "--ny", "8192", "--gpus", str(g), "--decomp", decomp,
                             "--plan"], tmp_path).stdout)
        assert (p["halo_passes"], p["resident"]) == (m, res), (decomp, g, p)
        assert p["halo"] == 12 * m
        px, py = map(int, p["process_grid"].split("x"))
        rm = resident_halo_passes(8192, 8192, px, py)
        assert m == (rm if rm >= 4 else 8)
    forced = json.loads(heat(["--nx", "8192", "--ny", "8192", "--gpus", "4", "--halo-passes", "8",
                              "--plan"], tmp_path).stdout)
    assert forced["halo_passes"] == 8 and not forced["resident"]


def _flags_of(text):
    import re
    return set(re.findall(r"(?<![\w-])(--[a-z][a-z0-9-]*)", text))


def test_cli_flag_parity():
    # The two front ends accept the same flags (SURVEY §5 config system; the
    # reference's -D macros, mpi/Makefile:12-22).  Help flags aside, the only
    # difference allowed is a VALUE: --transport torch is Python-only.
    native = heat(["--help"], ROOT).stdout
    from parallel_heat_amd.cli import build_parser
    py = {o for a in build_parser()._actions for o in a.option_strings if o.startswith("--")}
    nat = _flags_of(native)
    assert nat - py == set(), f"native-only flags: {sorted(nat - py)}"
    assert py - nat - {"--help"} == set(), f"python-only flags: {sorted(py - nat - {'--help'})}"


@pytest.mark.parametrize("args", [
    ["--nx", "20", "--ny", "20", "--steps", "100", "--naming", "mpi"],
    ["--nx", "24", "--ny", "30", "--steps", "10000", "--converge", "--naming", "mpi"],
    ["--nx", "24", "--ny", "30", "--steps", "10000", "--converge", "--naming", "cuda"],
    ["--nx", "17", "--ny", "23", "--steps", "40", "--init", "random", "--seed", "3",
     "--out-format", "checksum", "--out", "c.json"],
])
def test_cli_reference_lines_match(tmp_path, args):
    import re
    # Identical reference lines and identical output files from both CLIs
    # (elapsed-time values aside).
    outs = {}
    for name, cmd in (("native", [HEAT]), ("python", [sys.executable, "-m", "parallel_heat_amd"])):
        d = tmp_path / name
        d.mkdir()
        p = subprocess.run(cmd + ["--backend", "cpu"] + args, cwd=d, capture_output=True,
                           text=True, timeout=300, check=True,
                           env=dict(os.environ, PYTHONPATH=ROOT))
        lines = [re.sub(r"[0-9.]+ m?secs", "T (m)secs", l) if l.startswith("Elapsed time") else l
                 for l in p.stdout.splitlines()]
        files = {f.name: f.read_bytes() for f in sorted(d.iterdir())}
        outs[name] = (lines, files)
    assert outs["native"][0] == outs["python"][0]
    assert outs["native"][1].keys() == outs["python"][1].keys()
    for k, v in outs["native"][1].items():
        if k.endswith(".json"):
            a, b = json.loads(v), json.loads(outs["python"][1][k])
            assert a["hash"] == b["hash"] and a["step"] == b["step"]
        else:
            assert v == outs["python"][1][k], k


def test_plan_halo_rule_matches_the_model(tmp_path):
    # The native rule (plan.hpp resident_halo_passes + resident_fits_static,
    # what `heat --plan` prints) and its Python mirror in parallel/model.py
    # agree on the halo depth and resident fit over plate sizes and rank
    # counts, remainders included.
    from parallel_heat_amd.parallel.model import (RES_MIN_PASSES, resident_fits,
                                                  resident_halo_passes)
    for n in (3000, 5000, 8192, 10000):
        for g in (2, 3, 4, 6, 8):
            for decomp in ("rows", "auto"):
                p = json.loads(heat(["--nx", str(n), "--ny", str(n + 100), "--gpus", str(g),
                                     "--decomp", decomp, "--plan"], tmp_path).stdout)
                px, py = map(int, p["process_grid"].split("x"))
                rm = resident_halo_passes(n, n + 100, px, py)
                m = rm if rm >= RES_MIN_PASSES else 8
                assert p["halo_passes"] == m, (n, g, decomp, p, rm)
                # Resident iff every rank's span box at m fits (model mirror).
                rows = [n // px + (1 if i < n % px else 0) for i in range(px)]
                cols = [(n + 100) // py + (1 if j < (n + 100) % py else 0) for j in range(py)]
                gr, gc = (m - 1) * 12 if px > 1 else 0, ((m - 1) * 12) // 4 * 4 if py > 1 else 0
                fits = all(resident_fits(r + gr * ((i > 0) + (i < px - 1)),
                                         c + gc * ((j > 0) + (j < py - 1)))
                           for i, r in enumerate(rows) for j, c in enumerate(cols))
                assert p["resident"] == fits, (n, g, decomp, p)


def test_cli_warmup_restores_the_initial_state(tmp_path):
    # --warmup N: N untimed steps (graph capture on GPUs), then the initial
    # state again; the timed run's output is a cold run's, byte for byte.
    base = ["--backend", "cpu", "--nx", "50", "--ny", "40", "--steps", "33", "--init", "random",
            "--seed", "4", "--out-format", "checksum", "--json"]
    a = heat(base + ["--out", "a.json", "--warmup", "20"], tmp_path)
    heat(base + ["--out", "b.json"], tmp_path)
    assert json.loads(a.stdout.splitlines()[-1])["steps_done"] == 33
    assert (tmp_path / "a.json").read_text() == (tmp_path / "b.json").read_text()


def test_plan_tile_shape_matches_the_model(tmp_path):
    # The host planner mirror (topology.cpp resident_shape_static, what
    # `heat --plan` reports as resident_tile) and parallel/model.py's
    # resident_shape pick the same tile shape (tb_resident.hip plan_res's
    # lowest tile_step_estimate): 12 x 16 up to 1168 rows of 8192 columns,
    # 14 x 8 two per CU at 1192, 20 x 16 on the 4-GPU plates.
    from parallel_heat_amd.parallel.model import resident_shape
    want = {(1024, 8192): (12, 16), (1168, 8192): (12, 16), (1192, 8192): (14, 8),
            (2192, 4168): (12, 16), (2216, 4180): (14, 8), (4144, 4144): (20, 16),
            (4180, 4180): None, (2048, 8192): (20, 16), (300, 1000): (12, 8)}
    for (r, c), sh in want.items():
        assert resident_shape(r, c) == sh, (r, c)
    for r in (200, 640, 1000, 1100, 1500, 2100, 3000, 4100):
        for c in (500, 2000, 4100, 8192):
            p = json.loads(heat(["--nx", str(r), "--ny", str(c), "--tb-depth", "12", "--plan"],
                                tmp_path).stdout)
            sh = resident_shape(r, c)
            assert p["resident_tile"] == (f"{sh[0]}x{sh[1]}" if sh else "0x0"), (r, c, p)
