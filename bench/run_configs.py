#!/usr/bin/env python3
"""Run the BASELINE.json configurations that fit the visible hardware and write
one JSON line per config to bench/results/<name>.json.

  1  256x256, 100 iters, serial CPU reference            (no GPU)
  2  8192x8192 fp32, 1 MI355X, 1000 iters                 (1 GPU)
  3  16384x16384, 2 GPUs, 1-D decomposition, RCCL         (>= 2 GPUs)
  4  32768x32768, 8 GPUs, 2-D decomposition, overlap + hipGraph   (8 GPUs)
  5  131072x131072 fp32, 8 GPUs, convergence all-reduce every 50  (8 GPUs;
     with --capacity-1gpu the same grid also runs on ONE GPU: 2 x 68.7 GB fits
     in 288 GB HBM3E)

With --rehearse-1gpu, configs 3 and 4 run at full size on ONE GPU as N ranks
that are threads of one process (`heat --gpus N`, loopback transport: the same
message list and device-memory halo buffers as RCCL, moved by D2D copies).
That checks the decomposition, deep halos, schedules and graphs end to end on
real hardware; its throughput is one GPU's, not an N-GPU number.

Usage: python bench/run_configs.py [--configs 1,2] [--capacity-1gpu] [--rehearse-1gpu]
Multi-GPU configs are launched with torch.distributed.run (one rank per GPU).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "bench", "results")


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def gpus():
    try:
        import torch
        return torch.cuda.device_count()
    except Exception:
        return 0


def run(cmd, timeout=3000):
    t0 = time.time()
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    wall = time.time() - t0
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    if p.returncode != 0 or not lines:
        raise RuntimeError(f"{cmd} failed ({p.returncode}):\n{p.stdout[-2000:]}\n{p.stderr[-3000:]}")
    d = json.loads(lines[-1])
    d["wall_s"] = round(wall, 2)
    return d


def bench(n, args):
    if n == 1:
        return [sys.executable, "bench.py"] + args
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={free_port()}", "bench.py",
            "--gpus", str(n)] + args


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1,2,3,4,5")
    ap.add_argument("--capacity-1gpu", action="store_true")
    ap.add_argument("--rehearse-1gpu", action="store_true")
    ap.add_argument("--out", default=OUT, help="result directory (GPU box: under gpurun_out/)")
    a = ap.parse_args()
    out_dir = a.out
    os.makedirs(out_dir, exist_ok=True)
    ng = gpus()
    todo = [int(x) for x in a.configs.split(",")]
    results = {}
    for c in todo:
        try:
            if c == 1:
                cli = os.path.join(ROOT, "build", "heat")
                d = run([cli, "--backend", "cpu", "--threads", "1", "--nx", "256", "--ny", "256",
                         "--steps", "100", "--out", "none", "--json"])
                name = "c1_256_cpu_serial"
            elif c == 2 and ng >= 1:
                d = run(bench(1, ["--steps", "10", "--warmup", "2"]))
                name = "c2_8192_1gpu"
            elif c == 3 and ng >= 2:
                d = run(bench(2, ["--nx", "16384", "--ny", "16384", "--decomp", "rows",
                                  "--steps", "5", "--warmup", "1"]))
                name = "c3_16384_2gpu_1d"
            elif c in (3, 4) and a.rehearse_1gpu and ng >= 1:
                cli = os.path.join(ROOT, "build", "heat")
                if c == 3:
                    extra = ["--gpus", "2", "--nx", "16384", "--ny", "16384", "--decomp", "rows"]
                    name = "c3_16384_2ranks_rehearsal_1gpu"
                else:
                    extra = ["--gpus", "8", "--nx", "32768", "--ny", "32768", "--decomp", "2d",
                             "--schedule", "overlap"]
                    name = "c4_32768_8ranks_2d_overlap_rehearsal_1gpu"
                # Warm: 1000 untimed steps capture the graphs first (round 5's
                # rows were single cold runs with the capture inside the
                # timed steps).
                d = run([cli] + extra + ["--steps", "1000", "--warmup", "1000", "--init", "random",
                                         "--seed", "1234", "--out", "none", "--json"])
                d["note"] = "N ranks as threads on ONE GPU (loopback transport); not an N-GPU number"
            elif c == 4 and ng >= 8:
                d = run(bench(8, ["--nx", "32768", "--ny", "32768", "--decomp", "2d",
                                  "--steps", "3", "--warmup", "1"]))
                name = "c4_32768_8gpu_2d"
            elif c == 5 and (ng >= 8 or (a.capacity_1gpu and ng >= 1)):
                n = 8 if ng >= 8 else 1
                # 1000 timed iterations (a bench step), after one untimed
                # step that captures the graphs; the reference's initial
                # condition, which does not converge within the run.
                d = run(bench(n, ["--nx", "131072", "--ny", "131072", "--converge",
                                  "--check-interval", "50", "--steps", "1", "--warmup", "1",
                                  "--iters-per-step", "1000", "--init", "ref-wrap"]),
                        timeout=5000)
                name = f"c5_131072_{n}gpu_conv50"
            else:
                print(f"config {c}: skipped ({ng} GPU(s) visible)")
                continue
        except Exception as e:  # keep going; record the failure
            d = {"error": str(e)[-2000:]}
            name = f"c{c}_failed"
        results[name] = d
        with open(os.path.join(out_dir, name + ".json"), "w") as f:
            f.write(json.dumps(d) + "\n")
        print(name, json.dumps(d))
    return 0


if __name__ == "__main__":
    sys.exit(main())
