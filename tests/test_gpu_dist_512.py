"""GPU, BASELINE.json configs[2] at full size: the 7-point Poisson operator on a 512^3 grid
(134,217,728 rows, 937,951,232 nonzeros) row-partitioned over 8 ranks, as bench.py --gpus 8 --n 512
runs it (hybrid smoother: exact GS-CF on the red-black level 0 with a halo exchange between its
passes, C/F-Jacobi on level 1, two-stage from level 2, the long-row levels' second inner step;
explicit-inverse coarse solve), here with the 8 ranks sharing the one GPU of a test box over the
host transport.

One host process builds the global hierarchy once without touching the GPU (SSS_SETUP_GPU_RAP=0),
then forks: first the single-GPU engine (3 V-cycles, x saved), then the 8 ranks, each building its
own rows, ghosts and halo lists from the global hierarchy it shares copy-on-write with the parent
(sss_hip_dist_create: the same partition plan the partition files carry, tests/test_dist_cpu.py
pins the two bitwise) -- no rank copies the global hierarchy, and the 65 GB of partition files are
never written.  With stored-order sums (sum_order 0) every rank computes its rows from the same
entries in the same order as one GPU, so the gathered x after 3 V-cycles must equal the single-GPU
engine's bit for bit, and the residual norms agree to the reduction order (reference loop:
Solve/SSS_cycle.cu:861-964, norm Solve/SSS_SOLVE.c:59-64).

Progress goes to gpurun_out/test_dist_512.log (a long step that prints nothing is taken for a hang).
"""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
import threading
import time
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
WORLD, CYCLES = 8, 3
N_EDGE = int(os.environ.get("SSS_TEST_DIST_N", "512"))   # (a smaller grid only to rehearse the harness)
OPTS = dict(smoother="hybrid", coarse="direct", sum_order=0)

pytestmark = pytest.mark.gpu


def _log(msg: str):
    print(f"[dist512 {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _single(H, out: str):
    import amg_amd as A
    N = H.level(0).A.num_rows
    R = A.DeviceHierarchy(H, device=0, **OPTS)
    R.upload(0, "b", np.ones(N))
    R.upload(0, "x", np.ones(N))
    rel = []
    for _ in range(CYCLES):
        R.cycle()
        rel.append(R.residual_norm())
    np.save(f"{out}/single_x.npy", R.download(0, "x"))
    Path(f"{out}/single.json").write_text(json.dumps({"rel": rel}))
    R.close()
    _log(f"single GPU: 3 V-cycles, relres {[r / np.sqrt(N) for r in rel]}")


def _rank(rank: int, port: int, H, out: str):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    import amg_amd as A
    comm = A.Comm(WORLD, rank, "host", device=0)
    t0 = time.perf_counter()
    D = A.DistHierarchy(H, comm, device=0, **OPTS)
    own = D.hi - D.lo
    D.upload("b", np.ones(own))
    D.upload("x", np.ones(own))
    dist.barrier()
    if rank == 0:
        _log(f"ranks built ({time.perf_counter() - t0:.1f} s on rank 0, {D.nagg} partitioned levels)")
    rel = []
    for _ in range(CYCLES):
        D.cycle()
        rel.append(D.residual_norm())
    np.save(f"{out}/x_r{rank}.npy", D.download("x"))
    Path(f"{out}/rank{rank}.json").write_text(json.dumps({"lo": D.lo, "hi": D.hi, "rel": rel}))
    D.close()
    comm.close()
    dist.barrier()
    dist.destroy_process_group()


def _heartbeat(stop: threading.Event, what: list):
    while not stop.wait(20.0):
        _log(f"... {what[0]}")


def main(out: str) -> int:
    """The host process: global setup (no GPU), then forked children -- never a GPU call here, so
    the fork is safe for them."""
    import multiprocessing as mp
    os.environ["SSS_SETUP_GPU_RAP"] = "0"
    what = ["setup"]
    stop = threading.Event()
    threading.Thread(target=_heartbeat, args=(stop, what), daemon=True).start()
    sys.path.insert(0, str(ROOT))
    import ctypes as C
    import amg_amd as A
    t0 = time.perf_counter()
    M = A.generate(7, N_EDGE)
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        H = A.Hierarchy(M)
    finally:
        C.CDLL(None).fflush(None)
        os.dup2(saved, 1)
        os.close(saved)
    A.lib().SSS_mat_destroy(C.byref(M))
    N = H.level(0).A.num_rows
    assert N == N_EDGE ** 3 and H.level(0).A.num_nnzs == 7 * N - 6 * N_EDGE ** 2
    _log(f"global setup {time.perf_counter() - t0:.1f} s, {H.num_levels} levels")
    ctx = mp.get_context("fork")
    what[0] = "single-GPU engine"
    p = ctx.Process(target=_single, args=(H, out))
    p.start()
    p.join()
    if p.exitcode != 0:
        _log(f"single-GPU child exited {p.exitcode}")
        return 2
    what[0] = "8 ranks"
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = [ctx.Process(target=_rank, args=(r, port, H, out)) for r in range(WORLD)]
    for q in procs:
        q.start()
    for q in procs:
        q.join()
    if any(q.exitcode != 0 for q in procs):
        _log(f"rank exit codes {[q.exitcode for q in procs]}")
        return 3
    H.close()
    what[0] = "comparing"
    x_r = np.load(f"{out}/single_x.npy")
    rel_r = json.loads(Path(f"{out}/single.json").read_text())["rel"]
    x = np.empty_like(x_r)
    covered = 0
    for r in range(WORLD):
        meta = json.loads(Path(f"{out}/rank{r}.json").read_text())
        xo = np.load(f"{out}/x_r{r}.npy")
        x[meta["lo"]:meta["hi"]] = xo
        covered += meta["hi"] - meta["lo"]
        rel = meta["rel"]
    stop.set()
    res = {"rows": int(N), "covered": covered, "bitwise": bool(np.array_equal(x.view(np.uint64), x_r.view(np.uint64))),
           "max_abs_dx": float(np.max(np.abs(x - x_r))), "rel_single": rel_r, "rel_ranks": rel,
           "seconds": time.perf_counter() - t0}
    _log(json.dumps(res))
    print(json.dumps(res), flush=True)
    return 0


def test_p7_512_eight_ranks_bitwise_single_gpu(tmp_path):
    logd = ROOT / "gpurun_out"
    logd.mkdir(exist_ok=True)
    with open(logd / "test_dist_512.log", "w") as err:
        r = subprocess.run([sys.executable, "-u", __file__, str(tmp_path)], stdout=subprocess.PIPE, stderr=err,
                           text=True, timeout=840, cwd=str(ROOT))
    assert r.returncode == 0, (r.returncode, (logd / "test_dist_512.log").read_text()[-4000:])
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["covered"] == res["rows"] == N_EDGE ** 3
    assert res["bitwise"], res
    assert np.allclose(res["rel_ranks"], res["rel_single"], rtol=1e-12, atol=0), res


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
