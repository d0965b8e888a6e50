"""GPU, BASELINE.json configs[4] at full size: the 27-point anisotropic Poisson operator on a 256^3 grid
(16,777,216 rows, 449,455,096 nonzeros) row-partitioned over 4 ranks, as bench.py --gpus 4 --stencil 27
runs it (level 0 by C/F-Jacobi: its GS-CF chains cross the rank cuts; two-stage from level 2; explicit-
inverse coarse solve), here with the 4 ranks sharing the one GPU of a test box over the host transport.

The parent process builds the global hierarchy once, runs 3 V-cycles on the single-GPU engine and
writes the partition set; each rank then reads only its own partition file and the tail
(sss_hip_dist_create_from_files, bench.py's N > 1 path).  With stored-order sums every rank computes
its rows from the same entries in the same order as one GPU, so the gathered x after 3 V-cycles must
equal the single-GPU engine's bit for bit (reference loop: Solve/SSS_cycle.cu:861-964)."""
from __future__ import annotations

import os
import socket
import sys
import time
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

pytestmark = pytest.mark.gpu

WORLD, N_EDGE, CYCLES = 4, 256, 3
OPTS = dict(smoother="jacobi", coarse="direct", inner_from=2, sum_order=0)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, port, parts, ref_file, errq):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        import torch.distributed as dist

        dist.init_process_group("gloo", rank=rank, world_size=WORLD)
        import amg_amd as A

        comm = A.Comm(WORLD, rank, "host", device=0)
        D = A.DistHierarchy(None, comm, device=0, parts=parts, **OPTS)
        own = D.hi - D.lo
        D.upload("b", np.ones(own))
        D.upload("x", np.ones(own))
        rel = []
        for _ in range(CYCLES):
            D.cycle()
            rel.append(D.residual_norm())
        x_own = D.download("x")
        got = [None] * WORLD
        dist.all_gather_object(got, (D.lo, x_own))
        D.close()
        comm.close()
        if rank == 0:
            ref = np.load(ref_file)
            x_r, rel_r = ref["x"], ref["rel"]
            x = np.zeros_like(x_r)
            for lo, xo in got:
                x[lo:lo + len(xo)] = xo
            assert np.array_equal(x.view(np.uint64), x_r.view(np.uint64)), \
                f"max |dx| = {np.max(np.abs(x - x_r))}"
            assert np.allclose(rel, rel_r, rtol=1e-12, atol=0), (rel, rel_r)
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # noqa: BLE001
        import traceback
        errq.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")


def test_a27_256_four_ranks_bitwise_single_gpu(tmp_path):
    import amg_amd as A
    import torch.multiprocessing as mp
    from conftest import build_hierarchy, quiet_ctx

    t0 = time.perf_counter()
    H = build_hierarchy(A.generate(27, N_EDGE), quiet_ctx)
    N = H.level(0).A.num_rows
    assert N == N_EDGE ** 3 and H.level(0).A.num_nnzs == 449_455_096
    R = A.DeviceHierarchy(H, device=0, **OPTS)
    R.upload(0, "b", np.ones(N))
    R.upload(0, "x", np.ones(N))
    rel_r = []
    for _ in range(CYCLES):
        R.cycle()
        rel_r.append(R.residual_norm())
    x_r = R.download(0, "x")
    R.close()
    ref_file = tmp_path / "single.npz"
    np.savez(ref_file, x=x_r, rel=np.array(rel_r))
    del x_r
    A.part_save(H, WORLD, tmp_path / "part", 0)
    H.close()
    print(f"single GPU + partition set: {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)

    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, port, str(tmp_path / "part"), str(ref_file), errq))
             for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=900)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
