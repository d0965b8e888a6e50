"""GPU, world sizes 2, 4 and 8 on one device: the row-partitioned engine (sss_hip_dist_*) over the host
transport (torch.distributed gloo; RCCL refuses two ranks on one GPU).  Each rank's rows are
computed exactly as on one GPU, so after every V-cycle the gathered x equals the single-GPU
engine's x bitwise; the residual norm is reduced in another order (rtol 1e-12)."""
from __future__ import annotations

import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, kind, n, smoother, inner_from, agg_rows, cycles, errq, transport="host", sum_order=0,
            parts=None):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        if sum_order:   # every level on the free-order kernels, merged row groups wherever possible
            os.environ["SSS_HIP_FREE_MIN"] = "1"
            os.environ["SSS_HIP_MERGE_MIN_ROWS"] = "1"
        import torch
        import torch.distributed as dist

        dist.init_process_group("gloo", rank=rank, world_size=world)
        import amg_amd as A
        from conftest import build_hierarchy, quiet_ctx

        H = build_hierarchy(A.generate(kind, n), quiet_ctx)
        N = H.level(0).A.num_rows
        comm = A.Comm(world, rank, transport, device=0)
        if parts is None:
            D = A.DistHierarchy(H, comm, smoother=smoother, coarse="direct", device=0, agg_rows=agg_rows,
                                inner_from=inner_from, sum_order=sum_order)
        else:   # this rank's partition file and the tail file only
            D = A.DistHierarchy(None, comm, smoother=smoother, coarse="direct", device=0, inner_from=inner_from,
                                sum_order=sum_order, parts=parts)
        assert D.nagg >= 2, D.nagg
        if kind == 7 and smoother == "hybrid" and not sum_order:
            # red-black level 0: the fused C-row residual and the dead F-row prolongation hold
            # across the rank cut; every level's first pre-smoothing pass starts from zero
            f0 = D.level_flags(0)
            assert f0["fused_residual"] and f0["dead_prolong"], f0
        assert all(D.level_flags(l)["zero_first"] for l in range(D.nagg))
        own = D.hi - D.lo
        D.upload("b", np.ones(own))
        D.upload("x", np.ones(own))
        rel = []
        for _ in range(cycles):
            D.cycle()
            rel.append(D.residual_norm() / np.sqrt(N))
        if os.environ.get("SSS_HIP_DIST_GRAPH", "1") != "0" and transport == "rccl":   # coarse "direct": on the device
            assert D.level_flags(0)["cycle_graph"], "the distributed cycle was not captured"
        if os.environ.get("SSS_HIP_DIST_GRAPH") == "0" or transport != "rccl":
            assert not D.level_flags(0)["cycle_graph"]
        x_own = D.download("x")
        parts = [None] * world
        dist.all_gather_object(parts, (D.lo, x_own))
        D.close()
        comm.close()
        if rank == 0:
            x = np.zeros(N)
            for lo, xo in parts:
                x[lo:lo + len(xo)] = xo
            R = A.DeviceHierarchy(H, smoother=smoother, coarse="direct", device=0, inner_from=inner_from,
                                  sum_order=sum_order)
            R.upload(0, "b", np.ones(N))
            R.upload(0, "x", np.ones(N))
            rel_r = []
            for _ in range(cycles):
                R.cycle()
                rel_r.append(R.residual_norm() / np.sqrt(N))
            x_r = R.download(0, "x")
            R.close()
            if sum_order:   # tree-order sums over per-rank row groups: same iterates up to rounding
                assert np.linalg.norm(x - x_r) <= 1e-10 * np.linalg.norm(x_r), np.max(np.abs(x - x_r))
                assert np.allclose(rel, rel_r, rtol=1e-8, atol=0), (rel, rel_r)
            else:
                assert np.array_equal(x.view(np.uint64), x_r.view(np.uint64)), \
                    f"max |dx| = {np.max(np.abs(x - x_r))}"
                assert np.allclose(rel, rel_r, rtol=1e-12, atol=0), (rel, rel_r)
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # noqa: BLE001
        import traceback
        errq.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")


@pytest.mark.parametrize("kind,n,smoother,inner_from,agg", [
    (7, 24, "hybrid", 2, 100),     # level 0 exact red-black GS-CF, C/F-Jacobi, two-stage from level 2
    (7, 24, "jacobi", 0, 100),     # two-stage everywhere: lower-rank ghost rows are "lower" entries
    (27, 14, "jacobi", 2, 100),    # 27-point: not red-black, C/F-Jacobi forms only
])
def test_dist_equals_single_gpu(kind, n, smoother, inner_from, agg):
    _run(2, "host", kind, n, smoother, inner_from, agg)


@pytest.mark.parametrize("smoother", ["hybrid", "jacobi"])
def test_dist_rccl_single_rank(smoother, monkeypatch):
    """The RCCL transport on the one GPU a test box has, eager launches (SSS_HIP_DIST_GRAPH=0):
    communicator from a broadcast unique id, the grouped send/recv of the coarse all-gather (no
    peers) and the ncclAllReduce of ||r||^2 -- bitwise the single-GPU engine.  (Two ranks cannot
    share a GPU under RCCL; the halo send/recv pattern itself is covered by the host-transport
    tests above, which run the same plan.)"""
    monkeypatch.setenv("SSS_HIP_DIST_GRAPH", "0")
    _run(1, "rccl", 7, 24, smoother, 2, 100)


@pytest.mark.parametrize("smoother", ["hybrid", "jacobi"])
def test_dist_rccl_graph(smoother, monkeypatch):
    """The default over RCCL: the distributed cycle captured into one hipGraph and replayed --
    bitwise the single-GPU engine's cycles, and reported as captured."""
    monkeypatch.delenv("SSS_HIP_DIST_GRAPH", raising=False)
    _run(1, "rccl", 7, 24, smoother, 2, 100)


@pytest.mark.parametrize("kind,n,smoother", [(7, 24, "hybrid"), (27, 14, "jacobi")])
def test_dist_free_order(kind, n, smoother):
    """bench.py's N > 1 configuration: throughput mode with the free-order (merged-group) kernels
    on the row-partitioned engine, against the single-GPU engine in the same mode (27-point:
    level 0 is not red-black, so its exact GS-CF cannot be split across ranks -- C/F-Jacobi)."""
    _run(2, "host", kind, n, smoother, 2, 100, sum_order=1)


@pytest.mark.parametrize("kind,n,smoother", [(7, 24, "hybrid"), (7, 24, "jacobi"), (27, 14, "jacobi")])
def test_dist_overlap_split_launches(kind, n, smoother, monkeypatch):
    """The halo-overlap launch order (blocks that read no ghost first, the others after the
    halo; SSS_HIP_OVERLAP=2 applies it over the synchronous host transport too): every row block
    is launched exactly once with the right inputs -- still bitwise the single-GPU engine."""
    monkeypatch.setenv("SSS_HIP_OVERLAP", "2")
    _run(2, "host", kind, n, smoother, 2, 100)


@pytest.mark.parametrize("kind,n,smoother,sum_order", [(7, 24, "hybrid", 0), (27, 14, "jacobi", 0), (7, 24, "hybrid", 1)])
def test_dist_from_partition_files(kind, n, smoother, sum_order, tmp_path):
    """Engines built from a partition set (sss_part_save -> sss_hip_dist_create_from_files, the
    path bench.py takes at N > 1): every rank reads only its own file and the tail, and the
    iterates are those of one GPU."""
    import amg_amd as A
    from conftest import build_hierarchy, quiet_ctx
    H = build_hierarchy(A.generate(kind, n), quiet_ctx)
    A.part_save(H, 2, tmp_path / "part", 100)
    H.close()
    _run(2, "host", kind, n, smoother, 2, 100, sum_order=sum_order, parts=str(tmp_path / "part"))


@pytest.mark.parametrize("world,kind,n,smoother,agg", [
    (4, 7, 32, "hybrid", 60), (8, 7, 32, "hybrid", 60), (4, 27, 16, "jacobi", 40), (8, 27, 16, "jacobi", 40)])
def test_dist_multi_peer(world, kind, n, smoother, agg, monkeypatch):
    """4 and 8 ranks sharing the one GPU over the host transport: interior ranks exchange halos with
    two level-0 neighbours, and at 8 ranks the coarse levels gather ghosts from up to six peers,
    several of them non-adjacent; the replicated tail is all-gathered from every rank.  The halo
    overlap split is on (SSS_HIP_OVERLAP=2).  After 4 V-cycles x is bitwise the single-GPU engine's."""
    monkeypatch.setenv("SSS_HIP_OVERLAP", "2")
    _run(world, "host", kind, n, smoother, 2, agg)


@pytest.mark.parametrize("world,kind,n,smoother,agg,sum_order", [(4, 7, 32, "hybrid", 60, 1), (8, 27, 16, "jacobi", 40, 0)])
def test_dist_multi_peer_from_files(world, kind, n, smoother, agg, sum_order, tmp_path):
    """The bench's N > 1 path (partition set, each rank reading only its file) at 4 and 8 ranks."""
    import amg_amd as A
    from conftest import build_hierarchy, quiet_ctx
    H = build_hierarchy(A.generate(kind, n), quiet_ctx)
    A.part_save(H, world, tmp_path / "part", agg)
    H.close()
    _run(world, "host", kind, n, smoother, 2, agg, sum_order=sum_order, parts=str(tmp_path / "part"))


def _run(world, transport, kind, n, smoother, inner_from, agg, sum_order=0, parts=None):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker,
                         args=(r, world, port, kind, n, smoother, inner_from, agg, 4, errq, transport, sum_order,
                               parts))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=600)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_timing_comm_floor_and_level_times():
    """The floor instruments (tools/n8_floor.py): a rank built with the timing-only communicator
    (no transfer, no peer process) runs its whole cycle alone -- graph captured -- and reports its
    halo exchanges (rank 0 of 2 has a level-0 peer) and per-level times; the single-GPU engine's
    per-level times cover every level and add up to about one eager cycle."""
    import amg_amd as A
    from conftest import build_hierarchy, quiet_ctx
    H = build_hierarchy(A.generate(7, 32), quiet_ctx)
    comm = A.Comm(2, 0, "timing", device=0)
    D = A.DistHierarchy(H, comm, smoother="hybrid", coarse="direct", device=0, agg_rows=60)
    try:
        own = D.hi - D.lo
        D.upload("b", np.ones(own))
        D.upload("x", np.ones(own))
        D.halo_stats(reset=True)
        D.cycle()
        D.residual_norm()
        hs = D.halo_stats(reset=True)
        assert hs["exchanges"][0] > 0 and hs["doubles_sent"][0] >= hs["exchanges"][0] * 32 * 32
        assert hs["gather_all"] == H.level(D.nagg).A.num_rows and 0 < hs["gather_own"] < hs["gather_all"]
        assert hs["tail_levels"] == H.num_levels - D.nagg
        assert D.level_flags(0)["cycle_graph"]
        cyc, lv = D.time_levels(3)
        assert cyc > 0 and len(lv) == D.nagg + 1 and all(t > 0 for t in lv)
        tl = D.time_tail_levels(2)[:hs["tail_levels"]]
        assert tl[0] > 0 and all(t >= 0 for t in tl)   # (a single-workgroup tail counts at its first level)
    finally:
        D.close()
        comm.close()
    S = A.DeviceHierarchy(H, smoother="hybrid", coarse="direct")
    try:
        n = H.level(0).A.num_rows
        S.upload(0, "b", np.ones(n))
        S.upload(0, "x", np.ones(n))
        lv = S.time_levels(3)
        assert len(lv) == H.num_levels and lv[0] > 0 and all(t >= 0 for t in lv)
        S.cycle()   # the graph-replayed cycle is unaffected by the timing walk
        assert np.isfinite(S.residual_norm())
    finally:
        S.close()
