"""CPU, world sizes 2, 4 and 8 over gloo: the row partition of the distributed engine
(sss_part_plan_*).

Each rank builds the same global hierarchy, takes its partition, moves ghost values with the
plan's halo lists over torch.distributed (gloo) point-to-point, and checks that its local A, R
and P products equal the global products on its rows bitwise (same entries, same order): the
host-side contract the multi-GPU engine (amg_amd/csrc/sss_dist.hip) runs on.  At world 4 and 8
the interior ranks have two level-0 peers and the coarse levels (wider Galerkin stencils) couple
to non-adjacent ranks: ghosts arrive from up to seven peers.
"""
from __future__ import annotations

import ctypes as C
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _halo_exchange(dist, torch, halo, local, m):
    """local: own + ghost values (length m + g); fills the ghost part from the peers."""
    reqs, off, outs = [], 0, []
    for q, c in zip(halo["sdst"], halo["scount"]):
        t = torch.from_numpy(local[halo["sidx"][off:off + c]].copy())
        reqs.append(dist.isend(t, int(q)))
        off += c
    for q, c in zip(halo["rsrc"], halo["rcount"]):
        t = torch.empty(int(c), dtype=torch.float64)
        reqs.append(dist.irecv(t, int(q)))
        outs.append(t)
    for r in reqs:
        r.wait()
    off = m
    for t in outs:
        local[off:off + len(t)] = t.numpy()
        off += len(t)


def _worker(rank, world, port, kind, n, agg_rows, errq, prefix=None):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        import torch
        import torch.distributed as dist

        dist.init_process_group("gloo", rank=rank, world_size=world)
        import amg_amd as A
        import oracle
        from amg_amd._native import dptr
        from conftest import build_hierarchy, quiet_ctx

        H = build_hierarchy(A.generate(kind, n), quiet_ctx)
        if prefix is None:
            plan = A.PartPlan(H, world, rank, agg_rows)
        else:   # this rank's partition file only; the global H serves as the checker
            plan = A.PartPlan.load(f"{prefix}.r{rank}")
            ref = A.PartPlan(H, world, rank, agg_rows)
            assert plan.nagg == ref.nagg
            for l in range(plan.nagg):
                assert plan.level(l) == ref.level(l)
                for w in "APR":
                    a, b = A.csr_arrays(plan.matrix(l, w)), A.csr_arrays(ref.matrix(l, w))
                    assert all(np.array_equal(x.view(np.uint8), y.view(np.uint8)) for x, y in zip(a, b)), (l, w)
        ora = oracle.load()
        assert plan.nagg >= 2, plan.nagg
        # peers per level, gathered: slab interior ranks have two on level 0, and at world >= 4 some
        # coarse level couples a rank to a non-adjacent one
        peers = [len(plan.halo(l)["rsrc"]) for l in range(plan.nagg)]
        far = any(abs(int(q) - rank) > 1 for l in range(plan.nagg) for q in plan.halo(l)["rsrc"])
        allp = [None] * world
        dist.all_gather_object(allp, (peers, far))
        if 0 < rank < world - 1:
            assert peers[0] == 2, peers
        if world >= 8:
            assert any(f for _, f in allp), allp
            assert max(max(p) for p, _ in allp) >= 3, allp
        # ranges tile every partitioned level
        for l in range(plan.nagg + 1):
            lo, hi, _, _ = plan.level(l)
            got = [None] * world
            dist.all_gather_object(got, (lo, hi))
            assert got[0][0] == 0 and got[-1][1] == H.level(l).A.num_rows
            assert all(got[q][1] == got[q + 1][0] for q in range(world - 1))
        rng = np.random.default_rng(3)
        for l in range(plan.nagg):
            lo, hi, m, g = plan.level(l)
            perm, ghosts = plan.ids(l)
            assert sorted(perm.tolist()) == list(range(lo, hi))
            halo = plan.halo(l)
            Ag, Rg, Pg = H.level(l).A, H.level(l).R, H.level(l).P
            nl = Ag.num_rows
            x = rng.standard_normal(nl)           # same on every rank (same seed sequence)
            xc = rng.standard_normal(Pg.num_cols)
            loc = np.zeros(m + g)
            loc[:m] = x[perm]
            _halo_exchange(dist, torch, halo, loc, m)
            assert np.array_equal(loc[m:], x[ghosts]), ("halo", l)
            # A rows
            yg = np.zeros(nl)
            ora.ora_mv_mxy(C.byref(Ag), dptr(x), dptr(yg))
            Al = plan.matrix(l, "A")
            yl = np.zeros(m)
            ora.ora_mv_mxy(C.byref(Al), dptr(loc), dptr(yl))
            assert np.array_equal(yl.view(np.uint64), yg[perm].view(np.uint64)), ("A", l)
            # R rows (own coarse points, next level's local order or global order at nagg)
            rg = np.zeros(Rg.num_rows)
            ora.ora_mv_mxy(C.byref(Rg), dptr(x), dptr(rg))
            Rl = plan.matrix(l, "R")
            rl = np.zeros(Rl.num_rows)
            ora.ora_mv_mxy(C.byref(Rl), dptr(loc), dptr(rl))
            if l + 1 < plan.nagg:
                crow = plan.ids(l + 1)[0]
            else:
                clo, chi, _, _ = plan.level(l + 1)
                crow = np.arange(clo, chi)
            assert np.array_equal(rl.view(np.uint64), rg[crow].view(np.uint64)), ("R", l)
            # P rows: coarse vector in the next level's local numbering (with its halo)
            pg = np.zeros(nl)
            ora.ora_mv_mxy(C.byref(Pg), dptr(xc), dptr(pg))
            Pl = plan.matrix(l, "P")
            if l + 1 < plan.nagg:
                _, _, mc, gc = plan.level(l + 1)
                cperm, cghosts = plan.ids(l + 1)
                cl = np.zeros(mc + gc)
                cl[:mc] = xc[cperm]
                _halo_exchange(dist, torch, plan.halo(l + 1), cl, mc)
            else:
                cl = xc.copy()
            pl = np.zeros(m)
            ora.ora_mv_mxy(C.byref(Pl), dptr(cl), dptr(pl))
            assert np.array_equal(pl.view(np.uint64), pg[perm].view(np.uint64)), ("P", l)
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # noqa: BLE001
        import traceback
        errq.put(f"rank {rank}: {e!r}\n{traceback.format_exc()}")


def _run_world(world, kind, n, agg, prefix=None):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    errq = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, kind, n, agg, errq, prefix)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    errs = []
    while not errq.empty():
        errs.append(errq.get())
    assert not errs, "\n".join(errs)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


@pytest.mark.parametrize("kind,n,agg", [(7, 20, 60), (27, 12, 40)])
def test_partition_products_world2(kind, n, agg):
    _run_world(2, kind, n, agg)


@pytest.mark.parametrize("world,kind,n,agg", [(4, 7, 32, 60), (4, 27, 16, 40), (8, 7, 32, 60), (8, 27, 16, 40)])
def test_partition_products_multi_peer(world, kind, n, agg):
    """World 4 and 8: several peers per level, ghosts gathered from two or more neighbours, coarse
    levels coupled to non-adjacent ranks -- every local product still bitwise the global one."""
    _run_world(world, kind, n, agg)


@pytest.mark.parametrize("world,kind,n,agg", [(2, 7, 20, 60), (2, 27, 12, 40), (8, 7, 32, 60)])
def test_partition_files(world, kind, n, agg, tmp_path):
    """The same contract with each rank reading only its partition file (sss_part_save /
    sss_part_plan_load): the file round-trips the plan bitwise, and the products match."""
    import amg_amd as A
    from conftest import build_hierarchy, quiet_ctx
    H = build_hierarchy(A.generate(kind, n), quiet_ctx)
    prefix = tmp_path / "part"
    A.part_save(H, world, prefix, agg)
    assert all((tmp_path / f"part.r{r}").exists() for r in range(world)) and (tmp_path / "part.tail").exists()
    T = A.Hierarchy.load(tmp_path / "part.tail")
    plan0 = A.PartPlan.load(tmp_path / "part.r0")
    assert T.num_levels == H.num_levels - plan0.nagg
    for l in range(T.num_levels):   # the replicated tail is the global hierarchy's levels >= nagg
        a, b = A.csr_arrays(T.level(l).A), A.csr_arrays(H.level(plan0.nagg + l).A)
        assert all(np.array_equal(x.view(np.uint8), y.view(np.uint8)) for x, y in zip(a, b))
    _run_world(world, kind, n, agg, str(prefix))


def test_bench_gpus_n_launches_n_ranks():
    """`bench.py --gpus 2` without WORLD_SIZE launches two ranks itself (torch.distributed.run, a
    child process, before any GPU call); each rank sees world size 2."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--probe-ranks"], capture_output=True,
                       text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith('{"rank"')]
    assert sorted(x["rank"] for x in recs) == [0, 1]
    assert all(x["world"] == 2 for x in recs)


def test_bench_gpus_mismatch_fails_loudly():
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--probe-ranks"], capture_output=True,
                       text=True, env=env, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_gpus_n_selects_the_metric_problem(world):
    """The driver's `bench.py --gpus N` runs for N = 1, 2, 4, 8 measure ONE problem -- the metric's
    7-pt 400^3 -- so that they form a strong-scaling curve (BASELINE.json's 512^3/8 and 27-pt
    256^3/4 configs stay behind --n / --stencil).  Checked on the ranks the bench launches."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(world), "--probe-ranks"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    recs = [json.loads(l) for l in r.stdout.splitlines() if l.startswith('{"rank"')]
    assert sorted(x["rank"] for x in recs) == list(range(world))
    assert {x["workload"] for x in recs} == {"poisson7_400^3"}


def test_bench_workload_flags():
    import argparse
    import bench
    ns = lambda **kw: argparse.Namespace(**{"stencil": None, "n": None, "workload": "stencil", **kw})  # noqa: E731
    for world in (1, 2, 4, 8):
        assert bench.select_workload(ns(), world) == (7, 400)
    assert bench.select_workload(ns(n=512), 8) == (7, 512)
    assert bench.select_workload(ns(stencil=27), 4) == (27, 256)
    assert bench.select_workload(ns(stencil=27, n=64), 4) == (27, 64)


def test_bench_transport_policy_fails_loudly_on_distinct_gpus():
    """RCCL failing when every rank owns a GPU is a fault, not a reason to fall back to the host
    transport; the fallback is only for ranks sharing GPUs (the one-GPU test box)."""
    import bench
    assert bench.transport_policy(8, 8, True) == "rccl"
    assert bench.transport_policy(8, 8, False) == "fail"
    assert bench.transport_policy(2, 4, False) == "fail"
    assert bench.transport_policy(2, 1, False) == "host"
    assert bench.transport_policy(8, 1, True) == "rccl"


def test_bench_rccl_failure_exits_nonzero(tmp_path):
    """End to end on CPU: two ranks, RCCL creation fails on both (no GPU here) and the bench is told
    each rank owns a device (SSS_BENCH_FAKE_DEVICES) -- it must exit non-zero naming RCCL, before
    building anything, instead of printing a host-transport record."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(SSS_BENCH_FAKE_DEVICES="2", SSS_PART_DIR=str(tmp_path))
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--n", "12", "--no-cpu-baseline",
                        "--steps", "1", "--warmup", "0"], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode != 0
    assert "RCCL communicator creation failed" in r.stderr, r.stderr[-3000:]
    assert '"metric"' not in r.stdout


def test_bench_single_gpu_reference_matches_configuration(tmp_path):
    """parallel_efficiency's 1-GPU denominator must share workload, mode, smoother and sum order
    with the N > 1 run: a parity-mode (or differently smoothed) 1-GPU record is never used."""
    import json
    import bench
    cfg = {"workload": "poisson7_64^3", "mode": "throughput", "smoother": "hybrid", "sum_order": "tree (long rows)"}
    par = tmp_path / "parity.json"
    par.write_text(json.dumps({"value": 0.5, "n_gpus": 1, "config": dict(cfg, mode="parity", smoother="exact",
                                                                         sum_order="stored CSR order")}))
    assert bench.single_gpu_reference(str(par), dict(cfg, workload="poisson7_63^3")) is None
    thr = tmp_path / "thr.json"
    thr.write_text(json.dumps({"value": 50.0, "n_gpus": 1, "config": dict(cfg, workload="poisson7_63^3")}))
    ref = bench.single_gpu_reference(str(thr), dict(cfg, workload="poisson7_63^3"))
    assert ref and ref["value"] == 50.0 and ref["source"] == str(thr)
    # same workload, other smoother: not a denominator
    assert bench.single_gpu_reference(str(thr), dict(cfg, workload="poisson7_63^3", smoother="jacobi")) is None
    assert bench.single_ref_path("poisson7_64^3", "parity") != bench.single_ref_path("poisson7_64^3", "throughput")


def test_partition_set_versioned(tmp_path, monkeypatch):
    """A partition set names its file layout: the C writer's version word equals
    amg_amd.partition.PART_FORMAT, bench.py puts it (and a non-default tail threshold) in the set's
    directory name, and a manifest of another layout is not reused (it would abort the run with
    ERROR_WRONG_FILE instead of being regenerated)."""
    import json
    import struct
    import amg_amd as A
    import bench
    from amg_amd.partition import PART_FORMAT
    from conftest import build_hierarchy, quiet_ctx
    H = build_hierarchy(A.generate(7, 12), quiet_ctx)
    A.part_save(H, 2, tmp_path / "part", 60)
    raw = (tmp_path / "part.r0").read_bytes()
    assert raw[:8] == b"SSSPART1" and struct.unpack("<i", raw[8:12])[0] == PART_FORMAT
    monkeypatch.delenv("SSS_HIP_AGG_ROWS", raising=False)
    assert bench.part_set_name(7, 512, 8) == f"sss_parts_v{PART_FORMAT}_7pt_512_8r"
    monkeypatch.setenv("SSS_HIP_AGG_ROWS", "80000")
    assert bench.part_set_name(7, 512, 8).endswith("_agg80000")
    man = tmp_path / "part.json"
    man.write_text(json.dumps({"format": PART_FORMAT - 1}))
    assert not bench.part_set_usable(man)
    man.write_text(json.dumps({"format": PART_FORMAT}))
    assert bench.part_set_usable(man)
    assert not bench.part_set_usable(tmp_path / "missing.json")
