"""Multi-process halo exchange on the CPU (gloo, world_size 2 and 4): the N > 1 path's host logic.

Each rank takes its blocks from libocn_sw's own decomposition (``ocn_decompose``) and the
exchange schedule the RCCL path executes (``ocn_halo_schedule``), packs the messages, ships
them with torch.distributed/gloo, unpacks, and checks the reference's halo known-answer test
(shared/mpp/syncborder_block2D_gen_test.fi: fill the interior with a function of the global
(i, j), sync, every halo point that has a neighbour must hold that function of its own
global coordinates; domain-edge halos are never written)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import ocean_model_arch_amd as amd
from ocean_model_arch_amd import domain

FIELDS = ["ssh", "vort", "str_t"]


def kat(fi, m, n):
    return float(fi) * 1.0e7 + float(m) * 1.0e3 + float(n)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def strip_index(b, rect):
    x0, x1, y0, y1 = rect
    ii = []
    for n in range(y0, y1 + 1):           # column-major walk (m fastest)
        for m in range(x0, x1 + 1):
            ii.append((m - b.bnd_x1, n - b.bnd_y1))
    return tuple(np.array(ii).T)


def exchange(rank, world, basin, par):
    import torch
    blocks = domain.decompose(basin, par, rank, world)
    arrs = []
    for b in blocks:
        d = {}
        for fi, f in enumerate(FIELDS):
            a = np.full(b.shape, np.nan)
            for n in range(b.ny_start, b.ny_end + 1):
                for m in range(b.nx_start, b.nx_end + 1):
                    a[m - b.bnd_x1, n - b.bnd_y1] = kat(fi, m, n)
            d[f] = a
        arrs.append(d)
    sched = domain.halo_schedule(basin, par, FIELDS, rank, world)
    sizes = {}
    for e in sched:
        if e["kind"] != amd._lib.HALO_LOCAL:
            sizes[e["peer"]] = max(sizes.get(e["peer"], 0), e["offset"] + e["count"])
    send = {p: np.zeros(n) for p, n in sizes.items()}
    for e in sched:
        if e["kind"] == amd._lib.HALO_SEND:
            b = blocks[e["k_src"]]
            send[e["peer"]][e["offset"]:e["offset"] + e["count"]] = arrs[e["k_src"]][e["field"]][strip_index(b, e["src"])]
    recv = {p: torch.zeros(n, dtype=torch.float64) for p, n in sizes.items()}
    reqs = []
    for p in sorted(sizes):
        reqs.append(dist.isend(torch.from_numpy(send[p]), p))
        reqs.append(dist.irecv(recv[p], p))
    for r in reqs:
        r.wait()
    for e in sched:
        if e["kind"] == amd._lib.HALO_RECV:
            b = blocks[e["k"]]
            arrs[e["k"]][e["field"]][strip_index(b, e["dst"])] = \
                recv[e["peer"]].numpy()[e["offset"]:e["offset"] + e["count"]]
        elif e["kind"] == amd._lib.HALO_LOCAL:
            b, sb = blocks[e["k"]], blocks[e["k_src"]]
            arrs[e["k"]][e["field"]][strip_index(b, e["dst"])] = arrs[e["k_src"]][e["field"]][strip_index(sb, e["src"])]
    return blocks, arrs, sched


DIRS = {1: (1, 0), 2: (-1, 0), 3: (0, 1), 4: (0, -1), 5: (1, 1), 6: (1, -1), 7: (-1, 1), 8: (-1, -1)}


def check_kat(blocks, arrs):
    bad = 0
    for b, d in zip(blocks, arrs):
        for dd, (dm, dn) in DIRS.items():
            xs = [b.nx_end + 1] if dm > 0 else [b.nx_start - 1] if dm < 0 else range(b.nx_start, b.nx_end + 1)
            ys = [b.ny_end + 1] if dn > 0 else [b.ny_start - 1] if dn < 0 else range(b.ny_start, b.ny_end + 1)
            has = b.nbr_rank[dd - 1] >= 0
            for fi, f in enumerate(FIELDS):
                for m in xs:
                    for n in ys:
                        v = d[f][m - b.bnd_x1, n - b.bnd_y1]
                        if has and v != kat(fi, m, n):
                            bad += 1
                        if not has and not np.isnan(v):
                            bad += 1
    return bad


def _worker(rank, world, port, bxy, result):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        basin = amd.box_config(45)
        par = amd.ParallelConfig(*bxy)
        blocks, arrs, sched = exchange(rank, world, basin, par)
        result[rank] = (len(blocks), check_kat(blocks, arrs), len(sched))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,bxy", [(2, (2, 1)), (2, (4, 2)), (4, (2, 2)), (4, (4, 4))])
def test_halo_exchange_gloo(world, bxy):
    manager = mp.Manager()
    result = manager.dict()
    mp.spawn(_worker, args=(world, _free_port(), bxy, result), nprocs=world, join=True)
    assert sorted(result.keys()) == list(range(world))
    assert sum(r[0] for r in result.values()) == bxy[0] * bxy[1]      # every block owned once
    for rank, (nb, bad, nsched) in result.items():
        assert nb >= 1 and nsched > 0
        assert bad == 0, f"rank {rank}: {bad} halo points differ from the known answer"


def test_decomposition_is_consistent_across_ranks():
    basin, par, world = amd.box_config(64), amd.ParallelConfig(4, 2), 8
    owner = {}
    for r in range(world):
        for b in domain.decompose(basin, par, r, world):
            assert (b.bm, b.bn) not in owner
            owner[(b.bm, b.bn)] = (r, b.k)
    assert len(owner) == 8
    for r in range(world):
        for b in domain.decompose(basin, par, r, world):
            for d, (dm, dn) in DIRS.items():
                nb = owner.get((b.bm + dm, b.bn + dn))
                assert b.nbr_rank[d - 1] == (nb[0] if nb else -2)
                assert b.nbr_k[d - 1] == (nb[1] if nb else -1)
    # 8 GPUs = 4x2 blocks; process grid from MPI_Dims_create(8,2) = 4x2
    assert {owner[(bm, bn)][0] for bm in range(1, 5) for bn in range(1, 3)} == set(range(8))


def test_land_blocks_are_dropped():
    from tests.golden import cases
    case = cases.load_e2e("bs_b4x2_s60")
    b = case["basin"]
    basin = amd.BasinConfig(nx=b["nx"], ny=b["ny"], mask=case["mask"])
    blocks = domain.decompose(basin, amd.ParallelConfig(8, 8), 0, 1)
    assert 0 < len(blocks) < 64            # the Black Sea grid has all-land blocks
