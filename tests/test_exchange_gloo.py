"""Multi-process exchange (the CHOCO sync step) over gloo on CPU, world sizes 2, 3, 4 and 8
(rings larger than 3: each rank exchanges with 2 of its N - 1 peers)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from chocosgd_amd.communication import DecentralizedAggregation, neighborhood
        nb = neighborhood(rank, world)
        agg = DecentralizedAggregation(rank, nb)
        res = {}
        for dtype in (torch.int32, torch.uint8):
            msg = (torch.arange(37) * (rank + 1)).to(dtype)
            reqs, got = agg._agg(msg, op="get_raw_sync_data", force_wait=False)
            agg.complete_wait(reqs)
            res[str(dtype)] = {r: t.tolist() for r, t in got.items()}
        # range-by-range posting into one receive buffer per neighbour (_agg out=, the
        # chunked sign exchange): three slices, posted out of order
        msg = torch.arange(101, dtype=torch.int32) * (rank + 1)
        recv = {r: torch.full((101,), -1, dtype=torch.int32) for r in agg.neighbor_ranks}
        reqs = []
        for a, b in ((4, 40), (40, 101), (0, 4)):
            rq, got = agg._agg(msg[a:b], op="get_raw_sync_data", force_wait=False,
                               out={r: recv[r][a:b] for r in agg.neighbor_ranks})
            assert all(got[r].data_ptr() == recv[r][a:b].data_ptr() for r in agg.neighbor_ranks)
            reqs += rq
        agg.complete_wait(reqs)
        res["ranged"] = {r: t.tolist() for r, t in recv.items()}
        w = agg._agg(torch.full((4,), float(rank)), op="weighted", force_wait=True)
        res["weighted"] = w.tolist()
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_decentralized_exchange(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from chocosgd_amd.communication import neighborhood
    for rank in range(world):
        nb = neighborhood(rank, world)
        for dtype in (torch.int32, torch.uint8):
            got = out[rank][str(dtype)]
            assert sorted(got) == sorted(nb)
            assert len(nb) == min(world, 3)  # self + the two ring neighbours (both, for world 2)
            for r in nb:
                assert got[r] == (torch.arange(37) * (r + 1)).to(dtype).tolist()
        for r, got in out[rank]["ranged"].items():
            assert got == (torch.arange(101, dtype=torch.int32) * (r + 1)).tolist()
        exp = sum(float(r) * w for r, w in nb.items())
        assert all(abs(v - exp) < 1e-6 for v in out[rank]["weighted"])
