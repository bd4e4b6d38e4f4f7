"""Exchange step of the CHOCO gossip (drop-in for the decentralized half of
dl_code/pcode/utils/communication.py).

`DecentralizedAggregation._agg(data, op="get_raw_sync_data", force_wait=False)`
keeps the reference's contract (communication.py:246-291): send `data` to every
neighbour, receive each neighbour's message into a same-shaped buffer, return
`(reqs, {rank: tensor})` with the local entry being `data` itself.  On ROCm the
sends/receives are issued as ONE grouped batch (`dist.batch_isend_irecv`, i.e.
ncclGroupStart/End over RCCL), so both ring directions run concurrently on
their own xGMI links; on CPU the same code runs over gloo.

Messages are whatever the CHOCO compressors pack (uint8 / int32 wire buffers);
unlike the reference nothing is re-cast to the default float dtype.
"""
import torch
import torch.distributed as dist


def recover_device(data, device=None):
    return data.to(device) if device is not None else data


def neighborhood(rank, world_size):
    """Mixing-matrix row {rank: weight} incl. self, as the reference topologies give it.

    world 1: {0: 1.0}; world 2: CompleteGraph (topology.py:122-162, weight 1/2,
    RingGraph asserts n > 2 at topology.py:187); world >= 3: RingGraph
    (topology.py:174-299, weights 1/3 for r-1, r, r+1, keys in ascending order).
    """
    if world_size == 1:
        return {0: 1.0}
    if world_size == 2:
        return {0: 0.5, 1: 0.5}
    ranks = sorted({(rank - 1) % world_size, rank, (rank + 1) % world_size})
    return {r: 1.0 / 3 for r in ranks}


class _Works:
    def __init__(self, works):
        self.works = list(works)

    def wait(self):
        for w in self.works:
            w.wait()


class DecentralizedAggregation(object):
    """Aggregate updates in a decentralized manner (communication.py:230-291)."""

    def __init__(self, rank, neighbors_info):
        self.rank = rank
        self.neighbors_info = neighbors_info
        self.neighbor_ranks = [r for r in neighbors_info.keys() if r != rank]
        self.world_size = float(len(self.neighbor_ranks))

    def _agg(self, data, op, force_wait=True, out=None):
        """`out` (this drop-in's addition, default None = the reference's behaviour):
        {rank: buffer} to receive each neighbour's message into, e.g. slices of one
        message posted range by range (CHOCOSignCompressor exchange_chunks)."""
        if out is not None:
            local_data = {i: out[i] for i in self.neighbor_ranks}
        else:
            local_data = {i: torch.empty_like(data) for i in self.neighbor_ranks}
        local_data[self.rank] = data
        reqs = []
        if self.neighbor_ranks:
            ops = []
            for node_rank in self.neighbor_ranks:
                ops.append(dist.P2POp(dist.isend, data, node_rank))
                ops.append(dist.P2POp(dist.irecv, local_data[node_rank], node_rank))
            reqs = [_Works(dist.batch_isend_irecv(ops))]
        if force_wait:
            self.complete_wait(reqs)
            if op == "avg":
                return sum(local_data.values()) / (self.world_size + 1)
            if op == "weighted":
                return sum(t * self.neighbors_info[r] for r, t in local_data.items())
            if op == "get_raw_sync_data":
                return local_data
            raise NotImplementedError("op {} is not supported yet.".format(op))
        if op == "get_raw_sync_data":
            return reqs, local_data
        raise NotImplementedError("op {} is not supported yet.".format(op))

    def complete_wait(self, reqs):
        for req in reqs:
            req.wait()


class CentralizedAggregation(object):
    """The all-gather / all-reduce / reduce half of communication.py:138-226 that the
    EF-sign and DGC consumers use (`_agg(data, op=, communication_scheme=, async_op=)`):
    RCCL collectives on ROCm, gloo on CPU.

    Built as the reference builds it (communication.py:141-151; dgc.py:53-59 and
    ef_sign_sgd.py:41-47 pass `world=conf.graph.ranks`, a list, which the reference
    ignores): the group is `dist.new_group` of the neighbour ranks (every rank must make
    the same call, as with the reference) and the world size is the number of neighbour
    ranks.  `group=` overrides the group (e.g. an existing one); no neighbours -> the
    default group."""

    def __init__(self, rank, world=None, neighbors_info=None, group=None):
        self.rank = rank
        neighbor_ranks = list(neighbors_info.keys()) if neighbors_info else []
        if group is not None:
            self.group = group
        elif neighbor_ranks and dist.is_initialized():
            self.group = dist.new_group(neighbor_ranks)
        else:
            self.group = None
        if neighbor_ranks:
            self.world_size = float(len(neighbor_ranks))
        elif isinstance(world, (list, tuple)):
            self.world_size = float(len(world))
        else:
            self.world_size = float(world if world is not None else (dist.get_world_size() if dist.is_initialized()
                                                                      else 1))

    def _agg(self, data, op=None, distributed=True, communication_scheme="all_reduce", async_op=False, **kargs):
        if not distributed:
            return data
        if communication_scheme == "all_reduce":
            if op not in ("avg", "sum"):
                raise NotImplementedError
            req = dist.all_reduce(data, op=dist.ReduceOp.SUM, group=self.group, async_op=async_op)
            if async_op:
                return data, req
            return data / self.world_size if op == "avg" else data
        if communication_scheme == "reduce":
            if op != "sum":
                raise NotImplementedError
            req = dist.reduce(data, dst=kargs["dst_rank"], op=dist.ReduceOp.SUM, group=self.group, async_op=async_op)
            return (data, req) if async_op else data
        if communication_scheme == "all_gather":
            gathered = [torch.empty_like(data) for _ in range(int(self.world_size))]
            req = dist.all_gather(gathered, data, group=self.group, async_op=async_op)
            return (gathered, req) if async_op else gathered
        raise NotImplementedError

    def complete_wait(self, req):
        req.wait()


def get_aggregators(cur_rank, world, neighbors_info, aggregator_type):
    if aggregator_type == "decentralized":
        return DecentralizedAggregation(cur_rank, neighbors_info)
    if aggregator_type == "centralized":
        return CentralizedAggregation(cur_rank, world, neighbors_info)
    raise NotImplementedError(f"aggregator '{aggregator_type}' is outside the compressor path (see DESIGN.md)")
