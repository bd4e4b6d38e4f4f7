"""Multi-process CHOCO gossip round for tests/test_gpu_multiproc.py (not a test module).

    python tests/_mp_choco_worker.py <comm_op> <world> <outdir>

This launcher process never touches the GPU: it starts `world` rank processes
(spawn), each of which builds the drop-in CHOCOCompressor with the reference's
DecentralizedAggregation over gloo and comm_device="cpu" (pinned host staging,
parallel_choco_v.py:271-272), runs compress -> sync -> uncompress on the one
GPU, and saves its x_hat / memory and every received message to <outdir>.
"""
import os
import socket
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LENS = [3, 70_001, 5, 1_100_003, 17, 300]
RATIO = 0.9
CHUNKS = 4  # exchange_chunks of the *_chunked comm ops (ranges of 294,912 elements)


def inputs(rank):
    """Worker `rank`'s x, x_hat (its own flatten_hat_params), and its x_hat_i / memory state."""
    n = sum(LENS)
    rng = np.random.default_rng(100 + rank)
    x = rng.standard_normal(n).astype(np.float32)
    xh = (rng.standard_normal(n) * 0.5).astype(np.float32)
    hat0 = rng.standard_normal(n).astype(np.float32)
    mem0 = rng.standard_normal(n).astype(np.float32)
    return x, xh, hat0, mem0


DEFER_STEPS = 4
GAMMA = 0.5


def _defer_steps(rank, comp, nb, split, state, outdir, dist, torch):
    """`*_defer`: DEFER_STEPS fused CHOCO steps (sync_buffer["gossip"], x_hat_i itself as
    flatten_hat_params) twice over the same start state -- the receive applied at once, then
    deferred into the next step's first pass (sync_buffer["defer_receive"]) and flushed at the
    end; x after every step and the final x_hat / memory are saved for both runs."""
    from chocosgd_amd.tensor_buffer import TensorBuffer
    x0, hat0, mem0 = state
    shapes = [(torch.Size([m]), m) for m in LENS]
    out = {}
    for tag, defer in (("now", False), ("deferred", True)):
        x = TensorBuffer(split(x0))
        nhp = {rank: TensorBuffer(split(hat0)), "memory": TensorBuffer(split(mem0))}
        for step in range(DEFER_STEPS):
            sb = {"original_shapes": shapes, "flatten_params": x, "flatten_hat_params": nhp[rank],
                  "gossip": (nhp["memory"].buffer, GAMMA)}
            if defer:
                sb["defer_receive"] = True
            with torch.cuda.stream(comp.compressor_fn.gossip_stream):
                comp.compress(sb)
                comp.sync(sb)
                comp.uncompress(sb, nhp, nb)
            torch.cuda.synchronize()
            out[f"{tag}_x{step}"] = x.buffer.cpu().numpy()
        comp.flush_receive()
        torch.cuda.synchronize()
        out[f"{tag}_hat"] = nhp[rank].buffer.cpu().numpy()
        out[f"{tag}_mem"] = nhp["memory"].buffer.cpu().numpy()
        dist.barrier()
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), **out)
    dist.barrier()


def _rank_main(rank, world, port, comm_op, outdir):
    global LENS
    defer_steps = comm_op.endswith("_defer")
    comm_op = comm_op[:-len("_defer")] if defer_steps else comm_op
    if comm_op == "sign1":  # one segment: the single-kernel deferred sign receive
        LENS = [sum(LENS)]
        comm_op = "sign"
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from chocosgd_amd import parallel_choco
        from chocosgd_amd.communication import DecentralizedAggregation, neighborhood
        from chocosgd_amd.parallel_choco import CHOCOCompressor
        from chocosgd_amd.tensor_buffer import TensorBuffer
        parallel_choco._draw_seed = lambda: 1000 + rank  # pinned per-worker seeds (random-k, QSGD)
        nb = neighborhood(rank, world)
        if comm_op.endswith("_refagg"):
            class _RefAgg(DecentralizedAggregation):  # the reference's _agg signature (no out=)
                def _agg(self, data, op, force_wait=True):
                    return DecentralizedAggregation._agg(self, data, op, force_wait)
            agg = _RefAgg(rank, nb)
            comm_op = comm_op[:-len("_refagg")]
        else:
            agg = DecentralizedAggregation(rank, nb)
        chunks = CHUNKS if comm_op.endswith("_chunked") else 1
        comp = CHOCOCompressor(aggregator=agg, comm_op=comm_op.replace("_chunked", ""), comm_device="cpu",
                               compress_ratio=RATIO, quantize_level=4, is_biased=False, backend="gloo",
                               use_ipc=False, exchange_chunks=chunks)
        x, xh, hat0, mem0 = inputs(rank)

        def split(a):
            t = torch.from_numpy(a).cuda()
            out, p = [], 0
            for m in LENS:
                out.append(t[p:p + m].clone())
                p += m
            return out
        if defer_steps:
            return _defer_steps(rank, comp, nb, split, (x, hat0, mem0), outdir, dist, torch)
        sb = {"original_shapes": [(torch.Size([m]), m) for m in LENS],
              "flatten_params": TensorBuffer(split(x)), "flatten_hat_params": TensorBuffer(split(xh))}
        nhp = {rank: TensorBuffer(split(hat0)), "memory": TensorBuffer(split(mem0))}
        # pipeline() without its except-and-print, so a failure fails the test
        with torch.cuda.stream(comp.compressor_fn.gossip_stream):
            comp.compress(sb)
            comp.sync(sb)
            comp.uncompress(sb, nhp, nb)
        torch.cuda.synchronize()
        out = {"hat": nhp[rank].buffer.cpu().numpy(), "mem": nhp["memory"].buffer.cpu().numpy()}
        for r, m in sb["synced_message"].items():
            if isinstance(m, list):  # chunked wire: [norms header, range 0, range 1, ...]
                for i, part in enumerate(m):
                    out[f"msg{r}_{i}"] = part.cpu().numpy()
            else:
                out[f"msg{r}"] = m.cpu().numpy()
        np.savez(os.path.join(outdir, f"rank{rank}.npz"), **out)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def grads_of(rank):
    """Worker `rank`'s gradient, error-feedback memory and parameters (centralized consumers)."""
    n = sum(LENS)
    rng = np.random.default_rng(500 + rank)
    g = rng.standard_normal(n).astype(np.float32)
    mem = (rng.standard_normal(n) * 0.25).astype(np.float32)
    params = rng.standard_normal(n).astype(np.float32)
    return g, mem, params


LR = 0.1


def _rank_central(rank, world, port, comm_op, outdir):
    """EF-signSGD / DGC through the centralized aggregator built as the reference builds it
    (ef_sign_sgd.py:41-47, dgc.py:53-59: get_aggregators(cur_rank, world=ranks,
    neighbors_info={r: 1 / n_nodes}, "centralized") -> communication.py:138-224), all-gathers
    over gloo with comm_device="cpu"."""
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from chocosgd_amd.communication import get_aggregators
        from chocosgd_amd.tensor_buffer import TensorBuffer
        ranks = list(range(world))
        agg = get_aggregators(cur_rank=rank, world=ranks, neighbors_info={r: 1.0 / world for r in ranks},
                              aggregator_type="centralized")
        g, mem, params = grads_of(rank)

        def split(a):
            t = torch.from_numpy(a).cuda()
            out, p = [], 0
            for m in LENS:
                out.append(t[p:p + m].clone())
                p += m
            return out
        out = {}
        if comm_op == "efsign":
            from chocosgd_amd.ef_sign import EFSignCompressor
            comp = EFSignCompressor(rank=rank, world_size=world, aggregator=agg, comm_op="sign", comm_device="cpu",
                                    use_ipc=False)
            sb = comp.compress(TensorBuffer(split(g)))
            out["local"] = sb["synced_grads_tb"].buffer.cpu().numpy()
            comp.sync(sb)
            out["out"] = comp.decompress(sb).buffer.cpu().numpy()
            for r, m in enumerate(sb["synced_message"]):
                out[f"msg{r}"] = m.cpu().numpy()
        else:  # dgc_top_k: DGC's top-k with the reference's 255 / 254 memory mask (strict default)
            from chocosgd_amd.dgc import DGCCodec
            c = DGCCodec(world_aggregator=agg, comm_op="compress_top_k", comm_device="cpu", n_nodes=world)
            memory = TensorBuffer(split(mem))
            vals, idx, _ = c.compress(split(g), memory, RATIO)
            synced, size = c.sync(vals, idx)
            flat = torch.from_numpy(params).cuda()
            out["params"] = c.recover_info(flat, synced, size, LR).cpu().numpy()
            out["mem"] = memory.buffer.cpu().numpy()
            for r, m in enumerate(synced):
                out[f"msg{r}"] = m.cpu().numpy()
        torch.cuda.synchronize()
        np.savez(os.path.join(outdir, f"rank{rank}.npz"), **out)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def main():
    comm_op, world, outdir = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    import multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    target = _rank_central if comm_op in ("efsign", "dgc_top_k") else _rank_main
    procs = [ctx.Process(target=target, args=(r, world, port, comm_op, outdir)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    codes = [p.exitcode for p in procs]
    if any(c != 0 for c in codes):
        print(f"rank exit codes {codes}", file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()
