"""ParallelCHOCO's process variant for tests/test_gpu_multiproc.py (not a test module).

    python tests/_mp_ipc_worker.py <comm_op> <world> <outdir>

The reference's ParallelCHOCO (dl_code/pcode/optim/parallel_choco.py:64-87,
95-187) runs the compressor in a separate "sync" process: the trainer puts its
CUDA parameter tensors into a torch.multiprocessing queue (CUDA IPC), the sync
process opens its own process group (:127-130) and, when the trainer sets
`updated_local_model_flag`, runs CHOCOCompressor.pipeline on the SHARED tensors
(:153-187), writing x_hat / memory in place.

Here: this launcher never touches the GPU; it spawns one trainer per rank; each
trainer allocates x, x_hat and memory on the GPU and spawns its sync process
(spawn context), hands it the tensors through a queue (IPC handles), sets the
flag, waits for `gossiped` and saves what its own tensors hold afterwards.  The
sync processes of all ranks form the gloo group and exchange with
comm_device="cpu" through the drop-in DecentralizedAggregation.
"""
import os
import socket
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from _mp_choco_worker import LENS, RATIO, inputs  # noqa: E402


def _sync_main(rank, world, port, comm_op, queue, updated, gossiped, outdir):
    """The sync process: parallel_choco.py:_sync_thread_func with the drop-in compressor."""
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(0)
    x, xh, hat, mem = queue.get()  # CUDA tensors shared over IPC (no copy)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from chocosgd_amd import parallel_choco
        from chocosgd_amd.communication import DecentralizedAggregation, neighborhood
        from chocosgd_amd.parallel_choco import CHOCOCompressor
        from chocosgd_amd.tensor_buffer import TensorBuffer
        parallel_choco._draw_seed = lambda: 1000 + rank  # pinned per-worker seeds (random-k, QSGD)
        nb = neighborhood(rank, world)
        comp = CHOCOCompressor(aggregator=DecentralizedAggregation(rank, nb), comm_op=comm_op, comm_device="cpu",
                               compress_ratio=RATIO, quantize_level=4, is_biased=False, backend="gloo",
                               use_ipc=True)
        sizes = [(m,) for m in LENS]
        sb = {"original_shapes": [(torch.Size([m]), m) for m in LENS],
              "flatten_params": TensorBuffer.from_flat(x, sizes), "flatten_hat_params": TensorBuffer.from_flat(xh, sizes)}
        nhp = {rank: TensorBuffer.from_flat(hat, sizes), "memory": TensorBuffer.from_flat(mem, sizes)}
        updated.wait(timeout=120)
        comp.pipeline(sync_buffer=sb, neighbor_hat_params=nhp, neighbors_info=nb)  # the reference's own entry
        if hasattr(comp.compressor_fn, "check"):  # bad received indices: raise here, not later
            comp.compressor_fn.check(wait=True)
        torch.cuda.synchronize()
        np.savez(os.path.join(outdir, f"msgs{rank}.npz"),
                 **{f"msg{r}": m.cpu().numpy() for r, m in sb["synced_message"].items()})
        dist.barrier()
    finally:
        gossiped.set()
        dist.destroy_process_group()


def _trainer_main(rank, world, port, comm_op, outdir):
    sys.path.insert(0, ROOT)
    import torch
    import torch.multiprocessing as tmp
    # the sync process is started before this one touches the GPU (the reference starts
    # it from the optimizer's constructor, parallel_choco.py:66-82)
    ctx = tmp.get_context("spawn")
    queue, updated, gossiped = ctx.Queue(), ctx.Event(), ctx.Event()
    child = ctx.Process(target=_sync_main, args=(rank, world, port, comm_op, queue, updated, gossiped, outdir),
                        name="Sync-Thread", daemon=True)
    child.start()
    torch.cuda.set_device(0)
    x, xh, hat0, mem0 = inputs(rank)
    shared = [torch.from_numpy(a).cuda() for a in (x, xh, hat0, mem0)]
    torch.cuda.synchronize()
    queue.put(shared)
    updated.set()
    gossiped.wait(timeout=300)
    child.join(timeout=120)
    if child.exitcode != 0:
        raise SystemExit(f"sync process of rank {rank} exited with {child.exitcode}")
    # what the trainer's own tensors hold after the sync process worked on them
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), hat=shared[2].cpu().numpy(), mem=shared[3].cpu().numpy(),
             x=shared[0].cpu().numpy())


def main():
    comm_op, world, outdir = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    import multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_trainer_main, args=(r, world, port, comm_op, outdir)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=400)
    codes = [p.exitcode for p in procs]
    if any(c != 0 for c in codes):
        print(f"trainer exit codes {codes}", file=sys.stderr)
        sys.exit(1)
    for r in range(world):
        with np.load(os.path.join(outdir, f"msgs{r}.npz")) as z:
            d = dict(z)
        with np.load(os.path.join(outdir, f"rank{r}.npz")) as z:
            d.update(dict(z))
        np.savez(os.path.join(outdir, f"rank{r}.npz"), **d)


if __name__ == "__main__":
    main()
