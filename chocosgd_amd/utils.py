"""Gossip-step helpers: drop-in for the CHOCO half of dl_code/pcode/optim/utils.py."""
from . import codec
from .tensor_buffer import TensorBuffer


def _get_data(param_groups, idx, is_get_grad):
    if is_get_grad:
        return param_groups[idx]["params"][0].grad
    return param_groups[idx]["params"][0]


def recover_params(param_groups, param_names, rank=None, neighbor_hat_params=None, get_hat_params=True):
    """optim/utils.py:50-64: flat copies of the params (and of x_hat_i)."""
    params = [_get_data(param_groups, idx, False) for idx, _ in param_names]
    params = [p for p in params if p is not None]
    flatten_params = TensorBuffer(params)
    if get_hat_params:
        assert neighbor_hat_params is not None and rank is not None
        flatten_hat_params = TensorBuffer(params)
        flatten_hat_params.buffer.data[:] = neighbor_hat_params[rank].buffer
        return params, flatten_params, flatten_hat_params
    return params, flatten_params


def fused_step(compressor, param_groups, param_names, shapes, neighbor_hat_params, neighbors_info,
               consensus_stepsize, rank, defer_receive=False):
    """ParallelCHOCO_V.step after apply_gradient (parallel_choco_v.py:115-155), with the
    consensus step fused into the compressor's first pass: recover_params, then
    compress (x += gamma * (memory - x_hat_i) and d = x_new - x_hat_i in one pass), sync,
    uncompress, and the updated x unpacked into the model.  Returns the sync_buffer.
    The reference runs update_params_from_neighbor as its own pass before compress.

    defer_receive=True (QSGD, sign): this step's uncompress is applied by the NEXT step's
    compress, in the same pass as that step's consensus step (the reference's step runs
    the previous step's join, then update_params_from_neighbor, with only apply_gradient
    -- which touches x alone -- in between, parallel_choco_v.py:104-131).  x is the same
    after every step; x_hat / memory lag by one step until the next step or
    compressor.flush_receive() (call it before reading or saving them).  flatten_hat_params
    is x_hat_i itself, not a copy (the pass updates it in place)."""
    if defer_receive:
        params, flatten_params = recover_params(param_groups, param_names, get_hat_params=False)
        flatten_hat_params = neighbor_hat_params[rank]
    else:
        if hasattr(compressor, "flush_receive"):  # a receive an earlier deferred step left
            compressor.flush_receive()
        params, flatten_params, flatten_hat_params = recover_params(param_groups, param_names, rank,
                                                                    neighbor_hat_params, get_hat_params=True)
    sync_buffer = {"original_shapes": shapes, "flatten_params": flatten_params,
                   "flatten_hat_params": flatten_hat_params,
                   "gossip": (neighbor_hat_params["memory"].buffer, consensus_stepsize)}
    if defer_receive:
        sync_buffer["defer_receive"] = True
    compressor.pipeline(sync_buffer, neighbor_hat_params, neighbors_info)
    flatten_params.unpack(params)
    return sync_buffer


def update_params_from_neighbor(neighbor_hat_params, flatten_params, consensus_stepsize, self_rank):
    """optim/utils.py:67-72:  x += gamma * (memory - x_hat_i), one fused HIP pass."""
    codec.gossip_step(flatten_params.buffer, neighbor_hat_params["memory"].buffer,
                      neighbor_hat_params[self_rank].buffer, consensus_stepsize)
