"""Inputs of the ring fixtures (not a test module).

tests/golden/gen_golden.py `gen_ring` runs the reference's CHOCO compressors for every
worker of a ring of 8 (neighbourhoods from the reference's own RingGraph mixing matrix,
topology.py:186-202,295-299) on these inputs and records each worker's x_hat / memory;
the tests regenerate the same inputs from the seeds and replay the ring through the
oracle (CPU) and through the drop-in on the GPU.
"""
import numpy as np

RING_LAYOUT = [300, 5, 1029, 17, 2000, 3]
RING_WORLD = 8
RING_RATIO = 0.9


def ring_inputs(rank, lens=RING_LAYOUT):
    """Worker `rank`'s x, x_hat (flatten_hat_params), and its x_hat_i / memory state."""
    n = sum(lens)
    rng = np.random.default_rng(7000 + rank)
    x = rng.standard_normal(n).astype(np.float32)
    xh = (x + 0.1 * rng.standard_normal(n)).astype(np.float32)
    hat0 = (0.3 * rng.standard_normal(n)).astype(np.float32)
    mem0 = (0.3 * rng.standard_normal(n)).astype(np.float32)
    return x, xh, hat0, mem0
