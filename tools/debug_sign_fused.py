"""Diagnostic: the one-segment sign pack with the fused gossip step, and the deferred receive,
each against the oracle, array by array (first mismatching element printed)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from chocosgd_amd import _lib, codec  # noqa: E402
from oracle import choco_oracle as O  # noqa: E402

DEV = "cuda"
G = 0.9


def host(t):
    return t.cpu().numpy()


def cmp(name, a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    bad = np.nonzero(a.view(np.uint32) != b.view(np.uint32))[0]
    print(f"  {name}: {'ok' if bad.size == 0 else f'{bad.size} differ, first at {bad[0]}: {a[bad[0]]!r} vs {b[bad[0]]!r}'}",
          flush=True)


def main():
    if len(sys.argv) > 1:
        _lib.load(sys.argv[1])
    for n in (4_000_000, 1_234_567):
        g = torch.Generator(device=DEV).manual_seed(7)
        x = torch.randn(n, generator=g, device=DEV)
        h = x + 0.1 * torch.randn(n, generator=g, device=DEV)
        m = h + 0.05 * torch.randn(n, generator=g, device=DEV)
        x0, h0, m0 = host(x), host(h), host(m)
        print(f"n {n}: pack with the fused step")
        xa = x.clone()
        p, nm = codec.sign_compress(xa, xhat=h, gossip=(m, G))
        xo = O.gossip_step(x0, m0, h0, G)
        cmp("x", host(xa), xo)
        cmp("words", host(p).view(np.float32), O.sign_pack((xo - h0).astype(np.float32)).view(np.float32))
        d = torch.randn(n, generator=g, device=DEV)
        msg = codec.sign_compress(d)
        print(f"n {n}: deferred receive (one message, self)")
        xb, hb, mb = x.clone(), h.clone(), m.clone()
        pb, nb = codec.sign_recv_gossip_compress([msg], [0.5], 0, xb, mb, hb, G)
        hs, ms = h0.copy(), m0.copy()
        O.sign_accumulate(hs, ms, [(host(msg[0]), host(msg[1]))], [0.5], 0, [n])
        xo = O.gossip_step(x0, ms, hs, G)
        cmp("x", host(xb), xo)
        cmp("x_hat", host(hb), hs)
        cmp("memory", host(mb), ms)
        cmp("words", host(pb).view(np.float32), O.sign_pack((xo - hs).astype(np.float32)).view(np.float32))


if __name__ == "__main__":
    main()
