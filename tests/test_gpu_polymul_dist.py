"""Polynomial multiply on the GPU: squaring (a == b) on one GPU, and the distributed polymul of
BASELINE config 5 (forward(a), forward(b) in ONE all-to-all, local pointwise product
fused into the inverse's first column pass, inverse all-to-all back to the row layout).

The distributed result is compared bit for bit with the single-GPU ntt_polymul of the same vectors
(itself checked against the oracle's cyclic product in test_gpu_parity.py and below), through
virtual ranks (one GPU, exchange = device copies) at G = 1..8 up to C5's 2^24, the single-process
multi-GPU plan (ntt_polymul_multi, RCCL) and DistNTT over a torch.distributed RCCL group.
"""
import os

import numpy as np
import pytest
import torch

from oracle import ntt_ref as R
from oracle import oracle_c as OC

pytestmark = pytest.mark.gpu


def _plan(fid, log_n, L):
    from ntt_amd.ntt import NTTPlan
    return NTTPlan(field_id=fid, log_n=log_n, limbs64=L, device=0)


def _host(t, L):
    return t.cpu().numpy().view(np.uint64).reshape(-1, L)


@pytest.mark.parametrize("fid,L,log_n", [(1, 4, 12), (1, 4, 16), (2, 6, 13), (0, 1, 14), (0, 4, 12)])
def test_single_gpu_squaring_matches_oracle(fid, L, log_n):
    """polymul(a, a, c) used to forward-transform a twice."""
    p, g = R.FIELDS[fid]
    pl = _plan(fid, log_n, L)
    a = pl.fill(pl.empty(), "random", seed=80 + log_n)
    x = _host(a, L).copy()
    c = pl.empty()
    pl.polymul(a, a, c)
    if L == 1:
        A = OC.ntt_u64(x[:, 0].astype(np.int64), p, g)
        C2 = np.array([int(u) * int(u) % p for u in A], dtype=np.int64)
        exp = OC.ntt_u64(C2, p, g, True).astype(np.uint64).reshape(-1, 1)
    else:
        A = OC.ntt_mp(x, p, g)
        exp = OC.ntt_mp(OC.mul_mp(A, A, p), p, g, inverse=True)
    assert np.array_equal(_host(c, L), exp)


def _row_index(lay, device):
    i = torch.arange(lay.local_n, dtype=torch.int64, device=device)
    return lay.rank * lay.r + (i >> lay.log_n2) + lay.n1 * (i & (lay.n2 - 1))


def _single_gpu_product(fid, L, log_n, seed_a, seed_b):
    pl = _plan(fid, log_n, L)
    a = pl.fill(pl.empty(), "random", seed=seed_a)
    b = a if seed_b is None else pl.fill(pl.empty(), "random", seed=seed_b)
    c = pl.empty()
    pl.polymul(a, b, c)
    return c


@pytest.mark.parametrize("world,fid,L,log_n,square,pieces", [(1, 1, 4, 12, False, 1), (2, 1, 4, 13, False, 1),
                                                             (4, 1, 4, 16, False, 1), (8, 1, 4, 20, False, 1),
                                                             (8, 2, 6, 16, False, 1), (2, 0, 1, 14, False, 1),
                                                             (4, 1, 4, 14, True, 1), (4, 1, 4, 16, False, 4),
                                                             (8, 2, 6, 16, False, 3), (4, 1, 4, 14, True, 2),
                                                             (2, 0, 1, 14, False, 2), (2, 1, 4, 12, False, 2),
                                                             (2, 1, 4, 22, False, 4)])
def test_virtual_ranks_polymul_matches_single_gpu(world, fid, L, log_n, square, pieces):
    """pieces > 1: as many row and column pieces (VirtualRanks' default), exchanged as one
    multi-tensor copy per unit (batched); the P field (no fused
    product) and 2^12 over 2 (single-pass column transforms) take the gathered-product path of
    ntt_rplan_inverse_cols_piece."""
    from ntt_amd.distributed import VirtualRanks
    exp = _single_gpu_product(fid, L, log_n, 5, None if square else 6)
    vr = VirtualRanks(fid, log_n, L, world, pieces=pieces, batched=pieces > 1)
    As = vr.fill(vr.empty(), "random", seed=5)
    Bs = As if square else vr.fill(vr.empty(), "random", seed=6)
    Outs = vr.empty()
    vr.polymul(As, Bs, Outs)
    for lay, o in zip(vr.layouts, Outs):
        assert torch.equal(o, exp[_row_index(lay, o.device)]), (world, log_n, lay.rank)


@pytest.mark.parametrize("batched", [False, True])
def test_c5_polymul_2pow24_eight_virtual_ranks(batched):
    """BASELINE config 5's size and GPU count, on one GPU: bit-exact vs the single-GPU product.
    batched: each exchange unit's copies as one multi-tensor copy."""
    from ntt_amd.distributed import VirtualRanks
    fid, L, log_n, world = 1, 4, 24, 8
    exp = _single_gpu_product(fid, L, log_n, 5, 6)
    vr = VirtualRanks(fid, log_n, L, world, pieces=4, batched=batched)  # the pipelined exchange, as timed in bench_configs
    As = vr.fill(vr.empty(), "random", seed=5)
    Bs = vr.fill(vr.empty(), "random", seed=6)
    vr.polymul(As, Bs, As)  # out aliases a
    for lay, o in zip(vr.layouts, As):
        assert torch.equal(o, exp[_row_index(lay, o.device)]), lay.rank


@pytest.mark.parametrize("log_n,pieces,col_pieces", [(16, None, None), (24, None, None), (16, 4, None), (24, 8, None),
                                                     (16, 4, 4), (24, 2, 4), (14, 2, 2)])
def test_mplan_polymul_matches_single_gpu(log_n, pieces, col_pieces):
    """col_pieces: the two-sided schedule (a and b in every unit of the forward; the product fused
    into the inverse's column pieces, or gathered at 2^14 where the column transforms are one pass)."""
    from ntt_amd.distributed import MultiPlan
    fid, L = 1, 4
    exp = _single_gpu_product(fid, L, log_n, 5, 6)
    mp = MultiPlan(fid, log_n, L, devices=list(range(torch.cuda.device_count())), pieces=pieces,
                   col_pieces=col_pieces)
    As = mp.fill(mp.empty(), "random", seed=5)
    Bs = mp.fill(mp.empty(), "random", seed=6)
    Outs = mp.empty()
    mp.polymul(As, Bs, Outs)
    for lay, o in zip(mp.layouts, Outs):
        assert torch.equal(o.to("cuda:0"), exp[_row_index(lay, "cuda:0")]), lay.rank
    # squaring through the same entry point (a == b: one forward, single-vector exchange)
    exp2 = _single_gpu_product(fid, L, log_n, 5, None)
    As = mp.fill(mp.empty(), "random", seed=5)
    mp.polymul(As, As, Outs)
    for lay, o in zip(mp.layouts, Outs):
        assert torch.equal(o.to("cuda:0"), exp2[_row_index(lay, "cuda:0")]), lay.rank
    del mp


def test_mplan_polymul_2pow26_chunked_rows():
    """2^26 on the visible devices: at world size 1 the rank plan splits 2^16 x 2^10, so the row
    transforms of a and b (nvec = 2) run in launches of 2^15 rows; bit-exact vs the one-GPU product."""
    from ntt_amd.distributed import MultiPlan
    fid, L, log_n = 1, 4, 26
    exp = _single_gpu_product(fid, L, log_n, 5, 6)
    mp = MultiPlan(fid, log_n, L, devices=list(range(torch.cuda.device_count())))
    As = mp.fill(mp.empty(), "random", seed=5)
    Bs = mp.fill(mp.empty(), "random", seed=6)
    Outs = mp.empty()
    mp.polymul(As, Bs, Outs)
    chunk = 1 << 22  # one torch gather over 2^26 rows fails its launch configuration on this build
    for lay, o in zip(mp.layouts, Outs):
        idx = _row_index(lay, "cuda:0")
        o = o.to("cuda:0")
        for i in range(0, idx.numel(), chunk):
            assert torch.equal(o[i:i + chunk], exp[idx[i:i + chunk]]), (lay.rank, i)
    del mp


def test_dist_ntt_polymul_rccl_world1():
    import torch.distributed as dist
    from ntt_amd.distributed import DistNTT
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = "29563"
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    try:
        log_n = 18
        exp = _single_gpu_product(1, 4, log_n, 5, 6)
        # whole blocks; pipelined async RCCL units (a and b in each), row pieces only and both sides
        for pieces, col_pieces in ((None, None), (4, 1), (4, 4)):
            d = DistNTT(1, log_n, 4, device=0, pieces=pieces, col_pieces=col_pieces)
            a = d.fill(d.empty(), "random", seed=5)
            b = d.fill(d.empty(), "random", seed=6)
            out = d.empty()
            d.polymul(a, b, out)
            assert torch.equal(out, exp[_row_index(d.layout, "cuda:0")]), (pieces, col_pieces)
    finally:
        dist.destroy_process_group()
