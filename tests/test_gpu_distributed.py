"""GPU checks of the multi-GPU four-step (ntt_amd.distributed) on a single MI355X:

* G virtual ranks in one process (exchange = device copies), G = 1, 2, 4, 8: the gathered column
  layout equals the single-GPU transform (itself checked against the oracle in test_gpu_parity),
  and inverse(forward(x)) returns every rank's row-layout share;
* a real torch.distributed (RCCL) process group of world size 1 through DistNTT.
"""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _index(layout, kind):
    i = torch.arange(layout.local_n, dtype=torch.int64, device="cuda:0")
    if kind == "row":
        a, j2 = i >> layout.log_n2, i & (layout.n2 - 1)
        return layout.rank * layout.r + a + layout.n1 * j2
    k1, kc = i >> layout.log_c, i & (layout.c - 1)  # column layout [n1][c]
    return layout.rank * layout.c + kc + layout.n2 * k1


def _eq_at(t, src, idx, chunk=1 << 22):
    """t == src[idx], gathered in chunks (one torch gather over 2^26 rows fails its launch
    configuration on this ROCm build)."""
    return all(torch.equal(t[i:i + chunk], src[idx[i:i + chunk]]) for i in range(0, idx.numel(), chunk))


@pytest.mark.parametrize("batched", [False, True])
@pytest.mark.parametrize("world,log_n,field_id,L,pieces,col_pieces",
                         [(1, 12, 1, 4, 1, 1), (2, 12, 1, 4, 1, 1), (4, 16, 1, 4, 1, 1), (8, 20, 1, 4, 1, 1),
                          (8, 16, 2, 6, 1, 1), (2, 14, 0, 1, 1, 1), (2, 12, 1, 4, 4, 1), (8, 20, 1, 4, 4, 1),
                          (4, 16, 1, 4, 3, 1), (8, 16, 2, 6, 2, 1), (2, 14, 0, 1, 8, 1), (1, 22, 1, 4, 1, 1),
                          (4, 22, 1, 4, 2, 1), (8, 24, 1, 4, 1, 1), (2, 22, 2, 6, 1, 1), (1, 26, 1, 4, 1, 1),
                          (2, 12, 1, 4, 1, 4), (2, 12, 1, 4, 4, 4), (8, 20, 1, 4, 4, 4), (4, 16, 1, 4, 2, 8),
                          (2, 14, 0, 1, 2, 2), (8, 16, 2, 6, 2, 2), (4, 22, 1, 4, 4, 4), (2, 24, 1, 4, 2, 2),
                          (1, 26, 1, 4, 4, 8), (2, 21, 1, 4, 1, 1), (4, 21, 1, 4, 2, 2)])
def test_virtual_ranks_match_single_gpu(world, log_n, field_id, L, pieces, col_pieces, batched):
    """batched: each exchange unit's copies as one multi-tensor copy.  pieces / col_pieces > 1: the pipelined schedule (the exchange units copied on a side stream
    while the row transforms before them and the column transforms after them run) -- same column
    layout, same round trip.  2^22 / 2^24 / 2^26: the rank plans' unbalanced split (n2 = 2^10, one
    workgroup tile per row transform); 2^26 at world 1 has 2^16 rows per rank, launched in chunks of
    2^15 (grid.y).  2^21 splits 14 + 7: 2^7-point rows, eight per workgroup (KIND_ROWS) with the Mode B
    output map and the epilogue table; 2^12 (6 + 6) takes KIND_ROWS in Mode I too."""
    from ntt_amd.distributed import VirtualRanks
    from ntt_amd.ntt import NTTPlan
    ref = NTTPlan(field_id, log_n, L)
    x = ref.empty()
    ref.fill(x, "random", seed=42)
    x0 = x.clone()
    ref.forward(x)
    vr = VirtualRanks(field_id, log_n, L, world, pieces=pieces, col_pieces=col_pieces, batched=batched)
    xs = vr.fill(vr.empty(), "random", seed=42)
    for lay, t in zip(vr.layouts, xs):  # row-layout shares hold the right global elements
        assert _eq_at(t, x0, _index(lay, "row"))
    shares = [t.clone() for t in xs]
    vr.forward(xs)
    for lay, t in zip(vr.layouts, xs):
        assert _eq_at(t, x, _index(lay, "col")), (world, log_n, lay.rank)
    vr.inverse(xs)
    for s, t in zip(shares, xs):
        assert torch.equal(s, t)


def test_piece_entry_points_reject_bad_pieces():
    """ntt_rplan_*_piece: piece counts must be powers of two within the rows / columns and the piece
    index within its count; ntt_mplan_set_pieces2 likewise (NTT_ERR_ARG, nothing launched)."""
    import ctypes as C
    from ntt_amd import lib as L
    from ntt_amd.distributed import MultiPlan, RankPlan
    lib = L.load()
    rp = RankPlan(1, 12, 4, 2, 0, 0)  # rank 0 of 2; the split is read from the plan
    lay = rp.layout
    x, send = rp.empty(lay.local_n), rp.empty(lay.local_n)
    p = lambda t: C.c_void_p(t.data_ptr())
    h = rp.handle
    assert lib.ntt_rplan_forward_rows_piece(h, p(x), p(send), 1, 0, 0, 3, 1, None) == -1          # not 2^k
    assert lib.ntt_rplan_forward_rows_piece(h, p(x), p(send), 1, 0, 2, 2, 1, None) == -1          # index >= count
    assert lib.ntt_rplan_forward_rows_piece(h, p(x), p(send), 1, 0, 0, 2 * lay.r, 1, None) == -1  # > r rows
    assert lib.ntt_rplan_forward_cols_piece(h, p(send), p(x), 1, 0, 0, 1, 2 * lay.c, None) == -1  # > c columns
    assert lib.ntt_rplan_inverse_cols_piece(h, p(x), None, p(send), 4, 1, 4, None) == -1
    assert lib.ntt_rplan_inverse_rows_piece(h, p(send), p(x), 0, 0, 1, None) == -1                # zero pieces
    assert lib.ntt_rplan_forward_rows_piece(h, p(x), p(send), 3, 0, 0, 1, 1, None) == -1          # nvec 3
    mp = MultiPlan(1, 12, 4, devices=[0])
    assert lib.ntt_mplan_set_pieces2(mp.handle, 3, 1) == -1
    assert lib.ntt_mplan_set_pieces2(mp.handle, 1, 32) == -1
    assert lib.ntt_mplan_set_pieces2(mp.handle, 2, 2) == 0


def test_rank_plan_split_takes_fewest_passes():
    """ntt_rplan_create's split: fewest pass kernels, then the smallest largest radix, then the most
    balanced (round 5).  2^24 BN254: 16 + 8 (2 + 1 passes of radix <= 2^8; 12 + 12 takes 2 + 2, 14 + 10
    has a radix-2^10 row pass); 2^22: 14 + 8; 2^21: 14 + 7; 2^20 keeps 10 + 10 (1 + 1); C4's 2^28 keeps 14 + 14,
    asserted in test_gpu_fullsize."""
    from ntt_amd.distributed import RankPlan
    for log_n, world, n2 in ((24, 1, 8), (24, 8, 8), (22, 2, 8), (20, 4, 10), (16, 2, 8), (21, 2, 7)):
        rp = RankPlan(1, log_n, 4, world, 0, 0)
        assert (rp.layout.log_n1, rp.layout.log_n2) == (log_n - n2, n2), log_n
        del rp


def test_dist_ntt_rccl_world1():
    """DistNTT over a real RCCL group (world size 1): whole-block exchange, and the pipelined
    exchange (async RCCL all-to-all per unit; 3 rounds down to 2 pieces) forced on, on one side and
    on both."""
    import torch.distributed as dist
    from ntt_amd.distributed import DistNTT
    from ntt_amd.ntt import NTTPlan
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29561")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    try:
        log_n = 16
        ref = NTTPlan(1, log_n, 4)
        x = ref.fill(ref.empty(), "random", seed=3)
        ref.forward(x)
        for pieces, col_pieces in ((None, None), (4, 1), (3, 1), (1, 4), (4, 8)):
            d = DistNTT(1, log_n, 4, device=0, pieces=pieces, col_pieces=col_pieces)
            assert len(d.fs.pieces) == {None: 1, 4: 4, 3: 2, 1: 1}[pieces]
            assert d.fs.cp == (1 if col_pieces is None else col_pieces)
            t = d.fill(d.empty(), "random", seed=3)
            t0 = t.clone()
            d.forward(t)
            assert torch.equal(t, x[_index(d.layout, "col")]), pieces
            d.inverse(t)
            assert torch.equal(t, t0), pieces
        # the per-launch timings of one call report EVERY launch, with its label.
        # At 2^24 (16 + 8) the row transform runs as two launches of 2^15 rows, then the column
        # transforms' two passes: four launches, the first two of one kind.
        d = DistNTT(1, 24, 4, device=0)
        t = d.fill(d.empty(), "random", seed=2)
        d.set_profiling(True)
        for _ in range(3):
            d.forward(t)
        ms, labels = d.last_launch_ms(), d.last_launch_labels()
        d.set_profiling(False)
        assert len(ms) == 4 and len(labels) == 4, (ms, labels)
        assert labels[0] == labels[1] and all(labels) and all(m > 0 for m in ms), (ms, labels)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("log_n,field_id,L,pieces,col_pieces",
                         [(12, 1, 4, None, None), (17, 1, 4, None, None), (16, 2, 6, None, None),
                          (14, 0, 1, None, None), (12, 1, 4, 4, None), (17, 1, 4, 3, None), (16, 2, 6, 16, None),
                          (14, 0, 1, 2, None), (12, 1, 4, 1, 4), (16, 1, 4, 4, 8), (14, 0, 1, 2, 2),
                          (16, 2, 6, 2, 4), (24, 1, 4, None, None)])
def test_mplan_single_process_rccl(log_n, field_id, L, pieces, col_pieces):
    """ntt_mplan_* (one process, ncclCommInitAll over the visible devices, grouped all-to-all):
    the column-layout output equals the single-GPU transform; the inverse restores the rows.
    pieces / col_pieces: the pipelined exchange on both sides (grouped ncclSend/ncclRecv of the
    exchange units on the plan's communication streams; 3 rounds down to 2; 2^24 on one device: the
    default pieces)."""
    from ntt_amd.distributed import MultiPlan
    from ntt_amd.ntt import NTTPlan
    mp = MultiPlan(field_id, log_n, L, devices=list(range(torch.cuda.device_count())), pieces=pieces,
                   col_pieces=col_pieces)
    xs = mp.fill(mp.empty(), "random", seed=11)
    ref = NTTPlan(field_id, log_n, L)
    x = ref.fill(ref.empty(), "random", seed=11)
    x0 = x.clone()
    for lay, t in zip(mp.layouts, xs):
        assert torch.equal(t.to("cuda:0"), x0[_index(lay, "row")])
    shares = [t.clone() for t in xs]
    ref.forward(x)
    mp.forward(xs)
    for lay, t in zip(mp.layouts, xs):
        assert torch.equal(t.to("cuda:0"), x[_index(lay, "col")]), (log_n, lay.rank)
    mp.inverse(xs)
    for s, t in zip(shares, xs):
        assert torch.equal(s, t)


@pytest.mark.parametrize("fid,L", [(1, 4), (0, 1), (2, 6)])
def test_twiddle_pack_and_transpose_building_blocks(fid, L):
    """ntt_twiddle_pack_ex / ntt_transpose_ex (C-ABI building blocks; the rank plan fuses them into
    the transform passes): against the closed forms on the host."""
    from ntt_amd.ntt import NTTPlan
    from oracle import ntt_ref as R
    from oracle import oracle_c as OC
    import numpy as np
    p, g = R.FIELDS[fid]
    log_n, lr, ll, lb = 12, 3, 6, 4
    pl = NTTPlan(fid, log_n, L, twiddle_only=True)
    n = 1 << log_n
    w = R.root_of_unity(p, g, n)
    rows, length, bw = 1 << lr, 1 << ll, 1 << lb
    src_np = OC.random_limbs(fid, rows * length, seed=3, L=L)
    src = torch.from_numpy(src_np.view(np.int64)).to("cuda:0").reshape(-1, L) if L > 1 else \
        torch.from_numpy(src_np.view(np.int64).reshape(-1)).to("cuda:0")
    ps = 2 * rows * bw
    dst = torch.zeros((length // bw) * ps * L, dtype=torch.int64, device="cuda:0")
    dst = dst.reshape(-1, L) if L > 1 else dst
    row0 = 5
    pl.twiddle_pack(src, dst, lr, ll, lb, row0, False, peer_stride=ps)
    got = OC.limbs_to_ints(dst.cpu().numpy().view(np.uint64).reshape(-1, L))
    sv = OC.limbs_to_ints(src_np)
    for a in range(rows):
        for b in range(length):
            assert got[(b // bw) * ps + a * bw + b % bw] == sv[a * length + b] * pow(w, (row0 + a) * b % n, p) % p
    # transpose of a matrix whose row blocks are spread at block_stride
    lrows, lcols, lbr = 5, 3, 2
    bs = 3 * (1 << (lbr + lcols))
    nblk = 1 << (lrows - lbr)
    src2 = torch.arange(nblk * bs * L, dtype=torch.int64, device="cuda:0")
    src2 = src2.reshape(-1, L) if L > 1 else src2
    out = torch.empty(((1 << (lrows + lcols)), L) if L > 1 else (1 << (lrows + lcols),), dtype=torch.int64,
                      device="cuda:0")
    pl.transpose(src2, out, lrows, lcols, log_block_rows=lbr, block_stride=bs)
    s2 = src2.cpu().reshape(nblk * bs, -1)
    o = out.cpu().reshape(1 << lcols, 1 << lrows, -1)
    for r_ in range(1 << lrows):
        for c_ in range(1 << lcols):
            srow = (r_ >> lbr) * bs + (r_ & ((1 << lbr) - 1)) * (1 << lcols) + c_
            assert torch.equal(o[c_, r_], s2[srow])


def _dist_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    from ntt_amd.distributed import DistNTT
    from ntt_amd.ntt import NTTPlan
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    try:
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        log_n = 16
        ref = NTTPlan(1, log_n, 4)
        X = ref.fill(ref.empty(), "random", seed=8)
        ref.forward(X)
        A, B, C = ref.fill(ref.empty(), "random", seed=5), ref.fill(ref.empty(), "random", seed=6), ref.empty()
        ref.polymul(A, B, C)
        ok_f = ok_i = ok_p = True
        # whole blocks, then the two-sided pieces (units exchanged one by one between the processes)
        for pieces, col_pieces in ((None, None), (2, 4), (4, 2)):
            d = DistNTT(1, log_n, 4, device=0, host_exchange=True, pieces=pieces, col_pieces=col_pieces)
            x = d.fill(d.empty(), "random", seed=8)
            x0 = x.clone()
            d.forward(x)
            ok_f = ok_f and torch.equal(x, X[_index(d.layout, "col")])
            d.inverse(x)
            ok_i = ok_i and torch.equal(x, x0)
            a, b, c = d.fill(d.empty(), "random", seed=5), d.fill(d.empty(), "random", seed=6), d.empty()
            d.polymul(a, b, c)
            ok_p = ok_p and torch.equal(c, C[_index(d.layout, "row")])
        q.put((rank, ok_f, ok_i, ok_p))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((rank, repr(e), False, False))


def test_dist_ntt_two_processes_host_exchange():
    """DistNTT in two processes (ranks 0 and 1 of one transform) on one GPU: rank plans, layouts
    and the exchange schedule of the N > 1 bench path, with the all-to-all staged through host
    memory over gloo (RCCL refuses two ranks on one device).  Forward / inverse / polymul bit-exact
    against the single-GPU transform, with whole blocks and with 2 x 4 and 4 x 2 pieces."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_dist_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    assert all(r[1] is True and r[2] and r[3] for r in res), res
