"""The multi-GPU four-step schedule (ntt_amd.distributed.FourStep) on CPU: gloo all-to-all with
world_size 2, 4 and 8 (8: the rank count of the N = 8 bench line), local steps done by an
oracle-backed test engine.  Checks the layouts, the twiddle/pack index math and the exchange
against the single-transform oracle."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import ntt_ref as R
from oracle import oracle_c as OC


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _exchange(layout, pieces, col_pieces=1):
    """Whole-block all-to-all (plain callable, one piece) or the piece exchange interface."""
    from tests.dist_helpers import GlooPieceExchange
    if pieces == 1 and col_pieces == 1:
        return lambda s, r: dist.all_to_all_single(r.view(-1), s.view(-1))
    return GlooPieceExchange(layout)


def _worker(rank, world, port, field_id, log_n, L, q, pieces=1, log_n2=None, col_pieces=1):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from ntt_amd.distributed import FourStep, Layout, pow2_pieces
    from tests.dist_helpers import CpuOracleEngine, row_shares
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 1 << log_n
        x = R.random_vector(field_id, n, seed=77)
        share = row_shares(x, Layout, log_n, world, L, log_n2)[rank]
        eng = CpuOracleEngine(field_id, log_n, L, world, rank, log_n2)
        lay = Layout(log_n, world, rank, log_n2)
        fs = FourStep(lay, eng, _exchange(lay, pieces, col_pieces), pieces=pieces, col_pieces=col_pieces)
        assert len(fs.pieces) == pow2_pieces(pieces, lay.r) and fs.cp == pow2_pieces(col_pieces, lay.c)
        fs.forward(share)
        fwd = share.clone()
        fs.inverse(share)
        back = OC.limbs_to_ints(share.numpy().view("uint64").reshape(-1, L))
        ok_rt = back == [x[lay.row_global(i)] for i in range(lay.local_n)]
        q.put((rank, fwd.numpy().tobytes(), ok_rt))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,field_id,log_n,pieces,log_n2,col_pieces",
                         [(2, 1, 6, 1, None, 1), (2, 2, 7, 1, None, 1), (4, 1, 8, 1, None, 1), (2, 1, 6, 2, None, 1),
                          (2, 2, 7, 3, None, 1), (4, 1, 8, 4, None, 1), (2, 1, 8, 2, 3, 1), (4, 2, 9, 1, 3, 1),
                          (2, 1, 8, 1, None, 4), (2, 1, 8, 2, None, 2), (4, 1, 10, 4, None, 2),
                          (2, 2, 9, 4, 4, 8), (8, 1, 8, 1, None, 1), (8, 2, 10, 2, None, 2)])
def test_four_step_gloo(world, field_id, log_n, pieces, log_n2, col_pieces):
    """pieces / col_pieces > 1: the pipelined schedule (the all-to-all in row-piece x column-piece
    units overlapping the row transforms before it and the column transforms after it; a count that
    is not a power of two rounds down) gives the same column layout and round trip.  log_n2: an
    unbalanced split n1 > n2 (what the rank plans pick when it saves a pass, ntt_rplan.cpp
    choose_split)."""
    from ntt_amd.distributed import Layout
    from tests.dist_helpers import gather_cols
    L = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, field_id, log_n, L, q, pieces, log_n2, col_pieces))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, fwd, ok = q.get(timeout=240)
        res[rank] = (fwd, ok)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import numpy as np
    shares = [torch.from_numpy(np.frombuffer(res[r][0], dtype=np.int64).copy().reshape(-1, L)) for r in range(world)]
    X = gather_cols(shares, Layout, log_n, world, L, log_n2)
    p_, g_ = R.FIELDS[field_id]
    x = R.random_vector(field_id, 1 << log_n, seed=77)
    assert X == R.ntt_dit(x, p_, g_)
    assert all(res[r][1] for r in range(world)), "inverse round trip"


def test_layout_index_maps_are_bijections():
    from ntt_amd.distributed import Layout
    for log_n, world, log_n2 in ((6, 2, None), (9, 4, None), (12, 8, None), (12, 2, 4), (11, 4, 2)):
        n = 1 << log_n
        lays = [Layout(log_n, world, g, log_n2) for g in range(world)]
        rows = sorted(lay.row_global(i) for lay in lays for i in range(lay.local_n))
        cols = sorted(lay.col_global(i) for lay in lays for i in range(lay.local_n))
        assert rows == list(range(n)) and cols == list(range(n))


def test_layout_rejects_bad_world():
    from ntt_amd.distributed import Layout
    with pytest.raises(ValueError):
        Layout(10, 3, 0)
    with pytest.raises(ValueError):
        Layout(4, 8, 0)
    with pytest.raises(ValueError):
        Layout(10, 2, 0, 6)  # n2 > n1
    with pytest.raises(ValueError):
        Layout(10, 8, 0, 2)  # fewer columns than ranks


def _polymul_worker(rank, world, port, field_id, log_n, L, square, q, pieces=1, log_n2=None, col_pieces=1):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from ntt_amd.distributed import FourStep, Layout
    from tests.dist_helpers import CpuOracleEngine, row_shares
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 1 << log_n
        a = R.random_vector(field_id, n, seed=5)
        b = a if square else R.random_vector(field_id, n, seed=6)
        sa = row_shares(a, Layout, log_n, world, L, log_n2)[rank]
        sb = sa if square else row_shares(b, Layout, log_n, world, L, log_n2)[rank]
        out = torch.zeros_like(sa)
        eng = CpuOracleEngine(field_id, log_n, L, world, rank, log_n2)
        lay = Layout(log_n, world, rank, log_n2)
        fs = FourStep(lay, eng, _exchange(lay, pieces, col_pieces), pieces=pieces, col_pieces=col_pieces)
        fs.polymul(sa, sb, out)
        q.put((rank, out.numpy().tobytes()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,field_id,log_n,square,pieces,log_n2,col_pieces",
                         [(2, 1, 6, False, 1, None, 1), (4, 1, 8, False, 1, None, 1), (2, 2, 7, True, 1, None, 1),
                          (2, 1, 6, False, 2, None, 1), (4, 1, 8, False, 4, None, 1), (2, 2, 7, True, 2, None, 1),
                          (2, 1, 8, False, 2, 3, 1), (2, 1, 8, False, 2, None, 4), (4, 2, 10, True, 2, None, 2),
                          (8, 1, 8, False, 1, None, 1)])
def test_distributed_polymul_gloo(world, field_id, log_n, square, pieces, log_n2, col_pieces):
    """C5's schedule (forward(a), forward(b) in ONE all-to-all, local pointwise product fused into
    the inverse, inverse all-to-all) over gloo: the row-layout result equals the oracle's cyclic
    product; squaring (a is b) takes the single-vector exchange."""
    import numpy as np
    from ntt_amd.distributed import Layout
    L = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_polymul_worker,
                         args=(r, world, port, field_id, log_n, L, square, q, pieces, log_n2, col_pieces))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, out = q.get(timeout=240)
        res[rank] = out
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n = 1 << log_n
    p_, g_ = R.FIELDS[field_id]
    a = R.random_vector(field_id, n, seed=5)
    b = a if square else R.random_vector(field_id, n, seed=6)
    exp = R.polymul(a, b, p_, g_)
    got = [None] * n
    for r in range(world):
        lay = Layout(log_n, world, r, log_n2)
        vals = OC.limbs_to_ints(np.frombuffer(res[r], dtype=np.uint64).reshape(-1, L))
        for i, v in enumerate(vals):
            got[lay.row_global(i)] = v
    assert got == exp


def test_piece_ranges_and_auto_pieces():
    """Row ranges tile [0, r) exactly (uneven last piece allowed; the row-range entry points); the
    schedule's piece counts are powers of two <= the rows / columns; the automatic count keeps every
    piece's transforms >= 2^22 elements (full GPU launches) and never exceeds the cap."""
    from ntt_amd.distributed import DistNTT, FourStep, pow2_pieces
    assert [pow2_pieces(k, 8) for k in (0, 1, 2, 3, 4, 5, 7, 8, 9, 100)] == [1, 1, 2, 2, 4, 4, 4, 8, 8, 8]
    assert pow2_pieces(8, 2) == 2 and pow2_pieces(3, 1) == 1
    for r in (1, 2, 3, 4, 7, 512, 2048):
        for k in (1, 2, 3, 4, 8, 100):
            pr = FourStep.piece_ranges(r, k)
            assert len(pr) <= min(k, r)
            assert pr[0][0] == 0 and all(a + n == b for (a, n), (b, _) in zip(pr, pr[1:]))
            assert pr[-1][0] + pr[-1][1] == r and all(n >= 1 for _, n in pr)
    assert DistNTT.auto_pieces(1 << 21) == 1  # 2^24 over 8 GPUs: one piece
    assert DistNTT.auto_pieces(1 << 25) == 8  # C4: 2^28 over 8 GPUs
    assert DistNTT.auto_pieces(1 << 23) == 2
    for ln in range(10, 32):
        k = DistNTT.auto_pieces(1 << ln)
        assert k == 1 or (1 << ln) // k >= DistNTT.MIN_PIECE_ELEMS
        kc = DistNTT.auto_pieces(1 << ln, cap=4, min_elems=DistNTT.MIN_COL_PIECE_ELEMS)
        assert kc <= 4 and (kc == 1 or (1 << ln) // kc >= DistNTT.MIN_COL_PIECE_ELEMS)
    # 2^24 over 2 GPUs (2^23 per rank): 2 row pieces, 4 column pieces; over 8 (2^21): none
    assert DistNTT.auto_pieces(1 << 23, cap=4, min_elems=DistNTT.MIN_COL_PIECE_ELEMS) == 4
    assert DistNTT.auto_pieces(1 << 21, cap=4, min_elems=DistNTT.MIN_COL_PIECE_ELEMS) == 1


def test_piece_candidates_give_the_tuner_a_choice_at_every_world_size():
    """at 2^24 over 8 ranks (2^21 elements per rank, below both auto-piece
    minimums) round 4's candidate list was 1 x 1 alone.  Every N > 1 now measures at least 1 x 1,
    2 x 1, 1 x 2 and 2 x 2 (clipped to the rank's rows / columns); world size 1 only 1 x 1."""
    from ntt_amd.distributed import DistNTT, Layout
    for log_n, log_n2 in ((24, 10), (24, 12), (28, 14), (12, 6)):
        for world in (2, 4, 8):
            c = DistNTT.piece_candidates(Layout(log_n, world, 0, log_n2))
            assert len(c) >= 2 and c[0] == (1, 1) and len(set(c)) == len(c), (log_n, world, c)
            if log_n >= 24:
                assert {(1, 1), (2, 1), (1, 2), (2, 2)} <= set(c), (log_n, world, c)
        assert DistNTT.piece_candidates(Layout(log_n, 1, 0, log_n2)) == [(1, 1)]
    # 2^24 over 2 ranks: the size rule adds its 2 x 4
    assert (2, 4) in DistNTT.piece_candidates(Layout(24, 2, 0, 10))
    # 2^24 over 8 ranks (2^21 per rank): the four small schedules, no auto addition
    assert DistNTT.piece_candidates(Layout(24, 8, 0, 10)) == [(1, 1), (2, 1), (1, 2), (2, 2)]


def _tune_worker(rank, world, port, field_id, log_n, L, q, cands=None):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from ntt_amd.distributed import Layout, tune_four_step
    from tests.dist_helpers import CpuOracleEngine, GlooPieceExchange, row_shares
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = 1 << log_n
        x = R.random_vector(field_id, n, seed=78)
        share = row_shares(x, Layout, log_n, world, L)[rank]
        eng = CpuOracleEngine(field_id, log_n, L, world, rank)
        lay = Layout(log_n, world, rank)
        scratch = share.clone()
        if cands is None:
            cands = [(1, 1), (2, 2), (4, 1)]
        elif cands == "dist":  # the candidate list DistNTT.tune_pieces uses
            from ntt_amd.distributed import DistNTT
            cands = DistNTT.piece_candidates(lay)
        fs, res = tune_four_step(lay, eng, GlooPieceExchange(lay), dist, None, scratch, cands,
                                 steps=1, warmup=0, device=torch.device("cpu"), sync=lambda: None)
        fs.forward(share)  # the chosen schedule computes the same transform
        q.put((rank, share.numpy().tobytes(), res["chosen"], sorted(res["ms_per_transform"])))
    finally:
        dist.destroy_process_group()


def test_tune_four_step_picks_one_schedule_on_every_rank():
    """DistNTT.tune_pieces' collective core (tune_four_step): every rank times the candidates in the
    same order, takes the slowest rank's time, and so picks the SAME schedule; that schedule's
    forward equals the definition."""
    from ntt_amd.distributed import Layout
    from tests.dist_helpers import gather_cols
    world, field_id, log_n, L = 4, 1, 8, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tune_worker, args=(r, world, port, field_id, log_n, L, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, fwd, chosen, keys = q.get(timeout=240)
        res[rank] = (fwd, chosen, keys)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import numpy as np
    assert len({res[r][1] for r in range(world)}) == 1, res
    assert res[0][2] == ["1x1", "2x2", "4x1"]
    shares = [torch.from_numpy(np.frombuffer(res[r][0], dtype=np.int64).copy().reshape(-1, L)) for r in range(world)]
    X = gather_cols(shares, Layout, log_n, world, L)
    p_, g_ = R.FIELDS[field_id]
    assert X == R.ntt_dit(R.random_vector(field_id, 1 << log_n, seed=78), p_, g_)


def test_tune_four_step_world8_measures_several_candidates():
    """The N = 8 shape (world 8, gloo): the tuner times DistNTT.piece_candidates' schedules (more
    than one), every rank picks the same one, and its forward equals the definition."""
    from ntt_amd.distributed import Layout
    from tests.dist_helpers import gather_cols
    world, field_id, log_n, L = 8, 1, 8, 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tune_worker, args=(r, world, port, field_id, log_n, L, q, "dist"))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, fwd, chosen, keys = q.get(timeout=240)
        res[rank] = (fwd, chosen, keys)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import numpy as np
    assert len({res[r][1] for r in range(world)}) == 1, res
    assert len(res[0][2]) >= 2, res[0][2]
    shares = [torch.from_numpy(np.frombuffer(res[r][0], dtype=np.int64).copy().reshape(-1, L)) for r in range(world)]
    X = gather_cols(shares, Layout, log_n, world, L)
    p_, g_ = R.FIELDS[field_id]
    assert X == R.ntt_dit(R.random_vector(field_id, 1 << log_n, seed=78), p_, g_)
