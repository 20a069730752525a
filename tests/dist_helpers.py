"""Test doubles for the distributed four-step: a CPU engine backed by the C oracle (the checker),
used to run ntt_amd.distributed.FourStep over gloo on CPU.  Not product code.

It implements the rank plan's piece interface (ntt_rplan_*_piece, ntt_amd/csrc/ntt_rplan.cpp) with
the same layouts: row layout [r][n2], column layout [n1][c], exchange buffers of one block per peer q
(P_r row pieces of ra = r / P_r rows, P_c column pieces of cm = c / P_c columns):
  forward block [i][v][k][ra][cm]: row a = i ra + a' of this rank, column q c + k cm + kc' of vector v
  inverse block [k][i][ra][cm]:    row j1 = q r + i ra + a' of the peer, column g c + k cm + kc' of this rank
"""
import numpy as np
import torch

from oracle import ntt_ref as R
from oracle import oracle_c as OC


class CpuOracleEngine:
    def __init__(self, field_id, log_n, limbs64, world=1, rank=0, log_n2=None):
        from ntt_amd.distributed import Layout
        self.p, self.g = R.FIELDS[field_id]
        self.L = limbs64
        self.lay = Layout(log_n, world, rank, log_n2)
        n = 1 << log_n
        w = R.root_of_unity(self.p, self.g, n)
        self.w, self.winv, self.n = w, pow(w, self.p - 2, self.p), n

    def empty(self, count):
        return torch.zeros((count, self.L), dtype=torch.int64)

    def _ints(self, t):
        return OC.limbs_to_ints(t.numpy().view(np.uint64).reshape(-1, self.L))

    def _put(self, t, idx, vals):
        a = t.numpy().view(np.uint64).reshape(-1, self.L)
        a[np.asarray(idx)] = OC.ints_to_limbs(vals, self.L)

    def _ntt(self, vals, inverse):
        return OC.limbs_to_ints(OC.ntt_mp(OC.ints_to_limbs(vals, self.L), self.p, self.g, inverse))

    def _geom(self, rp, cp):
        L = self.lay
        assert L.r % rp == 0 and L.c % cp == 0
        return L.r // rp, L.c // cp

    def _fwd_idx(self, nvec, v, a, kc, rp, cp, peer):
        """forward block of `peer`: element (row a of the sender, column kc of the receiver) of vector v"""
        L = self.lay
        ra, cm = self._geom(rp, cp)
        i, a1 = divmod(a, ra)
        k, kc1 = divmod(kc, cm)
        return peer * nvec * L.chunk + i * nvec * ra * L.c + v * ra * L.c + k * ra * cm + a1 * cm + kc1

    def _inv_idx(self, a, kc, rp, cp, peer):
        """inverse block of `peer`: element (row a of the receiver, column kc of the sender)"""
        L = self.lay
        ra, cm = self._geom(rp, cp)
        k, kc1 = divmod(kc, cm)
        return peer * L.chunk + k * L.r * cm + a * cm + kc1

    def forward_rows_piece(self, x, send, nvec, slot, i, rp, cp):
        L, p = self.lay, self.p
        ra, _ = self._geom(rp, cp)
        xs = self._ints(x)
        idx, vals = [], []
        for a in range(i * ra, (i + 1) * ra):
            X = self._ntt(xs[a * L.n2:(a + 1) * L.n2], False)
            j1 = L.rank * L.r + a
            for k2 in range(L.n2):
                q, kc = divmod(k2, L.c)
                idx.append(self._fwd_idx(nvec, slot, a, kc, rp, cp, q))
                vals.append(X[k2] * pow(self.w, j1 * k2 % self.n, p) % p)
        self._put(send, idx, vals)

    def forward_cols_piece(self, recv, x, nvec, slot, k, rp, cp):
        L = self.lay
        _, cm = self._geom(rp, cp)
        rv = self._ints(recv)
        idx, vals = [], []
        for kc in range(k * cm, (k + 1) * cm):
            col = [rv[self._fwd_idx(nvec, slot, j1 % L.r, kc, rp, cp, j1 // L.r)] for j1 in range(L.n1)]
            for k1, v in enumerate(self._ntt(col, False)):
                idx.append(k1 * L.c + kc)
                vals.append(v)
        self._put(x, idx, vals)

    def inverse_cols_piece(self, x, y, send, k, rp, cp):
        L, p = self.lay, self.p
        _, cm = self._geom(rp, cp)
        xs = self._ints(x)
        if y is not None:
            ys = self._ints(y)
            xs = [u * v % p for u, v in zip(xs, ys)]
        idx, vals = [], []
        for kc in range(k * cm, (k + 1) * cm):
            k2 = L.rank * L.c + kc
            col = self._ntt([xs[k1 * L.c + kc] for k1 in range(L.n1)], True)
            for j1, v in enumerate(col):
                idx.append(self._inv_idx(j1 % L.r, kc, rp, cp, j1 // L.r))
                vals.append(v * pow(self.winv, j1 * k2 % self.n, p) % p)
        self._put(send, idx, vals)

    def inverse_rows_piece(self, recv, out, i, rp, cp):
        L = self.lay
        ra, _ = self._geom(rp, cp)
        rv = self._ints(recv)
        res = []
        for a in range(i * ra, (i + 1) * ra):
            row = [rv[self._inv_idx(a, k2 % L.c, rp, cp, k2 // L.c)] for k2 in range(L.n2)]
            res += self._ntt(row, True)
        self._put(out, range(i * ra * L.n2, (i + 1) * ra * L.n2), res)


class GlooPieceExchange:
    """FourStep exchange interface over any torch.distributed backend: runs of every peer block, one
    all_to_all_single per run (synchronous; the handle is unused)."""

    def __init__(self, layout):
        self.L = layout

    def start(self, send, recv, peer_stride, runs):
        import torch.distributed as dist
        from ntt_amd.distributed import run_views
        L = self.L
        sv = run_views(send, L.world, peer_stride, runs)
        rv = run_views(recv, L.world, peer_stride, runs)
        for u in range(len(runs)):
            ins = torch.cat([sv[g][u] for g in range(L.world)])
            out = torch.empty_like(ins)
            dist.all_to_all_single(out, ins)
            for g in range(L.world):
                m = rv[g][u].shape[0]
                rv[g][u].copy_(out[g * m:(g + 1) * m])

    def wait(self, handle):
        pass


def row_shares(x_ints, layout_cls, log_n, world, L, log_n2=None):
    """Split a global vector into the row-layout shares of every rank (limb arrays)."""
    shares = []
    for g in range(world):
        lay = layout_cls(log_n, world, g, log_n2)
        vals = [x_ints[lay.row_global(i)] for i in range(lay.local_n)]
        shares.append(torch.from_numpy(OC.ints_to_limbs(vals, L).view(np.int64)))
    return shares


def gather_cols(shares, layout_cls, log_n, world, L, log_n2=None):
    n = 1 << log_n
    X = [None] * n
    for g, t in enumerate(shares):
        lay = layout_cls(log_n, world, g, log_n2)
        vals = OC.limbs_to_ints(t.numpy().view(np.uint64).reshape(-1, L))
        for i, v in enumerate(vals):
            X[lay.col_global(i)] = v
    return X
