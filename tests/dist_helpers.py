"""Test doubles for the distributed four-step: a CPU engine backed by the C oracle (the checker),
used to run ntt_amd.distributed.FourStep over gloo on CPU.  Not product code.

It implements the rank-plan interface (ntt_rplan_*, ntt_amd/csrc/ntt_rplan.cpp) with the same
layouts: row layout [r][n2], column layout [n1][c], send / receive buffers [G][nvec][r c] where the
forward's chunk for peer q holds [a][kc] (rows a of this rank, columns q c + kc) and the inverse's
chunk for peer q holds [j1 - q r][kc] (this rank's columns).
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

    def forward_rows(self, x, send, nvec, slot, row0=0, nrows=None):
        L, p = self.lay, self.p
        nrows = L.r - row0 if nrows is None else nrows
        xs = self._ints(x)
        idx, vals = [], []
        for a in range(row0, row0 + nrows):
            X = self._ntt(xs[a * L.n2:(a + 1) * L.n2], False)
            j1 = L.rank * L.r + a
            for k2 in range(L.n2):
                q, kc = divmod(k2, L.c)
                idx.append((q * nvec + slot) * L.chunk + a * L.c + kc)
                vals.append(X[k2] * pow(self.w, j1 * k2 % self.n, p) % p)
        self._put(send, idx, vals)

    def forward_cols(self, recv, x, nvec, slot):
        L = self.lay
        rv = self._ints(recv)
        out = [0] * L.local_n
        for kc in range(L.c):
            col = [rv[((j1 // L.r) * nvec + slot) * L.chunk + (j1 % L.r) * L.c + kc] for j1 in range(L.n1)]
            for k1, v in enumerate(self._ntt(col, False)):
                out[k1 * L.c + kc] = v
        self._put(x, range(L.local_n), out)

    def inverse_cols(self, x, y, send):
        L, p = self.lay, self.p
        xs = self._ints(x)
        if y is not None:
            ys = self._ints(y)
            xs = [u * v % p for u, v in zip(xs, ys)]
        out = [0] * L.local_n
        for kc in range(L.c):
            k2 = L.rank * L.c + kc
            col = self._ntt([xs[k1 * L.c + kc] for k1 in range(L.n1)], True)
            for j1, v in enumerate(col):
                out[j1 * L.c + kc] = v * pow(self.winv, j1 * k2 % self.n, p) % p
        self._put(send, range(L.local_n), out)

    def inverse_rows(self, recv, out, row0=0, nrows=None):
        L = self.lay
        nrows = L.r - row0 if nrows is None else nrows
        rv = self._ints(recv)
        res = []
        for a in range(row0, row0 + nrows):
            row = [rv[(k2 // L.c) * L.chunk + a * L.c + (k2 % L.c)] for k2 in range(L.n2)]
            res += self._ntt(row, True)
        self._put(out, range(row0 * L.n2, (row0 + nrows) * L.n2), res)


class GlooPieceExchange:
    """FourStep exchange interface over any torch.distributed backend: rows [row0, row0 + nrows) of
    every peer chunk, one all_to_all_single per vector (synchronous; the handle is unused)."""

    def __init__(self, layout):
        self.L = layout

    def start(self, send, recv, nvec, row0, nrows):
        import torch.distributed as dist
        from ntt_amd.distributed import piece_views
        L = self.L
        sv = piece_views(send, L.world, nvec, L.r, L.c, row0, nrows)
        rv = piece_views(recv, L.world, nvec, L.r, L.c, row0, nrows)
        for v in range(nvec):
            ins = torch.cat([sv[g][v] for g in range(L.world)])
            out = torch.empty_like(ins)
            dist.all_to_all_single(out, ins)
            for g in range(L.world):
                m = rv[g][v].shape[0]
                rv[g][v].copy_(out[g * m:(g + 1) * m])

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
