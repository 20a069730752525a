"""Test doubles for the distributed four-step: a CPU engine backed by the C oracle (the checker),
used to run ntt_amd.distributed.FourStep over gloo on CPU.  Not product code."""
import numpy as np
import torch

from oracle import ntt_ref as R
from oracle import oracle_c as OC


class CpuOracleEngine:
    def __init__(self, field_id, log_n, limbs64):
        from ntt_amd.distributed import Layout
        self.p, self.g = R.FIELDS[field_id]
        self.L = limbs64
        self.log_n = log_n
        lay = Layout(log_n, 1, 0)
        self.n1, self.n2 = lay.n1, lay.n2
        n = 1 << log_n
        w = R.root_of_unity(self.p, self.g, n)
        self.pw = [pow(w, e, self.p) for e in range(n)]
        winv = pow(w, self.p - 2, self.p)
        self.pw_inv = [pow(winv, e, self.p) for e in range(n)]

    def empty(self, count):
        return torch.zeros((count, self.L), dtype=torch.int64)

    def _rows(self, t, batch, inverse):
        a = t.numpy().view(np.uint64).reshape(batch, -1, self.L)
        for i in range(batch):
            a[i] = OC.ntt_mp(a[i], self.p, self.g, inverse)

    def rows_forward(self, t, batch):
        self._rows(t, batch, False)

    def rows_inverse(self, t, batch):
        self._rows(t, batch, True)

    cols_forward = rows_forward
    cols_inverse = rows_inverse

    def cols_inverse_pointwise(self, a, b, out, batch):
        n = a.shape[0] // batch
        prod = OC.mul_mp(a.numpy().view(np.uint64).reshape(-1, self.L), b.numpy().view(np.uint64).reshape(-1, self.L),
                         self.p)
        for i in range(batch):
            prod[i * n:(i + 1) * n] = OC.ntt_mp(prod[i * n:(i + 1) * n], self.p, self.g, True)
        out.numpy().view(np.uint64).reshape(-1, self.L)[:] = prod

    def twiddle_pack(self, src, dst, log_rows, log_len, log_block, row0, inverse, peer_stride=None):
        n = 1 << self.log_n
        table = self.pw_inv if inverse else self.pw
        s = OC.limbs_to_ints(src.numpy().view(np.uint64).reshape(-1, self.L))
        rows, length, bw = 1 << log_rows, 1 << log_len, 1 << log_block
        ps = rows * bw if peer_stride is None else peer_stride
        d = dst.numpy().view(np.uint64).reshape(-1, self.L)
        for a in range(rows):
            for b in range(length):
                v = s[a * length + b] * table[((row0 + a) * b) % n] % self.p
                d[(b // bw) * ps + a * bw + (b % bw)] = OC.ints_to_limbs([v], self.L)[0]

    def transpose(self, src, dst, log_rows, log_cols, log_block_rows=None, block_stride=None):
        lb = log_rows if log_block_rows is None else log_block_rows
        bs = (1 << (lb + log_cols)) if block_stride is None else block_stride
        s = src.numpy().view(np.uint64).reshape(-1, self.L)
        rows, cols = 1 << log_rows, 1 << log_cols
        m = np.stack([s[(r >> lb) * bs + (r & ((1 << lb) - 1)) * cols:][:cols] for r in range(rows)])
        dst.numpy().view(np.uint64).reshape(-1, self.L)[:] = np.ascontiguousarray(m.transpose(1, 0, 2)).reshape(-1, self.L)


def row_shares(x_ints, layout_cls, log_n, world, L):
    """Split a global vector into the row-layout shares of every rank (limb arrays)."""
    shares = []
    for g in range(world):
        lay = layout_cls(log_n, world, g)
        vals = [x_ints[lay.row_global(i)] for i in range(lay.local_n)]
        shares.append(torch.from_numpy(OC.ints_to_limbs(vals, L).view(np.int64)))
    return shares


def gather_cols(shares, layout_cls, log_n, world, L):
    n = 1 << log_n
    X = [None] * n
    for g, t in enumerate(shares):
        lay = layout_cls(log_n, world, g)
        vals = OC.limbs_to_ints(t.numpy().view(np.uint64).reshape(-1, L))
        for i, v in enumerate(vals):
            X[lay.col_global(i)] = v
    return X
