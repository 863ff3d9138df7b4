"""Backward of one nn.Linear on the small-GEMM kernels (shared by the AVMNIST head / encoder fc, the
monomodal classifier and the MMIMDb path)."""
from __future__ import annotations

from . import _lib as L


def linear_bwd(n, fin, fout, x, ldx, dy, ldy, w, dw, db, dx, lddx, stream) -> None:
    """dw = dy^T @ x (+ db = column sums of dy) and, if dx is given, dx = dy @ w — ONE ``tspm_linear_bwd``
    launch (bitwise the two separate products; 2.88 -> 2.81 ms per AVMNIST step when introduced)."""
    L.check(L.lib().tspm_linear_bwd(n, fin, fout, x, ldx, dy, ldy, w, dw, db, dx, lddx, stream), "linear_bwd")
