"""Backward of one nn.Linear on the small-GEMM kernels (shared by the AVMNIST head / encoder fc, the
monomodal classifier and the MMIMDb path)."""
from __future__ import annotations

import os

from . import _lib as L

# TSPM_LINEAR_PAIR=0: the two products as separate launches (A/B measurement; bitwise the same result)
PAIR = os.environ.get("TSPM_LINEAR_PAIR", "1") != "0"


def linear_bwd(n, fin, fout, x, ldx, dy, ldy, w, dw, db, dx, lddx, stream) -> None:
    """dw = dy^T @ x (+ db = column sums of dy) and, if dx is given, dx = dy @ w — ONE
    ``tspm_linear_bwd`` launch (bitwise the two separate products) unless TSPM_LINEAR_PAIR=0."""
    lib = L.lib()
    if PAIR:
        L.check(lib.tspm_linear_bwd(n, fin, fout, x, ldx, dy, ldy, w, dw, db, dx, lddx, stream), "linear_bwd")
        return
    L.check(lib.tspm_linear_bwd_weight(n, fin, fout, x, ldx, dy, ldy, dw, db, stream), "linear_bwd_weight")
    if dx is not None:
        L.check(lib.tspm_linear_bwd_data(n, fin, fout, dy, ldy, w, dx, lddx, stream), "linear_bwd_data")
