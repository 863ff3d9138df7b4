"""Test helpers: call libtspm entry points on torch tensors and convert NCHW <-> HWNC."""
from __future__ import annotations

import ctypes

import torch

import tspm_amd
from tspm_amd import _lib as L


def to_hwnc(x: torch.Tensor) -> torch.Tensor:
    n, c, h, w = x.shape
    return x.permute(2, 3, 0, 1).contiguous().view(h * w * n, c)


def from_hwnc(y: torch.Tensor, n: int, h: int, w: int, c: int) -> torch.Tensor:
    return y.view(h, w, n, c).permute(2, 3, 0, 1).contiguous()


def shape(n, h, w, c, k, r, s, stride, pad):
    p = (h + 2 * pad - r) // stride + 1
    q = (w + 2 * pad - s) // stride + 1
    return L.ConvShape(n, h, w, c, k, r, s, stride, pad, p, q)


def sh():
    return L.stream_handle()


def conv_fwd(x_nchw: torch.Tensor, w_oihw: torch.Tensor, stride: int, pad: int, algo=(0, 0, 0, 0, 0),
             nchw_input: bool = False) -> torch.Tensor:
    """Returns NCHW output computed by tspm_conv_fwd (input passed HWNC, or NCHW strided when asked)."""
    n, c, h, w = x_nchw.shape
    k, _, r, s = w_oihw.shape
    shp = shape(n, h, w, c, k, r, s, stride, pad)
    a = L.ConvAlgo(*algo)
    dev = x_nchw.device
    if nchw_input:
        xd = x_nchw.contiguous()
        st = L.Strides4(*[int(v) for v in (xd.stride(0), xd.stride(2), xd.stride(3), xd.stride(1))])
    else:
        xd = to_hwnc(x_nchw)
        st = L.hwnc_strides(n, h, w, c)
    wd = w_oihw.contiguous(memory_format=torch.channels_last)
    y = torch.empty(shp.p * shp.q * n, k, device=dev)
    lib = L.lib()
    wsb = lib.tspm_conv_fwd_workspace(ctypes.byref(shp), ctypes.byref(a))
    ws = torch.zeros(max(wsb, 16), dtype=torch.uint8, device=dev)  # counter header starts zero
    L.check(lib.tspm_conv_fwd(ctypes.byref(shp), ctypes.byref(a), xd.data_ptr(), ctypes.byref(st), wd.data_ptr(),
                              y.data_ptr(), None, ws.data_ptr(), wsb, sh()), "conv_fwd")
    return from_hwnc(y, n, shp.p, shp.q, k)


def zeroed_counters(k: int, dev) -> torch.Tensor:
    return torch.zeros(k // 32 + 1, dtype=torch.int32, device=dev)


def conv_fwd_with_stats(x_nchw, w_oihw, stride, pad, algo=(0, 0, 0, 0, 0), fused=True, counters=None,
                        running=None, two_level=False):
    """conv forward whose epilogue emits BN partials — merged in-launch by the last workgroup of
    each channel block (fused; with two_level, the buffers sized for the two-level merge) or by
    tspm_bn_finalize — returns (y NCHW, mean, invstd)."""
    n, c, h, w = x_nchw.shape
    k, _, r, s = w_oihw.shape
    shp = shape(n, h, w, c, k, r, s, stride, pad)
    a = L.ConvAlgo(*algo)
    dev = x_nchw.device
    xd = to_hwnc(x_nchw)
    st = L.hwnc_strides(n, h, w, c)
    wd = w_oihw.contiguous(memory_format=torch.channels_last)
    m = shp.p * shp.q * n
    y = torch.empty(m, k, device=dev)
    lib = L.lib()
    tiles = lib.tspm_conv_fwd_tiles(ctypes.byref(shp), ctypes.byref(a))
    rows = lib.tspm_conv_fwd_tile_rows(ctypes.byref(shp), ctypes.byref(a))
    nfl = lib.tspm_conv_fwd_bn_partial_floats(ctypes.byref(shp), ctypes.byref(a)) if two_level else 3 * tiles * k
    part = torch.empty(nfl, device=dev)
    mean = torch.empty(k, device=dev)
    inv = torch.empty(k, device=dev)
    rm, rv = running if running is not None else (None, None)
    if fused:
        if counters is not None:
            cnt = counters
        elif two_level:
            cnt = torch.zeros(lib.tspm_conv_fwd_bn_counters(ctypes.byref(shp), ctypes.byref(a)), dtype=torch.int32,
                              device=dev)
        else:
            cnt = zeroed_counters(k, dev)
        bnf = L.BnFuse(part.data_ptr(), cnt.data_ptr(), L.ptr(rm), L.ptr(rv), 0.1, 1e-5, mean.data_ptr(),
                       inv.data_ptr(), cnt.numel() if two_level else 0, 0, nfl if two_level else 0)
    else:
        bnf = L.BnFuse(part.data_ptr(), None, None, None, 0.1, 1e-5, None, None)
    wsb = lib.tspm_conv_fwd_workspace(ctypes.byref(shp), ctypes.byref(a))
    ws = torch.zeros(max(wsb, 16), dtype=torch.uint8, device=dev)
    L.check(lib.tspm_conv_fwd(ctypes.byref(shp), ctypes.byref(a), xd.data_ptr(), ctypes.byref(st), wd.data_ptr(),
                              y.data_ptr(), ctypes.byref(bnf), ws.data_ptr(), wsb, sh()), "conv_fwd")
    if not fused:
        L.check(lib.tspm_bn_finalize(m, k, tiles, rows, part.data_ptr(), L.ptr(rm), L.ptr(rv), 0.1, 1e-5,
                                     mean.data_ptr(), inv.data_ptr(), sh()), "bn_finalize")
    return from_hwnc(y, n, shp.p, shp.q, k), mean, inv


def conv_dgrad(dy_nchw: torch.Tensor, w_oihw: torch.Tensor, in_hw, stride: int, pad: int, algo=(0, 0, 0, 0, 0),
               beta_init: torch.Tensor = None) -> torch.Tensor:
    n, k, p, q = dy_nchw.shape
    _, c, r, s = w_oihw.shape
    h, w = in_hw
    shp = shape(n, h, w, c, k, r, s, stride, pad)
    assert (shp.p, shp.q) == (p, q)
    a = L.ConvAlgo(*algo)
    dev = dy_nchw.device
    dyd = to_hwnc(dy_nchw)
    wd = w_oihw.contiguous(memory_format=torch.channels_last)
    if beta_init is not None:
        dx = to_hwnc(beta_init)
    else:
        dx = torch.empty(h * w * n, c, device=dev)
    lib = L.lib()
    wsb = lib.tspm_conv_dgrad_workspace(ctypes.byref(shp), ctypes.byref(a))
    ws = torch.zeros(max(wsb, 16), dtype=torch.uint8, device=dev)  # counter header starts zero
    L.check(lib.tspm_conv_dgrad(ctypes.byref(shp), ctypes.byref(a), dyd.data_ptr(), wd.data_ptr(), dx.data_ptr(),
                                1 if beta_init is not None else 0, ws.data_ptr(), wsb, sh()), "conv_dgrad")
    return from_hwnc(dx, n, h, w, c)


def conv_wgrad(x_nchw: torch.Tensor, dy_nchw: torch.Tensor, rs, stride: int, pad: int, algo=(0, 0, 0, 0, 0),
               nchw_input: bool = False) -> torch.Tensor:
    n, c, h, w = x_nchw.shape
    _, k, p, q = dy_nchw.shape
    r, s = rs
    shp = shape(n, h, w, c, k, r, s, stride, pad)
    a = L.ConvAlgo(*algo)
    dev = x_nchw.device
    if nchw_input:
        xd = x_nchw.contiguous()
        st = L.Strides4(*[int(v) for v in (xd.stride(0), xd.stride(2), xd.stride(3), xd.stride(1))])
    else:
        xd = to_hwnc(x_nchw)
        st = L.hwnc_strides(n, h, w, c)
    dyd = to_hwnc(dy_nchw)
    dw = torch.empty(k, c, r, s, device=dev).contiguous(memory_format=torch.channels_last)
    lib = L.lib()
    wsb = lib.tspm_conv_wgrad_workspace(ctypes.byref(shp), ctypes.byref(a))
    ws = torch.zeros(max(wsb, 16), dtype=torch.uint8, device=dev)  # counter header must start zero
    L.check(lib.tspm_conv_wgrad(ctypes.byref(shp), ctypes.byref(a), xd.data_ptr(), ctypes.byref(st), dyd.data_ptr(),
                                dw.data_ptr(), ws.data_ptr(), wsb, sh()), "conv_wgrad")
    return dw.contiguous()


def lds_supported(kind: str, case, algo) -> bool:
    """Mirror of the variant-1/2/4 (LDS-staged) support rules in include/tspm.h."""
    n, c, h, w, k, r, s, st, pad = case
    tm, tn, wn, wk, sp = algo[:5]
    if len(algo) < 6 or algo[5] not in (1, 2, 4):
        return True
    if wn * wk == 0 or 4 % (wn * wk):
        return False
    if algo[5] == 4 and wk > 2:  # variant 4 (bf16-piece products): waves take whole 16-deep steps
        return False
    wm = 4 // (wn * wk)
    bm, bn = wm * tm * 32, wn * tn * 32
    if kind == "fwd":
        return c % 32 == 0 and n % bm == 0
    if kind == "dgrad":
        return k % 32 == 0 and c % 4 == 0 and n % bm == 0
    return n % 32 == 0 and k % 4 == 0 and c % bn == 0


def conv_bound(x: torch.Tensor, w: torch.Tensor, stride: int, pad: int) -> torch.Tensor:
    """sum |w||x| per output element (fp64, CPU) — the scale of the fp32 rounding error bound."""
    import torch.nn.functional as F
    return F.conv2d(x.double().abs().cpu(), w.double().abs().cpu(), None, stride, pad)
