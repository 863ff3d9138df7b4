"""The C-ABI library loads and exports exactly what include/tspm.h declares (no GPU needed: only
symbol lookup, version / status queries, workspace-size queries and argument validation that
returns before any HIP call)."""
import ctypes
import os
import re

import pytest

import tspm_amd
from tspm_amd import _lib as L

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "tspm.h")


def header_prototypes():
    src = open(HEADER).read()
    return dict(re.findall(r"\n(?:int|int32_t|int64_t|uint32_t|size_t|const char\*)\s+(tspm_\w+)\(([^;]*?)\);", src, re.S))


def test_library_loads_and_version():
    lib = L.load()
    assert lib.tspm_abi_version() == L.ABI_VERSION
    assert lib.tspm_status_string(0) == b"ok"
    assert lib.tspm_status_string(3) == b"workspace too small"


def test_every_header_symbol_is_exported_and_bound():
    protos = header_prototypes()
    assert len(protos) >= 28
    lib = ctypes.CDLL(L.LIB_PATH)
    for name, params in protos.items():
        assert hasattr(lib, name), f"{name} declared in tspm.h but not exported"
        assert name in L._SIGS, f"{name} has no ctypes binding"
        n = 0 if params.strip() in ("void", "") else len(params.split(","))
        assert n == len(L._SIGS[name][1]), f"{name}: header has {n} params, binding {len(L._SIGS[name][1])}"
    assert set(L._SIGS) == set(protos)


def test_no_unexpected_exports():
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T tspm_" in l}
    assert exported == set(header_prototypes())


def test_invalid_arguments_are_rejected_before_launch():
    lib = L.load()
    s = L.ConvShape(2, 8, 8, 64, 64, 3, 3, 1, 1, 7, 8)  # wrong p
    a = L.ConvAlgo()
    assert lib.tspm_conv_fwd(ctypes.byref(s), ctypes.byref(a), 1, None, 1, 1, None, None, 0, None) == 1
    assert lib.tspm_conv_fwd_tiles(ctypes.byref(s), ctypes.byref(a)) == 0
    good = L.ConvShape(2, 8, 8, 64, 64, 3, 3, 1, 1, 8, 8)
    assert lib.tspm_conv_fwd(ctypes.byref(good), ctypes.byref(a), None, None, 1, 1, None, None, 0, None) == 1
    for bad in [(3, 1, 1, 1, 1), (2, 1, 1, 1, 1), (1, 1, 3, 1, 1), (1, 1, 2, 8, 1), (1, 1, 2, 16, 1), (2, 2, 1, 16, 1)]:
        bad_algo = L.ConvAlgo(*bad)
        assert lib.tspm_conv_fwd(ctypes.byref(good), ctypes.byref(bad_algo), 16, None, 16, 16, None, None, 0, None) == 1, bad
    assert lib.tspm_bn_finalize(128, 64, 2, 32, 16, None, None, 0.1, 1e-5, 16, 16, None) == 1  # tiles*rows < m
    # dgrad needs K % 8 == 0
    odd = L.ConvShape(2, 8, 8, 64, 12, 3, 3, 1, 1, 8, 8)
    assert lib.tspm_conv_dgrad(ctypes.byref(odd), ctypes.byref(a), 16, 16, 16, 0, None, 0, None) == 1
    assert lib.tspm_bn_stats(0, 64, 16, 1, 0, None, None, None, 0.1, 1e-5, 16, 16, 16, 1 << 20, None) == 1
    assert lib.tspm_bn_stats(128, 66, 16, 1, 0, None, None, None, 0.1, 1e-5, 16, 16, 16, 1 << 20, None) == 1
    assert lib.tspm_bn_stats(128, 64, 16, 1, 0, None, None, None, 0.1, 1e-5, 16, 16, 16, 0, None) == 3
    assert lib.tspm_maxpool_fwd(2, 8, 8, 64, 3, 2, 1, 5, 4, 16, 16, 16, None, 0, None) == 1
    # variant 1 (LDS-staged): n % BM != 0 and wm*wn*wk != 4 are rejected, split-K needs its workspace
    s64 = L.ConvShape(64, 8, 8, 64, 64, 3, 3, 1, 1, 8, 8)
    v1 = L.ConvAlgo(1, 1, 1, 1, 1, 1)  # wm = 4: BM = 128 > n
    for v in (1, 2):  # the 2x2 wave tiles are not built (round 5)
        assert lib.tspm_conv_fwd(ctypes.byref(good), ctypes.byref(L.ConvAlgo(2, 2, 2, 1, 1, v)), 16, None, 16, 16, None,
                                 None, 0, None) == 1
    assert lib.tspm_conv_fwd(ctypes.byref(s64), ctypes.byref(v1), 16, None, 16, 16, None, None, 0, None) == 1
    assert lib.tspm_conv_dgrad(ctypes.byref(s64), ctypes.byref(v1), 16, 16, 16, 0, None, 0, None) == 1
    v3 = L.ConvAlgo(1, 1, 3, 1, 1, 1)
    assert lib.tspm_conv_fwd(ctypes.byref(good), ctypes.byref(v3), 16, None, 16, 16, None, None, 0, None) == 1
    stem_only = L.ConvAlgo(0, 0, 0, 0, 0, 3)  # variant 3: the 1-channel 7x7/2 stems only
    assert lib.tspm_conv_fwd(ctypes.byref(good), ctypes.byref(stem_only), 16, None, 16, 16, None, None, 0, None) == 1
    assert lib.tspm_conv_wgrad(ctypes.byref(good), ctypes.byref(stem_only), 16, None, 16, 16, None, 0, None) == 1
    vs = L.ConvAlgo(1, 1, 1, 4, 2, 1)  # BM = 32, split-K 2 without workspace
    s32 = L.ConvShape(32, 8, 8, 64, 64, 3, 3, 1, 1, 8, 8)
    assert lib.tspm_conv_fwd(ctypes.byref(s32), ctypes.byref(vs), 16, None, 16, 16, None, None, 0, None) == 3
    assert lib.tspm_adam_step(10, 17, 16, 16, 16, 16, None) == 1   # misaligned
    assert lib.tspm_dropout_mask(10, 1.0, 0, None, 16, None) == 1   # p must be < 1
    hd = L.HeadDesc(n=8, in_=192, hidden=128, hidden2=64, classes=10, ldx=192, lddx=192)
    assert lib.tspm_head_train_step(ctypes.byref(hd), None) == 1       # null buffers
    assert lib.tspm_head_train_step(None, None) == 1


def test_workspace_queries():
    lib = L.load()
    s = L.ConvShape(128, 7, 7, 64, 64, 3, 3, 1, 1, 7, 7)
    assert lib.tspm_conv_fwd_workspace(ctypes.byref(s), ctypes.byref(L.ConvAlgo(1, 1, 1, 4, 1))) == 0
    assert lib.tspm_conv_fwd_tiles(ctypes.byref(s), ctypes.byref(L.ConvAlgo(1, 1, 1, 4, 1))) == 7 * 7 * 128 // 32
    assert lib.tspm_conv_fwd_tile_rows(ctypes.byref(s), ctypes.byref(L.ConvAlgo(2, 2, 1, 1, 1))) == 64
    w3 = lib.tspm_conv_wgrad_workspace(ctypes.byref(s), ctypes.byref(L.ConvAlgo(1, 1, 1, 4, 3)))
    assert w3 == L.COUNTER_BYTES + 3 * 64 * 9 * 64 * 4
    v = L.ConvAlgo(1, 1, 1, 1, 4, 1)  # variant 1, split-K 4
    assert lib.tspm_conv_fwd_workspace(ctypes.byref(s), ctypes.byref(v)) == L.COUNTER_BYTES + 4 * 7 * 7 * 128 * 64 * 4
    assert lib.tspm_conv_dgrad_workspace(ctypes.byref(s), ctypes.byref(v)) == L.COUNTER_BYTES + 4 * 7 * 7 * 128 * 64 * 4
    assert lib.tspm_conv_wgrad_workspace(ctypes.byref(s), ctypes.byref(v)) == L.COUNTER_BYTES + 4 * 64 * 9 * 64 * 4
    assert lib.tspm_conv_fwd_tile_rows(ctypes.byref(s), ctypes.byref(L.ConvAlgo(2, 1, 1, 1, 1, 1))) == 64
    assert lib.tspm_bn_stats_workspace(6272, 64) > 0
    assert lib.tspm_bn_bwd_workspace(6272, 64) >= lib.tspm_bn_stats_workspace(6272, 64)


def test_abi_version_consistent_everywhere():
    """include/tspm.h's TSPM_ABI_VERSION, the Python binding's expectation and the version the
    INTEGRATION.md binding snippet asserts are the same number (the snippet must keep working)."""
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with open(os.path.join(root, "include", "tspm.h")) as f:
        hdr = int(re.search(r"#define TSPM_ABI_VERSION (\d+)", f.read()).group(1))
    with open(os.path.join(root, "INTEGRATION.md")) as f:
        doc = [int(v) for v in re.findall(r"tspm_abi_version\(\) == (\d+)", f.read())]
    assert doc and all(v == hdr for v in doc)
    assert L.ABI_VERSION == hdr


def test_launch_options_are_per_call_and_validated():
    """ABI 21: the LDS floor and the hand-off mode are tspm_conv_algo fields (no process-wide setter); values out of
    range are refused before any launch."""
    lib = L.load()
    assert ctypes.sizeof(L.ConvAlgo) == 32
    assert not hasattr(L, "tspm_set_conv_lds_floor") and "tspm_set_conv_lds_floor" not in L._SIGS
    a = L.ConvAlgo(1, 1, 1, 4, 1, 1)
    b = a.with_options(82000, L.ALGO_HANDOFF_ACQUIRE)
    assert (b.tm, b.tn, b.wn, b.wk, b.splits, b.variant, b.lds_floor, b.flags) == (1, 1, 1, 4, 1, 1, 82000, 1)
    assert (a.lds_floor, a.flags) == (0, 0)  # the tuned configuration itself is not modified
    s = L.ConvShape(128, 7, 7, 64, 64, 3, 3, 1, 1, 7, 7)
    st = L.hwnc_strides(128, 7, 7, 64)
    for bad in (a.with_options(160 * 1024 + 1), a.with_options(-1), a.with_options(0, 2)):
        B = ctypes.byref(bad)
        assert lib.tspm_conv_fwd(ctypes.byref(s), B, 16, ctypes.byref(st), 16, 16, None, None, 0, None) == 1
        assert lib.tspm_conv_dgrad(ctypes.byref(s), B, 16, 16, 16, 0, None, 0, None) == 1
        assert lib.tspm_conv_wgrad(ctypes.byref(s), B, 16, ctypes.byref(st), 16, 16, None, 0, None) == 1
        assert lib.tspm_conv_bwd(ctypes.byref(s), B, ctypes.byref(a), 16, ctypes.byref(st), 16, 16, 16, 0, 16,
                                 None, 0, None, 0, None) == 1
    hd = L.HeadDesc(n=8, in_=192, hidden=128, hidden2=64, classes=10, ldx=192, lddx=192, rows_per_block=2)
    assert lib.tspm_head_train_step(ctypes.byref(hd), None) == 1


def test_library_sources_read_no_environment_and_keep_no_mutable_globals():
    """nothing under csrc/ reads the environment, and no product translation unit defines a
    mutable file-scope variable (the stamp buffers exist only in the TSPM_STAMPS diagnostic build)."""
    csrc = os.path.join(REPO, "task-specific-pretraining-multimodal_amd", "csrc")
    for f in sorted(os.listdir(csrc)):
        if not f.endswith((".hip", ".h")):
            continue
        src = open(os.path.join(csrc, f)).read()
        assert "getenv" not in src, f
        product = re.sub(r"#if(def TSPM_STAMPS| defined\(TSPM_STAMPS\)).*?#endif", "", src, flags=re.S)
        for line in product.splitlines():
            if re.match(r"^(static\s+)?(__device__\s+)?(unsigned|int|long|size_t|float|double|bool|char)\b[\w\s\*]*\s\w+\s*(=|;|\[)",
                        line) and "constexpr" not in line and "(" not in line:
                raise AssertionError(f"{f}: file-scope variable: {line.strip()}")


def test_round6_entry_points_validate_before_launch():
    """The round-6 entry points refuse bad arguments before any launch (no GPU here: an accepted call would fail with
    TSPM_ERR_LAUNCH = 2, a refused one returns TSPM_ERR_INVALID = 1)."""
    lib = L.load()
    # tspm_bn_bwd_apply_part: more tiles than the merge prologue takes, a missing ReLU output
    assert lib.tspm_bn_bwd_apply_part(512, 256, 1025, *([16] * 10), *([None] * 7), None, None) == 1
    assert lib.tspm_bn_bwd_apply_part(512, 256, 16, 16, 16, None, *([16] * 7), *([None] * 7), None, None) == 1
    # tspm_bn_apply_merge: more than 256 tiles, channels not a multiple of 16
    assert lib.tspm_bn_apply_merge(6272, 64, 257, 32, 16, None, None, 0.1, 1e-5, 16, 16, 16, 16, 16, 0, None, None,
                                   None, None, None, 1, 16, None) == 1
    assert lib.tspm_bn_apply_merge(6272, 72, 196, 32, 16, None, None, 0.1, 1e-5, 16, 16, 16, 16, 16, 0, None, None,
                                   None, None, None, 1, 16, None) == 1
    # tspm_conv_fwd_pair: tile shapes differ; both halves split-K on one workspace
    s1, s2 = L.ConvShape(128, 4, 4, 128, 256, 3, 3, 2, 1, 2, 2), L.ConvShape(128, 4, 4, 128, 256, 1, 1, 2, 0, 2, 2)
    xs = L.hwnc_strides(128, 4, 4, 128)
    a1, a2, a3 = L.ConvAlgo(1, 1, 2, 2, 1, 1), L.ConvAlgo(1, 1, 1, 4, 1, 1), L.ConvAlgo(1, 1, 2, 2, 2, 1)
    B = ctypes.byref
    assert not lib.tspm_conv_fwd_pair_supported(B(s1), B(a1), B(xs), B(s2), B(a2), B(xs))
    assert lib.tspm_conv_fwd_pair_supported(B(s1), B(a1), B(xs), B(s2), B(a3), B(xs))
    assert lib.tspm_conv_fwd_pair(B(s1), B(a1), 16, B(xs), 16, 16, None, 16, 1 << 30, B(s2), B(a2), 16, B(xs), 16, 16,
                                  None, 32, 1 << 30, None) == 1
    assert lib.tspm_conv_fwd_pair(B(s1), B(a3), 16, B(xs), 16, 16, None, 16, 1 << 30, B(s2), B(a3), 16, B(xs), 16, 16,
                                  None, 16, 1 << 30, None) == 1
    # tspm_conv_bwd_ex: the whole-BN-backward mode without its tickets
    assert ctypes.sizeof(L.BnBwdPart) == 160
    bs, ba, bw = L.ConvShape(128, 2, 2, 256, 256, 3, 3, 1, 1, 2, 2), L.ConvAlgo(1, 1, 2, 2, 4, 1), L.ConvAlgo(1, 1, 1, 2, 1, 1)
    d = L.BnBwdPart(16, 16, 16, None, None, 16)
    d.dy = 16
    assert lib.tspm_conv_bwd_ex(B(bs), B(ba), B(bw), 16, B(L.hwnc_strides(128, 2, 2, 256)), 16, 16, 16, 0, 16, None, B(d),
                                16, 1 << 30, 32, 1 << 30, None) == 1
    # tspm_conv_bwd_quad: the downsample's wgrad tile differs from conv2's
    c2, ds = L.ConvShape(128, 2, 2, 256, 256, 3, 3, 1, 1, 2, 2), L.ConvShape(128, 4, 4, 128, 256, 1, 1, 2, 0, 2, 2)
    xs2 = L.hwnc_strides(128, 2, 2, 256)
    ad, aw, aw_other = L.ConvAlgo(1, 1, 2, 2, 1, 1), L.ConvAlgo(1, 1, 2, 1, 1, 1), L.ConvAlgo(1, 1, 1, 4, 1, 1)
    assert lib.tspm_conv_bwd_quad_supported(B(c2), B(ad), B(aw), B(xs2), B(ds), B(ad), B(aw), B(xs))
    assert not lib.tspm_conv_bwd_quad_supported(B(c2), B(ad), B(aw), B(xs2), B(ds), B(ad), B(aw_other), B(xs))
    assert lib.tspm_conv_bwd_quad(B(c2), B(ad), B(aw), 16, B(xs2), 16, 16, 16, 0, 16, None, 16, 1 << 30, 32, 1 << 30,
                                  B(ds), B(ad), B(aw_other), 16, B(xs), 16, 16, 16, 16, 48, 1 << 30, 64, 1 << 30, None,
                                  None) == 1
