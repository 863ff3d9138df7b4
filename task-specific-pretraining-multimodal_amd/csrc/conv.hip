// Implicit-GEMM convolution on v_mfma_f32_32x32x2_f32 (exact fp32, gfx950).
//
// Replaces nn.Conv2d fwd / dgrad / wgrad of MML_Suite/models/msa/networks/resnet.py:25,30,137,176.
//
// Operand delivery (no LDS staging): with the 32x32x2 f32 MFMA a lane supplies ONE A element (row
// l&31, k = l>>5) and ONE B element (k = l>>5, col l&31) per instruction.  Each lane loads 4
// consecutive reduction elements as one 16-byte load and feeds them to 4 consecutive MFMAs: half
// h = lane>>5 covers reduction indices c0+4h..c0+4h+3, so MFMA j reduces over {c0+j, c0+4+j}.  Any
// fixed permutation of the reduction order is a valid GEMM, so A and B only have to agree on it.
//   fwd   : A = x rows (HWNC, C contiguous) 16 B/lane; B = w[co][tap][c] (OHWI) 16 B/lane.
//   dgrad : A = dy rows (K contiguous) 16 B/lane; B = w[co][tap][ci] read as 4 coalesced dwords.
//   wgrad : A = dy[m][co], B = x[in(m,tap)][ci] as coalesced dwords (reduction over rows m).
// Waves whose 32*TM rows share one output position (batch % (32*TM) == 0 with the HWNC row order)
// know the valid (non-padding) taps uniformly and skip the rest; other waves mask per lane.
//
// Work decomposition (the layers are small: R34 layer4 at batch 128 is a 128x512x512 GEMM):
//   * a workgroup = WN x WK waves; the WN waves take neighbouring 32*TN-column tiles of the same
//     rows (A re-read from L1), the WK waves split the reduction of the SAME tile and combine their
//     accumulators through LDS in fixed order (deterministic, no HBM slabs, no extra launch);
//   * wgrad additionally splits its (long) reduction over rows across workgroups (grid.z) into fp32
//     slabs summed by tspm_reduce_slabs in slab order.
// The forward epilogue can also emit BatchNorm partial statistics of its output tile (per column:
// shift K = the tile's first row, mean offset and corrected sum of squared deviations), so the BN
// statistics never re-read the conv output (tspm_bn_finalize merges them).
#include "conv_common.h"

#ifdef TSPM_STAMPS
__device__ unsigned long long tspm_g_stamps[TSPM_STAMP_WAVES * TSPM_STAMP_SLOTS];
extern "C" int tspm_debug_stamps(void* host_dst, size_t bytes) {
  if (bytes > sizeof(tspm_g_stamps)) bytes = sizeof(tspm_g_stamps);
  return hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(tspm_g_stamps), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 2;
}
extern "C" int tspm_debug_stamps_clear(void) {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(tspm_g_stamps)) != hipSuccess) return 2;
  return hipMemset(p, 0, sizeof(tspm_g_stamps)) == hipSuccess ? 0 : 2;
}
#endif

namespace {

// =============================================================================================
// Forward, vector path: HWNC input, C % 8 == 0.
// =============================================================================================
template <int TM, int TN, int WN, int WK, bool F_>
__global__ __launch_bounds__(64 * WN * WK) void k_conv_fwd_vec(ConvArgs g, const float* __restrict__ x,
                                                              const float* __restrict__ w, float* __restrict__ y,
                                                              tspm_bn_fuse bf) {
  extern __shared__ float lds[];
  TSPM_STAMP(tspm_g_stamps, 0);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wn = wave % WN, wk = wave / WN;
  const int row0 = blockIdx.x * (TM * 32);
  const int col0 = (blockIdx.y * WN + wn) * (TN * 32);
  const bool active = col0 < g.k;
  const int li = lane & 31, hh = lane >> 5;
  const int C = g.c, N = g.n, RSC = g.r * g.s * C;
  const int cch = C >> 3;

  Acc<TM, TN> acc;
  acc.zero();
  if (active) {
    int nb[TM], hb[TM], wb[TM];
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      int m = min(row0 + a * 32 + li, g.m - 1);
      int pos = m / N;
      nb[a] = m - pos * N;
      int pp = pos / g.q, qq = pos - pp * g.q;
      hb[a] = pp * g.st - g.pad;
      wb[a] = qq * g.st - g.pad;
    }
    const float* wrow[TN];
#pragma unroll
    for (int b = 0; b < TN; ++b) wrow[b] = w + (long long)min(col0 + b * 32 + li, g.k - 1) * RSC + 4 * hh;

    const int pos_first = row0 / N;
    const int pos_last = (min(row0 + TM * 32, g.m) - 1) / N;
    if (pos_first == pos_last) {
      // ---- uniform position: iterate over the valid taps only ----
      const int pp = pos_first / g.q, qq = pos_first - pp * g.q;
      const int h0 = pp * g.st - g.pad, w0 = qq * g.st - g.pad;
      const int r_lo = max(0, -h0), r_hi = min(g.r - 1, g.h - 1 - h0);
      const int s_lo = max(0, -w0), s_hi = min(g.s - 1, g.w - 1 - w0);
      const int nr = r_hi - r_lo + 1, ns = s_hi - s_lo + 1;
      const int T = (nr > 0 && ns > 0) ? nr * ns * cch : 0;
      const int it0 = split_lo(T, wk, WK), it1 = split_lo(T, wk + 1, WK);
      const float* xa[TM];
#pragma unroll
      for (int a = 0; a < TM; ++a) xa[a] = x + (long long)nb[a] * C + 4 * hh;
      // iteration it = (valid tap, 8-channel chunk), taps row-major over the valid window
      run_pipelined<TM, TN, prefetch_depth<TM, TN>()>(acc, it0, it1, [&](int it, f32x4 (&A)[TM], f32x4 (&B)[TN]) {
        const int tap = it / cch, ci = (it - tap * cch) * 8;
        const int tr = tap / ns;
        const int r = r_lo + tr, s = s_lo + (tap - tr * ns);
        const long long ao = ((long long)(h0 + r) * g.w + (w0 + s)) * N * C + ci;
        const int bo = (r * g.s + s) * C + ci;
#pragma unroll
        for (int a = 0; a < TM; ++a) A[a] = ld4(xa[a] + ao);
#pragma unroll
        for (int b = 0; b < TN; ++b) B[b] = ld4(wrow[b] + bo);
      });
    } else {
      // ---- mixed positions: all taps, per-lane padding masks ----
      const int T = g.r * g.s * cch;
      const int it0 = split_lo(T, wk, WK), it1 = split_lo(T, wk + 1, WK);
      bool rowok[TM];
#pragma unroll
      for (int a = 0; a < TM; ++a) rowok[a] = (row0 + a * 32 + li) < g.m;
      for (int it = it0; it < it1; ++it) {
        const int tap = it / cch, ci = (it - tap * cch) * 8;
        const int r = tap / g.s, s = tap - r * g.s;
        f32x4 A[TM], B[TN];
#pragma unroll
        for (int a = 0; a < TM; ++a) {
          const int hi = hb[a] + r, wi = wb[a] + s;
          const bool ok = rowok[a] && hi >= 0 && hi < g.h && wi >= 0 && wi < g.w;
          const long long off = (((long long)hi * g.w + wi) * N + nb[a]) * C + ci + 4 * hh;
          A[a] = ok ? ld4(x + off) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int b = 0; b < TN; ++b) B[b] = ld4(wrow[b] + (r * g.s + s) * C + ci);
        acc.mma4(A, B);
      }
    }
  }
  TSPM_STAMP(tspm_g_stamps, 1);
  acc.template combine<WN, WK>(lds, wn, wk, lane, active);
  TSPM_STAMP(tspm_g_stamps, 2);
  if (wk == 0 && active) {
    acc.store(y, row0, col0, g.m, g.k, g.k, lane, false);
    if (bf.partial)
      acc.bn_partials(bf.partial, (long long)gridDim.x * g.k, blockIdx.x, row0, col0, g.m, g.k, lane, bf.counters != nullptr);
  }
  TSPM_STAMP(tspm_g_stamps, 3);
  fwd_bn_tail<TM, TN, WN>(g, bf, lds);
  TSPM_STAMP(tspm_g_stamps, 4);
}

// =============================================================================================
// Forward, gather path: arbitrary input strides / any C (the Cin=1 7x7 stem reads the reference's
// NCHW input directly).  Reduction index kidx = (r*S + s)*C + c, chunks of 8, scalar loads.
// =============================================================================================
template <int TM, int TN, int WN, int WK, bool F_>
__global__ __launch_bounds__(64 * WN * WK) void k_conv_fwd_gather(ConvArgs g, const float* __restrict__ x,
                                                                 const float* __restrict__ w, float* __restrict__ y,
                                                                 tspm_bn_fuse bf) {
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wn = wave % WN, wk = wave / WN;
  const int row0 = blockIdx.x * (TM * 32);
  const int col0 = (blockIdx.y * WN + wn) * (TN * 32);
  const bool active = col0 < g.k;
  const int li = lane & 31, hh = lane >> 5;
  const int C = g.c, N = g.n, RSC = g.r * g.s * C;

  Acc<TM, TN> acc;
  acc.zero();
  if (active) {
    int hb[TM], wb[TM];
    long long xb[TM];
    bool rowok[TM];
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      int mr = row0 + a * 32 + li;
      rowok[a] = mr < g.m;
      int m = min(mr, g.m - 1);
      int pos = m / N, nbv = m - pos * N;
      int pp = pos / g.q, qq = pos - pp * g.q;
      hb[a] = pp * g.st - g.pad;
      wb[a] = qq * g.st - g.pad;
      xb[a] = (long long)nbv * g.sn;
    }
    int co[TN];
#pragma unroll
    for (int b = 0; b < TN; ++b) co[b] = min(col0 + b * 32 + li, g.k - 1);
    const int T = cdiv_dev(RSC, 8);
    const int it0 = split_lo(T, wk, WK), it1 = split_lo(T, wk + 1, WK);
    for (int it = it0; it < it1; ++it) {
      f32x4 A[TM], B[TN];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int kidx = it * 8 + 4 * hh + j;
        const bool kok = kidx < RSC;
        const int kk = kok ? kidx : 0;
        const int tap = kk / C, cc = kk - tap * C;
        const int r = tap / g.s, s = tap - r * g.s;
#pragma unroll
        for (int a = 0; a < TM; ++a) {
          const int hi = hb[a] + r, wi = wb[a] + s;
          const bool ok = kok && rowok[a] && hi >= 0 && hi < g.h && wi >= 0 && wi < g.w;
          A[a][j] = ok ? x[xb[a] + hi * g.sh + wi * g.sw + cc * g.sc] : 0.f;
        }
#pragma unroll
        for (int b = 0; b < TN; ++b) B[b][j] = kok ? w[(long long)co[b] * RSC + kk] : 0.f;
      }
      acc.mma4(A, B);
    }
  }
  acc.template combine<WN, WK>(lds, wn, wk, lane, active);
  if (wk == 0 && active) {
    acc.store(y, row0, col0, g.m, g.k, g.k, lane, false);
    if (bf.partial)
      acc.bn_partials(bf.partial, (long long)gridDim.x * g.k, blockIdx.x, row0, col0, g.m, g.k, lane, bf.counters != nullptr);
  }
  fwd_bn_tail<TM, TN, WN>(g, bf, lds);
}

// =============================================================================================
// Data gradient: dx[h,w,n,ci] = sum_{r,s,co} dy[(h+pad-r)/st, (w+pad-s)/st, n, co] * w[co,r,s,ci]
// GEMM rows m = (h,w,n) of the input, cols = ci, reduction over (valid tap, co) in chunks of 8 co.
// =============================================================================================
template <int TM, int TN, int WN, int WK, bool F_>
__global__ __launch_bounds__(64 * WN * WK) void k_conv_dgrad(ConvArgs g, const float* __restrict__ dy,
                                                            const float* __restrict__ w, float* __restrict__ dx) {
  extern __shared__ float lds[];
  TSPM_STAMP(tspm_g_stamps, 0);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wn = wave % WN, wk = wave / WN;
  const int row0 = blockIdx.x * (TM * 32);
  const int col0 = (blockIdx.y * WN + wn) * (TN * 32);
  const bool active = col0 < g.c;
  const int li = lane & 31, hh = lane >> 5;
  const int C = g.c, N = g.n, K = g.k, RSC = g.r * g.s * C;
  const int kch = K >> 3;

  Acc<TM, TN> acc;
  acc.zero();
  if (active) {
    int nb[TM], hp[TM], wp[TM];
    bool rowok[TM];
#pragma unroll
    for (int a = 0; a < TM; ++a) {
      int mr = row0 + a * 32 + li;
      rowok[a] = mr < g.m;
      int m = min(mr, g.m - 1);
      int pos = m / N;
      nb[a] = m - pos * N;
      int hi = pos / g.w, wi = pos - hi * g.w;
      hp[a] = hi + g.pad;
      wp[a] = wi + g.pad;
    }
    int ci[TN];
#pragma unroll
    for (int b = 0; b < TN; ++b) ci[b] = min(col0 + b * 32 + li, C - 1);

    const int pos_first = row0 / N;
    const int pos_last = (min(row0 + TM * 32, g.m) - 1) / N;
    if (pos_first == pos_last) {
      const int hi = pos_first / g.w, wi = pos_first - hi * g.w;
      unsigned rmask = 0, smask = 0;
      for (int r = 0; r < g.r; ++r) {
        int t = hi + g.pad - r;
        if (t >= 0 && t % g.st == 0 && t / g.st < g.p) rmask |= 1u << r;
      }
      for (int s = 0; s < g.s; ++s) {
        int t = wi + g.pad - s;
        if (t >= 0 && t % g.st == 0 && t / g.st < g.q) smask |= 1u << s;
      }
      const int nr = __builtin_popcount(rmask), ns = __builtin_popcount(smask);
      const int T = nr * ns * kch;
      const int it0 = split_lo(T, wk, WK), it1 = split_lo(T, wk + 1, WK);
      const float* dya[TM];
#pragma unroll
      for (int a = 0; a < TM; ++a) dya[a] = dy + (long long)nb[a] * K + 4 * hh;
      run_pipelined<TM, TN, prefetch_depth<TM, TN>()>(acc, it0, it1, [&](int it, f32x4 (&A)[TM], f32x4 (&B)[TN]) {
        const int t = it / kch, c0 = (it - t * kch) * 8;
        const int ri = t / ns, si = t - ri * ns;
        unsigned rm = rmask, sm = smask;
        for (int i = 0; i < ri; ++i) rm &= rm - 1;
        for (int i = 0; i < si; ++i) sm &= sm - 1;
        const int r = __builtin_ctz(rm), s = __builtin_ctz(sm);
        const int pp = (hi + g.pad - r) / g.st, qq = (wi + g.pad - s) / g.st;
        const long long aoff = ((long long)pp * g.q + qq) * N * K + c0;
#pragma unroll
        for (int a = 0; a < TM; ++a) A[a] = ld4(dya[a] + aoff);
        const long long wbase = (long long)(c0 + 4 * hh) * RSC + (r * g.s + s) * C;
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
          for (int j = 0; j < 4; ++j) B[b][j] = w[wbase + (long long)j * RSC + ci[b]];
      });
    } else {
      const int T = g.r * g.s * kch;
      const int it0 = split_lo(T, wk, WK), it1 = split_lo(T, wk + 1, WK);
      for (int it = it0; it < it1; ++it) {
        const int tap = it / kch, c0 = (it - tap * kch) * 8;
        const int r = tap / g.s, s = tap - r * g.s;
        f32x4 A[TM], B[TN];
#pragma unroll
        for (int a = 0; a < TM; ++a) {
          const int th = hp[a] - r, tw = wp[a] - s;
          const int pp = th / g.st, qq = tw / g.st;
          const bool ok = rowok[a] && th >= 0 && tw >= 0 && pp * g.st == th && qq * g.st == tw && pp < g.p && qq < g.q;
          const long long off = (((long long)pp * g.q + qq) * N + nb[a]) * K + c0 + 4 * hh;
          A[a] = ok ? ld4(dy + off) : f32x4{0.f, 0.f, 0.f, 0.f};
        }
        const long long wbase = (long long)(c0 + 4 * hh) * RSC + (r * g.s + s) * C;
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
          for (int j = 0; j < 4; ++j) B[b][j] = w[wbase + (long long)j * RSC + ci[b]];
        acc.mma4(A, B);
      }
    }
  }
  TSPM_STAMP(tspm_g_stamps, 1);
  acc.template combine<WN, WK>(lds, wn, wk, lane, active);
  TSPM_STAMP(tspm_g_stamps, 2);
  if (wk == 0 && active) acc.store(dx, row0, col0, g.m, C, C, lane, g.beta != 0);
  TSPM_STAMP(tspm_g_stamps, 3);
}

// =============================================================================================
// Weight gradient: dw[co, (r,s,c)] = sum_m dy[m, co] * x[in(m, r, s), c]
// GEMM rows = co (K), cols = kidx = (r*S+s)*C + c, reduction over output rows m in chunks of 8,
// split over WK waves in the workgroup and `splits` workgroups (grid.z, fp32 slabs).
// FAST: N % 8 == 0 so an 8-row chunk shares one output position (uniform decomposition).
// =============================================================================================
template <int TM, int TN, int WN, int WK, bool FAST>
__global__ __launch_bounds__(64 * WN * WK) void k_conv_wgrad(ConvArgs g, const float* __restrict__ x,
                                                            const float* __restrict__ dy, float* __restrict__ dw,
                                                            float* __restrict__ dw_final) {
  extern __shared__ float lds[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wn = wave % WN, wk = wave / WN;
  const int K = g.k, C = g.c, N = g.n;
  const int RSC = g.r * g.s * C;
  const int row0 = blockIdx.x * (TM * 32);   // co
  const int col0 = (blockIdx.y * WN + wn) * (TN * 32);   // kidx
  const bool active = col0 < RSC;
  const int z = blockIdx.z;
  const int li = lane & 31, hh = lane >> 5;
  const int Mout = g.p * g.q * N;

  Acc<TM, TN> acc;
  acc.zero();
  if (active) {
    int co[TM];
#pragma unroll
    for (int a = 0; a < TM; ++a) co[a] = min(row0 + a * 32 + li, K - 1);
    int kr[TN], ks[TN], kc[TN];
    bool kok[TN];
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      int kidx = col0 + b * 32 + li;
      kok[b] = kidx < RSC;
      kidx = min(kidx, RSC - 1);
      int tap = kidx / C;
      kc[b] = kidx - tap * C;
      kr[b] = tap / g.s;
      ks[b] = tap - kr[b] * g.s;
    }
    const int tap_first = col0 / C, tap_last = (min(col0 + TN * 32, RSC) - 1) / C;
    const bool one_tap = tap_first == tap_last;
    const int S = g.splits * WK, zz = z * WK + wk;
    if (FAST && one_tap) {
      // The tile's columns share one tap (r, s): only output positions whose input tap lies inside
      // the image contribute — a rectangle [pp_lo, pp_hi] x [qq_lo, qq_hi].  Enumerate its 8-row
      // chunks (rows (pp*Q + qq)*N + n, n in chunk), split evenly over the S reducers.
      const int r = tap_first / g.s, s = tap_first - r * g.s;
      const int pp_lo = max(0, cdiv_dev(g.pad - r, g.st)), pp_hi = min(g.p - 1, (g.h - 1 + g.pad - r) / g.st);
      const int qq_lo = max(0, cdiv_dev(g.pad - s, g.st)), qq_hi = min(g.q - 1, (g.w - 1 + g.pad - s) / g.st);
      const int npp = max(0, pp_hi - pp_lo + 1), nqq = max(0, qq_hi - qq_lo + 1), n8 = N >> 3;
      const int T = npp * nqq * n8;
      const int it0 = split_lo(T, zz, S), it1 = split_lo(T, zz + 1, S);
      long long xoff[TN];
#pragma unroll
      for (int b = 0; b < TN; ++b) xoff[b] = (long long)kc[b] * g.sc;
      run_pipelined<TM, TN, prefetch_depth<TM, TN>()>(acc, it0, it1, [&](int it, f32x4 (&A)[TM], f32x4 (&B)[TN]) {
        const int pc = it / n8, nch = it - pc * n8;
        const int ip = pc / nqq, iq = pc - ip * nqq;
        const int pp = pp_lo + ip, qq = qq_lo + iq;
        const int n0 = nch * 8 + hh;
        const long long mrow = ((long long)pp * g.q + qq) * N + n0;
        const long long xb = (long long)n0 * g.sn + (long long)(pp * g.st - g.pad + r) * g.sh +
                             (long long)(qq * g.st - g.pad + s) * g.sw;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
          for (int a = 0; a < TM; ++a) A[a][j] = dy[(mrow + 2 * j) * K + co[a]];
#pragma unroll
          for (int b = 0; b < TN; ++b) B[b][j] = x[xb + 2 * j * g.sn + xoff[b]];
        }
      });
    } else {
    const int T = cdiv_dev(Mout, 8);
    const int it0 = split_lo(T, zz, S), it1 = split_lo(T, zz + 1, S);
    for (int it = it0; it < it1; ++it) {
      const int mbase = it * 8;
      int pp_u = 0, qq_u = 0, nb_u = 0;
      if (FAST) {
        const int pos = mbase / N;
        nb_u = mbase - pos * N;
        pp_u = pos / g.q;
        qq_u = pos - pp_u * g.q;
        if (one_tap) {
          const int r = tap_first / g.s, s = tap_first - r * g.s;
          const int hi = pp_u * g.st - g.pad + r, wi = qq_u * g.st - g.pad + s;
          if (hi < 0 || hi >= g.h || wi < 0 || wi >= g.w) continue;  // padding tap for the whole chunk
        }
      }
      f32x4 A[TM], B[TN];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int m = mbase + 2 * j + hh;
        const bool mok = m < Mout;
        const int mm = mok ? m : 0;
#pragma unroll
        for (int a = 0; a < TM; ++a) A[a][j] = mok ? dy[(long long)mm * K + co[a]] : 0.f;
        int pp, qq, nbv;
        if (FAST) {
          pp = pp_u; qq = qq_u; nbv = nb_u + 2 * j + hh;
        } else {
          const int pos = mm / N;
          nbv = mm - pos * N;
          pp = pos / g.q;
          qq = pos - pp * g.q;
        }
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          const int hi = pp * g.st - g.pad + kr[b], wi = qq * g.st - g.pad + ks[b];
          const bool ok = mok && kok[b] && hi >= 0 && hi < g.h && wi >= 0 && wi < g.w;
          B[b][j] = ok ? x[nbv * g.sn + hi * g.sh + wi * g.sw + kc[b] * g.sc] : 0.f;
        }
      }
      acc.mma4(A, B);
    }
    }
  }
  acc.template combine<WN, WK>(lds, wn, wk, lane, active);
  if (wk == 0 && active) {
    float* out = g.splits > 1 ? dw + (long long)z * g.slab : dw;
    acc.store(out, row0, col0, K, RSC, RSC, lane, false, g.cnt != nullptr);
  }
  if (g.splits > 1 && g.cnt) slab_tail<TM, TN, WN>(g, dw, dw_final, RSC, lds);
}

__global__ __launch_bounds__(256) void k_reduce_slabs(long long count, int nslab, long long slab_stride,
                                                      const float* __restrict__ slabs, float* __restrict__ out,
                                                      int beta) {
  const long long n4 = count >> 2;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    f32x4 s = beta ? ld4(out + 4 * i) : f32x4{0.f, 0.f, 0.f, 0.f};
    for (int z = 0; z < nslab; ++z) s += ld4(slabs + z * slab_stride + 4 * i);
    st4(out + 4 * i, s);
  }
  if (blockIdx.x == 0 && threadIdx.x < (count & 3)) {
    long long i = (n4 << 2) + threadIdx.x;
    float s = beta ? out[i] : 0.f;
    for (int z = 0; z < nslab; ++z) s += slabs[z * slab_stride + i];
    out[i] = s;
  }
}

// Many slabs of a small output (the 7x7 stem weight gradient: 64 x 49 floats split over 64 slabs): the
// loop above would give each of a handful of workgroups a serial chain of nslab loads per element.  Here
// Q slab groups x (256 / Q) elements per workgroup: group q sums slabs q, q+Q, q+2Q, ... in order (four
// loads in flight), then the Q partial sums are added in group order — a fixed order, so deterministic.
template <int Q>
__global__ __launch_bounds__(256) void k_reduce_slabs_wide(long long count, int nslab, long long slab_stride,
                                                           const float* __restrict__ slabs, float* __restrict__ out,
                                                           int beta) {
  constexpr int E = 256 / Q;
  __shared__ float part[Q][E];
  const int e = threadIdx.x % E, q = threadIdx.x / E;
  const long long i = blockIdx.x * (long long)E + e;
  float s = 0.f;
  if (i < count) {
    int z = q;
    for (; z + 3 * Q < nslab; z += 4 * Q) {
      const float a = slabs[z * slab_stride + i], b = slabs[(z + Q) * slab_stride + i];
      const float c = slabs[(z + 2 * Q) * slab_stride + i], d = slabs[(z + 3 * Q) * slab_stride + i];
      s += a;
      s += b;
      s += c;
      s += d;
    }
    for (; z < nslab; z += Q) s += slabs[z * slab_stride + i];
  }
  part[q][e] = s;
  __syncthreads();
  if (q == 0 && i < count) {
    float t = beta ? out[i] : 0.f;
#pragma unroll
    for (int k = 0; k < Q; ++k) t += part[k][e];
    out[i] = t;
  }
}

void launch_reduce_slabs(long long count, int nslab, long long slab_stride, const float* slabs, float* out, int beta,
                         hipStream_t st) {
  constexpr int kQ = 8;
  if (nslab >= 2 * kQ && count <= (1LL << 18)) {  // slab-parallel: many slabs of a small output
    hipLaunchKernelGGL((k_reduce_slabs_wide<kQ>), dim3((unsigned)cdiv64(count, 256 / kQ)), dim3(256), 0, st, count,
                       nslab, slab_stride, slabs, out, beta);
    return;
  }
  const int blocks = (int)std::min<long long>(cdiv64(count / 4 + 1, 256), 2048);
  hipLaunchKernelGGL(k_reduce_slabs, dim3(blocks), dim3(256), 0, st, count, nslab, slab_stride, slabs, out, beta);
}

// ---------------------------------------------------------------------------------------------
// host-side dispatch
// ---------------------------------------------------------------------------------------------
bool shape_ok(const tspm_conv_shape* s) {
  if (!s) return false;
  if (s->n <= 0 || s->h <= 0 || s->w <= 0 || s->c <= 0 || s->k <= 0 || s->r <= 0 || s->s <= 0) return false;
  if (s->stride <= 0 || s->pad < 0 || s->r > 31 || s->s > 31) return false;
  if (s->p != (s->h + 2 * s->pad - s->r) / s->stride + 1) return false;
  if (s->q != (s->w + 2 * s->pad - s->s) / s->stride + 1) return false;
  return s->p > 0 && s->q > 0;
}

struct Algo {
  int tm, tn, wn, wk, splits;
};

int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
int pow2_floor(int v) { int p = 1; while (p * 2 <= v) p *= 2; return p; }

// heuristic (used when no tuned table entry exists): spread over >= ~256 workgroups (one per CU)
// with >= 4 waves each, 32x32 tiles when the output is small, >= 4 reduction iterations per wave
Algo pick(const tspm_conv_algo* user, long long rows, long long cols, long long red_iters, bool allow_global) {
  Algo a{1, 1, 1, 1, 1};
  if (user && user->tm > 0) {
    a.tm = user->tm; a.tn = user->tn; a.wn = user->wn > 0 ? user->wn : 1; a.wk = user->wk > 0 ? user->wk : 1;
    a.splits = user->splits > 0 ? user->splits : 1;
    return a;
  }
  if (cols >= 64 && rows * cols >= (long long)256 * 32 * 64) a.tn = 2;
  if (a.tn == 2 && rows * cols >= (long long)512 * 64 * 64) a.tm = 2;
  const long long tiles = cdiv64(rows, 32 * a.tm) * cdiv64(cols, 32 * a.tn);
  int wk = 1;
  while (wk < 8 && tiles * wk < 1024 && red_iters / (wk * 2) >= 4) wk *= 2;
  a.wk = wk;
  a.wn = 1;
  if (allow_global) {
    long long want = cdiv64(1024, tiles * wk);
    int sp = (int)std::min<long long>(want, 64);
    while (sp > 1 && red_iters / ((long long)sp * wk) < 8) --sp;
    a.splits = sp < 1 ? 1 : sp;
  }
  return a;
}

size_t lds_bytes(const Algo& a) { return (size_t)(a.wk - 1) * a.wn * a.tm * a.tn * 16 * 64 * sizeof(float); }

bool algo_supported(const Algo& a) {
  if (a.splits < 1) return false;
  if (!((a.tm == 1 && a.tn == 1) || (a.tm == 1 && a.tn == 2) || (a.tm == 2 && a.tn == 2))) return false;
  if (!(a.wn == 1 || a.wn == 2 || a.wn == 4)) return false;
  if (!(a.wk == 1 || a.wk == 2 || a.wk == 4 || a.wk == 8 || a.wk == 16)) return false;
  if (a.wk == 16 && a.wn != 1) return false;
  if (a.wn * a.wk > 16 || (a.wn > 1 && a.wn * a.wk > 8)) return false;
  return lds_bytes(a) <= 160 * 1024;
}

#define TSPM_L(KERNEL, TM_, TN_, WN_, WK_, F_, ...) \
  hipLaunchKernelGGL((KERNEL<TM_, TN_, WN_, WK_, F_>), grid, dim3(64 * WN_ * WK_), lds, st, __VA_ARGS__)

#define TSPM_WK_SWITCH(KERNEL, TM_, TN_, WN_, F_, ...)                  \
  switch (al.wk) {                                                      \
    case 1: TSPM_L(KERNEL, TM_, TN_, WN_, 1, F_, __VA_ARGS__); break;   \
    case 2: TSPM_L(KERNEL, TM_, TN_, WN_, 2, F_, __VA_ARGS__); break;   \
    case 4: TSPM_L(KERNEL, TM_, TN_, WN_, 4, F_, __VA_ARGS__); break;   \
    case 8: TSPM_L(KERNEL, TM_, TN_, WN_, 8, F_, __VA_ARGS__); break;   \
    default: TSPM_L(KERNEL, TM_, TN_, WN_, 16, F_, __VA_ARGS__); break; \
  }

#define TSPM_WN_SWITCH(KERNEL, TM_, TN_, F_, ...)                                             \
  if (al.wn == 1) {                                                                           \
    TSPM_WK_SWITCH(KERNEL, TM_, TN_, 1, F_, __VA_ARGS__)                                      \
  } else if (al.wn == 2) {                                                                    \
    switch (al.wk) {                                                                          \
      case 1: TSPM_L(KERNEL, TM_, TN_, 2, 1, F_, __VA_ARGS__); break;                         \
      case 2: TSPM_L(KERNEL, TM_, TN_, 2, 2, F_, __VA_ARGS__); break;                         \
      default: TSPM_L(KERNEL, TM_, TN_, 2, 4, F_, __VA_ARGS__); break;                        \
    }                                                                                         \
  } else {                                                                                    \
    if (al.wk == 1) TSPM_L(KERNEL, TM_, TN_, 4, 1, F_, __VA_ARGS__);                          \
    else TSPM_L(KERNEL, TM_, TN_, 4, 2, F_, __VA_ARGS__);                                     \
  }

#define TSPM_DISPATCH(KERNEL, F_, ...)                                                   \
  do {                                                                                   \
    if (al.tm == 1 && al.tn == 1) { TSPM_WN_SWITCH(KERNEL, 1, 1, F_, __VA_ARGS__) }       \
    else if (al.tm == 1 && al.tn == 2) { TSPM_WN_SWITCH(KERNEL, 1, 2, F_, __VA_ARGS__) }  \
    else { TSPM_WN_SWITCH(KERNEL, 2, 2, F_, __VA_ARGS__) }                                \
  } while (0)

ConvArgs make_args(const tspm_conv_shape* s) {
  ConvArgs g{};
  g.n = s->n; g.h = s->h; g.w = s->w; g.c = s->c; g.k = s->k; g.r = s->r; g.s = s->s;
  g.st = s->stride; g.pad = s->pad; g.p = s->p; g.q = s->q;
  g.sn = (long long)s->c; g.sh = (long long)s->w * s->n * s->c; g.sw = (long long)s->n * s->c; g.sc = 1;
  g.m = 0; g.splits = 1; g.slab = 0; g.beta = 0; g.cnt = nullptr;
  g.xcd = 0;
  g.acq = 1;  // register-direct kernels: acquire-based hand-offs (conv_common.h tails)
  return g;
}

constexpr int kMaxFusedSplits = 16;   // wgrad: in-launch slab reduction up to this many slabs
constexpr int kMaxFusedMergeIters = 16;  // fwd: in-launch BN merge when each thread reads <= this many tiles

// In-launch hand-offs (BN merge / slab reduction by the last arriving workgroup) are always on.
constexpr bool inlaunch_enabled() { return true; }

bool is_hwnc(const tspm_conv_shape* s, const tspm_strides4* st) {
  if (!st) return true;
  return st->sc == 1 && st->sn == s->c && st->sw == (long long)s->n * s->c && st->sh == (long long)s->w * s->n * s->c;
}

Algo fwd_algo(const tspm_conv_shape* s, const tspm_conv_algo* user) {
  long long rows = (long long)s->p * s->q * s->n;
  long long iters = (long long)s->r * s->s * cdiv(s->c, 8);
  Algo a = pick(user, rows, s->k, iters, false);
  a.splits = 1;
  return a;
}
Algo dgrad_algo(const tspm_conv_shape* s, const tspm_conv_algo* user) {
  long long rows = (long long)s->h * s->w * s->n;
  long long iters = (long long)s->r * s->s * (s->k / 8);
  Algo a = pick(user, rows, s->c, iters, false);
  a.splits = 1;
  return a;
}
Algo wgrad_algo(const tspm_conv_shape* s, const tspm_conv_algo* user) {
  long long cols = (long long)s->r * s->s * s->c;
  long long iters = cdiv64((long long)s->p * s->q * s->n, 8);
  return pick(user, s->k, cols, iters, true);
}

// variants 1, 2 and 4 (LDS-staged, conv_lds.hip: register-staged loader waves / single-role LDS-DMA ring / the
// register-staged kernels with exact three-piece bf16 products):
// wm = 4 / (wn * wk)
// the per-call launch options of ABI 21 (tspm_conv_algo.lds_floor / flags) are in range
bool opts_ok(const tspm_conv_algo* u) {
  return !u || (u->lds_floor >= 0 && u->lds_floor <= 160 * 1024 && (u->flags & ~TSPM_ALGO_HANDOFF_ACQUIRE) == 0);
}
bool is_lds(const tspm_conv_algo* user) {
  return user && (user->variant == 1 || user->variant == 2 || user->variant == 4);
}
bool is_stem(const tspm_conv_algo* user) { return user && user->variant == 3; }
const tspm_detail::LdsImpl& lds_of(const tspm_conv_algo* user) {
  return user->variant == 2 ? tspm_detail::lds_impl_dma()
                            : (user->variant == 4 ? tspm_detail::lds_impl_x9() : tspm_detail::lds_impl_reg());
}
tspm_detail::LdsAlgo lds_algo(const tspm_conv_algo* u) {
  tspm_detail::LdsAlgo a{u->tm, u->tn, 0, u->wn, u->wk, u->splits > 0 ? u->splits : 1,
                         (size_t)std::max(0, u->lds_floor), (u->flags & TSPM_ALGO_HANDOFF_ACQUIRE) ? 1 : 0};
  const int wnk = a.wn * a.wk;
  a.wm = (wnk > 0 && 4 % wnk == 0) ? 4 / wnk : 0;
  return a;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
extern "C" size_t tspm_conv_fwd_workspace(const tspm_conv_shape* s, const tspm_conv_algo* user) {
  if (!shape_ok(s) || !is_lds(user)) return 0;  // register-direct: in-workgroup split-K only
  return lds_of(user).fwd_workspace(s, lds_algo(user));
}

extern "C" int32_t tspm_conv_fwd_tiles(const tspm_conv_shape* s, const tspm_conv_algo* user) {
  if (!shape_ok(s)) return 0;
  if (is_stem(user)) return tspm_detail::stem_supported(s) ? tspm_detail::stem_tiles(s) : 0;
  const int rows = is_lds(user) ? user->tm * 32 : fwd_algo(s, user).tm * 32;
  return rows > 0 ? cdiv(s->p * s->q * s->n, rows) : 0;
}

// 1 when tspm_conv_fwd with a BN fuse that has counters (and no two-level buffers) merges the statistics inside
// the launch, 0 when it follows the launch with tspm_bn_finalize (round 6: the caller may instead pass no counters
// and merge in the apply, tspm_bn_apply_merge)
extern "C" int32_t tspm_conv_fwd_bn_inlaunch(const tspm_conv_shape* s, const tspm_conv_algo* user) {
  if (!shape_ok(s) || is_stem(user)) return 0;
  if (is_lds(user)) return lds_of(user).fwd_bn_inlaunch(s, lds_algo(user));
  const Algo al = fwd_algo(s, user);
  const int tiles = cdiv(s->p * s->q * s->n, al.tm * 32), groups = 2 * al.wk / al.tn;
  return (cdiv(tiles, groups) <= kMaxFusedMergeIters && inlaunch_enabled()) ? 1 : 0;
}

extern "C" int32_t tspm_conv_fwd_tile_rows(const tspm_conv_shape* s, const tspm_conv_algo* user) {
  if (!shape_ok(s)) return 0;
  if (is_stem(user)) return tspm_detail::stem_supported(s) ? tspm_detail::stem_tile_rows(s) : 0;
  return is_lds(user) ? user->tm * 32 : fwd_algo(s, user).tm * 32;
}

extern "C" int32_t tspm_conv_fwd_bn_counters(const tspm_conv_shape* s, const tspm_conv_algo* user) {
  if (!shape_ok(s)) return 0;
  const int single = cdiv(s->k, 32);
  return is_lds(user) ? std::max(single, lds_of(user).fwd_bn_counters(s, lds_algo(user))) : single;
}

extern "C" int64_t tspm_conv_fwd_bn_partial_floats(const tspm_conv_shape* s, const tspm_conv_algo* user) {
  if (!shape_ok(s)) return 0;
  if (is_lds(user)) return lds_of(user).fwd_bn_partial_floats(s, lds_algo(user));
  if (is_stem(user)) return tspm_detail::stem_supported(s) ? 3LL * tspm_detail::stem_tiles(s) * s->k : 0;
  return 3LL * tspm_conv_fwd_tiles(s, user) * s->k;
}

extern "C" int tspm_conv_fwd(const tspm_conv_shape* s, const tspm_conv_algo* user, const float* x,
                             const tspm_strides4* xs, const float* w, float* y, const tspm_bn_fuse* bn, void* ws,
                             size_t ws_bytes, tspm_stream_t stream) {
  if (!shape_ok(s) || !x || !w || !y || !opts_ok(user)) return TSPM_ERR_INVALID;
  tspm_bn_fuse bf{};
  if (bn) {
    bf = *bn;
    if (!bf.partial && bf.counters) return TSPM_ERR_INVALID;
    if (bf.counters && (!bf.save_mean || !bf.save_invstd)) return TSPM_ERR_INVALID;
  }
  if (is_lds(user)) {
    const tspm_detail::LdsAlgo la = lds_algo(user);
    if (!lds_of(user).fwd_supported(s, xs, la)) return TSPM_ERR_INVALID;
    return lds_of(user).fwd(s, la, x, w, y, bn ? &bf : nullptr, ws, ws_bytes, static_cast<hipStream_t>(stream));
  }
  if (is_stem(user)) {  // per-band partials, merged by tspm_bn_finalize when the caller asked for the merge
    if (!tspm_detail::stem_supported(s)) return TSPM_ERR_INVALID;
    const int rc = tspm_detail::stem_fwd(s, x, xs, w, y, bn ? bf.partial : nullptr, static_cast<hipStream_t>(stream));
    if (rc != TSPM_OK || !bn || !bf.counters) return rc;
    return tspm_bn_finalize((long long)s->p * s->q * s->n, s->k, tspm_detail::stem_tiles(s),
                            tspm_detail::stem_tile_rows(s), bf.partial, bf.running_mean, bf.running_var, bf.momentum,
                            bf.eps, bf.save_mean, bf.save_invstd, stream);
  }
  (void)ws; (void)ws_bytes;
  Algo al = fwd_algo(s, user);
  if (!algo_supported(al)) return TSPM_ERR_INVALID;
  ConvArgs g = make_args(s);
  if (xs) { g.sn = xs->sn; g.sh = xs->sh; g.sw = xs->sw; g.sc = xs->sc; }
  g.m = s->p * s->q * s->n;
  hipStream_t st = static_cast<hipStream_t>(stream);
  dim3 grid(cdiv(g.m, al.tm * 32), cdiv(s->k, al.wn * al.tn * 32), 1);
  // in-launch merge only when the last arriver's per-thread read is short (tiles / thread groups);
  // otherwise the parallel tspm_bn_finalize pass follows
  const int tiles = (int)grid.x, groups = 2 * al.wk / al.tn;
  const tspm_bn_fuse want = bf;
  if (bf.counters && (cdiv(tiles, groups) > kMaxFusedMergeIters || !inlaunch_enabled())) bf.counters = nullptr;
  size_t lds = lds_bytes(al);
  if (bf.counters) lds = std::max(lds, (size_t)16 + 8 * (size_t)(64 * al.wn * al.wk + 32 * al.wn * al.tn));
  const bool vec = is_hwnc(s, xs) && (s->c % 8 == 0);
  if (vec) TSPM_DISPATCH(k_conv_fwd_vec, false, g, x, w, y, bf);
  else TSPM_DISPATCH(k_conv_fwd_gather, false, g, x, w, y, bf);
  TSPM_LAUNCH_CHECK();
  if (want.counters && !bf.counters)
    return tspm_bn_finalize(g.m, s->k, tiles, al.tm * 32, want.partial, want.running_mean, want.running_var,
                            want.momentum, want.eps, want.save_mean, want.save_invstd, stream);
  return TSPM_OK;
}

namespace {
int bnf_ok(const tspm_bn_fuse* bn) {
  if (!bn) return 1;
  if (!bn->partial && bn->counters) return 0;
  if (bn->counters && (!bn->save_mean || !bn->save_invstd)) return 0;
  return 1;
}
}  // namespace

extern "C" int32_t tspm_conv_fwd_pair_supported(const tspm_conv_shape* s1, const tspm_conv_algo* a1,
                                                const tspm_strides4* xs1, const tspm_conv_shape* s2,
                                                const tspm_conv_algo* a2, const tspm_strides4* xs2) {
  if (!shape_ok(s1) || !shape_ok(s2) || !is_lds(a1) || !is_lds(a2) || a1->variant != a2->variant) return 0;
  if (a1->tm != a2->tm || a1->tn != a2->tn || a1->wn != a2->wn || a1->wk != a2->wk) return 0;
  const tspm_detail::LdsImpl& v = lds_of(a1);
  return (v.fwd_supported(s1, xs1, lds_algo(a1)) && v.fwd_supported(s2, xs2, lds_algo(a2))) ? 1 : 0;
}

extern "C" int tspm_conv_fwd_pair(const tspm_conv_shape* s1, const tspm_conv_algo* a1, const float* x1,
                                  const tspm_strides4* xs1, const float* w1, float* y1, const tspm_bn_fuse* bn1,
                                  void* ws1, size_t ws1_bytes, const tspm_conv_shape* s2, const tspm_conv_algo* a2,
                                  const float* x2, const tspm_strides4* xs2, const float* w2, float* y2,
                                  const tspm_bn_fuse* bn2, void* ws2, size_t ws2_bytes, tspm_stream_t stream) {
  if (!x1 || !w1 || !y1 || !x2 || !w2 || !y2 || !opts_ok(a1) || !opts_ok(a2) || !bnf_ok(bn1) || !bnf_ok(bn2))
    return TSPM_ERR_INVALID;
  if (!tspm_conv_fwd_pair_supported(s1, a1, xs1, s2, a2, xs2)) return TSPM_ERR_INVALID;
  return lds_of(a1).fwd_pair(s1, lds_algo(a1), x1, w1, y1, bn1, ws1, ws1_bytes, s2, lds_algo(a2), x2, w2, y2, bn2, ws2,
                             ws2_bytes, static_cast<hipStream_t>(stream));
}

extern "C" size_t tspm_conv_dgrad_workspace(const tspm_conv_shape* s, const tspm_conv_algo* user) {
  if (!shape_ok(s) || !is_lds(user)) return 0;
  return lds_of(user).dgrad_workspace(s, lds_algo(user));
}

extern "C" int tspm_conv_dgrad(const tspm_conv_shape* s, const tspm_conv_algo* user, const float* dy,
                               const float* w, float* dx, int32_t beta, void* ws, size_t ws_bytes,
                               tspm_stream_t stream) {
  if (!shape_ok(s) || !dy || !w || !dx || !opts_ok(user)) return TSPM_ERR_INVALID;
  if (is_lds(user)) {
    const tspm_detail::LdsAlgo la = lds_algo(user);
    if (!lds_of(user).dgrad_supported(s, la)) return TSPM_ERR_INVALID;
    return lds_of(user).dgrad(s, la, dy, w, dx, beta, ws, ws_bytes, static_cast<hipStream_t>(stream));
  }
  (void)ws; (void)ws_bytes;
  if (s->k % 8 != 0) return TSPM_ERR_INVALID;
  Algo al = dgrad_algo(s, user);
  if (!algo_supported(al)) return TSPM_ERR_INVALID;
  ConvArgs g = make_args(s);
  g.m = s->h * s->w * s->n;
  g.beta = beta ? 1 : 0;
  hipStream_t st = static_cast<hipStream_t>(stream);
  dim3 grid(cdiv(g.m, al.tm * 32), cdiv(s->c, al.wn * al.tn * 32), 1);
  const size_t lds = lds_bytes(al);
  TSPM_DISPATCH(k_conv_dgrad, false, g, dy, w, dx);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" size_t tspm_conv_wgrad_workspace(const tspm_conv_shape* s, const tspm_conv_algo* user) {
  if (!shape_ok(s)) return 0;
  if (is_lds(user)) return lds_of(user).wgrad_workspace(s, lds_algo(user));
  if (is_stem(user)) return tspm_detail::stem_wgrad_supported(s) ? tspm_detail::stem_wgrad_workspace(s) : 0;
  Algo al = wgrad_algo(s, user);
  if (al.splits <= 1) return 0;
  return TSPM_COUNTER_BYTES + (size_t)al.splits * s->k * s->r * s->s * s->c * sizeof(float);
}

extern "C" int tspm_conv_wgrad(const tspm_conv_shape* s, const tspm_conv_algo* user, const float* x,
                               const tspm_strides4* xs, const float* dy, float* dw, void* ws, size_t ws_bytes,
                               tspm_stream_t stream) {
  if (!shape_ok(s) || !x || !dy || !dw || !opts_ok(user)) return TSPM_ERR_INVALID;
  if (is_lds(user)) {
    const tspm_detail::LdsAlgo la = lds_algo(user);
    if (!lds_of(user).wgrad_supported(s, xs, la)) return TSPM_ERR_INVALID;
    return lds_of(user).wgrad(s, la, x, dy, dw, ws, ws_bytes, static_cast<hipStream_t>(stream));
  }
  if (is_stem(user)) {
    if (!tspm_detail::stem_wgrad_supported(s)) return TSPM_ERR_INVALID;
    return tspm_detail::stem_wgrad(s, x, xs, dy, dw, ws, ws_bytes, static_cast<hipStream_t>(stream));
  }
  Algo al = wgrad_algo(s, user);
  if (!algo_supported(al)) return TSPM_ERR_INVALID;
  ConvArgs g = make_args(s);
  if (xs) { g.sn = xs->sn; g.sh = xs->sh; g.sw = xs->sw; g.sc = xs->sc; }
  const int RSC = s->r * s->s * s->c;
  g.m = s->k;
  g.splits = al.splits;
  g.slab = (long long)s->k * RSC;
  hipStream_t st = static_cast<hipStream_t>(stream);
  float* out = dw;
  dim3 grid(cdiv(s->k, al.tm * 32), cdiv(RSC, al.wn * al.tn * 32), al.splits);
  if (al.splits > 1) {
    if (!ws || ws_bytes < tspm_conv_wgrad_workspace(s, user)) return TSPM_ERR_WORKSPACE;
    out = reinterpret_cast<float*>(static_cast<char*>(ws) + TSPM_COUNTER_BYTES);
    // in-launch reduction when the last arriver's serial read is short; else a separate pass
    if (al.splits <= kMaxFusedSplits && (size_t)grid.x * grid.y <= TSPM_COUNTER_BYTES / sizeof(unsigned) &&
        inlaunch_enabled())
      g.cnt = static_cast<unsigned*>(ws);
  }
  const size_t lds = std::max(lds_bytes(al), (size_t)16);
  if (s->n % 8 == 0) TSPM_DISPATCH(k_conv_wgrad, true, g, x, dy, out, dw);
  else TSPM_DISPATCH(k_conv_wgrad, false, g, x, dy, out, dw);
  TSPM_LAUNCH_CHECK();
  if (al.splits > 1 && !g.cnt) {  // separate slab reduction
    launch_reduce_slabs(g.slab, al.splits, g.slab, static_cast<const float*>(out), dw, 0, st);
    TSPM_LAUNCH_CHECK();
  }
  return TSPM_OK;
}

extern "C" int32_t tspm_conv_bwd_supported(const tspm_conv_shape* s, const tspm_conv_algo* dg,
                                          const tspm_conv_algo* wg, const tspm_strides4* xs) {
  if (!shape_ok(s) || !is_lds(dg) || !is_lds(wg) || dg->variant != wg->variant) return 0;
  const tspm_detail::LdsAlgo ad = lds_algo(dg), aw = lds_algo(wg);
  const tspm_detail::LdsImpl& v = lds_of(dg);
  return (v.dgrad_supported(s, ad) && v.wgrad_supported(s, xs, aw) && v.bwd_built(ad, aw)) ? 1 : 0;
}

extern "C" int tspm_conv_bwd(const tspm_conv_shape* s, const tspm_conv_algo* dg, const tspm_conv_algo* wg,
                             const float* x, const tspm_strides4* xs, const float* dy, const float* w, float* dx,
                             int32_t beta, float* dw, void* ws_d, size_t ws_d_bytes, void* ws_w, size_t ws_w_bytes,
                             tspm_stream_t stream) {
  if (!shape_ok(s) || !x || !dy || !w || !dx || !dw || !opts_ok(dg) || !opts_ok(wg)) return TSPM_ERR_INVALID;
  if (!tspm_conv_bwd_supported(s, dg, wg, xs)) return TSPM_ERR_INVALID;
  return lds_of(dg).bwd(s, lds_algo(dg), lds_algo(wg), x, dy, w, dx, beta, dw, nullptr, nullptr, ws_d, ws_d_bytes, ws_w,
                        ws_w_bytes, static_cast<hipStream_t>(stream));
}

extern "C" int tspm_conv_bwd_adam(const tspm_conv_shape* s, const tspm_conv_algo* dg, const tspm_conv_algo* wg,
                                  const float* x, const tspm_strides4* xs, const float* dy, const float* w, float* dx,
                                  int32_t beta, float* dw, const tspm_adam_job* job, void* ws_d, size_t ws_d_bytes,
                                  void* ws_w, size_t ws_w_bytes, tspm_stream_t stream) {
  if (!shape_ok(s) || !x || !dy || !w || !dx || !dw || !job || !opts_ok(dg) || !opts_ok(wg)) return TSPM_ERR_INVALID;
  if (job->count < 0 || job->blocks < 0 || (job->count > 0 && (!job->param || !job->grad || !job->exp_avg ||
                                                               !job->exp_avg_sq || !job->hyper || job->blocks < 1)))
    return TSPM_ERR_INVALID;
  if (!tspm_conv_bwd_supported(s, dg, wg, xs)) return TSPM_ERR_INVALID;
  return lds_of(dg).bwd(s, lds_algo(dg), lds_algo(wg), x, dy, w, dx, beta, dw, job->count > 0 ? job : nullptr, nullptr,
                        ws_d, ws_d_bytes, ws_w, ws_w_bytes, static_cast<hipStream_t>(stream));
}

extern "C" int tspm_conv_bwd_ex(const tspm_conv_shape* s, const tspm_conv_algo* dg, const tspm_conv_algo* wg,
                                const float* x, const tspm_strides4* xs, const float* dy, const float* w, float* dx,
                                int32_t beta, float* dw, const tspm_adam_job* job, const tspm_bn_bwd_part* bnp,
                                void* ws_d, size_t ws_d_bytes, void* ws_w, size_t ws_w_bytes, tspm_stream_t stream) {
  if (!shape_ok(s) || !x || !dy || !w || !dx || !dw || !opts_ok(dg) || !opts_ok(wg)) return TSPM_ERR_INVALID;
  if (job && (job->count < 0 || job->blocks < 0 ||
              (job->count > 0 && (!job->param || !job->grad || !job->exp_avg || !job->exp_avg_sq || !job->hyper ||
                                  job->blocks < 1))))
    return TSPM_ERR_INVALID;
  if (bnp && (!bnp->out || !bnp->y || !bnp->mean || !bnp->part || (bnp->y2 && !bnp->mean2) ||
              ((long long)s->h * s->w * s->n) % 32 != 0 || (bnp->dy && (!bnp->counters || bnp->idx))))
    return TSPM_ERR_INVALID;
  if (!tspm_conv_bwd_supported(s, dg, wg, xs)) return TSPM_ERR_INVALID;
  return lds_of(dg).bwd(s, lds_algo(dg), lds_algo(wg), x, dy, w, dx, beta, dw, (job && job->count > 0) ? job : nullptr,
                        bnp, ws_d, ws_d_bytes, ws_w, ws_w_bytes, static_cast<hipStream_t>(stream));
}

extern "C" int32_t tspm_conv_bwd_quad_supported(const tspm_conv_shape* s, const tspm_conv_algo* dg,
                                                const tspm_conv_algo* wg, const tspm_strides4* xs,
                                                const tspm_conv_shape* s2, const tspm_conv_algo* dg2,
                                                const tspm_conv_algo* wg2, const tspm_strides4* xs2) {
  if (!tspm_conv_bwd_supported(s, dg, wg, xs) || !tspm_conv_bwd_supported(s2, dg2, wg2, xs2)) return 0;
  if (dg->variant != dg2->variant) return 0;
  auto same = [](const tspm_conv_algo* a, const tspm_conv_algo* b) {
    return a->tm == b->tm && a->tn == b->tn && a->wn == b->wn && a->wk == b->wk;
  };
  return (same(dg, dg2) && same(wg, wg2)) ? 1 : 0;
}

extern "C" int tspm_conv_bwd_quad(const tspm_conv_shape* s, const tspm_conv_algo* dg, const tspm_conv_algo* wg,
                                  const float* x, const tspm_strides4* xs, const float* dy, const float* w, float* dx,
                                  int32_t beta, float* dw, const tspm_bn_bwd_part* bnp, void* ws_d, size_t ws_d_bytes,
                                  void* ws_w, size_t ws_w_bytes, const tspm_conv_shape* s2, const tspm_conv_algo* dg2,
                                  const tspm_conv_algo* wg2, const float* x2, const tspm_strides4* xs2,
                                  const float* dy2, const float* w2, float* dx2, float* dw2, void* ws_d2,
                                  size_t ws_d2_bytes, void* ws_w2, size_t ws_w2_bytes, const tspm_adam_job* job,
                                  tspm_stream_t stream) {
  if (!shape_ok(s) || !x || !dy || !w || !dx || !dw || !opts_ok(dg) || !opts_ok(wg)) return TSPM_ERR_INVALID;
  if (!shape_ok(s2) || !x2 || !dy2 || !w2 || !dx2 || !dw2 || !opts_ok(dg2) || !opts_ok(wg2)) return TSPM_ERR_INVALID;
  if (job && (job->count < 0 || job->blocks < 0 ||
              (job->count > 0 && (!job->param || !job->grad || !job->exp_avg || !job->exp_avg_sq || !job->hyper ||
                                  job->blocks < 1))))
    return TSPM_ERR_INVALID;
  if (!tspm_conv_bwd_quad_supported(s, dg, wg, xs, s2, dg2, wg2, xs2)) return TSPM_ERR_INVALID;
  return lds_of(dg).bwd_quad(s, lds_algo(dg), lds_algo(wg), x, dy, w, dx, beta, dw, bnp, ws_d, ws_d_bytes, ws_w,
                             ws_w_bytes, s2, lds_algo(dg2), lds_algo(wg2), x2, dy2, w2, dx2, dw2, ws_d2, ws_d2_bytes,
                             ws_w2, ws_w2_bytes, (job && job->count > 0) ? job : nullptr,
                             static_cast<hipStream_t>(stream));
}

extern "C" int tspm_reduce_slabs(int64_t count, int32_t nslab, int64_t slab_stride, const float* slabs,
                                 float* out, tspm_stream_t stream) {
  if (count < 0 || nslab < 1 || !slabs || !out) return TSPM_ERR_INVALID;
  if (count == 0) return TSPM_OK;
  if ((reinterpret_cast<uintptr_t>(slabs) | reinterpret_cast<uintptr_t>(out)) & 15) return TSPM_ERR_INVALID;
  if (nslab > 1 && (slab_stride & 3)) return TSPM_ERR_INVALID;
  launch_reduce_slabs(count, nslab, slab_stride, slabs, out, 0, static_cast<hipStream_t>(stream));
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}
