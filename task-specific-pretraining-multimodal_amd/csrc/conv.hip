// Implicit-GEMM convolution on v_mfma_f32_32x32x2_f32 (exact fp32, gfx950).
//
// Replaces nn.Conv2d fwd / dgrad / wgrad of MML_Suite/models/msa/networks/resnet.py:25,30,137,176.
//
// Operand delivery (no LDS): with the 32x32x2 f32 MFMA a lane supplies ONE A element (row l&31,
// k = l>>5) and ONE B element (k = l>>5, col l&31) per instruction.  Each lane loads 4 consecutive
// reduction elements as one 16-byte load and feeds them to 4 consecutive MFMAs: half h = lane>>5
// covers reduction indices c0+4h..c0+4h+3, so MFMA j reduces over {c0+j, c0+4+j}.  Any fixed
// permutation of the reduction order is a valid GEMM, so A and B only have to agree on it.
//   fwd   : A = x rows (HWNC, C contiguous) 16 B/lane; B = w[co][tap][c] (OHWI) 16 B/lane.
//   dgrad : A = dy rows (K contiguous) 16 B/lane; B = w[co][tap][ci] read as 4 coalesced dwords.
//   wgrad : A = dy[m][co], B = x[in(m,tap)][ci] as coalesced dwords (reduction over rows m).
// Waves whose 32*TM rows share one output position (batch % (32*TM) == 0 with the HWNC row order)
// know the valid (non-padding) taps uniformly and skip the rest; other waves mask per lane.
// Split-K writes fp32 slabs that the consumer (BN stats or tspm_reduce_slabs) sums in slab order.
#include "common.h"

namespace {

struct ConvArgs {
  int n, h, w, c, k, r, s, st, pad, p, q;
  long long sn, sh, sw, sc;  // input strides (fwd / wgrad)
  int m;                     // GEMM rows: fwd P*Q*N, dgrad H*W*N, wgrad K
  int splits;
  long long slab;            // elements per split slab
  int beta;                  // dgrad accumulate
};

template <int TM, int TN>
struct Acc {
  f32x16 v[TM][TN];
  TSPM_DEV void zero() {
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int i = 0; i < 16; ++i) v[a][b][i] = 0.f;
  }
  TSPM_DEV void mma4(const f32x4 (&A)[TM], const f32x4 (&B)[TN]) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) v[a][b] = mfma32(A[a][j], B[b][j], v[a][b]);
  }
  // store rows row0 + a*32 + acc_row, cols col0 + b*32 + (lane&31) of a [rows, ld] matrix
  TSPM_DEV void store(float* out, int row0, int col0, int rows, int cols, long long ld, int lane, bool accumulate) const {
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int col = col0 + b * 32 + (lane & 31);
        if (col >= cols) continue;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int row = row0 + a * 32 + acc_row(i, lane);
          if (row < rows) {
            float* p = out + (long long)row * ld + col;
            *p = accumulate ? (*p + v[a][b][i]) : v[a][b][i];
          }
        }
      }
  }
};

TSPM_DEV int split_lo(int T, int z, int S) { return (int)(((long long)T * z) / S); }

// =============================================================================================
// Forward, vector path: HWNC input, C % 8 == 0.
// =============================================================================================
template <int TM, int TN, int WM, int WN>
__global__ __launch_bounds__(256) void k_conv_fwd_vec(ConvArgs g, const float* __restrict__ x,
                                                      const float* __restrict__ w, float* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int row0 = (blockIdx.x * WM + wave % WM) * (TM * 32);
  const int col0 = (blockIdx.y * WN + wave / WM) * (TN * 32);
  if (row0 >= g.m || col0 >= g.k) return;
  const int z = blockIdx.z;
  const int li = lane & 31, hh = lane >> 5;
  const int C = g.c, N = g.n, RSC = g.r * g.s * C;
  const int cch = C >> 3;

  // per-lane rows (clamped for loads)
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

  Acc<TM, TN> acc;
  acc.zero();

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
    const int it0 = split_lo(T, z, g.splits), it1 = split_lo(T, z + 1, g.splits);
    if (it0 < it1) {
      int tap = it0 / cch, ci = (it0 - tap * cch) * 8;
      int r = r_lo + tap / ns, s = s_lo + tap % ns;
      const float* xa[TM];
#pragma unroll
      for (int a = 0; a < TM; ++a) xa[a] = x + (long long)nb[a] * C + 4 * hh;
      auto a_off = [&](int rr, int ss, int cc) -> long long {
        return ((long long)(h0 + rr) * g.w + (w0 + ss)) * N * C + cc;
      };
      auto b_off = [&](int rr, int ss, int cc) -> int { return (rr * g.s + ss) * C + cc; };
      f32x4 A[TM], B[TN];
      {
        long long ao = a_off(r, s, ci);
        int bo = b_off(r, s, ci);
#pragma unroll
        for (int a = 0; a < TM; ++a) A[a] = ld4(xa[a] + ao);
#pragma unroll
        for (int b = 0; b < TN; ++b) B[b] = ld4(wrow[b] + bo);
      }
      for (int it = it0; it < it1; ++it) {
        // advance (ci, s, r) to the next iteration (clamped re-load of the last one at the end)
        int ci2 = ci + 8, s2 = s, r2 = r;
        if (ci2 == C) { ci2 = 0; ++s2; if (s2 > s_hi) { s2 = s_lo; ++r2; } }
        const bool more = it + 1 < it1;
        const int rl = more ? r2 : r, sl = more ? s2 : s, cl = more ? ci2 : ci;
        f32x4 An[TM], Bn[TN];
        long long ao = a_off(rl, sl, cl);
        int bo = b_off(rl, sl, cl);
#pragma unroll
        for (int a = 0; a < TM; ++a) An[a] = ld4(xa[a] + ao);
#pragma unroll
        for (int b = 0; b < TN; ++b) Bn[b] = ld4(wrow[b] + bo);
        acc.mma4(A, B);
#pragma unroll
        for (int a = 0; a < TM; ++a) A[a] = An[a];
#pragma unroll
        for (int b = 0; b < TN; ++b) B[b] = Bn[b];
        ci = ci2; s = s2; r = r2;
      }
    }
  } else {
    // ---- mixed positions: all taps, per-lane padding masks ----
    const int T = g.r * g.s * cch;
    const int it0 = split_lo(T, z, g.splits), it1 = split_lo(T, z + 1, g.splits);
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
  float* out = g.splits > 1 ? y + (long long)z * g.slab : y;
  acc.store(out, row0, col0, g.m, g.k, g.k, lane, false);
}

// =============================================================================================
// Forward, gather path: arbitrary input strides / any C (the Cin=1 7x7 stem reads the reference's
// NCHW input directly).  Reduction index kidx = (r*S + s)*C + c, chunks of 8, scalar loads.
// =============================================================================================
template <int TM, int TN, int WM, int WN>
__global__ __launch_bounds__(256) void k_conv_fwd_gather(ConvArgs g, const float* __restrict__ x,
                                                         const float* __restrict__ w, float* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int row0 = (blockIdx.x * WM + wave % WM) * (TM * 32);
  const int col0 = (blockIdx.y * WN + wave / WM) * (TN * 32);
  if (row0 >= g.m || col0 >= g.k) return;
  const int z = blockIdx.z;
  const int li = lane & 31, hh = lane >> 5;
  const int C = g.c, N = g.n, RSC = g.r * g.s * C;

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

  Acc<TM, TN> acc;
  acc.zero();
  const int T = cdiv_dev(RSC, 8);
  const int it0 = split_lo(T, z, g.splits), it1 = split_lo(T, z + 1, g.splits);
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
  float* out = g.splits > 1 ? y + (long long)z * g.slab : y;
  acc.store(out, row0, col0, g.m, g.k, g.k, lane, false);
}

// =============================================================================================
// Data gradient: dx[h,w,n,ci] = sum_{r,s,co} dy[(h+pad-r)/st, (w+pad-s)/st, n, co] * w[co,r,s,ci]
// GEMM rows m = (h,w,n) of the input, cols = ci, reduction over (valid tap, co) in chunks of 8 co.
// =============================================================================================
template <int TM, int TN, int WM, int WN>
__global__ __launch_bounds__(256) void k_conv_dgrad(ConvArgs g, const float* __restrict__ dy,
                                                    const float* __restrict__ w, float* __restrict__ dx) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int row0 = (blockIdx.x * WM + wave % WM) * (TM * 32);
  const int col0 = (blockIdx.y * WN + wave / WM) * (TN * 32);
  if (row0 >= g.m || col0 >= g.c) return;
  const int z = blockIdx.z;
  const int li = lane & 31, hh = lane >> 5;
  const int C = g.c, N = g.n, K = g.k, RSC = g.r * g.s * C;
  const int kch = K >> 3;

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

  Acc<TM, TN> acc;
  acc.zero();
  const int pos_first = row0 / N;
  const int pos_last = (min(row0 + TM * 32, g.m) - 1) / N;
  if (pos_first == pos_last) {
    const int hi = pos_first / g.w, wi = pos_first - hi * g.w;
    // valid r: (hi+pad-r) % st == 0 and 0 <= (hi+pad-r)/st < P  (bitmasks, R,S <= 31)
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
    const int it0 = split_lo(T, z, g.splits), it1 = split_lo(T, z + 1, g.splits);
    const float* dya[TM];
#pragma unroll
    for (int a = 0; a < TM; ++a) dya[a] = dy + (long long)nb[a] * K + 4 * hh;
    for (int it = it0; it < it1; ++it) {
      const int t = it / kch, c0 = (it - t * kch) * 8;
      const int ri = t / ns, si = t - ri * ns;
      // ri-th / si-th set bits
      unsigned rm = rmask, sm = smask;
      for (int i = 0; i < ri; ++i) rm &= rm - 1;
      for (int i = 0; i < si; ++i) sm &= sm - 1;
      const int r = __builtin_ctz(rm), s = __builtin_ctz(sm);
      const int pp = (hi + g.pad - r) / g.st, qq = (wi + g.pad - s) / g.st;
      const long long aoff = ((long long)pp * g.q + qq) * N * K + c0;
      f32x4 A[TM], B[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) A[a] = ld4(dya[a] + aoff);
      const long long wbase = (long long)(c0 + 4 * hh) * RSC + (r * g.s + s) * C;
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int j = 0; j < 4; ++j) B[b][j] = w[wbase + (long long)j * RSC + ci[b]];
      acc.mma4(A, B);
    }
  } else {
    const int T = g.r * g.s * kch;
    const int it0 = split_lo(T, z, g.splits), it1 = split_lo(T, z + 1, g.splits);
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
  if (g.splits > 1) {
    acc.store(dx + (long long)z * g.slab, row0, col0, g.m, C, C, lane, false);
  } else {
    acc.store(dx, row0, col0, g.m, C, C, lane, g.beta != 0);
  }
}

// =============================================================================================
// Weight gradient: dw[co, (r,s,c)] = sum_m dy[m, co] * x[in(m, r, s), c]
// GEMM rows = co (K), cols = kidx = (r*S+s)*C + c, reduction over output rows m in chunks of 8.
// FAST: N % 8 == 0 so an 8-row chunk shares one output position (uniform decomposition).
// =============================================================================================
template <int TM, int TN, int WM, int WN, bool FAST>
__global__ __launch_bounds__(256) void k_conv_wgrad(ConvArgs g, const float* __restrict__ x,
                                                    const float* __restrict__ dy, float* __restrict__ dw) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int K = g.k, C = g.c, N = g.n;
  const int RSC = g.r * g.s * C;
  const int row0 = (blockIdx.x * WM + wave % WM) * (TM * 32);   // co
  const int col0 = (blockIdx.y * WN + wave / WM) * (TN * 32);   // kidx
  if (row0 >= K || col0 >= RSC) return;
  const int z = blockIdx.z;
  const int li = lane & 31, hh = lane >> 5;
  const int Mout = g.p * g.q * N;

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
  // single-tap column tile: all lanes share (r, s) -> whole chunks can be skipped when padded
  const int tap_first = col0 / C, tap_last = (min(col0 + TN * 32, RSC) - 1) / C;
  const bool one_tap = tap_first == tap_last;

  Acc<TM, TN> acc;
  acc.zero();
  const int T = cdiv_dev(Mout, 8);
  const int it0 = split_lo(T, z, g.splits), it1 = split_lo(T, z + 1, g.splits);
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
  float* out = g.splits > 1 ? dw + (long long)z * g.slab : dw;
  acc.store(out, row0, col0, K, RSC, RSC, lane, false);
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
  // tail
  if (blockIdx.x == 0 && threadIdx.x < (count & 3)) {
    long long i = (n4 << 2) + threadIdx.x;
    float s = beta ? out[i] : 0.f;
    for (int z = 0; z < nslab; ++z) s += slabs[z * slab_stride + i];
    out[i] = s;
  }
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
  int tm, tn, wm, wn, splits;
};

int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// heuristic: aim for >= ~1024 waves in flight (4 per SIMD-quad of the 256 CUs) with >= 8
// reduction iterations per split
Algo pick(const tspm_conv_algo* user, long long rows, long long cols, long long red_iters) {
  Algo a{1, cols >= 64 ? 2 : 1, 0, 0, 1};
  if (user && user->tm > 0) {
    a.tm = user->tm; a.tn = user->tn; a.wm = user->wm; a.wn = user->wn; a.splits = user->splits > 0 ? user->splits : 1;
  } else {
    if (rows >= 8192 && cols >= 64) a.tm = 2;
    long long waves = cdiv64(rows, 32 * a.tm) * cdiv64(cols, 32 * a.tn);
    int sp = (int)cdiv64(1024, waves);
    int maxsp = (int)(red_iters / 8);
    a.splits = clampi(sp, 1, maxsp < 1 ? 1 : maxsp);
    if (a.splits > 64) a.splits = 64;
    if (user && user->splits > 0) a.splits = user->splits;
  }
  if (a.wm <= 0 || a.wn <= 0) {
    long long wn_need = cdiv64(cols, 32 * a.tn);
    a.wn = wn_need >= 4 ? 4 : (wn_need >= 2 ? 2 : 1);
    a.wm = 4 / a.wn;
  }
  return a;
}

bool algo_supported(const Algo& a) {
  if (a.wm * a.wn != 4 || a.splits < 1) return false;
  return (a.tm == 1 || a.tm == 2) && (a.tn == 1 || a.tn == 2);
}

#define TSPM_DISPATCH_TILES(KERNEL, TEMPLATE_EXTRA, ...)                                            \
  do {                                                                                              \
    const Algo& A_ = al;                                                                            \
    if (A_.tm == 1 && A_.tn == 1) {                                                                 \
      if (A_.wm == 4) hipLaunchKernelGGL((KERNEL<1, 1, 4, 1 TEMPLATE_EXTRA>), grid, dim3(256), 0, st, __VA_ARGS__); \
      else if (A_.wm == 2) hipLaunchKernelGGL((KERNEL<1, 1, 2, 2 TEMPLATE_EXTRA>), grid, dim3(256), 0, st, __VA_ARGS__); \
      else hipLaunchKernelGGL((KERNEL<1, 1, 1, 4 TEMPLATE_EXTRA>), grid, dim3(256), 0, st, __VA_ARGS__); \
    } else if (A_.tm == 1 && A_.tn == 2) {                                                          \
      if (A_.wm == 4) hipLaunchKernelGGL((KERNEL<1, 2, 4, 1 TEMPLATE_EXTRA>), grid, dim3(256), 0, st, __VA_ARGS__); \
      else if (A_.wm == 2) hipLaunchKernelGGL((KERNEL<1, 2, 2, 2 TEMPLATE_EXTRA>), grid, dim3(256), 0, st, __VA_ARGS__); \
      else hipLaunchKernelGGL((KERNEL<1, 2, 1, 4 TEMPLATE_EXTRA>), grid, dim3(256), 0, st, __VA_ARGS__); \
    } else if (A_.tm == 2 && A_.tn == 1) {                                                          \
      if (A_.wm == 4) hipLaunchKernelGGL((KERNEL<2, 1, 4, 1 TEMPLATE_EXTRA>), grid, dim3(256), 0, st, __VA_ARGS__); \
      else if (A_.wm == 2) hipLaunchKernelGGL((KERNEL<2, 1, 2, 2 TEMPLATE_EXTRA>), grid, dim3(256), 0, st, __VA_ARGS__); \
      else hipLaunchKernelGGL((KERNEL<2, 1, 1, 4 TEMPLATE_EXTRA>), grid, dim3(256), 0, st, __VA_ARGS__); \
    } else {                                                                                        \
      if (A_.wm == 4) hipLaunchKernelGGL((KERNEL<2, 2, 4, 1 TEMPLATE_EXTRA>), grid, dim3(256), 0, st, __VA_ARGS__); \
      else if (A_.wm == 2) hipLaunchKernelGGL((KERNEL<2, 2, 2, 2 TEMPLATE_EXTRA>), grid, dim3(256), 0, st, __VA_ARGS__); \
      else hipLaunchKernelGGL((KERNEL<2, 2, 1, 4 TEMPLATE_EXTRA>), grid, dim3(256), 0, st, __VA_ARGS__); \
    }                                                                                               \
  } while (0)

#define TSPM_NOEXTRA
#define TSPM_FAST_T , true
#define TSPM_FAST_F , false

ConvArgs make_args(const tspm_conv_shape* s) {
  ConvArgs g;
  g.n = s->n; g.h = s->h; g.w = s->w; g.c = s->c; g.k = s->k; g.r = s->r; g.s = s->s;
  g.st = s->stride; g.pad = s->pad; g.p = s->p; g.q = s->q;
  g.sn = (long long)s->c; g.sh = (long long)s->w * s->n * s->c; g.sw = (long long)s->n * s->c; g.sc = 1;
  g.m = 0; g.splits = 1; g.slab = 0; g.beta = 0;
  return g;
}

bool is_hwnc(const tspm_conv_shape* s, const tspm_strides4* st) {
  if (!st) return true;
  return st->sc == 1 && st->sn == s->c && st->sw == (long long)s->n * s->c && st->sh == (long long)s->w * s->n * s->c;
}

Algo fwd_algo(const tspm_conv_shape* s, const tspm_conv_algo* user) {
  long long rows = (long long)s->p * s->q * s->n;
  long long iters = (long long)s->r * s->s * cdiv(s->c, 8);
  return pick(user, rows, s->k, iters);
}
Algo dgrad_algo(const tspm_conv_shape* s, const tspm_conv_algo* user) {
  long long rows = (long long)s->h * s->w * s->n;
  long long iters = (long long)s->r * s->s * (s->k / 8);
  return pick(user, rows, s->c, iters);
}
Algo wgrad_algo(const tspm_conv_shape* s, const tspm_conv_algo* user) {
  long long cols = (long long)s->r * s->s * s->c;
  long long iters = cdiv64((long long)s->p * s->q * s->n, 8);
  return pick(user, s->k, cols, iters);
}

}  // namespace

// ---------------------------------------------------------------------------------------------
extern "C" size_t tspm_conv_fwd_workspace(const tspm_conv_shape* s, const tspm_conv_algo* user) {
  if (!shape_ok(s)) return 0;
  Algo al = fwd_algo(s, user);
  if (al.splits <= 1) return 0;
  return (size_t)al.splits * s->p * s->q * s->n * s->k * sizeof(float);
}

extern "C" int tspm_conv_fwd(const tspm_conv_shape* s, const tspm_conv_algo* user, const float* x,
                             const tspm_strides4* xs, const float* w, float* y, void* ws, size_t ws_bytes,
                             tspm_stream_t stream) {
  if (!shape_ok(s) || !x || !w || !y) return TSPM_ERR_INVALID;
  Algo al = fwd_algo(s, user);
  if (!algo_supported(al)) return TSPM_ERR_INVALID;
  ConvArgs g = make_args(s);
  if (xs) { g.sn = xs->sn; g.sh = xs->sh; g.sw = xs->sw; g.sc = xs->sc; }
  g.m = s->p * s->q * s->n;
  g.splits = al.splits;
  g.slab = (long long)g.m * s->k;
  float* out = y;
  if (al.splits > 1) {
    if (!ws || ws_bytes < tspm_conv_fwd_workspace(s, user)) return TSPM_ERR_WORKSPACE;
    out = static_cast<float*>(ws);
  }
  hipStream_t st = static_cast<hipStream_t>(stream);
  dim3 grid(cdiv(g.m, al.wm * al.tm * 32), cdiv(s->k, al.wn * al.tn * 32), al.splits);
  const bool vec = is_hwnc(s, xs) && (s->c % 8 == 0);
  if (vec) TSPM_DISPATCH_TILES(k_conv_fwd_vec, TSPM_NOEXTRA, g, x, w, out);
  else TSPM_DISPATCH_TILES(k_conv_fwd_gather, TSPM_NOEXTRA, g, x, w, out);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" size_t tspm_conv_dgrad_workspace(const tspm_conv_shape* s, const tspm_conv_algo* user) {
  if (!shape_ok(s)) return 0;
  Algo al = dgrad_algo(s, user);
  if (al.splits <= 1) return 0;
  return (size_t)al.splits * s->h * s->w * s->n * s->c * sizeof(float);
}

extern "C" int tspm_conv_dgrad(const tspm_conv_shape* s, const tspm_conv_algo* user, const float* dy,
                               const float* w, float* dx, int32_t beta, void* ws, size_t ws_bytes,
                               tspm_stream_t stream) {
  if (!shape_ok(s) || !dy || !w || !dx) return TSPM_ERR_INVALID;
  if (s->k % 8 != 0) return TSPM_ERR_INVALID;
  Algo al = dgrad_algo(s, user);
  if (!algo_supported(al)) return TSPM_ERR_INVALID;
  ConvArgs g = make_args(s);
  g.m = s->h * s->w * s->n;
  g.splits = al.splits;
  g.slab = (long long)g.m * s->c;
  g.beta = beta ? 1 : 0;
  hipStream_t st = static_cast<hipStream_t>(stream);
  float* out = dx;
  if (al.splits > 1) {
    if (!ws || ws_bytes < tspm_conv_dgrad_workspace(s, user)) return TSPM_ERR_WORKSPACE;
    out = static_cast<float*>(ws);
  }
  dim3 grid(cdiv(g.m, al.wm * al.tm * 32), cdiv(s->c, al.wn * al.tn * 32), al.splits);
  TSPM_DISPATCH_TILES(k_conv_dgrad, TSPM_NOEXTRA, g, dy, w, out);
  TSPM_LAUNCH_CHECK();
  if (al.splits > 1) {
    long long count = (long long)g.m * s->c;
    int blocks = (int)std::min<long long>(cdiv64(count / 4 + 1, 256), 2048);
    hipLaunchKernelGGL(k_reduce_slabs, dim3(blocks), dim3(256), 0, st, count, al.splits, g.slab,
                       static_cast<const float*>(ws), dx, g.beta);
    TSPM_LAUNCH_CHECK();
  }
  return TSPM_OK;
}

extern "C" size_t tspm_conv_wgrad_workspace(const tspm_conv_shape* s, const tspm_conv_algo* user) {
  if (!shape_ok(s)) return 0;
  Algo al = wgrad_algo(s, user);
  if (al.splits <= 1) return 0;
  return (size_t)al.splits * s->k * s->r * s->s * s->c * sizeof(float);
}

extern "C" int tspm_conv_wgrad(const tspm_conv_shape* s, const tspm_conv_algo* user, const float* x,
                               const tspm_strides4* xs, const float* dy, float* dw, void* ws, size_t ws_bytes,
                               tspm_stream_t stream) {
  if (!shape_ok(s) || !x || !dy || !dw) return TSPM_ERR_INVALID;
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
  if (al.splits > 1) {
    if (!ws || ws_bytes < tspm_conv_wgrad_workspace(s, user)) return TSPM_ERR_WORKSPACE;
    out = static_cast<float*>(ws);
  }
  dim3 grid(cdiv(s->k, al.wm * al.tm * 32), cdiv(RSC, al.wn * al.tn * 32), al.splits);
  if (s->n % 8 == 0) TSPM_DISPATCH_TILES(k_conv_wgrad, TSPM_FAST_T, g, x, dy, out);
  else TSPM_DISPATCH_TILES(k_conv_wgrad, TSPM_FAST_F, g, x, dy, out);
  TSPM_LAUNCH_CHECK();
  if (al.splits > 1) {
    long long count = g.slab;
    int blocks = (int)std::min<long long>(cdiv64(count / 4 + 1, 256), 2048);
    hipLaunchKernelGGL(k_reduce_slabs, dim3(blocks), dim3(256), 0, st, count, al.splits, g.slab,
                       static_cast<const float*>(ws), dw, 0);
    TSPM_LAUNCH_CHECK();
  }
  return TSPM_OK;
}

extern "C" int tspm_reduce_slabs(int64_t count, int32_t nslab, int64_t slab_stride, const float* slabs,
                                 float* out, tspm_stream_t stream) {
  if (count < 0 || nslab < 1 || !slabs || !out) return TSPM_ERR_INVALID;
  if (count == 0) return TSPM_OK;
  if ((reinterpret_cast<uintptr_t>(slabs) | reinterpret_cast<uintptr_t>(out)) & 15) return TSPM_ERR_INVALID;
  if (nslab > 1 && (slab_stride & 3)) return TSPM_ERR_INVALID;
  int blocks = (int)std::min<long long>(cdiv64(count / 4 + 1, 256), 2048);
  hipLaunchKernelGGL(k_reduce_slabs, dim3(blocks), dim3(256), 0, static_cast<hipStream_t>(stream),
                     (long long)count, nslab, (long long)slab_stride, slabs, out, 0);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}
