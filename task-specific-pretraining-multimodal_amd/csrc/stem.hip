// The ResNet stems' 7x7 / stride-2 / pad-3 convolution of a one-channel input into 64 channels
// (MML_Suite/models/msa/networks/resnet.py:137, the first op of both encoders; the audio one heads the
// step's critical path) — tspm_conv_algo.variant 3.
//
// The generic gather kernel (conv.hip k_conv_fwd_gather) assigns a 32-row MFMA tile 32 different images
// at one output position (HWNC rows), so every operand load touches 32 scattered lines of the NCHW input.
// Here a workgroup owns one image and a band of PB output rows: it stages the band's (2*PB + 5) input rows
// (zero-padded to W + 6 columns) in LDS with coalesced loads, keeps the 64 x 49 filter in registers (the
// MFMA B operand: lane (column, half) holds 25 taps), and runs the band's PB*Q output rows x 64 channels as
// 32x32 tiles of v_mfma_f32_32x32x2_f32 whose A operand is read from LDS.  The 49 taps are split 25 / 24
// (+ one zero-weight tap) between the two lane halves, the same permutation on both operands.
// The epilogue writes the HWNC output rows and the tile's BatchNorm partial statistics in the format the
// conv epilogues use (conv_common.h Acc::bn_partials: per channel {K, mean - K, M2}; one tile = one band of
// PB*Q rows), merged by tspm_bn_finalize.
#include "conv_common.h"

#ifdef TSPM_STAMPS
// Diagnostic build only: phase stamps of the stem kernels (read back by scripts/stem_bench.py --stamps)
__device__ unsigned long long tspm_g_stamps_stem[TSPM_STAMP_WAVES * TSPM_STAMP_SLOTS];
extern "C" int tspm_debug_stamps_stem(void* host_dst, size_t bytes) {
  if (bytes > sizeof(tspm_g_stamps_stem)) bytes = sizeof(tspm_g_stamps_stem);
  return hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(tspm_g_stamps_stem), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? 0 : 2;
}
extern "C" int tspm_debug_stamps_stem_clear(void) {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(tspm_g_stamps_stem)) != hipSuccess) return 2;
  return hipMemset(p, 0, sizeof(tspm_g_stamps_stem)) == hipSuccess ? 0 : 2;
}
#endif

namespace {

constexpr int STEM_K = 64;     // output channels
constexpr int STEM_TAPS = 49;  // 7 x 7, one input channel
constexpr int STEM_HALF = 25;  // taps per lane half (the second half's last is tap 49: zero weight)
constexpr int STEM_WAVES = 4;
constexpr int STEM_JOBS = 4;   // (row tile, column tile) jobs per wave: <= 8 row tiles (256 rows) per workgroup

struct StemArgs {
  int n, h, w, p, q, pb, nb, R, RT;
  long long sn, sh, sw;
  const float* x;
  const float* wt;
  float* y;
  float* part;
};

TSPM_DEV int stem_tapoff(int t, int LW) { return t < STEM_TAPS ? (t / 7) * LW + (t % 7) : 0; }

// i / d for 0 <= i < 2^22 without an integer division (a 32-bit udiv is ~40 VALU instructions; the row decodes
// in these kernels' epilogues and loops were VALU-bound on them): float reciprocal estimate, corrected by one
// step either way
TSPM_DEV int div_small(int i, int d, float inv) {
  int r = (int)((float)i * inv);
  r -= r * d > i ? 1 : 0;
  r += (r + 1) * d <= i ? 1 : 0;
  return r;
}

__global__ __launch_bounds__(64 * STEM_WAVES) void k_stem_fwd(StemArgs a) {
  extern __shared__ float lds[];
  const int tile = blockIdx.x, n = tile / a.nb, band = tile - n * a.nb, p0 = band * a.pb;
  const int IH = 2 * a.pb + 5, LW = a.w + 6, NE = IH * LW;
  float* sw = lds;                     // [64][49] filter (coalesced staging; lanes read their taps from here)
  float* sx = sw + STEM_K * STEM_TAPS; // [IH][LW] input band, zero padded
  float* sK = sx + ((NE + 3) & ~3);    // [64] shift K of the BN partials (row 0 of the band)
  float* sOff = sK + STEM_K;           // [64] mean - K
  float* sS = sOff + STEM_K;           // [RT][64] per row tile sums
  float* sQ = sS + a.RT * STEM_K;      // [RT][64] per row tile sums of squares
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, li = lane & 31, kh = lane >> 5;
  constexpr int NT = 64 * STEM_WAVES;
  TSPM_STAMP(tspm_g_stamps_stem, 0);
  TSPM_STAMP_CLK(tspm_g_stamps_stem, 6);

  // the filter (12.5 KB, contiguous) and the band's input rows 2*p0-3 .. 2*p0-3+IH-1, columns -3 .. W+2
  // (zeros outside the image); every load of a round is unconditional (clamped addresses), so they are all in
  // flight before the first LDS store.  (Per-lane filter loads straight from global — 32 lines per
  // instruction — cost more than the MFMAs.)
  {
    constexpr int WU = (STEM_K * STEM_TAPS / 4 + NT - 1) / NT;
    f32x4 wv[WU];
#pragma unroll
    for (int u = 0; u < WU; ++u) wv[u] = ld4(a.wt + 4 * min(u * NT + t, STEM_K * STEM_TAPS / 4 - 1));
    const long long xb = (long long)n * a.sn;
    const float inv_lw = 1.0f / (float)LW;
    constexpr int SU = 8;
    for (int e0 = 0; e0 < NE; e0 += SU * NT) {
      float v[SU];
      bool ok[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int e = min(e0 + u * NT + t, NE - 1);
        const int i = div_small(e, LW, inv_lw), j = e - i * LW;
        const int ih = 2 * p0 - 3 + i, iw = j - 3;
        ok[u] = ih >= 0 && ih < a.h && iw >= 0 && iw < a.w;
        v[u] = a.x[xb + (long long)min(max(ih, 0), a.h - 1) * a.sh + (long long)min(max(iw, 0), a.w - 1) * a.sw];
      }
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const int e = e0 + u * NT + t;
        if (e < NE) sx[e] = ok[u] ? v[u] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < WU; ++u)
      if (u * NT + t < STEM_K * STEM_TAPS / 4) st4(sw + 4 * (u * NT + t), wv[u]);
  }
  __syncthreads();
  TSPM_STAMP(tspm_g_stamps_stem, 1);
  // filter registers: lane (column li, half kh) holds w[ct*32 + li][i + 25*kh]
  float wr0[STEM_HALF], wr1[STEM_HALF];
  int toff[STEM_HALF];
#pragma unroll
  for (int i = 0; i < STEM_HALF; ++i) {
    const int tap = i + STEM_HALF * kh, tc = min(tap, STEM_TAPS - 1);
    wr0[i] = tap < STEM_TAPS ? sw[li * STEM_TAPS + tc] : 0.f;
    wr1[i] = tap < STEM_TAPS ? sw[(32 + li) * STEM_TAPS + tc] : 0.f;
    toff[i] = stem_tapoff(tap, LW);
  }

  const float inv_q = 1.0f / (float)a.q;
  // jobs j = wave + 4*jr over (row tile j >> 1, column tile j & 1): every SIMD gets the same MFMA count
  f32x16 acc[STEM_JOBS];
#pragma unroll
  for (int jr = 0; jr < STEM_JOBS; ++jr) {
    acc[jr] = f32x16{};
    const int j = wave + STEM_WAVES * jr;
    if (j < 2 * a.RT) {
      const int rt = j >> 1;
      const bool c1 = (j & 1) != 0;
      const int ml = min(rt * 32 + li, a.R - 1);
      const int pl = div_small(ml, a.q, inv_q), qq = ml - pl * a.q;
      const float* xp = sx + 2 * pl * LW + 2 * qq;
      float av[STEM_HALF];
#pragma unroll
      for (int i = 0; i < STEM_HALF; ++i) av[i] = xp[toff[i]];
#pragma unroll
      for (int i = 0; i < STEM_HALF; ++i) acc[jr] = mfma32(av[i], c1 ? wr1[i] : wr0[i], acc[jr]);
    }
  }

  TSPM_STAMP(tspm_g_stamps_stem, 2);
  // HWNC output rows ((p0 + pl) * Q + q) * N + n
#pragma unroll
  for (int jr = 0; jr < STEM_JOBS; ++jr) {
    const int j = wave + STEM_WAVES * jr;
    if (j >= 2 * a.RT) continue;
    const int rt = j >> 1, ct = j & 1;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ml = rt * 32 + acc_row(r, lane);
      if (ml < a.R) {
        const int pl = div_small(ml, a.q, inv_q), qq = ml - pl * a.q;
        a.y[((long long)((p0 + pl) * a.q + qq) * a.n + n) * STEM_K + ct * 32 + li] = acc[jr][r];
      }
    }
  }
  TSPM_STAMP(tspm_g_stamps_stem, 3);
  if (!a.part) return;

  // BN partials of the band: K = row 0's value, then the shifted two-pass mean / M2 (fixed order over tiles)
  if (wave < 2 && lane < 32) sK[wave * 32 + li] = acc[0][0];  // jobs 0 / 1 = row tile 0, column tiles 0 / 1
  __syncthreads();
#pragma unroll
  for (int jr = 0; jr < STEM_JOBS; ++jr) {
    const int j = wave + STEM_WAVES * jr;
    if (j >= 2 * a.RT) continue;
    const int rt = j >> 1, ct = j & 1;
    const float K = sK[ct * 32 + li];
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (rt * 32 + acc_row(r, lane) < a.R) s += acc[jr][r] - K;
    s += __shfl_xor(s, 32, 64);
    if (lane < 32) sS[rt * STEM_K + ct * 32 + li] = s;
  }
  __syncthreads();
  if (t < STEM_K) {
    float tot = 0.f;
    for (int rt = 0; rt < a.RT; ++rt) tot += sS[rt * STEM_K + t];
    sOff[t] = tot * (1.0f / (float)a.R);
  }
  __syncthreads();
#pragma unroll
  for (int jr = 0; jr < STEM_JOBS; ++jr) {
    const int j = wave + STEM_WAVES * jr;
    if (j >= 2 * a.RT) continue;
    const int rt = j >> 1, ct = j & 1;
    const float K = sK[ct * 32 + li], off = sOff[ct * 32 + li];
    float sd = 0.f, s2 = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (rt * 32 + acc_row(r, lane) < a.R) {
        const float d = (acc[jr][r] - K) - off;
        sd += d;
        s2 += d * d;
      }
    sd += __shfl_xor(sd, 32, 64);
    s2 += __shfl_xor(s2, 32, 64);
    if (lane < 32) {
      sS[rt * STEM_K + ct * 32 + li] = sd;
      sQ[rt * STEM_K + ct * 32 + li] = s2;
    }
  }
  __syncthreads();
  if (t < STEM_K) {
    float sd = 0.f, s2 = 0.f;
    for (int rt = 0; rt < a.RT; ++rt) {
      sd += sS[rt * STEM_K + t];
      s2 += sQ[rt * STEM_K + t];
    }
    const double cnt = (double)a.R;
    const long long plane = (long long)gridDim.x * STEM_K, o = (long long)tile * STEM_K + t;
    a.part[o] = sK[t];
    a.part[plane + o] = (float)((double)sOff[t] + (double)sd / cnt);
    a.part[2 * plane + o] = (float)((double)s2 - (double)sd * (double)sd / cnt);
  }
  TSPM_STAMP(tspm_g_stamps_stem, 4);
  TSPM_STAMP_CLK(tspm_g_stamps_stem, 7);
}

// Weight gradient of the stem: dw[c][tap] = sum over rows (p, q, n) of dy[row][c] * x_patch(row)[tap].  A
// workgroup runs a contiguous run of bands (one image x PB output rows each; at most 256 workgroups, so at
// most 256 partial slabs): per band it stages the input band AND the band's dy rows in LDS (coalesced 16-byte
// loads, all in flight together), then 8 waves = 4 output tiles (2 channel tiles x 2 tap tiles of 32; taps
// >= 49 discarded) x 2 halves of the band's rows run v_mfma_f32_32x32x2_f32 with both operands from LDS
// (A = dy, B = the patch value), accumulating across the workgroup's bands.  The halves combine in LDS in fixed
// order and the 64 x 49 partial goes to the workgroup's slab, summed in slab order by tspm_reduce_slabs.
// (Reading dy from global inside the MMA loop, 8 rows in flight per lane, was slower than the gather kernel:
// a full memory round trip per 8 steps.)
constexpr int STEMW_WAVES = 8;

struct StemWArgs {
  int n, h, w, p, q, pb, nb, R, ldd, bands, bpw;
  long long sn, sh, sw;
  const float* x;
  const float* dy;
  float* slab;
};

__global__ __launch_bounds__(64 * STEMW_WAVES) void k_stem_wgrad(StemWArgs a) {
  extern __shared__ float lds[];
  const int IH = 2 * a.pb + 5, LW = a.w + 6, NE = IH * LW, LDD = a.ldd;
  float* sx = lds;                    // [IH][LW]
  float* sdy = sx + ((NE + 3) & ~3);  // [R][LDD] the band's dy rows; then the second half's accumulators
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, li = lane & 31, kh = lane >> 5;
  const int ot = wave & 3, half = wave >> 2, ct = ot >> 1, tt = ot & 1;
  const int tap = tt * 32 + li;
  const int toffl = stem_tapoff(tap, LW);  // taps >= 49: offset 0 (a finite value; the column is discarded)
  const int S = (a.R + 1) / 2, s0 = half ? S / 2 : 0, s1 = half ? S : S / 2;
  constexpr int NT = 64 * STEMW_WAVES;
  const float inv_lw = 1.0f / (float)LW, inv_q = 1.0f / (float)a.q;
  f32x16 acc = {};
  TSPM_STAMP(tspm_g_stamps_stem, 0);
  TSPM_STAMP_CLK(tspm_g_stamps_stem, 6);
  const int b0 = blockIdx.x * a.bpw, b1 = min(a.bands, b0 + a.bpw);
  for (int bnd = b0; bnd < b1; ++bnd) {
    const int n = bnd / a.nb, p0 = (bnd - n * a.nb) * a.pb;
    __syncthreads();  // the previous band's LDS reads are done
    {
      const long long xb = (long long)n * a.sn;
      constexpr int SU = 4;
      for (int e0 = 0; e0 < NE; e0 += SU * NT) {
        float v[SU];
        bool ok[SU];
#pragma unroll
        for (int u = 0; u < SU; ++u) {
          const int e = min(e0 + u * NT + t, NE - 1);
          const int i = div_small(e, LW, inv_lw), j = e - i * LW;
          const int ih = 2 * p0 - 3 + i, iw = j - 3;
          ok[u] = ih >= 0 && ih < a.h && iw >= 0 && iw < a.w;
          v[u] = a.x[xb + (long long)min(max(ih, 0), a.h - 1) * a.sh + (long long)min(max(iw, 0), a.w - 1) * a.sw];
        }
#pragma unroll
        for (int u = 0; u < SU; ++u) {
          const int e = e0 + u * NT + t;
          if (e < NE) sx[e] = ok[u] ? v[u] : 0.f;
        }
      }
      const int ND = a.R * (STEM_K / 4);  // float4 of the band's dy rows
      constexpr int DU = 12;
      for (int e0 = 0; e0 < ND; e0 += DU * NT) {
        f32x4 v[DU];
#pragma unroll
        for (int u = 0; u < DU; ++u) {
          const int e = min(e0 + u * NT + t, ND - 1);
          const int m = e >> 4, c4 = e & 15;
          const int pl = div_small(m, a.q, inv_q), qq = m - pl * a.q;
          v[u] = ld4(a.dy + ((long long)((p0 + pl) * a.q + qq) * a.n + n) * STEM_K + 4 * c4);
        }
#pragma unroll
        for (int u = 0; u < DU; ++u) {
          const int e = e0 + u * NT + t;
          if (e < ND) st4(sdy + (e >> 4) * LDD + 4 * (e & 15), v[u]);
        }
      }
    }
    __syncthreads();
    if (bnd == b0) TSPM_STAMP(tspm_g_stamps_stem, 1);
    const float* ap = sdy + ct * 32 + li;
    int m = 2 * s0 + kh;
    int pl = div_small(m, a.q, inv_q), qq = m - pl * a.q;
    for (int sb = s0; sb < s1; sb += 8) {
      float av[8], bv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const bool ok = sb + u < s1 && m < a.R;
        const int mc = ok ? m : 0;
        const int plc = ok ? pl : 0, qqc = ok ? qq : 0;
        av[u] = ok ? ap[mc * LDD] : 0.f;
        bv[u] = sx[2 * plc * LW + 2 * qqc + toffl];
        m += 2;
        qq += 2;  // q >= 1: at most two wraps
        if (qq >= a.q) { qq -= a.q; ++pl; }
        if (qq >= a.q) { qq -= a.q; ++pl; }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) acc = mfma32(av[u], bv[u], acc);
    }
  }
  TSPM_STAMP(tspm_g_stamps_stem, 2);
  __syncthreads();  // the last band's reads of sdy are done: reuse it for the second half's accumulators
  float* sc = sdy;  // [4 tiles][16][64]
  if (half == 1) {
#pragma unroll
    for (int r = 0; r < 16; ++r) sc[(ot * 16 + r) * 64 + lane] = acc[r];
  }
  __syncthreads();
  if (half == 0) {
    float* sl = a.slab + (long long)blockIdx.x * (STEM_K * STEM_TAPS);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float v = acc[r] + sc[(ot * 16 + r) * 64 + lane];
      const int c = ct * 32 + acc_row(r, lane);
      if (tap < STEM_TAPS) sl[c * STEM_TAPS + tap] = v;
    }
  }
  TSPM_STAMP(tspm_g_stamps_stem, 3);
  TSPM_STAMP_CLK(tspm_g_stamps_stem, 7);
}

}  // namespace

namespace tspm_detail {

// Output rows per band: the largest divisor PB of P with PB*Q <= 256 that still gives >= 256 workgroups,
// else the one giving the most workgroups (PB = 1); 0 when even one output row exceeds 256.
int stem_pb(const tspm_conv_shape* s) {
  if (s->q > 16 * STEM_WAVES * STEM_JOBS) return 0;
  for (int pb = s->p; pb >= 1; --pb) {
    if (s->p % pb || pb * s->q > 16 * STEM_WAVES * STEM_JOBS) continue;
    if ((long long)s->n * (s->p / pb) >= 256) return pb;
  }
  return 1;
}

bool stem_supported(const tspm_conv_shape* s) {
  return s->c == 1 && s->r == 7 && s->s == 7 && s->stride == 2 && s->pad == 3 && s->k == STEM_K && s->p >= 1 &&
         s->q >= 1 && s->w + 6 <= 4096 && stem_pb(s) > 0;
}

int stem_tiles(const tspm_conv_shape* s) { return s->n * (s->p / stem_pb(s)); }
int stem_tile_rows(const tspm_conv_shape* s) { return stem_pb(s) * s->q; }

int stem_fwd(const tspm_conv_shape* s, const float* x, const tspm_strides4* xs, const float* w, float* y, float* part,
             hipStream_t st) {
  StemArgs a{};
  a.n = s->n; a.h = s->h; a.w = s->w; a.p = s->p; a.q = s->q;
  a.pb = stem_pb(s);
  a.nb = s->p / a.pb;
  a.R = a.pb * s->q;
  a.RT = cdiv(a.R, 32);
  if (xs) {
    a.sn = xs->sn; a.sh = xs->sh; a.sw = xs->sw;
  } else {  // HWNC, one channel
    a.sn = 1; a.sh = (long long)s->w * s->n; a.sw = s->n;
  }
  a.x = x; a.wt = w; a.y = y; a.part = part;
  const int NE = (2 * a.pb + 5) * (s->w + 6);
  const size_t lds =
      ((size_t)STEM_K * STEM_TAPS + ((NE + 3) & ~3) + 2 * STEM_K + 2 * (size_t)a.RT * STEM_K) * sizeof(float);
  hipLaunchKernelGGL(k_stem_fwd, dim3(s->n * a.nb), dim3(64 * STEM_WAVES), lds, st, a);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

// Weight-gradient bands: the largest divisor PB of P with PB*Q <= 384 rows (the band's dy in LDS) that gives
// >= 256 bands, else PB = 1; bands are dealt to at most 256 workgroups in contiguous runs (256 slabs).
int stem_wgrad_pb(const tspm_conv_shape* s) {
  for (int pb = s->p; pb >= 1; --pb) {
    if (s->p % pb || pb * s->q > 384) continue;
    if ((long long)s->n * (s->p / pb) >= 256) return pb;
  }
  return 1;
}

struct StemWPlan {
  int pb, nb, R, ldd, bands, bpw, wgs;
  size_t lds;
};

StemWPlan stem_wgrad_plan(const tspm_conv_shape* s) {
  StemWPlan pl{};
  pl.pb = stem_wgrad_pb(s);
  pl.nb = s->p / pl.pb;
  pl.R = pl.pb * s->q;
  pl.bands = s->n * pl.nb;
  pl.bpw = (int)cdiv64(pl.bands, 256);
  pl.wgs = (int)cdiv64(pl.bands, pl.bpw);
  const size_t nx = (size_t)(((2 * pl.pb + 5) * (s->w + 6) + 3) & ~3);
  // dy row pitch 96 floats: the two lane halves of an MFMA A read (rows m, m+1) land on disjoint banks; 64
  // (2-way conflicts) when 96 does not fit the LDS
  pl.ldd = (nx + (size_t)pl.R * 96) * sizeof(float) <= 160 * 1024 ? 96 : 64;
  const size_t ndy = std::max((size_t)pl.R * pl.ldd, (size_t)4 * 16 * 64);
  pl.lds = (nx + ndy) * sizeof(float);
  return pl;
}

bool stem_wgrad_supported(const tspm_conv_shape* s) {
  return s->c == 1 && s->r == 7 && s->s == 7 && s->stride == 2 && s->pad == 3 && s->k == STEM_K && s->p >= 1 &&
         s->q >= 1 && s->q <= 384 && stem_wgrad_plan(s).lds <= 160 * 1024;
}

// The slabs start after the workspace's counter header (TSPM_COUNTER_BYTES): other conv launches of the
// engine share the workspace and rely on those counters staying zero.
size_t stem_wgrad_workspace(const tspm_conv_shape* s) {
  return TSPM_COUNTER_BYTES + (size_t)stem_wgrad_plan(s).wgs * STEM_K * STEM_TAPS * sizeof(float);
}

int stem_wgrad(const tspm_conv_shape* s, const float* x, const tspm_strides4* xs, const float* dy, float* dw, void* ws,
               size_t ws_bytes, hipStream_t st) {
  const StemWPlan pl = stem_wgrad_plan(s);
  StemWArgs a{};
  a.n = s->n; a.h = s->h; a.w = s->w; a.p = s->p; a.q = s->q;
  a.pb = pl.pb; a.nb = pl.nb; a.R = pl.R; a.ldd = pl.ldd; a.bands = pl.bands; a.bpw = pl.bpw;
  if (xs) {
    a.sn = xs->sn; a.sh = xs->sh; a.sw = xs->sw;
  } else {
    a.sn = 1; a.sh = (long long)s->w * s->n; a.sw = s->n;
  }
  if (!ws || ws_bytes < stem_wgrad_workspace(s) || (reinterpret_cast<uintptr_t>(ws) & 15) ||
      (reinterpret_cast<uintptr_t>(dy) & 15))
    return TSPM_ERR_WORKSPACE;
  a.x = x; a.dy = dy; a.slab = reinterpret_cast<float*>(static_cast<char*>(ws) + TSPM_COUNTER_BYTES);
  hipLaunchKernelGGL(k_stem_wgrad, dim3(pl.wgs), dim3(64 * STEMW_WAVES), pl.lds, st, a);
  TSPM_LAUNCH_CHECK();
  return tspm_reduce_slabs(STEM_K * STEM_TAPS, pl.wgs, STEM_K * STEM_TAPS, a.slab, dw, st);
}

}  // namespace tspm_detail
