// Device helpers shared by the register-direct (conv.hip) and LDS-staged (conv_lds.hip)
// implicit-GEMM convolution kernels: argument block, MFMA accumulator tile with its epilogues
// (stores, split-K combine, BatchNorm partial statistics), split-K slab reduction and the in-launch
// BatchNorm merge.  Replaces nn.Conv2d of MML_Suite/models/msa/networks/resnet.py:25,30,137,176.
#pragma once
#include "common.h"

namespace {

struct ConvArgs {
  int n, h, w, c, k, r, s, st, pad, p, q;
  long long sn, sh, sw, sc;  // input strides (fwd / wgrad)
  int m;                     // GEMM rows: fwd P*Q*N, dgrad H*W*N, wgrad K
  int splits;                // wgrad global split
  long long slab;            // elements per split slab
  int beta;                  // dgrad accumulate
  unsigned* cnt;             // wgrad: per-tile arrival counters (in-launch slab reduction), or null
  int xcd;                   // LDS-staged kernels: XCD-aware workgroup -> tile mapping (1) or identity (0)
  int acq;                   // LDS-staged kernels: agent acquire before reading split-K slabs / BN partials
                             // (1), or sc1 loads only (0, default; TSPM_ALGO_HANDOFF_ACQUIRE for A/B)
  // LDS-staged dgrad epilogue (round 6, tspm_conv_bwd_ex): the BatchNorm-backward partial sums of the gradient
  // being written — g' = dx * [bnb_out > 0], per 32-row tile and channel sum(g'), sum(g' (bnb_y - mean)) [and
  // sum(g' (bnb_y2 - mean2))] into bnb_part [3][tiles][C] — so the BN backward that consumes dx needs no partial
  // pass of its own.  bnb_part == nullptr: off.
  const float* bnb_out;
  const float* bnb_y;
  const float* bnb_mean;
  const float* bnb_y2;
  const float* bnb_mean2;
  float* bnb_part;
  const uint8_t* bnb_idx;    // max-pool gather mode (tspm_bn_bwd_part.idx): bnb_out / bnb_y are [bnb_H][bnb_W][n][c]
  int bnb_H, bnb_W;
  // whole-BN-backward mode (tspm_bn_bwd_part.dy): the last tile of each column block applies the BN backward
  const float *bnx_inv, *bnx_gamma, *bnx_inv2, *bnx_gamma2;
  float *bnx_dgamma, *bnx_dbeta, *bnx_dy, *bnx_dgamma2, *bnx_dbeta2, *bnx_dy2, *bnx_dres;
  unsigned* bnx_cnt;
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
#ifdef TSPM_EXP_NOMFMA  // diagnostic ablation (stamped build only): consume operands without MFMA
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) v[a][b][0] += A[a][0] * B[b][0] + A[a][3] * B[b][3];
#else
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) v[a][b] = mfma32(A[a][j], B[b][j], v[a][b]);
#endif
  }
  // store rows row0 + a*32 + acc_row, cols col0 + b*32 + (lane&31) of a [rows, ld] matrix
  // (sc1: write-through, the payload of an in-launch hand-off)
  TSPM_DEV void store(float* out, int row0, int col0, int rows, int cols, long long ld, int lane, bool accumulate,
                      bool sc1 = false) const {
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
            if (sc1) st_sc1(p, v[a][b][i]);
            else *p = accumulate ? (*p + v[a][b][i]) : v[a][b][i];
          }
        }
      }
  }
  // store (or accumulate onto) rows x cols as store() does — bitwise the same dx — and emit the BatchNorm-backward
  // partial sums of the stored values per 32-row tile and column (ConvArgs.bnb_*): the mask / y / y2 / old-dx
  // loads of 8 rows are issued together, the two lane halves' 16 rows each combined with one xor shuffle.
  TSPM_DEV void store_bnb(float* out, int row0, int col0, int rows, int cols, long long ld, int lane,
                          bool accumulate, const ConvArgs& g) const {
    const long long plane = (long long)(rows >> 5) * cols;
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int col = col0 + b * 32 + (lane & 31);
      const bool colok = col < cols;
      const int c = colok ? col : cols - 1;
      const float mu = g.bnb_mean[c];
      const float mu2 = g.bnb_y2 ? g.bnb_mean2[c] : 0.f;
#pragma unroll
      for (int a = 0; a < TM; ++a) {
        float sg = 0.f, sx = 0.f, sx2 = 0.f;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          float old[8], msk[8], yy[8], yy2[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int row = min(row0 + a * 32 + acc_row(h * 8 + j, lane), rows - 1);
            const long long off = (long long)row * ld + c;
            old[j] = accumulate ? out[off] : 0.f;
            long long src = off;
            if (g.bnb_idx) {  // the element the max pool took this output from (dx rows = (p, q, n) of the pool output)
              const int tap = g.bnb_idx[off];
              const int pos = row / g.n, nn = row - pos * g.n;
              const int pp = pos / g.w, qq = pos - pp * g.w;
              const int hh = 2 * pp - 1 + tap / 3, ww = 2 * qq - 1 + tap % 3;
              src = (((long long)hh * g.bnb_W + ww) * g.n + nn) * ld + c;
            }
            msk[j] = g.bnb_out[src];
            yy[j] = g.bnb_y[src];
            yy2[j] = g.bnb_y2 ? g.bnb_y2[src] : 0.f;
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int row = row0 + a * 32 + acc_row(h * 8 + j, lane);
            const float val = accumulate ? (old[j] + v[a][b][h * 8 + j]) : v[a][b][h * 8 + j];
            if (row < rows && colok) {
              if (g.bnx_dy) st_sc1(out + (long long)row * ld + col, val);  // read by the column block's last tile
              else out[(long long)row * ld + col] = val;
              const float gm = msk[j] > 0.f ? val : 0.f;
              sg += gm;
              sx += gm * (yy[j] - mu);
              sx2 += gm * (yy2[j] - mu2);
            }
          }
        }
        sg += __shfl_xor(sg, 32, 64);
        sx += __shfl_xor(sx, 32, 64);
        sx2 += __shfl_xor(sx2, 32, 64);
        if (lane < 32 && colok) {
          float* p = g.bnb_part + (long long)((row0 + a * 32) >> 5) * cols + col;
          if (g.bnx_dy) {
            st_sc1(p, sg);
            st_sc1(p + plane, sx);
            if (g.bnb_y2) st_sc1(p + 2 * plane, sx2);
          } else {
            p[0] = sg;
            p[plane] = sx;
            if (g.bnb_y2) p[2 * plane] = sx2;
          }
        }
      }
    }
  }
  // split-K combine of the WK waves of one tile through LDS (wave wk > 0 writes, wave 0 sums in
  // order).  Every wave of the workgroup must call this (it contains barriers).
  template <int WN, int WK>
  TSPM_DEV void combine(float* lds, int wn, int wk, int lane, bool active) {
    if constexpr (WK > 1) {
      constexpr int TILE = TM * TN * 16 * 64;
      if (wk > 0 && active) {
        float* dst = lds + ((wk - 1) * WN + wn) * TILE;
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
#pragma unroll
            for (int i = 0; i < 16; ++i) dst[((a * TN + b) * 16 + i) * 64 + lane] = v[a][b][i];
      }
      __syncthreads();
      if (wk == 0 && active) {
        for (int k = 1; k < WK; ++k) {
          const float* src = lds + ((k - 1) * WN + wn) * TILE;
#pragma unroll
          for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < TN; ++b)
#pragma unroll
              for (int i = 0; i < 16; ++i) v[a][b][i] += src[((a * TN + b) * 16 + i) * 64 + lane];
        }
      }
    }
  }
  // BatchNorm partial statistics of this tile's valid rows, per column (channel):
  //   part[0][mt][col] = K (the tile's first row), part[1][..] = mean - K, part[2][..] = M2
  TSPM_DEV void bn_partials(float* part, long long plane, int mt, int row0, int col0, int rows, int cols,
                            int lane, bool sc1) const {
    const int cnt = min(TM * 32, rows - row0);
    const float inv = 1.0f / (float)cnt;
#pragma unroll
    for (int b = 0; b < TN; ++b) {
      const int col = col0 + b * 32 + (lane & 31);
      const float K = __shfl(v[0][b][0], lane & 31, 64);  // row 0 of the tile lives in lane (col, half 0), reg 0
      float s = 0.f;
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (row0 + a * 32 + acc_row(i, lane) < rows) s += v[a][b][i] - K;
      s += __shfl_xor(s, 32, 64);
      const float off = s * inv;
      float sd = 0.f, s2 = 0.f;
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (row0 + a * 32 + acc_row(i, lane) < rows) {
            const float d = (v[a][b][i] - K) - off;
            sd += d;
            s2 += d * d;
          }
      sd += __shfl_xor(sd, 32, 64);
      s2 += __shfl_xor(s2, 32, 64);
      if (lane < 32 && col < cols) {
        const double n = (double)cnt;
        const float v0 = K, v1 = (float)((double)off + (double)sd / n), v2 = (float)((double)s2 - (double)sd * (double)sd / n);
        float* p0 = part + (long long)mt * cols + col;
        if (sc1) {
          st_sc1(p0, v0); st_sc1(p0 + plane, v1); st_sc1(p0 + 2 * plane, v2);
        } else {
          p0[0] = v0; p0[plane] = v1; p0[2 * plane] = v2;
        }
      }
    }
  }
};

TSPM_DEV int split_lo(int T, int z, int S) { return (int)(((long long)T * z) / S); }

// Register prefetch depth of the main loops: loads of PF reduction iterations are in flight while
// one is multiplied, so a wave pays one memory round trip per PF iterations instead of one per
// iteration (at batch 128 most layers give a wave 4-20 iterations: with a one-deep prefetch the
// loop was a chain of dependent L2/HBM round trips, 2-5x the MFMA time).
template <int TM, int TN>
constexpr int prefetch_depth() {
  return TM * TN == 1 ? 8 : (TM * TN == 2 ? 4 : 3);
}

// Runs iterations [it0, it1) through a PF-slot register ring: slot d holds iteration
// base + d; right after slot d is multiplied it is refilled with iteration base + PF + d.  The main
// loop has no data-dependent branches around its loads (past the end a slot reloads iteration
// it1-1, which is never multiplied), so the compiler's counted vmcnt waits keep PF-1 loads in
// flight.  load(it, A, B) fills the operands of reduction iteration it.
template <int TM, int TN, int PF, class LoadFn>
TSPM_DEV void run_pipelined(Acc<TM, TN>& acc, int it0, int it1, LoadFn&& load) {
  const int n = it1 - it0;
  if (n <= 0) return;
  f32x4 A[PF][TM], B[PF][TN];
#pragma unroll
  for (int d = 0; d < PF; ++d) load(min(it0 + d, it1 - 1), A[d], B[d]);
  const int nfull = n / PF;
  for (int bt = 0; bt < nfull; ++bt) {
    const int nb = it0 + (bt + 1) * PF;
#pragma unroll
    for (int d = 0; d < PF; ++d) {
      acc.mma4(A[d], B[d]);
      load(min(nb + d, it1 - 1), A[d], B[d]);
    }
  }
  const int rem = n - nfull * PF;
#pragma unroll
  for (int d = 0; d < PF; ++d)
    if (d < rem) acc.mma4(A[d], B[d]);
}

// wgrad tail with split-K over workgroups: the last of the `splits` workgroups of this tile sums
// the slabs in slab order (bitwise equal to tspm_reduce_slabs) and writes dw.
template <int TM, int TN, int WN>
TSPM_DEV void slab_tail(const ConvArgs& g, const float* slabs, float* dw_final, int RSC, float* lds) {
  if (!last_arriver(g.cnt + (blockIdx.y * gridDim.x + blockIdx.x), g.splits, reinterpret_cast<int*>(lds))) return;
  const int r0 = blockIdx.x * (TM * 32), rn = min(TM * 32, g.k - r0);
  const int cb0 = blockIdx.y * (WN * TN * 32), cn = min(WN * TN * 32, RSC - cb0);
  for (int e = threadIdx.x; e < rn * cn; e += blockDim.x) {
    const int rr = e / cn, cc = e - rr * cn;
    const long long off = (long long)(r0 + rr) * RSC + cb0 + cc;
    float sum = 0.f;
    int zz = 0;
    for (; zz + 8 <= g.splits; zz += 8) {  // 8 independent loads in flight, summed in slab order
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = slabs[(zz + u) * g.slab + off];
#pragma unroll
      for (int u = 0; u < 8; ++u) sum += v[u];
    }
    for (; zz < g.splits; ++zz) sum += slabs[zz * g.slab + off];
    dw_final[off] = sum;
  }
}

// Forward tail with in-launch BatchNorm: the last workgroup of each column block (all row tiles
// of its WN*TN*32 channels have written their partials) merges them (no finalize launch).
template <int TM, int TN, int WN>
TSPM_DEV void fwd_bn_tail(const ConvArgs& g, const tspm_bn_fuse& bf, float* lds) {
  if (!bf.counters) return;
  if (!last_arriver(bf.counters + blockIdx.y, gridDim.x, reinterpret_cast<int*>(lds))) return;
  constexpr int CB = WN * TN * 32;
  double* red = reinterpret_cast<double*>(lds) + 2;
  double* smu = red + blockDim.x;
  bn_merge_block(g.m, g.k, gridDim.x, TM * 32, bf.partial, blockIdx.y * CB, CB, bf.running_mean, bf.running_var,
                 bf.momentum, bf.eps, bf.save_mean, bf.save_invstd, red, smu);
}

}  // namespace

// Host-side launchers of the LDS-staged kernels (conv_lds.hip), called by the C ABI entry points
// in conv.hip for tspm_conv_algo.variant == 1.  Return a TSPM status.
namespace tspm_detail {
struct LdsAlgo {
  int tm, tn, wm, wn, wk, splits;
  size_t floor;  // tspm_conv_algo.lds_floor: minimum dynamic LDS of the launch (ABI 21; per call, no global state)
  int acq;       // tspm_conv_algo.flags & TSPM_ALGO_HANDOFF_ACQUIRE
};
// The LDS-staged kernels (conv_lds.hip) are built twice, with different operand loaders, and reached through
// these tables: variant 1 = register-staged loader waves (lds_impl_reg), variant 2 = single-role waves with
// an LDS-DMA ring (lds_impl_dma, built with TSPM_LOADER_WAVES=0).
struct LdsImpl {
  bool (*fwd_supported)(const tspm_conv_shape* s, const tspm_strides4* xs, const LdsAlgo& a);
  bool (*dgrad_supported)(const tspm_conv_shape* s, const LdsAlgo& a);
  bool (*wgrad_supported)(const tspm_conv_shape* s, const tspm_strides4* xs, const LdsAlgo& a);
  size_t (*fwd_workspace)(const tspm_conv_shape* s, const LdsAlgo& a);
  int (*fwd_bn_counters)(const tspm_conv_shape* s, const LdsAlgo& a);
  long long (*fwd_bn_partial_floats)(const tspm_conv_shape* s, const LdsAlgo& a);
  size_t (*dgrad_workspace)(const tspm_conv_shape* s, const LdsAlgo& a);
  size_t (*wgrad_workspace)(const tspm_conv_shape* s, const LdsAlgo& a);
  int (*fwd)(const tspm_conv_shape* s, const LdsAlgo& a, const float* x, const float* w, float* y,
             const tspm_bn_fuse* bn, void* ws, size_t ws_bytes, hipStream_t st);
  int (*dgrad)(const tspm_conv_shape* s, const LdsAlgo& a, const float* dy, const float* w, float* dx, int beta,
               void* ws, size_t ws_bytes, hipStream_t st);
  int (*wgrad)(const tspm_conv_shape* s, const LdsAlgo& a, const float* x, const float* dy, float* dw, void* ws,
               size_t ws_bytes, hipStream_t st);
  bool (*bwd_built)(const LdsAlgo& ad, const LdsAlgo& aw);
  int (*bwd)(const tspm_conv_shape* s, const LdsAlgo& ad, const LdsAlgo& aw, const float* x, const float* dy,
             const float* w, float* dx, int beta, float* dw, const tspm_adam_job* adam, const tspm_bn_bwd_part* bnp,
             void* wsd, size_t wsd_bytes, void* wsw, size_t wsw_bytes, hipStream_t st);
  int (*fwd_pair)(const tspm_conv_shape* s1, const LdsAlgo& a1, const float* x1, const float* w1, float* y1,
                  const tspm_bn_fuse* bn1, void* ws1, size_t ws1_bytes, const tspm_conv_shape* s2, const LdsAlgo& a2,
                  const float* x2, const float* w2, float* y2, const tspm_bn_fuse* bn2, void* ws2, size_t ws2_bytes,
                  hipStream_t st);
  int (*fwd_bn_inlaunch)(const tspm_conv_shape* s, const LdsAlgo& a);
  int (*bwd_quad)(const tspm_conv_shape* s, const LdsAlgo& ad, const LdsAlgo& aw, const float* x, const float* dy,
                  const float* w, float* dx, int beta, float* dw, const tspm_bn_bwd_part* bnp, void* wsd,
                  size_t wsd_bytes, void* wsw, size_t wsw_bytes, const tspm_conv_shape* s2, const LdsAlgo& ad2,
                  const LdsAlgo& aw2, const float* x2, const float* dy2, const float* w2, float* dx2, float* dw2,
                  void* wsd2, size_t wsd2_bytes, void* wsw2, size_t wsw2_bytes, const tspm_adam_job* adam,
                  hipStream_t st);
};
const LdsImpl& lds_impl_reg();
const LdsImpl& lds_impl_dma();
const LdsImpl& lds_impl_x9();  // variant 4: variant 1 with the fp32 products on bf16 MFMA (exact 3-piece split)
// Minimum dynamic LDS of an LDS-staged launch (tspm_conv_algo.lds_floor, ABI 21): a caller-chosen floor caps how
// many of the launch's workgroups share a CU, leaving room for a concurrent stream's kernels.  Passed per call.
inline size_t lds_with_floor(size_t lds, const LdsAlgo& a) { return std::max(lds, std::min(a.floor, (size_t)160 * 1024)); }
// The 1-channel 7x7/2 stems, tspm_conv_algo.variant 3 (stem.hip)
bool stem_supported(const tspm_conv_shape* s);
int stem_pb(const tspm_conv_shape* s);
int stem_tiles(const tspm_conv_shape* s);
int stem_tile_rows(const tspm_conv_shape* s);
int stem_fwd(const tspm_conv_shape* s, const float* x, const tspm_strides4* xs, const float* w, float* y, float* part,
             hipStream_t st);
bool stem_wgrad_supported(const tspm_conv_shape* s);
size_t stem_wgrad_workspace(const tspm_conv_shape* s);
int stem_wgrad(const tspm_conv_shape* s, const float* x, const tspm_strides4* xs, const float* dy, float* dw, void* ws,
               size_t ws_bytes, hipStream_t st);
}  // namespace tspm_detail
