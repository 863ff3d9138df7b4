// BatchNorm2d (training + eval) forward/backward for HWNC activations — HBM-bound kernels.
//
// Replaces nn.BatchNorm2d at MML_Suite/models/msa/networks/resnet.py:26,31,138,177 together with the
// ReLU (:27,42,52,139) and the residual add (:51) that follow it.
//
// Statistics are carried as per-tile partials {K (a data value of the tile), mean-K, M2 (sum of
// squared deviations from the tile mean)}: produced either by the conv epilogue (tspm_conv_fwd with
// bn_partial, no re-read of the conv output) or by a shifted two-pass kernel over a [rows x 64-chan]
// tile (tspm_bn_stats).  tspm_bn_finalize merges them per channel in double with a fixed-order
// parallel reduction: mean = sum(n_t * mean_t)/n, M2 = sum(M2_t + n_t (mean_t - mean)^2).  No
// E[y^2] - E[y]^2 cancellation anywhere: the audio stem produces |y| ~ 1e8, and border positions of
// tiny feature maps sit many standard deviations away from the channel mean.
#include "common.h"

namespace {

constexpr int kChanPerBlock = 64;  // 16 float4 lanes
constexpr int kRowGroups = 16;     // 256 threads = 16 lanes x 16 row groups

int row_blocks(long long m, int c, int target = 1024) {
  const long long cg = cdiv64(c, kChanPerBlock);
  long long g = cdiv64(target, cg);
  const long long max_g = cdiv64(m, kRowGroups);
  if (g > max_g) g = max_g;
  if (g < 1) g = 1;
  return (int)g;
}

// ------------------------------------------------------------------------------------------------
// standalone forward statistics partials (shifted two-pass per [rows x 64 channels] tile)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_bn_stats_partial(long long M, int C, const float* __restrict__ y,
                                                          int nslab, long long slab_stride, float* __restrict__ y_out,
                                                          long long rows_per_block, float* __restrict__ part) {
  __shared__ f32x4 sh[256], sh2[256];
  __shared__ f32x4 soff[16];
  const int t = threadIdx.x;
  const int lane = t & 15, rg = t >> 4;
  const int c4 = blockIdx.y * 16 + lane;
  const bool cok = 4 * c4 < C;
  const long long r_begin = blockIdx.x * rows_per_block;
  const long long r_end = min(M, r_begin + rows_per_block);
  const double n = (double)(r_end - r_begin);
  const float inv_n = (float)(1.0 / n);
  auto load = [&](long long off) -> f32x4 {
    f32x4 v = ld4(y + off);
    for (int z = 1; z < nslab; ++z) v += ld4(y + z * slab_stride + off);
    return v;
  };
  f32x4 K = {0.f, 0.f, 0.f, 0.f}, s1 = K;
  if (cok) {
    K = load(r_begin * C + 4 * c4);
    for (long long row = r_begin + rg; row < r_end; row += kRowGroups) {
      const long long off = row * C + 4 * c4;
      const f32x4 v = load(off);
      if (nslab > 1) st4(y_out + off, v);
      s1 += v - K;
    }
  }
  sh[t] = s1;
  __syncthreads();
  if (rg == 0) {
    for (int k = 1; k < kRowGroups; ++k) s1 += sh[k * 16 + lane];
    soff[lane] = s1 * inv_n;
  }
  __syncthreads();
  const f32x4 off = soff[lane];
  f32x4 sd = {0.f, 0.f, 0.f, 0.f}, s2 = sd;
  if (cok) {
    for (long long row = r_begin + rg; row < r_end; row += kRowGroups) {
      const f32x4 d = (load(row * C + 4 * c4) - K) - off;
      sd += d;
      s2 += d * d;
    }
  }
  __syncthreads();
  sh[t] = sd;
  sh2[t] = s2;
  __syncthreads();
  if (rg == 0 && cok) {
    for (int k = 1; k < kRowGroups; ++k) { sd += sh[k * 16 + lane]; s2 += sh2[k * 16 + lane]; }
    f32x4 lo, m2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      lo[j] = (float)((double)off[j] + (double)sd[j] / n);
      m2[j] = (float)((double)s2[j] - (double)sd[j] * (double)sd[j] / n);
    }
    const long long plane = (long long)gridDim.x * C;
    st4(part + (long long)blockIdx.x * C + 4 * c4, K);
    st4(part + plane + (long long)blockIdx.x * C + 4 * c4, lo);
    st4(part + 2 * plane + (long long)blockIdx.x * C + 4 * c4, m2);
  }
}

// per-channel merge of G partial tiles: 4 channels x 64 tile groups per workgroup, double, fixed
// order, 8 tile loads in flight per thread (bn_merge_block)
constexpr int kFinChan = 4;
template <int CH>
__global__ __launch_bounds__(256) void k_bn_finalize(long long M, int C, int G, long long rows_per_tile,
                                                     const float* __restrict__ part, float* __restrict__ rmean,
                                                     float* __restrict__ rvar, float momentum, float eps,
                                                     float* __restrict__ smean, float* __restrict__ sinv) {
  __shared__ double red[256];
  __shared__ double smu[CH];
  bn_merge_block(M, C, G, rows_per_tile, part, blockIdx.x * CH, CH, rmean, rvar, momentum, eps, smean,
                 sinv, red, smu);
}

// "Wide" BN launches for the few-channel layers (measured: BN 1.04 -> 1.02 ms): the statistics
// merge with fewer channels per workgroup (64 workgroups at C = 64 instead of 16, each merging its tiles
// with all 256 threads) and the backward partial sums with more rows' loads in flight per thread (the
// C = 64 layers' partial pass has only 64 workgroups: 1/4 of the CUs, so each must keep more bytes in
// flight).  Both change only the (fixed) order of the double-precision sums.
constexpr bool bn_wide() { return true; }


// ------------------------------------------------------------------------------------------------
// apply: out = act(y*scale + shift [+ res | + res*scale2 + shift2])
// ------------------------------------------------------------------------------------------------
template <int RES, bool RELU, bool EVAL>
__global__ __launch_bounds__(256) void k_bn_apply(long long n4, int C, const float* __restrict__ y,
                                                  const float* __restrict__ mean, const float* __restrict__ inv,
                                                  const float* __restrict__ gamma, const float* __restrict__ beta,
                                                  const float* __restrict__ res, const float* __restrict__ mean2,
                                                  const float* __restrict__ inv2, const float* __restrict__ gamma2,
                                                  const float* __restrict__ beta2, float eps, float* __restrict__ out) {
  const int L = C >> 2;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    const int c4 = (int)(i % L);
    f32x4 mu = ld4(mean + 4 * c4), iv = ld4(inv + 4 * c4);
    if (EVAL) {
#pragma unroll
      for (int j = 0; j < 4; ++j) iv[j] = 1.0f / sqrtf(iv[j] + eps);
    }
    const f32x4 sc = ld4(gamma + 4 * c4) * iv;
    const f32x4 sf = ld4(beta + 4 * c4) - mu * sc;
    f32x4 v = ld4(y + 4 * i);
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = fmaf(v[j], sc[j], sf[j]);
    if (RES == 1) {
      o += ld4(res + 4 * i);
    } else if (RES == 2) {
      f32x4 mu2 = ld4(mean2 + 4 * c4), iv2 = ld4(inv2 + 4 * c4);
      if (EVAL) {
#pragma unroll
        for (int j = 0; j < 4; ++j) iv2[j] = 1.0f / sqrtf(iv2[j] + eps);
      }
      const f32x4 sc2 = ld4(gamma2 + 4 * c4) * iv2;
      const f32x4 sf2 = ld4(beta2 + 4 * c4) - mu2 * sc2;
      const f32x4 v2 = ld4(res + 4 * i);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] += fmaf(v2[j], sc2[j], sf2[j]);
    }
    if (RELU) {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = relu_f(o[j]);
    }
    st4(out + 4 * i, o);
  }
}

// Round 6: the training-mode apply with the statistics merge folded into its prologue, for the layers whose conv
// forward cannot merge its per-tile partials in-launch (they used a tspm_bn_finalize launch between the conv and the
// apply).  Workgroup = 16 channels x a block of rows: the 16 x 16 threads first merge the G <= 256 partial tiles
// {K, mean - K, M2} of their 16 channels in double (thread (cl, gg) takes tiles gg, gg + 16, ... — at most 16, all
// loaded at once — then a fixed-order sum over the 16 groups; every workgroup derives the same statistics), row
// block 0 writes save_mean / save_invstd and the running statistics, then the block's rows are normalised as
// k_bn_apply does (+ReLU, + residual / + BN(downsample)).  One launch instead of finalize + apply.
constexpr int kApplyMergeTiles = 256;
template <int RES, bool RELU>
__global__ __launch_bounds__(256) void k_bn_apply_merge(long long M, int C, int G, long long rpt,
                                                        const float* __restrict__ part, float* __restrict__ rmean,
                                                        float* __restrict__ rvar, float momentum, float eps,
                                                        float* __restrict__ smean, float* __restrict__ sinv,
                                                        const float* __restrict__ y, const float* __restrict__ gamma,
                                                        const float* __restrict__ beta, const float* __restrict__ res,
                                                        const float* __restrict__ mean2, const float* __restrict__ inv2,
                                                        const float* __restrict__ gamma2,
                                                        const float* __restrict__ beta2, long long rows_per_block,
                                                        float* __restrict__ out) {
  __shared__ double red[256];
  __shared__ double smu[16];
  __shared__ float ssc[16], ssf[16];
  const int t = threadIdx.x, cl = t & 15, gg = t >> 4;
  const int c = blockIdx.y * 16 + cl;
  const bool cok = c < C;
  const int cc = cok ? c : C - 1;
  const long long plane = (long long)G * C;
  float k0[16], k1[16], k2[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) {  // unconditional (clamped) loads, weight 0 past G
    const long long o = (long long)min(gg + 16 * u, G - 1) * C + cc;
    k0[u] = part[o];
    k1[u] = part[plane + o];
    k2[u] = part[2 * plane + o];
  }
  auto nb_of = [&](int g) -> double { return g < G ? (double)min(rpt, M - (long long)g * rpt) : 0.0; };
  double s = 0.0;
#pragma unroll
  for (int u = 0; u < 16; ++u) s += nb_of(gg + 16 * u) * ((double)k0[u] + (double)k1[u]);
  red[t] = s;
  __syncthreads();
  if (gg == 0) {
    double a = red[cl];
    for (int k = 1; k < 16; ++k) a += red[k * 16 + cl];
    smu[cl] = a / (double)M;
  }
  __syncthreads();
  const double mean = smu[cl];
  double q = 0.0;
#pragma unroll
  for (int u = 0; u < 16; ++u) {
    const int g = gg + 16 * u;
    if (g < G) {
      const double mb = (double)k0[u] + (double)k1[u];
      q += (double)k2[u] + nb_of(g) * (mb - mean) * (mb - mean);
    }
  }
  __syncthreads();
  red[t] = q;
  __syncthreads();
  if (gg == 0) {
    double m2 = red[cl];
    for (int k = 1; k < 16; ++k) m2 += red[k * 16 + cl];
    const double n = (double)M;
    double var = m2 / n;
    if (var < 0.0) var = 0.0;
    const float fmean = (float)mean, fvar = (float)var;
    const float inv = 1.0f / sqrtf(fvar + eps);
    if (cok) {
      const float sc = gamma[c] * inv;
      ssc[cl] = sc;
      ssf[cl] = beta[c] - fmean * sc;
      if (blockIdx.x == 0) {
        smean[c] = fmean;
        sinv[c] = inv;
        if (rmean) rmean[c] = momentum * fmean + (1.f - momentum) * rmean[c];
        if (rvar) {
          const float unb = M > 1 ? (float)(m2 / (n - 1.0)) : fvar;
          rvar[c] = momentum * unb + (1.f - momentum) * rvar[c];
        }
      }
    }
  }
  __syncthreads();
  // apply: thread = (row, 4 channels); 64 rows per pass
  const int q4 = t & 3, rr = t >> 2;
  const int c4 = blockIdx.y * 4 + q4;
  if (4 * c4 >= C) return;
  f32x4 sc, sf, sc2 = {0.f, 0.f, 0.f, 0.f}, sf2 = sc2;
#pragma unroll
  for (int j = 0; j < 4; ++j) { sc[j] = ssc[4 * q4 + j]; sf[j] = ssf[4 * q4 + j]; }
  if (RES == 2) {
    sc2 = ld4(gamma2 + 4 * c4) * ld4(inv2 + 4 * c4);
    sf2 = ld4(beta2 + 4 * c4) - ld4(mean2 + 4 * c4) * sc2;
  }
  const long long r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  for (long long row = r0 + rr; row < r1; row += 64) {
    const long long off = row * C + 4 * c4;
    const f32x4 v = ld4(y + off);
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = fmaf(v[j], sc[j], sf[j]);
    if (RES == 1) {
      o += ld4(res + off);
    } else if (RES == 2) {
      const f32x4 v2 = ld4(res + off);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] += fmaf(v2[j], sc2[j], sf2[j]);
    }
    if (RELU) {
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = relu_f(o[j]);
    }
    st4(out + off, o);
  }
}

// The stem's BN apply + ReLU with the MaxPool2d(3, 2, 1) that follows it folded in (resnet.py:138-140; round 5):
// thread = (pooled output (p, q, n), 4 channels).  It forms relu(bn(y)) for the 3 x 3 window (k_bn_apply's
// arithmetic), keeps the first maximum in row-major window order with NaN winning (k_maxpool_fwd's rule) and
// writes the pooled value and its argmax tap; it also stores the activation `out` of the window elements it owns
// — rows 2p, 2p+1 x columns 2q, 2q+1, which tile the map exactly once — for the BN backward's ReLU mask.  Bitwise
// tspm_bn_apply + tspm_maxpool_fwd, one launch and one re-read of the activation fewer.
template <bool EVAL>
__global__ __launch_bounds__(256) void k_bn_apply_maxpool(int N, int H, int W, int C, int P, int Q,
                                                          const float* __restrict__ y, const float* __restrict__ mean,
                                                          const float* __restrict__ inv, const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float eps,
                                                          float* __restrict__ out, float* __restrict__ pooled,
                                                          uint8_t* __restrict__ idx) {
  const int L = C >> 2;
  const long long total = (long long)P * Q * N * L;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c4 = (int)(i % L);
    const long long row = i / L;  // (p, q, n)
    const int n = (int)(row % N);
    const int pos = (int)(row / N);
    const int p = pos / Q, q = pos - p * Q;
    f32x4 mu = ld4(mean + 4 * c4), iv = ld4(inv + 4 * c4);
    if (EVAL) {
#pragma unroll
      for (int j = 0; j < 4; ++j) iv[j] = 1.0f / sqrtf(iv[j] + eps);
    }
    const f32x4 sc = ld4(gamma + 4 * c4) * iv;
    const f32x4 sf = ld4(beta + 4 * c4) - mu * sc;
    f32x4 v[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int h = min(max(2 * p - 1 + t / 3, 0), H - 1), w = min(max(2 * q - 1 + t % 3, 0), W - 1);
      v[t] = ld4(y + (((long long)h * W + w) * N + n) * C + 4 * c4);
    }
    f32x4 best = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    int bi[4] = {0, 0, 0, 0};
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int h = 2 * p - 1 + t / 3, w = 2 * q - 1 + t % 3;
      if (h < 0 || h >= H || w < 0 || w >= W) continue;
      f32x4 a;
#pragma unroll
      for (int j = 0; j < 4; ++j) a[j] = relu_f(fmaf(v[t][j], sc[j], sf[j]));
      if (out && t / 3 >= 1 && t % 3 >= 1) st4(out + (((long long)h * W + w) * N + n) * C + 4 * c4, a);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (a[j] > best[j] || isnan(a[j])) { best[j] = a[j]; bi[j] = t; }
    }
    st4(pooled + row * C + 4 * c4, best);
    uchar4 u;
    u.x = (uint8_t)bi[0]; u.y = (uint8_t)bi[1]; u.z = (uint8_t)bi[2]; u.w = (uint8_t)bi[3];
    *reinterpret_cast<uchar4*>(idx + row * C + 4 * c4) = u;
  }
}

// The encoder's last BasicBlock apply with the adaptive average pool over its npos positions folded in
// (resnet.py:55-57 then :59-60): thread = (sample n, 4 channels), looping the positions — out as k_bn_apply
// writes it (the backward reads it) and pooled[n] = (sum over p in order) / npos, as k_avgpool_fwd computes it.
// One launch instead of apply + pool at the tail of each encoder's forward.
template <int RES, bool RELU, bool EVAL>
__global__ __launch_bounds__(256) void k_bn_apply_pool(int npos, int N, int C, const float* __restrict__ y,
                                                       const float* __restrict__ mean, const float* __restrict__ inv,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       const float* __restrict__ res, const float* __restrict__ mean2,
                                                       const float* __restrict__ inv2, const float* __restrict__ gamma2,
                                                       const float* __restrict__ beta2, float eps, float* __restrict__ out,
                                                       float* __restrict__ pooled) {
  const int L = C >> 2;
  const long long total = (long long)N * L, plane = (long long)N * C;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c4 = (int)(i % L);
    f32x4 mu = ld4(mean + 4 * c4), iv = ld4(inv + 4 * c4);
    if (EVAL) {
#pragma unroll
      for (int j = 0; j < 4; ++j) iv[j] = 1.0f / sqrtf(iv[j] + eps);
    }
    const f32x4 sc = ld4(gamma + 4 * c4) * iv;
    const f32x4 sf = ld4(beta + 4 * c4) - mu * sc;
    f32x4 sc2 = {0.f, 0.f, 0.f, 0.f}, sf2 = sc2;
    if (RES == 2) {
      f32x4 mu2 = ld4(mean2 + 4 * c4), iv2 = ld4(inv2 + 4 * c4);
      if (EVAL) {
#pragma unroll
        for (int j = 0; j < 4; ++j) iv2[j] = 1.0f / sqrtf(iv2[j] + eps);
      }
      sc2 = ld4(gamma2 + 4 * c4) * iv2;
      sf2 = ld4(beta2 + 4 * c4) - mu2 * sc2;
    }
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < npos; ++p) {
      const long long off = p * plane + 4 * i;
      const f32x4 v = ld4(y + off);
      f32x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = fmaf(v[j], sc[j], sf[j]);
      if (RES == 1) {
        o += ld4(res + off);
      } else if (RES == 2) {
        const f32x4 v2 = ld4(res + off);
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] += fmaf(v2[j], sc2[j], sf2[j]);
      }
      if (RELU) {
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = relu_f(o[j]);
      }
      st4(out + off, o);
      s += o;
    }
    f32x4 q;
#pragma unroll
    for (int j = 0; j < 4; ++j) q[j] = s[j] / (float)npos;
    st4(pooled + 4 * i, q);
  }
}

// Transposed-store helper of the tiled kernels: a [64 rows x 64 channels] tile staged in LDS
// (tile[row][65]) is written as dst[c][ld_t] rows-contiguous (the wgrad operand layout) with 16-byte
// stores, 4 consecutive threads per channel.  Requires (m % 4 == 0) and 16-byte aligned dst/ld_t.
TSPM_DEV void store_tile_t(const float (*tile)[65], long long r0, long long M, int c0, int C, float* dst,
                           long long ld_t) {
  const int t = threadIdx.x;
  const int cl = t >> 2, qq = t & 3;
  const int c = c0 + cl;
  if (c >= C) return;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int rl = qq * 16 + 4 * k;
    if (r0 + rl < M) {
      const f32x4 v = {tile[rl][cl], tile[rl + 1][cl], tile[rl + 2][cl], tile[rl + 3][cl]};
      st4(dst + (long long)c * ld_t + r0 + rl, v);
    }
  }
}

// Tiled train-mode apply: a workgroup owns [64 rows x 64 channels]; writes out (HWNC) and out_t
// ([C][ld_t]) through an LDS transpose.
template <int RES, bool RELU>
__global__ __launch_bounds__(256) void k_bn_apply_t(long long M, int C, const float* __restrict__ y,
                                                    const float* __restrict__ mean, const float* __restrict__ inv,
                                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                                    const float* __restrict__ res, const float* __restrict__ mean2,
                                                    const float* __restrict__ inv2, const float* __restrict__ gamma2,
                                                    const float* __restrict__ beta2, float* __restrict__ out,
                                                    float* __restrict__ out_t, long long ld_t) {
  __shared__ float tile[64][65];
  const int t = threadIdx.x, l16 = t & 15, rg = t >> 4;
  const int c4 = blockIdx.y * 16 + l16;
  const bool cok = 4 * c4 < C;
  const long long r0 = (long long)blockIdx.x * 64;
  f32x4 sc = {0.f, 0.f, 0.f, 0.f}, sf = sc, sc2 = sc, sf2 = sc;
  if (cok) {
    sc = ld4(gamma + 4 * c4) * ld4(inv + 4 * c4);
    sf = ld4(beta + 4 * c4) - ld4(mean + 4 * c4) * sc;
    if (RES == 2) {
      sc2 = ld4(gamma2 + 4 * c4) * ld4(inv2 + 4 * c4);
      sf2 = ld4(beta2 + 4 * c4) - ld4(mean2 + 4 * c4) * sc2;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rl = rg + 16 * i;
    const long long row = r0 + rl;
    f32x4 o = {0.f, 0.f, 0.f, 0.f};
    if (cok && row < M) {
      const long long off = row * C + 4 * c4;
      const f32x4 v = ld4(y + off);
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = fmaf(v[j], sc[j], sf[j]);
      if (RES == 1) o += ld4(res + off);
      if (RES == 2) {
        const f32x4 v2 = ld4(res + off);
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] += fmaf(v2[j], sc2[j], sf2[j]);
      }
      if (RELU) {
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = relu_f(o[j]);
      }
      st4(out + off, o);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) tile[rl][4 * l16 + j] = o[j];
  }
  __syncthreads();
  store_tile_t(tile, r0, M, blockIdx.y * 64, C, out_t, ld_t);
}

// ------------------------------------------------------------------------------------------------
// backward: partial sums of g', g'*(y-mean) [, g'*(y2-mean2)] over [rows x 64 channels] tiles
// ------------------------------------------------------------------------------------------------
// backward pass 1: partial sums of g', g'*(y-mean) [, g'*(y2-mean2)] over [rows x 64 channels]
// tiles (rows in batches of 4 per thread so their loads are in flight together).  An in-launch
// merge by the last workgroup was measured slower than the parallel pass 2 below (the merge of
// >= 64 tiles per channel block serialises on one CU), so pass 2 stays a launch.
// RG row groups of 16 lanes: 16 (256 threads), or 64 (1,024 threads) for the long tiles of the 64-channel
// layers, whose partial pass has only 64 workgroups — four times the loads in flight per CU.
// ------------------------------------------------------------------------------------------------
// Where the BN backward reads its incoming gradient g[row][4 channels] (row = (h*W + w)*N + n, HWNC):
//   GDense — a materialised [M, C] tensor (every BN of the blocks);
//   GAvg   — the adaptive average pool's backward folded in (the encoder's last BN): g = gp[n] / npos, exactly
//            k_avgpool_bwd's value, so the pooled-gradient broadcast is never written (one launch fewer);
//   GMax   — the stem's MaxPool2d(3, 2, 1) backward folded in: g = the sum, over the <= 2 x 2 pool windows that
//            contain the element and chose it (argmax tap), of the pooled gradient, in k_maxpool_bwd's order
//            (windows p then q ascending) — bitwise that kernel's dx, never written (one launch and a 25 MB
//            write + two reads fewer on the audio stem).
// Round 5 (tspm_bn_bwd_src).  Row decodes use a float reciprocal corrected by one step (rows < 2^24 are exact
// floats), not integer divisions.
TSPM_DEV int fdiv_row(long long a, int b, float inv_b) {
  int q = (int)((float)a * inv_b);
  q -= (long long)q * b > a ? 1 : 0;
  q += (long long)(q + 1) * b <= a ? 1 : 0;
  return q;
}
struct GDense {
  const float* g;
  int C;
  TSPM_DEV f32x4 at(long long row, int c4) const { return ld4(g + row * C + 4 * c4); }
};
struct GAvg {
  const float* gp;
  int ldg, N, npos;
  float invN;
  TSPM_DEV f32x4 at(long long row, int c4) const {
    const int q = fdiv_row(row, N, invN);
    const int n = (int)(row - (long long)q * N);
    const f32x4 v = ld4(gp + (long long)n * ldg + 4 * c4);
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = v[j] / (float)npos;
    return o;
  }
};
struct GMax {  // 3x3, stride 2, pad 1 (the ResNet stem pool)
  const float* gp;
  const uint8_t* idx;
  int N, W, P, Q, C;
  float invN, invW;
  TSPM_DEV f32x4 at(long long row, int c4) const {
    const int pos = fdiv_row(row, N, invN);
    const int n = (int)(row - (long long)pos * N);
    const int h = fdiv_row(pos, W, invW), w = pos - h * W;
    const int p_lo = max(0, (h + 1 - 3 + 2) / 2), p_hi = min(P - 1, (h + 1) / 2);
    const int q_lo = max(0, (w + 1 - 3 + 2) / 2), q_hi = min(Q - 1, (w + 1) / 2);
    uchar4 u4[4];
    f32x4 g4[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int pc = min(p_lo + (t >> 1), P - 1), qc = min(q_lo + (t & 1), Q - 1);
      const long long o = (((long long)pc * Q + qc) * N + n) * C + 4 * c4;
      u4[t] = *reinterpret_cast<const uchar4*>(idx + o);
      g4[t] = ld4(gp + o);
    }
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int p = p_lo + (t >> 1), q = q_lo + (t & 1);
      const int kh = h - (p * 2 - 1), kw = w - (q * 2 - 1);
      if (p > p_hi || q > q_hi || kh < 0 || kh >= 3 || kw < 0 || kw >= 3) continue;
      const int tap = kh * 3 + kw;
      if (u4[t].x == tap) acc[0] += g4[t][0];
      if (u4[t].y == tap) acc[1] += g4[t][1];
      if (u4[t].z == tap) acc[2] += g4[t][2];
      if (u4[t].w == tap) acc[3] += g4[t][3];
    }
    return acc;
  }
};

template <bool HAS_OUT, bool TWO, int U, int RG = kRowGroups, class GS = GDense>
__global__ __launch_bounds__(16 * RG) void k_bn_bwd_partial(long long M, int C, GS gs,
                                                        const float* __restrict__ out, const float* __restrict__ y,
                                                        const float* __restrict__ mean, const float* __restrict__ y2,
                                                        const float* __restrict__ mean2, long long rows_per_block,
                                                        float* __restrict__ part) {
  __shared__ f32x4 sh[3][16 * RG];
  const int t = threadIdx.x;
  const int lane = t & 15, rg = t >> 4;
  const int c4 = blockIdx.y * 16 + lane;
  const bool cok = 4 * c4 < C;
  const long long r_begin = blockIdx.x * rows_per_block;
  const long long r_end = min(M, r_begin + rows_per_block);
  f32x4 sg = {0.f, 0.f, 0.f, 0.f}, sx = sg, sx2 = sg;
  if (cok) {
    const f32x4 mu = ld4(mean + 4 * c4);
    const f32x4 mu2 = TWO ? ld4(mean2 + 4 * c4) : f32x4{0.f, 0.f, 0.f, 0.f};
    // U rows per batch: all their loads in flight together.  The loads are unconditional (rows past the
    // tile re-read its last row and are masked out of the sums): with a conditional load per row the
    // compiler waited for each row's loads before the next row's (vmcnt(1)/(2) after every row: ~21 GB/s
    // per CU on the 64-workgroup audio stem pass, 54.6 us for 74 MB)
    for (long long rb = r_begin + rg; rb < r_end; rb += U * RG) {
      f32x4 gv[U], ov[U], yv[U], y2v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const long long row = min(rb + u * RG, r_end - 1);
        const long long off = row * C + 4 * c4;
        gv[u] = gs.at(row, c4);
        if (HAS_OUT) ov[u] = ld4(out + off);
        yv[u] = ld4(y + off);
        if (TWO) y2v[u] = ld4(y2 + off);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool in = rb + u * RG < r_end;
        f32x4 gm;
#pragma unroll
        for (int j = 0; j < 4; ++j) gm[j] = (in && (!HAS_OUT || ov[u][j] > 0.f)) ? gv[u][j] : 0.f;
        sg += gm;
        sx += gm * (in ? yv[u] - mu : f32x4{0.f, 0.f, 0.f, 0.f});
        if (TWO) sx2 += gm * (in ? y2v[u] - mu2 : f32x4{0.f, 0.f, 0.f, 0.f});
      }
    }
  }
  sh[0][t] = sg;
  sh[1][t] = sx;
  if (TWO) sh[2][t] = sx2;
  __syncthreads();
  const long long plane = (long long)gridDim.x * C;
  if (rg == 0 && cok) {
    for (int k = 1; k < RG; ++k) {
      sg += sh[0][k * 16 + lane];
      sx += sh[1][k * 16 + lane];
      if (TWO) sx2 += sh[2][k * 16 + lane];
    }
    st4(part + (long long)blockIdx.x * C + 4 * c4, sg);
    st4(part + plane + (long long)blockIdx.x * C + 4 * c4, sx);
    if (TWO) st4(part + 2 * plane + (long long)blockIdx.x * C + 4 * c4, sx2);
  }
}

// coef layout [6][C]: ca, cb, cm (first BN), ca2, cb2, cm2 (second BN); 8 channels x 32 groups
__global__ __launch_bounds__(256) void k_bn_bwd_final(long long M, int C, int G, int two, const float* __restrict__ part,
                                                      const float* __restrict__ inv, const float* __restrict__ gamma,
                                                      const float* __restrict__ inv2, const float* __restrict__ gamma2,
                                                      float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                      float* __restrict__ dgamma2, float* __restrict__ dbeta2,
                                                      float* __restrict__ coef) {
  __shared__ double red[3][256];
  const int t = threadIdx.x;
  const int cl = t & 7, gg = t >> 3;
  const int c = blockIdx.x * 8 + cl;
  const bool cok = c < C;
  const long long plane = (long long)G * C;
  double sg = 0.0, sx = 0.0, sx2 = 0.0;
  if (cok)
    for (int g = gg; g < G; g += 32) {
      sg += (double)part[(long long)g * C + c];
      sx += (double)part[plane + (long long)g * C + c];
      if (two) sx2 += (double)part[2 * plane + (long long)g * C + c];
    }
  red[0][t] = sg;
  red[1][t] = sx;
  red[2][t] = sx2;
  __syncthreads();
  for (int w = 16; w > 0; w >>= 1) {
    if (gg < w) {
      red[0][t] += red[0][t + w * 8];
      red[1][t] += red[1][t + w * 8];
      red[2][t] += red[2][t + w * 8];
    }
    __syncthreads();
  }
  if (gg != 0 || !cok) return;
  sg = red[0][cl];
  sx = red[1][cl];
  sx2 = red[2][cl];
  const double n = (double)M;
  {
    const double iv = inv[c], ga = gamma[c];
    const double dg = sx * iv;
    if (dgamma) dgamma[c] = (float)dg;
    if (dbeta) dbeta[c] = (float)sg;
    const double ca = ga * iv;
    coef[c] = (float)ca;
    coef[C + c] = (float)(ca * iv * dg / n);
    coef[2 * C + c] = (float)(ca * sg / n);
  }
  if (two) {
    const double iv = inv2[c], ga = gamma2[c];
    const double dg = sx2 * iv;
    if (dgamma2) dgamma2[c] = (float)dg;
    if (dbeta2) dbeta2[c] = (float)sg;
    const double ca = ga * iv;
    coef[3 * C + c] = (float)ca;
    coef[4 * C + c] = (float)(ca * iv * dg / n);
    coef[5 * C + c] = (float)(ca * sg / n);
  }
}

// Backward apply with the per-channel merge folded in (no separate final launch): workgroup =
// [rows x 64 channels] (16 float4 lanes x 16 row groups).  Prologue: merge the G partial tiles of
// its 64 channels in double, in a fixed order (thread (lane, rg) sums tiles rg, rg+16, ... then a
// fixed 16-way LDS reduction), so every workgroup derives bitwise the same coefficients; the
// workgroups of row block 0 also write dgamma / dbeta.  Body: dy = ca*g' - cm - cb*(y - mean).
// G is kept <= kMergeTiles by the host, so the merge is <= 3 * kMergeTiles / 16 float4 loads per thread, all
// in flight together.
#ifndef TSPM_MERGE_TILES
#define TSPM_MERGE_TILES 128
#endif
constexpr int kMergeTiles = TSPM_MERGE_TILES;
template <bool HAS_OUT, bool TWO, bool DRES, class GS = GDense>
__global__ __launch_bounds__(256) void k_bn_bwd_apply_m(long long M, int C, int G, const float* __restrict__ part,
                                                        const float* __restrict__ inv, const float* __restrict__ gamma,
                                                        const float* __restrict__ inv2, const float* __restrict__ gamma2,
                                                        float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                        float* __restrict__ dgamma2, float* __restrict__ dbeta2,
                                                        GS gs, const float* __restrict__ out,
                                                        const float* __restrict__ y, const float* __restrict__ mean,
                                                        const float* __restrict__ y2, const float* __restrict__ mean2,
                                                        long long rows_per_block, float* __restrict__ dy,
                                                        float* __restrict__ dy2, float* __restrict__ dres) {
  __shared__ double red[3][4][256];
  __shared__ f32x4 scoef[6][16];
  const int t = threadIdx.x;
  const int lane = t & 15, rg = t >> 4;
  const int c4 = blockIdx.y * 16 + lane;
  const bool cok = 4 * c4 < C;
  const long long plane = (long long)G * C;
  {
    double a[3][4] = {};
    // G <= kMergeTiles: one batch of loads; more tiles (tspm_bn_bwd_apply_part, round 6) in further batches of
    // kMergeTiles — thread (lane, rg) still sums tiles rg, rg + 16, ... in order
    for (int base = 0; cok && base < G; base += kMergeTiles) {
      f32x4 v[kMergeTiles / 16][3];
#pragma unroll
      for (int u = 0; u < kMergeTiles / 16; ++u) {  // unconditional loads (tile clamped), then masked
        const int gt = base + rg + 16 * u;
        const bool ok = gt < G;
        const long long off = (long long)min(gt, G - 1) * C + 4 * c4;
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        const f32x4 l0 = ld4(part + off), l1 = ld4(part + plane + off);
        v[u][0] = ok ? l0 : z;
        v[u][1] = ok ? l1 : z;
        if constexpr (TWO) {
          const f32x4 l2 = ld4(part + 2 * plane + off);
          v[u][2] = ok ? l2 : z;
        } else {
          v[u][2] = z;
        }
      }
#pragma unroll
      for (int u = 0; u < kMergeTiles / 16; ++u)
#pragma unroll
        for (int k = 0; k < 3; ++k)
#pragma unroll
          for (int j = 0; j < 4; ++j) a[k][j] += (double)v[u][k][j];
    }
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) red[k][j][t] = a[k][j];
  }
  __syncthreads();
  if (rg == 0 && cok) {
    double sg[4], sx[4], sx2[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      sg[j] = red[0][j][lane];
      sx[j] = red[1][j][lane];
      sx2[j] = red[2][j][lane];
    }
    for (int k = 1; k < 16; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sg[j] += red[0][j][k * 16 + lane];
        sx[j] += red[1][j][k * 16 + lane];
        sx2[j] += red[2][j][k * 16 + lane];
      }
    const double n = (double)M;
    f32x4 ca, cb, cm, ca2 = {0.f, 0.f, 0.f, 0.f}, cb2 = ca2, cm2 = ca2;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = 4 * c4 + j;
      const double iv = inv[c], ga = gamma[c];
      const double dg = sx[j] * iv;
      const double a_ = ga * iv;
      ca[j] = (float)a_;
      cb[j] = (float)(a_ * iv * dg / n);
      cm[j] = (float)(a_ * sg[j] / n);
      if (blockIdx.x == 0) {
        if (dgamma) dgamma[c] = (float)dg;
        if (dbeta) dbeta[c] = (float)sg[j];
      }
      if (TWO) {
        const double iv2 = inv2[c], ga2 = gamma2[c];
        const double dg2 = sx2[j] * iv2;
        const double a2 = ga2 * iv2;
        ca2[j] = (float)a2;
        cb2[j] = (float)(a2 * iv2 * dg2 / n);
        cm2[j] = (float)(a2 * sg[j] / n);
        if (blockIdx.x == 0) {
          if (dgamma2) dgamma2[c] = (float)dg2;
          if (dbeta2) dbeta2[c] = (float)sg[j];
        }
      }
    }
    scoef[0][lane] = ca; scoef[1][lane] = cb; scoef[2][lane] = cm;
    scoef[3][lane] = ca2; scoef[4][lane] = cb2; scoef[5][lane] = cm2;
  }
  __syncthreads();
  if (!cok) return;
  const f32x4 ca = scoef[0][lane], cb = scoef[1][lane], cm = scoef[2][lane];
  const f32x4 ca2 = scoef[3][lane], cb2 = scoef[4][lane], cm2 = scoef[5][lane];
  const f32x4 mu = ld4(mean + 4 * c4);
  const f32x4 mu2 = TWO ? ld4(mean2 + 4 * c4) : f32x4{0.f, 0.f, 0.f, 0.f};
  const long long r_begin = blockIdx.x * rows_per_block;
  const long long r_end = min(M, r_begin + rows_per_block);
  constexpr int U = 4;
  for (long long rb = r_begin + rg; rb < r_end; rb += U * kRowGroups) {
    f32x4 gv[U], yv[U], y2v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long row = min(rb + u * kRowGroups, r_end - 1);
      const long long off = row * C + 4 * c4;
      gv[u] = gs.at(row, c4);
      if (HAS_OUT) {
        const f32x4 ov = ld4(out + off);
#pragma unroll
        for (int j = 0; j < 4; ++j) gv[u][j] = ov[j] > 0.f ? gv[u][j] : 0.f;
      }
      yv[u] = ld4(y + off);
      if (TWO) y2v[u] = ld4(y2 + off);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long row = rb + u * kRowGroups;
      if (row < r_end) {
        const long long off = row * C + 4 * c4;
        st4(dy + off, ca * gv[u] - cm - cb * (yv[u] - mu));
        if (TWO) st4(dy2 + off, ca2 * gv[u] - cm2 - cb2 * (y2v[u] - mu2));
        if (DRES) st4(dres + off, gv[u]);
      }
    }
  }
}

// Tiled backward apply: [64 rows x 64 channels] per workgroup; also writes dy_t (and dy2_t) in
// the transposed wgrad operand layout through LDS.
template <bool HAS_OUT, bool TWO, bool DRES>
__global__ __launch_bounds__(256) void k_bn_bwd_apply_t(long long M, int C, const float* __restrict__ g,
                                                        const float* __restrict__ out, const float* __restrict__ y,
                                                        const float* __restrict__ mean, const float* __restrict__ y2,
                                                        const float* __restrict__ mean2, const float* __restrict__ coef,
                                                        float* __restrict__ dy, float* __restrict__ dy2,
                                                        float* __restrict__ dres, float* __restrict__ dy_t,
                                                        float* __restrict__ dy2_t, long long ld_t) {
  __shared__ float tile[TWO ? 2 : 1][64][65];
  const int t = threadIdx.x, l16 = t & 15, rg = t >> 4;
  const int c4 = blockIdx.y * 16 + l16;
  const bool cok = 4 * c4 < C;
  const long long r0 = (long long)blockIdx.x * 64;
  f32x4 ca = {0.f, 0.f, 0.f, 0.f}, cb = ca, cm = ca, mu = ca, ca2 = ca, cb2 = ca, cm2 = ca, mu2 = ca;
  if (cok) {
    ca = ld4(coef + 4 * c4); cb = ld4(coef + C + 4 * c4); cm = ld4(coef + 2 * C + 4 * c4);
    mu = ld4(mean + 4 * c4);
    if (TWO) {
      ca2 = ld4(coef + 3 * C + 4 * c4); cb2 = ld4(coef + 4 * C + 4 * c4); cm2 = ld4(coef + 5 * C + 4 * c4);
      mu2 = ld4(mean2 + 4 * c4);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rl = rg + 16 * i;
    const long long row = r0 + rl;
    f32x4 o = {0.f, 0.f, 0.f, 0.f}, o2 = o;
    if (cok && row < M) {
      const long long off = row * C + 4 * c4;
      f32x4 gv = ld4(g + off);
      if (HAS_OUT) {
        const f32x4 ov = ld4(out + off);
#pragma unroll
        for (int j = 0; j < 4; ++j) gv[j] = ov[j] > 0.f ? gv[j] : 0.f;
      }
      o = ca * gv - cm - cb * (ld4(y + off) - mu);
      st4(dy + off, o);
      if (TWO) {
        o2 = ca2 * gv - cm2 - cb2 * (ld4(y2 + off) - mu2);
        st4(dy2 + off, o2);
      }
      if (DRES) st4(dres + off, gv);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      tile[0][rl][4 * l16 + j] = o[j];
      if (TWO) tile[TWO ? 1 : 0][rl][4 * l16 + j] = o2[j];
    }
  }
  __syncthreads();
  store_tile_t(tile[0], r0, M, blockIdx.y * 64, C, dy_t, ld_t);
  if (TWO && dy2_t) store_tile_t(tile[TWO ? 1 : 0], r0, M, blockIdx.y * 64, C, dy2_t, ld_t);
}

int ew_blocks(long long n4) {
  long long b = cdiv64(n4, 256);
  if (b > 2048) b = 2048;
  return (int)(b < 1 ? 1 : b);
}

bool c_ok(int C) { return C >= 4 && C % 4 == 0; }

}  // namespace

extern "C" int tspm_bn_finalize(int64_t m, int32_t c, int32_t ntiles, int64_t rows_per_tile, const float* partial,
                                float* running_mean, float* running_var, float momentum, float eps, float* save_mean,
                                float* save_invstd, tspm_stream_t stream) {
  if (m <= 0 || c <= 0 || ntiles <= 0 || rows_per_tile <= 0 || !partial || !save_mean || !save_invstd)
    return TSPM_ERR_INVALID;
  if ((long long)ntiles * rows_per_tile < m || (long long)(ntiles - 1) * rows_per_tile >= m) return TSPM_ERR_INVALID;
  const hipStream_t st = static_cast<hipStream_t>(stream);
  const int ch = bn_wide() ? (c <= 64 ? 1 : c <= 128 ? 2 : kFinChan) : kFinChan;
#define BN_FIN(CH)                                                                                               \
  hipLaunchKernelGGL((k_bn_finalize<CH>), dim3(cdiv(c, CH)), dim3(256), 0, st, (long long)m, c, ntiles,          \
                     (long long)rows_per_tile, partial, running_mean, running_var, momentum, eps, save_mean, save_invstd)
  if (ch == 1) BN_FIN(1);
  else if (ch == 2) BN_FIN(2);
  else BN_FIN(kFinChan);
#undef BN_FIN
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" size_t tspm_bn_stats_workspace(int64_t m, int32_t c) {
  if (m <= 0 || !c_ok(c)) return 0;
  return (size_t)3 * row_blocks(m, c) * c * sizeof(float);
}

extern "C" int tspm_bn_stats(int64_t m, int32_t c, const float* y, int32_t nslab, int64_t slab_stride, float* y_out,
                             float* running_mean, float* running_var, float momentum, float eps, float* save_mean,
                             float* save_invstd, void* ws, size_t ws_bytes, tspm_stream_t stream) {
  if (m <= 0 || !c_ok(c) || !y || nslab < 1 || !save_mean || !save_invstd) return TSPM_ERR_INVALID;
  if (nslab > 1 && !y_out) return TSPM_ERR_INVALID;
  if (!ws || ws_bytes < tspm_bn_stats_workspace(m, c)) return TSPM_ERR_WORKSPACE;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int G = row_blocks(m, c);
  const long long rpb = cdiv64(m, G);
  const int Greal = (int)cdiv64(m, rpb);
  float* part = static_cast<float*>(ws);
  hipLaunchKernelGGL(k_bn_stats_partial, dim3(Greal, cdiv(c, kChanPerBlock)), dim3(256), 0, st, (long long)m, c, y,
                     nslab, (long long)slab_stride, y_out, rpb, part);
  TSPM_LAUNCH_CHECK();
  return tspm_bn_finalize(m, c, Greal, rpb, part, running_mean, running_var, momentum, eps, save_mean, save_invstd,
                          stream);
}

#define BN_APPLY_LAUNCH(RES, RELU, EVAL)                                                                   \
  hipLaunchKernelGGL((k_bn_apply<RES, RELU, EVAL>), dim3(ew_blocks(n4)), dim3(256), 0, st, n4, c, y, mean, \
                     inv, gamma, beta, res, mean2, inv2, gamma2, beta2, eps, out)

static bool t_ok(long long m, const float* p, long long ld_t) {
  return m % 4 == 0 && ld_t >= m && ld_t % 4 == 0 && (reinterpret_cast<uintptr_t>(p) & 15) == 0;
}

#define BN_APPLY_T_LAUNCH(RES, RELU)                                                                          \
  hipLaunchKernelGGL((k_bn_apply_t<RES, RELU>), tgrid, dim3(256), 0, st, (long long)m, c, y, mean, inv, gamma, \
                     beta, res, mean2, inv2, gamma2, beta2, out, out_t, (long long)ld_t)

static int bn_apply_common(int64_t m, int32_t c, const float* y, const float* mean, const float* inv,
                           const float* gamma, const float* beta, int32_t res_mode, const float* res,
                           const float* mean2, const float* inv2, const float* gamma2, const float* beta2,
                           int32_t relu, float* out, float* out_t, int64_t ld_t, bool eval, float eps,
                           tspm_stream_t stream) {
  if (m <= 0 || !c_ok(c) || !y || !mean || !inv || !gamma || !beta || !out) return TSPM_ERR_INVALID;
  if (res_mode < 0 || res_mode > 2) return TSPM_ERR_INVALID;
  if (res_mode >= 1 && !res) return TSPM_ERR_INVALID;
  if (res_mode == 2 && (!mean2 || !inv2 || !gamma2 || !beta2)) return TSPM_ERR_INVALID;
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (out_t) {
    if (eval || !t_ok(m, out_t, ld_t)) return TSPM_ERR_INVALID;
    const dim3 tgrid((unsigned)cdiv64(m, 64), cdiv(c, 64));
    const bool r = relu != 0;
    if (res_mode == 0) { if (r) BN_APPLY_T_LAUNCH(0, true); else BN_APPLY_T_LAUNCH(0, false); }
    else if (res_mode == 1) { if (r) BN_APPLY_T_LAUNCH(1, true); else BN_APPLY_T_LAUNCH(1, false); }
    else { if (r) BN_APPLY_T_LAUNCH(2, true); else BN_APPLY_T_LAUNCH(2, false); }
    TSPM_LAUNCH_CHECK();
    return TSPM_OK;
  }
  const long long n4 = (long long)m * c / 4;
  const bool r = relu != 0;
  if (!eval) {
    if (res_mode == 0) { if (r) BN_APPLY_LAUNCH(0, true, false); else BN_APPLY_LAUNCH(0, false, false); }
    else if (res_mode == 1) { if (r) BN_APPLY_LAUNCH(1, true, false); else BN_APPLY_LAUNCH(1, false, false); }
    else { if (r) BN_APPLY_LAUNCH(2, true, false); else BN_APPLY_LAUNCH(2, false, false); }
  } else {
    if (res_mode == 0) { if (r) BN_APPLY_LAUNCH(0, true, true); else BN_APPLY_LAUNCH(0, false, true); }
    else if (res_mode == 1) { if (r) BN_APPLY_LAUNCH(1, true, true); else BN_APPLY_LAUNCH(1, false, true); }
    else { if (r) BN_APPLY_LAUNCH(2, true, true); else BN_APPLY_LAUNCH(2, false, true); }
  }
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_bn_apply(int64_t m, int32_t c, const float* y, const float* mean, const float* invstd,
                             const float* gamma, const float* beta, int32_t res_mode, const float* res,
                             const float* res_mean, const float* res_invstd, const float* res_gamma,
                             const float* res_beta, int32_t relu, float* out, float* out_t, int64_t ld_t,
                             tspm_stream_t stream) {
  return bn_apply_common(m, c, y, mean, invstd, gamma, beta, res_mode, res, res_mean, res_invstd, res_gamma,
                         res_beta, relu, out, out_t, ld_t, false, 0.f, stream);
}

extern "C" int tspm_bn_apply_merge(int64_t m, int32_t c, int32_t tiles, int64_t rows_per_tile, const float* partial,
                                   float* running_mean, float* running_var, float momentum, float eps,
                                   float* save_mean, float* save_invstd, const float* y, const float* gamma,
                                   const float* beta, int32_t res_mode, const float* res, const float* res_mean,
                                   const float* res_invstd, const float* res_gamma, const float* res_beta,
                                   int32_t relu, float* out, tspm_stream_t stream) {
  if (m <= 0 || !c_ok(c) || c % 16 || tiles < 1 || tiles > kApplyMergeTiles || rows_per_tile <= 0 || !partial ||
      !save_mean || !save_invstd || !y || !gamma || !beta || !out)
    return TSPM_ERR_INVALID;
  if ((long long)tiles * rows_per_tile < m || (long long)(tiles - 1) * rows_per_tile >= m) return TSPM_ERR_INVALID;
  if (res_mode < 0 || res_mode > 2 || (res_mode >= 1 && !res)) return TSPM_ERR_INVALID;
  if (res_mode == 2 && (!res_mean || !res_invstd || !res_gamma || !res_beta)) return TSPM_ERR_INVALID;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int cblk = c / 16;
  long long rb = cdiv64(m, std::max(1, 128 / cblk));  // ~128 workgroups, >= 64 rows each
  if (rb < 64) rb = 64;
  const dim3 grid((unsigned)cdiv64(m, rb), cblk);
#define BN_AM(RES, RELU)                                                                                             \
  hipLaunchKernelGGL((k_bn_apply_merge<RES, RELU>), grid, dim3(256), 0, st, (long long)m, c, tiles,                  \
                     (long long)rows_per_tile, partial, running_mean, running_var, momentum, eps, save_mean,          \
                     save_invstd, y, gamma, beta, res, res_mean, res_invstd, res_gamma, res_beta, rb, out)
  const bool r = relu != 0;
  if (res_mode == 0) { if (r) BN_AM(0, true); else BN_AM(0, false); }
  else if (res_mode == 1) { if (r) BN_AM(1, true); else BN_AM(1, false); }
  else { if (r) BN_AM(2, true); else BN_AM(2, false); }
#undef BN_AM
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_bn_apply_eval(int64_t m, int32_t c, const float* y, const float* running_mean,
                                  const float* running_var, float eps, const float* gamma, const float* beta,
                                  int32_t res_mode, const float* res, const float* res_rmean, const float* res_rvar,
                                  const float* res_gamma, const float* res_beta, int32_t relu, float* out,
                                  tspm_stream_t stream) {
  return bn_apply_common(m, c, y, running_mean, running_var, gamma, beta, res_mode, res, res_rmean, res_rvar,
                         res_gamma, res_beta, relu, out, nullptr, 0, true, eps, stream);
}

#define BN_APPLY_POOL_LAUNCH(RES, RELU, EVAL)                                                               \
  hipLaunchKernelGGL((k_bn_apply_pool<RES, RELU, EVAL>), dim3(ew_blocks(total)), dim3(256), 0, st, npos, n, c, y, \
                     mean, inv, gamma, beta, res, mean2, inv2, gamma2, beta2, eps, out, pooled)

extern "C" int tspm_bn_apply_pool(int32_t npos, int32_t n, int32_t c, const float* y, const float* mean,
                                  const float* inv, const float* gamma, const float* beta, int32_t res_mode,
                                  const float* res, const float* mean2, const float* inv2, const float* gamma2,
                                  const float* beta2, int32_t relu, int32_t eval, float eps, float* out,
                                  float* pooled, tspm_stream_t stream) {
  if (npos <= 0 || n <= 0 || !c_ok(c) || !y || !mean || !inv || !gamma || !beta || !out || !pooled)
    return TSPM_ERR_INVALID;
  if (res_mode < 0 || res_mode > 2) return TSPM_ERR_INVALID;
  if (res_mode >= 1 && !res) return TSPM_ERR_INVALID;
  if (res_mode == 2 && (!mean2 || !inv2 || !gamma2 || !beta2)) return TSPM_ERR_INVALID;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const long long total = (long long)n * c / 4;
  const bool r = relu != 0;
  if (!eval) {
    if (res_mode == 0) { if (r) BN_APPLY_POOL_LAUNCH(0, true, false); else BN_APPLY_POOL_LAUNCH(0, false, false); }
    else if (res_mode == 1) { if (r) BN_APPLY_POOL_LAUNCH(1, true, false); else BN_APPLY_POOL_LAUNCH(1, false, false); }
    else { if (r) BN_APPLY_POOL_LAUNCH(2, true, false); else BN_APPLY_POOL_LAUNCH(2, false, false); }
  } else {
    if (res_mode == 0) { if (r) BN_APPLY_POOL_LAUNCH(0, true, true); else BN_APPLY_POOL_LAUNCH(0, false, true); }
    else if (res_mode == 1) { if (r) BN_APPLY_POOL_LAUNCH(1, true, true); else BN_APPLY_POOL_LAUNCH(1, false, true); }
    else { if (r) BN_APPLY_POOL_LAUNCH(2, true, true); else BN_APPLY_POOL_LAUNCH(2, false, true); }
  }
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_bn_apply_maxpool(int32_t n, int32_t h, int32_t w, int32_t c, const float* y, const float* mean,
                                     const float* inv, const float* gamma, const float* beta, int32_t eval, float eps,
                                     float* out, float* pooled, uint8_t* idx, int32_t p, int32_t q,
                                     tspm_stream_t stream) {
  if (n <= 0 || h <= 0 || w <= 0 || !c_ok(c) || !y || !mean || !inv || !gamma || !beta || !pooled || !idx)
    return TSPM_ERR_INVALID;
  if (p != (h - 1) / 2 + 1 || q != (w - 1) / 2 + 1) return TSPM_ERR_INVALID;
  const long long total = (long long)p * q * n * (c / 4);
  const dim3 grid((unsigned)std::min<long long>(cdiv64(total, 256), 8192));
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (eval)
    hipLaunchKernelGGL(k_bn_apply_maxpool<true>, grid, dim3(256), 0, st, n, h, w, c, p, q, y, mean, inv, gamma, beta,
                       eps, out, pooled, idx);
  else
    hipLaunchKernelGGL(k_bn_apply_maxpool<false>, grid, dim3(256), 0, st, n, h, w, c, p, q, y, mean, inv, gamma, beta,
                       eps, out, pooled, idx);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" size_t tspm_bn_bwd_workspace(int64_t m, int32_t c) {
  if (m <= 0 || !c_ok(c)) return 0;
  return ((size_t)3 * row_blocks(m, c) * c + 6 * (size_t)c) * sizeof(float);
}

namespace {
// The two launches of the merged BN backward (partial sums, then the apply with the merge in its prologue) for
// a gradient source GS; returns false when the caller must take the transposed-copy path instead (dy_t).
template <class GS>
int bn_bwd_merged(int64_t m, int32_t c, const GS& gs, bool gather, const float* out, const float* y,
                  const float* mean, const float* invstd, const float* gamma, float* dgamma, float* dbeta, float* dy,
                  const float* y2, const float* mean2, const float* invstd2, const float* gamma2, float* dgamma2,
                  float* dbeta2, float* dy2, float* dres, float* part, int G, hipStream_t st) {
  const bool two = y2 != nullptr, ho = out != nullptr, dr = dres != nullptr;
  const long long rpb = cdiv64(m, G);
  const int Greal = (int)cdiv64(m, rpb);
  const dim3 pgrid(Greal, cdiv(c, kChanPerBlock));
  // rows per thread per batch: 4, or 8 / 16 for the long tiles of the few-channel layers (bn_wide).  16 from
  // 32 rows per thread on: with 128 tiles the audio stem's 96,256 rows give 752-row tiles, which the old
  // 64-rows-per-thread threshold ran at 8 (half the loads in flight: 39.7 vs 31.6 us with 64 tiles of 16;
  // 20.4 us with 128 tiles of 16, profiles/r4/r4l_serial_step.txt; step 2.597 vs 2.599 ms, r4m2_pu*).  A
  // gathering source (GMax: 8 loads per row) keeps 4.  (1,024-thread workgroups for the C = 64 partial pass:
  // BN 1.020 -> 0.972 ms of device time but the step 2.778 -> 2.786 ms — the wide workgroups crowd the other
  // encoder's stream; not built)
  //
  // The stems' long tiles (more than 192 rows: 752 / 196 rows at batch 128) run 1,024-thread workgroups, 64 row
  // groups, so the gathering max-pool source (4 rows per batch) needs a quarter of the serial load batches (round
  // 5: step 2.4175 vs 2.4293 ms, BN family 0.98 -> 0.95 ms, profiles/r5/r5rg_ab_stem_bn_rg64.json; the audio stem's
  // gathered partial pass was 56-65 us).  Chosen from (m, c) alone, so a shape's gathered and dense partial sums keep
  // the same order (bitwise).  (Round 6: a fixed threshold; the environment knob that moved it is gone — the
  // library reads no environment and keeps no mutable global state.)
  constexpr long long rg64_rows = 193;
  const bool rg64 = bn_wide() && c <= kChanPerBlock && rpb >= rg64_rows;
  const int pu = (!bn_wide() || gather || rg64) ? 4 : rpb >= 32LL * kRowGroups ? 16 : rpb >= 16LL * kRowGroups ? 8 : 4;
#define BNB_P(HO, TW, U)                                                                                       \
  hipLaunchKernelGGL((k_bn_bwd_partial<HO, TW, U, kRowGroups, GS>), pgrid, dim3(256), 0, st, (long long)m, c, gs, \
                     out, y, mean, y2, mean2, rpb, part)
#define BNB_P64(HO, TW)                                                                                          \
  hipLaunchKernelGGL((k_bn_bwd_partial<HO, TW, 4, 4 * kRowGroups, GS>), pgrid, dim3(64 * kRowGroups), 0, st,     \
                     (long long)m, c, gs, out, y, mean, y2, mean2, rpb, part)
#define BNB_PU(HO, TW)                                                                                    \
  if (rg64) { BNB_P64(HO, TW); } else if (pu == 16) { BNB_P(HO, TW, 16); } else if (pu == 8) { BNB_P(HO, TW, 8); } \
  else { BNB_P(HO, TW, 4); }
  if (ho) { if (two) { BNB_PU(true, true) } else { BNB_PU(true, false) } }
  else { if (two) { BNB_PU(false, true) } else { BNB_PU(false, false) } }
#undef BNB_PU
#undef BNB_P64
#undef BNB_P
  TSPM_LAUNCH_CHECK();
  const int cblk = cdiv(c, kChanPerBlock);
  long long rb = cdiv64(m, std::max(1, 512 / cblk));  // ~512 workgroups, >= 64 rows each
  if (rb < 64) rb = 64;
  const dim3 agrid((unsigned)cdiv64(m, rb), cblk);
#define BNB_M(HO, TW, DR)                                                                                         \
  hipLaunchKernelGGL((k_bn_bwd_apply_m<HO, TW, DR, GS>), agrid, dim3(256), 0, st, (long long)m, c, Greal, part,     \
                     invstd, gamma, invstd2, gamma2, dgamma, dbeta, dgamma2, dbeta2, gs, out, y, mean, y2, mean2, rb, \
                     dy, dy2, dres)
  if (ho) {
    if (two) { if (dr) BNB_M(true, true, true); else BNB_M(true, true, false); }
    else { if (dr) BNB_M(true, false, true); else BNB_M(true, false, false); }
  } else {
    if (two) { if (dr) BNB_M(false, true, true); else BNB_M(false, true, false); }
    else { if (dr) BNB_M(false, false, true); else BNB_M(false, false, false); }
  }
#undef BNB_M
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}
}  // namespace

extern "C" int tspm_bn_bwd_apply_part(int64_t m, int32_t c, int32_t tiles, const float* part, const float* g,
                                      const float* out, const float* y, const float* mean, const float* invstd,
                                      const float* gamma, float* dgamma, float* dbeta, float* dy, const float* y2,
                                      const float* mean2, const float* invstd2, const float* gamma2, float* dgamma2,
                                      float* dbeta2, float* dy2, float* dres, tspm_stream_t stream) {
  if (m <= 0 || !c_ok(c) || tiles < 1 || tiles > 8 * kMergeTiles || !part || !g || !out || !y || !mean || !invstd ||
      !gamma || !dy)
    return TSPM_ERR_INVALID;
  const bool two = y2 != nullptr;
  if (two && (!mean2 || !invstd2 || !gamma2 || !dy2)) return TSPM_ERR_INVALID;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const GDense gs{g, c};
  // the apply launch shape of bn_bwd_merged (~512 workgroups, >= 64 rows each)
  const int cblk = cdiv(c, kChanPerBlock);
  long long rb = cdiv64(m, std::max(1, 512 / cblk));
  if (rb < 64) rb = 64;
  const dim3 agrid((unsigned)cdiv64(m, rb), cblk);
#define BNB_MP(TW, DR)                                                                                            \
  hipLaunchKernelGGL((k_bn_bwd_apply_m<true, TW, DR, GDense>), agrid, dim3(256), 0, st, (long long)m, c, tiles, part, \
                     invstd, gamma, invstd2, gamma2, dgamma, dbeta, dgamma2, dbeta2, gs, out, y, mean, y2, mean2, rb,  \
                     dy, dy2, dres)
  if (two) { if (dres) BNB_MP(true, true); else BNB_MP(true, false); }
  else { if (dres) BNB_MP(false, true); else BNB_MP(false, false); }
#undef BNB_MP
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_bn_bwd_apply_part_src(int64_t m, int32_t c, int32_t tiles, const float* part,
                                          const tspm_bn_gsrc* src, const float* out, const float* y, const float* mean,
                                          const float* invstd, const float* gamma, float* dgamma, float* dbeta,
                                          float* dy, tspm_stream_t stream) {
  if (m <= 0 || !c_ok(c) || tiles < 1 || tiles > 8 * kMergeTiles || !part || !src || !src->gp || !out || !y || !mean ||
      !invstd || !gamma || !dy)
    return TSPM_ERR_INVALID;
  const tspm_bn_gsrc& g = *src;
  if (g.n <= 0 || g.h <= 0 || g.w <= 0 || (long long)g.h * g.w * g.n != m || m >= (1LL << 24)) return TSPM_ERR_INVALID;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int cblk = cdiv(c, kChanPerBlock);
  long long rb = cdiv64(m, std::max(1, 512 / cblk));
  if (rb < 64) rb = 64;
  const dim3 agrid((unsigned)cdiv64(m, rb), cblk);
  if (g.kind == TSPM_GSRC_MAXPOOL) {
    if (!g.idx || g.p != (g.h + 2 - 3) / 2 + 1 || g.q != (g.w + 2 - 3) / 2 + 1) return TSPM_ERR_INVALID;
    const GMax gs{g.gp, g.idx, g.n, g.w, g.p, g.q, c, 1.0f / (float)g.n, 1.0f / (float)g.w};
    hipLaunchKernelGGL((k_bn_bwd_apply_m<true, false, false, GMax>), agrid, dim3(256), 0, st, (long long)m, c, tiles,
                       part, invstd, gamma, nullptr, nullptr, dgamma, dbeta, nullptr, nullptr, gs, out, y, mean, nullptr,
                       nullptr, rb, dy, nullptr, nullptr);
  } else {
    return TSPM_ERR_INVALID;
  }
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_bn_bwd_src(int64_t m, int32_t c, const tspm_bn_gsrc* src, const float* out, const float* y,
                               const float* mean, const float* invstd, const float* gamma, float* dgamma, float* dbeta,
                               float* dy, const float* y2, const float* mean2, const float* invstd2,
                               const float* gamma2, float* dgamma2, float* dbeta2, float* dy2, float* dres, void* ws,
                               size_t ws_bytes, tspm_stream_t stream) {
  if (m <= 0 || !c_ok(c) || !src || !src->gp || !y || !mean || !invstd || !gamma || !dy) return TSPM_ERR_INVALID;
  const tspm_bn_gsrc& g = *src;
  if (g.n <= 0 || g.h <= 0 || g.w <= 0 || (long long)g.h * g.w * g.n != m || m >= (1LL << 24)) return TSPM_ERR_INVALID;
  const bool two = y2 != nullptr;
  if (two && (!mean2 || !invstd2 || !gamma2 || !dy2)) return TSPM_ERR_INVALID;
  if (!ws || ws_bytes < tspm_bn_bwd_workspace(m, c)) return TSPM_ERR_WORKSPACE;
  hipStream_t st = static_cast<hipStream_t>(stream);
  float* part = static_cast<float*>(ws);
  const int G = std::min(row_blocks(m, c), kMergeTiles);
  if (g.kind == TSPM_GSRC_AVGPOOL) {
    if (g.npos != g.h * g.w || g.ldg < c || g.ldg % 4) return TSPM_ERR_INVALID;
    const GAvg gs{g.gp, g.ldg, g.n, g.npos, 1.0f / (float)g.n};
    return bn_bwd_merged(m, c, gs, false, out, y, mean, invstd, gamma, dgamma, dbeta, dy, y2, mean2, invstd2, gamma2,
                         dgamma2, dbeta2, dy2, dres, part, G, st);
  }
  if (g.kind == TSPM_GSRC_MAXPOOL) {
    // MaxPool2d(3, 2, 1) of the h x w map into p x q (the ResNet stem pool)
    if (!g.idx || g.p != (g.h + 2 - 3) / 2 + 1 || g.q != (g.w + 2 - 3) / 2 + 1) return TSPM_ERR_INVALID;
    const GMax gs{g.gp, g.idx, g.n, g.w, g.p, g.q, c, 1.0f / (float)g.n, 1.0f / (float)g.w};
    return bn_bwd_merged(m, c, gs, true, out, y, mean, invstd, gamma, dgamma, dbeta, dy, y2, mean2, invstd2, gamma2,
                         dgamma2, dbeta2, dy2, dres, part, G, st);
  }
  return TSPM_ERR_INVALID;
}

extern "C" int tspm_bn_bwd(int64_t m, int32_t c, const float* g, const float* out, const float* y, const float* mean,
                           const float* invstd, const float* gamma, float* dgamma, float* dbeta, float* dy,
                           const float* y2, const float* mean2, const float* invstd2, const float* gamma2,
                           float* dgamma2, float* dbeta2, float* dy2, float* dres, float* dy_t, float* dy2_t,
                           int64_t ld_t, void* ws, size_t ws_bytes, tspm_stream_t stream) {
  if (m <= 0 || !c_ok(c) || !g || !y || !mean || !invstd || !gamma || !dy) return TSPM_ERR_INVALID;
  const bool two = y2 != nullptr;
  if (two && (!mean2 || !invstd2 || !gamma2 || !dy2)) return TSPM_ERR_INVALID;
  if (!ws || ws_bytes < tspm_bn_bwd_workspace(m, c)) return TSPM_ERR_WORKSPACE;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const bool ho = out != nullptr;
  const bool dr = dres != nullptr;
  float* part = static_cast<float*>(ws);
  // the merged path (no dy_t) keeps the partial tiles few enough for every apply workgroup to
  // merge them in its prologue; the transposed-copy path keeps the separate final pass
  if (!dy_t) {
    if (dy2_t) return TSPM_ERR_INVALID;
    return bn_bwd_merged(m, c, GDense{g, c}, false, out, y, mean, invstd, gamma, dgamma, dbeta, dy, y2, mean2, invstd2,
                         gamma2, dgamma2, dbeta2, dy2, dres, part, std::min(row_blocks(m, c), kMergeTiles), st);
  }
  const int G = row_blocks(m, c);
  const long long rpb = cdiv64(m, G);
  const int Greal = (int)cdiv64(m, rpb);
  float* coef = part + (size_t)3 * G * c;
  const dim3 pgrid(Greal, cdiv(c, kChanPerBlock));
  const GDense gs{g, c};
#define BNB_P(HO, TW) \
  hipLaunchKernelGGL((k_bn_bwd_partial<HO, TW, 4>), pgrid, dim3(256), 0, st, (long long)m, c, gs, out, y, mean, y2, \
                     mean2, rpb, part)
  if (ho) { if (two) { BNB_P(true, true); } else { BNB_P(true, false); } }
  else { if (two) { BNB_P(false, true); } else { BNB_P(false, false); } }
#undef BNB_P
  TSPM_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_bn_bwd_final, dim3(cdiv(c, 8)), dim3(256), 0, st, (long long)m, c, Greal, two ? 1 : 0, part,
                     invstd, gamma, invstd2, gamma2, dgamma, dbeta, dgamma2, dbeta2, coef);
  TSPM_LAUNCH_CHECK();
  {
    if (!t_ok(m, dy_t, ld_t) || (two && dy2_t && !t_ok(m, dy2_t, ld_t)) || (!two && dy2_t)) return TSPM_ERR_INVALID;
    const dim3 tgrid((unsigned)cdiv64(m, 64), cdiv(c, 64));
#define BNB_AT(HO, TW, DR)                                                                                  \
  hipLaunchKernelGGL((k_bn_bwd_apply_t<HO, TW, DR>), tgrid, dim3(256), 0, st, (long long)m, c, g, out, y, mean, \
                     y2, mean2, coef, dy, dy2, dres, dy_t, dy2_t, (long long)ld_t)
    if (ho) {
      if (two) { if (dr) BNB_AT(true, true, true); else BNB_AT(true, true, false); }
      else { if (dr) BNB_AT(true, false, true); else BNB_AT(true, false, false); }
    } else {
      if (two) { if (dr) BNB_AT(false, true, true); else BNB_AT(false, true, false); }
      else { if (dr) BNB_AT(false, false, true); else BNB_AT(false, false, false); }
    }
#undef BNB_AT
    TSPM_LAUNCH_CHECK();
    return TSPM_OK;
  }
  return TSPM_OK;
}
