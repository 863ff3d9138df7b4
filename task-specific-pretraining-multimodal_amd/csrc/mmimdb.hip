// MMIMDb late-fusion path (BASELINE configs[3]): the element-wise and row-reduction
// pieces around the small GEMMs —
//   * GatedBiModalNetwork (MML_Suite/models/gates/gated_bimodal.py): tanh of both projections, the
//     scalar gate sigmoid(w_z · [h1, h2]) per row, and z = g*h1 + (1-g)*h2, plus its backward;
//   * MaxOut(num_units=2, no bias) (models/maxout.py) fused with the Dropout(0.5) that follows it in
//     MLPGenreClassifier (models/mmimdb.py:38-47), plus the backward of torch.maximum (ties split the
//     gradient in half, as ATen's derivative of maximum does);
//   * BCEWithLogitsLoss(mean) (experiment_utils/loss.py:52) with on-device multilabel counts for the
//     f1_{samples,macro,weighted,micro} metrics of configs/mmimdb/centralised/mmimdb_baseline.yaml
//     (prediction = sigmoid(x) > threshold, models/mmimdb.py:236-237).
// Every kernel is HBM/latency bound (a few hundred KB per launch); rows map to workgroups so the
// row reductions are wave shuffles + one LDS step in a fixed order (deterministic).
#include "common.h"

namespace {

constexpr int kRowThreads = 256;
constexpr int kLossThreads = 1024;

// Block-wide sum in a fixed order: wave shuffle tree, then wave 0 adds the 4 wave totals.
template <int NT = kRowThreads>
TSPM_DEV float block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) t += red[w];
  return t;
}

// One workgroup per row.  u: [n, 2d] (fc_one output in columns [0,d), fc_two output in [d,2d)).
__global__ __launch_bounds__(kRowThreads) void k_gmu_fwd(int d, const float* __restrict__ u, int ldu,
                                                         const float* __restrict__ wz, float* __restrict__ h,
                                                         int ldh, float* __restrict__ gate, float* __restrict__ z,
                                                         int ldz) {
  __shared__ float red[kRowThreads / 64];
  const long long r = blockIdx.x;
  const float* ur = u + r * ldu;
  float* hr = h + r * ldh;
  float s = 0.f;
  for (int j = threadIdx.x; j < 2 * d; j += kRowThreads) {
    const float t = tanhf(ur[j]);
    hr[j] = t;
    s = fmaf(wz[j], t, s);
  }
  s = block_sum(s, red);
  const float g = 1.f / (1.f + expf(-s));
  if (threadIdx.x == 0) gate[r] = g;
  const float g1 = 1.f - g;
  float* zr = z + r * ldz;
  for (int j = threadIdx.x; j < d; j += kRowThreads) zr[j] = g * hr[j] + g1 * hr[d + j];
}

// dz -> du [n,2d] (through gate and tanh) and ds[n] = d(loss)/d(gate pre-activation) (the weight
// gradient of hidden_sigmoid is then ds^T @ h, a small GEMM).
__global__ __launch_bounds__(kRowThreads) void k_gmu_bwd(int d, const float* __restrict__ dz, int lddz,
                                                         const float* __restrict__ h, int ldh,
                                                         const float* __restrict__ gate,
                                                         const float* __restrict__ wz, float* __restrict__ du,
                                                         int lddu, float* __restrict__ ds) {
  __shared__ float red[kRowThreads / 64];
  const long long r = blockIdx.x;
  const float* hr = h + r * ldh;
  const float* dzr = dz + r * lddz;
  float a = 0.f;
  for (int j = threadIdx.x; j < d; j += kRowThreads) a = fmaf(dzr[j], hr[j] - hr[d + j], a);
  a = block_sum(a, red);
  const float g = gate[r];
  const float dsv = a * g * (1.f - g);
  if (threadIdx.x == 0) ds[r] = dsv;
  float* dur = du + r * lddu;
  for (int j = threadIdx.x; j < d; j += kRowThreads) {
    const float h1 = hr[j], h2 = hr[d + j];
    const float d1 = fmaf(dsv, wz[j], g * dzr[j]);
    const float d2 = fmaf(dsv, wz[d + j], (1.f - g) * dzr[j]);
    dur[j] = d1 * (1.f - h1 * h1);
    dur[d + j] = d2 * (1.f - h2 * h2);
  }
}

// y[r,j] = max(a[r,j], a[r,d+j]) [* (keep ? scale : 0)]
__global__ __launch_bounds__(256) void k_maxout_fwd(int n, int d, const float* __restrict__ a, int lda,
                                                    const uint8_t* __restrict__ keep, float scale,
                                                    float* __restrict__ y, int ldy) {
  const long long total = (long long)n * d;
  for (long long t = blockIdx.x * 256LL + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const long long r = t / d;
    const int j = (int)(t - r * d);
    const float a0 = a[r * lda + j], a1 = a[r * lda + d + j];
    float v = (a1 > a0 || a1 != a1) ? a1 : a0;  // NaN in either unit propagates (torch.max)
    if (keep) v = v * (keep[t] ? scale : 0.f);
    y[r * ldy + j] = v;
  }
}

// MaxOut forward that draws its dropout mask in-launch (the bits tspm_dropout_mask would write for
// elements index_offset + t) and stores it for the backward.
__global__ __launch_bounds__(256) void k_maxout_fwd_rng(int n, int d, const float* __restrict__ a, int lda, float p,
                                                        uint64_t seed, const uint64_t* __restrict__ ctr,
                                                        long long index_offset, uint8_t* __restrict__ keep,
                                                        float scale, float* __restrict__ y, int ldy) {
  const uint64_t base = tspm_dropout_base(seed, ctr ? *ctr : 0ULL);
  const long long total = (long long)n * d;
  for (long long t = blockIdx.x * 256LL + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const long long r = t / d;
    const int j = (int)(t - r * d);
    const float a0 = a[r * lda + j], a1 = a[r * lda + d + j];
    const bool k = tspm_dropout_keep(base, index_offset + t, p);
    keep[t] = k ? 1 : 0;
    const float v = (a1 > a0 || a1 != a1) ? a1 : a0;  // NaN in either unit propagates (torch.max)
    y[r * ldy + j] = v * (k ? scale : 0.f);
  }
}

__global__ __launch_bounds__(256) void k_maxout_bwd(int n, int d, const float* __restrict__ dy, int lddy,
                                                    const float* __restrict__ a, int lda,
                                                    const uint8_t* __restrict__ keep, float scale,
                                                    float* __restrict__ da, int ldda) {
  const long long total = (long long)n * d;
  for (long long t = blockIdx.x * 256LL + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const long long r = t / d;
    const int j = (int)(t - r * d);
    float g = dy[r * lddy + j];
    if (keep) g = g * (keep[t] ? scale : 0.f);
    const float a0 = a[r * lda + j], a1 = a[r * lda + d + j];
    const float half = 0.5f * g;
    // torch.maximum's derivative: where(a0 == a1, g/2, g) masked to 0 where the unit is the smaller one
    // (so a NaN in either unit sends the full gradient to both, as ATen does)
    da[r * ldda + j] = a0 == a1 ? half : (a0 < a1 ? 0.f : g);
    da[r * ldda + d + j] = a0 == a1 ? half : (a1 < a0 ? 0.f : g);
  }
}

// Single workgroup: loss (mean over n*c), dlogits, and the metric counts.
__global__ __launch_bounds__(kLossThreads) void k_bce_logits(int n, int c, const float* __restrict__ x,
                                                            const float* __restrict__ t, float* __restrict__ loss,
                                                            float* __restrict__ dx, float grad_scale, float threshold,
                                                            float* __restrict__ stats) {
  __shared__ float red[kLossThreads / 64];
  const long long total = (long long)n * c;
  const float inv = 1.f / (float)total;
  float acc = 0.f;
  for (long long i = threadIdx.x; i < total; i += kLossThreads) {
    const float xv = x[i], tv = t[i];
    // ATen: (1 - t) * x - log_sigmoid(x),  log_sigmoid(x) = min(x, 0) - log1p(exp(-|x|))
    const float ls = fminf(xv, 0.f) - log1pf(expf(-fabsf(xv)));
    acc += (1.f - tv) * xv - ls;
    if (dx) dx[i] = (1.f / (1.f + expf(-xv)) - tv) * inv * grad_scale;
  }
  const float sum = block_sum<kLossThreads>(acc, red);
  const float mean = sum * inv * grad_scale;
  if (threadIdx.x == 0) {
    loss[0] = mean;
    if (stats) {
      stats[0] += mean * (float)n;
      stats[1] += (float)n;
    }
  }
  if (!stats) return;
  // stats[2] += sum over rows of the per-sample F1 (zero_division = 0); per class k:
  // stats[3+3k+{0,1,2}] += tp, fp, fn.  Thread-exclusive slots, so plain read-modify-write.
  float f1 = 0.f;
  for (int r = threadIdx.x; r < n; r += kLossThreads) {
    int tp = 0, fp = 0, fn = 0;
    for (int k = 0; k < c; ++k) {
      const bool p = 1.f / (1.f + expf(-x[(long long)r * c + k])) > threshold;
      const bool y = t[(long long)r * c + k] > 0.5f;
      tp += p && y;
      fp += p && !y;
      fn += !p && y;
    }
    const int den = 2 * tp + fp + fn;
    f1 += den > 0 ? (2.f * tp) / (float)den : 0.f;
  }
  const float f1s = block_sum<kLossThreads>(f1, red);
  if (threadIdx.x == 0) stats[2] += f1s;
  for (int k = threadIdx.x; k < c; k += kLossThreads) {
    float tp = 0.f, fp = 0.f, fn = 0.f;
    for (int r = 0; r < n; ++r) {
      const bool p = 1.f / (1.f + expf(-x[(long long)r * c + k])) > threshold;
      const bool y = t[(long long)r * c + k] > 0.5f;
      tp += (p && y) ? 1.f : 0.f;
      fp += (p && !y) ? 1.f : 0.f;
      fn += (!p && y) ? 1.f : 0.f;
    }
    stats[3 + 3 * k] += tp;
    stats[4 + 3 * k] += fp;
    stats[5 + 3 * k] += fn;
  }
}

// BatchNorm1d over [m, c] rows in ONE launch each way (m = the batch, at most a few thousand rows on
// this path): one workgroup per kBnCh channels, kBnGroups row groups — lane = channel, so every row
// read is one coalesced segment; two-pass statistics (sum, then centred squares), row groups
// combined through LDS in a fixed order (deterministic).  Replaces the stats/finalize/apply triple
// (forward) and the partial/apply pair (backward) used for BatchNorm2d, whose launch overhead
// dominates at these sizes.
#ifndef TSPM_BN1D_CH
#define TSPM_BN1D_CH 32
#endif
// 1024 threads: 32 channels (one 128-byte line per row) x 32 row groups keep the per-lane row chain
// short and put c/32 workgroups on the chip (64 channels x 16 groups: 6.2-6.8 us per launch at c=512)
constexpr int kBnCh = TSPM_BN1D_CH, kBnGroups = 1024 / TSPM_BN1D_CH;

// Per-channel sums of the row groups, in double and in fixed group order.  BatchNorm1d runs over as
// few as 4 rows here, where the backward's projection (g - mean(g) - xhat * mean(g xhat)) cancels
// most of g: the statistics and sums are formed in double (as ATen's CPU kernels accumulate) so the
// cancellation does not amplify fp32 rounding.
TSPM_DEV double bn_group_sum(double v, double* red) {
  const int ch = threadIdx.x % kBnCh, grp = threadIdx.x / kBnCh;
  __syncthreads();
  red[grp * kBnCh + ch] = v;
  __syncthreads();
  // one row group forms each channel's total (same order as before) and publishes it: every thread
  // summing all kBnGroups doubles itself read 256 KB of LDS per call (≈ 1 µs at these sizes)
  if (grp == 0) {
    double t = 0.0;
#pragma unroll
    for (int q = 0; q < kBnGroups; ++q) t += red[q * kBnCh + ch];
    red[ch] = t;
  }
  __syncthreads();
  return red[ch];
}

struct Bn1dFwd {
  int c;
  const float* x;
  const float* gamma;
  const float* beta;
  float* rmean;
  float* rvar;
  float momentum, eps;
  float* smean;
  float* sinvstd;
  float* y;
  const uint8_t* keep;  // optional Dropout after the BN (tspm_bn1d_fwd_drop): y *= keep ? keep_scale : 0
  float keep_scale;
};

// DROP: the Dropout-after-BN variant (tspm_bn1d_fwd_drop) — a template parameter so the plain
// BatchNorm1d launches compile exactly as before (a runtime branch in the row loop cost them 1-2 us).
template <bool DROP = false>
TSPM_DEV void bn1d_fwd_body(int m, const Bn1dFwd& p, int bid, double* red);

template <bool DROP>
__global__ __launch_bounds__(kBnCh * kBnGroups) void k_bn1d_fwd(int m, Bn1dFwd p) {
  __shared__ double red[kBnCh * kBnGroups];
  bn1d_fwd_body<DROP>(m, p, blockIdx.x, red);
}

// Two independent BatchNorm1d layers over the same rows (the MMIMDb image and text encoders' input
// BNs) in one launch: blocks [0, nb0) take p0.
__global__ __launch_bounds__(kBnCh * kBnGroups) void k_bn1d_fwd2(int m, Bn1dFwd p0, Bn1dFwd p1, int nb0) {
  __shared__ double red[kBnCh * kBnGroups];
  if ((int)blockIdx.x < nb0)
    bn1d_fwd_body(m, p0, blockIdx.x, red);
  else
    bn1d_fwd_body(m, p1, blockIdx.x - nb0, red);
}

template <bool DROP>
TSPM_DEV void bn1d_fwd_body(int m, const Bn1dFwd& p, int bid, double* red) {
  const int c = p.c;
  const float* __restrict__ x = p.x;
  const float momentum = p.momentum, eps = p.eps;
  float* __restrict__ rmean = p.rmean;
  float* __restrict__ rvar = p.rvar;
  const int ch = bid * kBnCh + threadIdx.x % kBnCh, grp = threadIdx.x / kBnCh;
  const bool ok = ch < c;
  double s = 0.0;
  if (ok)
#pragma unroll 4
    for (int r = grp; r < m; r += kBnGroups) s += (double)x[(long long)r * c + ch];
  const double meand = bn_group_sum(s, red) / (double)m;
  double q = 0.0;
  if (ok)
#pragma unroll 4
    for (int r = grp; r < m; r += kBnGroups) {
      const double d = (double)x[(long long)r * c + ch] - meand;
      q = fma(d, d, q);
    }
  const double m2 = bn_group_sum(q, red);
  const float mean = (float)meand;
  const float invstd = (float)(1.0 / sqrt(m2 / (double)m + (double)eps));
  if (!ok) return;
  if (grp == 0) {
    p.smean[ch] = mean;
    p.sinvstd[ch] = invstd;
    if (rmean) rmean[ch] = (1.f - momentum) * rmean[ch] + momentum * mean;
    if (rvar) rvar[ch] = (1.f - momentum) * rvar[ch] + momentum * (float)(m > 1 ? m2 / (double)(m - 1) : m2);
  }
  const float ga = p.gamma[ch], be = p.beta[ch];
  for (int r = grp; r < m; r += kBnGroups) {
    const long long i = (long long)r * c + ch;
    const float v = (x[i] - mean) * invstd * ga + be;
    p.y[i] = (DROP && p.keep) ? v * (p.keep[i] ? p.keep_scale : 0.f) : v;
  }
}

struct Bn1dBwd {
  int c;
  const float* g;
  const float* x;
  const float* mean;
  const float* invstd;
  const float* gamma;
  float* dgamma;
  float* dbeta;
  float* dx;
  const uint8_t* g_keep;  // tspm_bn1d_bwd_drop_relu: g is the gradient of Dropout(BN(x)) -> g*keep*g_scale,
  float g_scale;          // and x is a ReLU output: dx = 0 where x <= 0
  int relu_x;
};

// DR: the Dropout-gradient-in / ReLU-mask-out variant (tspm_bn1d_bwd_drop_relu), compiled separately.
template <bool DR = false>
TSPM_DEV void bn1d_bwd_body(int m, const Bn1dBwd& p, int bid, double* red);

template <bool DR>
__global__ __launch_bounds__(kBnCh * kBnGroups) void k_bn1d_bwd(int m, Bn1dBwd p) {
  __shared__ double red[kBnCh * kBnGroups];
  bn1d_bwd_body<DR>(m, p, blockIdx.x, red);
}

__global__ __launch_bounds__(kBnCh * kBnGroups) void k_bn1d_bwd2(int m, Bn1dBwd p0, Bn1dBwd p1, int nb0) {
  __shared__ double red[kBnCh * kBnGroups];
  if ((int)blockIdx.x < nb0)
    bn1d_bwd_body(m, p0, blockIdx.x, red);
  else
    bn1d_bwd_body(m, p1, blockIdx.x - nb0, red);
}

template <bool DR>
TSPM_DEV void bn1d_bwd_body(int m, const Bn1dBwd& p, int bid, double* red) {
  const int c = p.c;
  const float* __restrict__ g = p.g;
  const float* __restrict__ x = p.x;
  const float* __restrict__ mean_ = p.mean;
  const float* __restrict__ invstd_ = p.invstd;
  const float* __restrict__ gamma = p.gamma;
  float* __restrict__ dgamma = p.dgamma;
  float* __restrict__ dbeta = p.dbeta;
  float* __restrict__ dx = p.dx;
  const int ch = bid * kBnCh + threadIdx.x % kBnCh, grp = threadIdx.x / kBnCh;
  const bool ok = ch < c;
  const float mean = ok ? mean_[ch] : 0.f, invstd = ok ? invstd_[ch] : 0.f;
  const uint8_t* __restrict__ gk = p.g_keep;
  const float gs = p.g_scale;
  auto gval = [&](long long i) -> float { return (DR && gk) ? g[i] * (gk[i] ? gs : 0.f) : g[i]; };
  double sg = 0.0, sgx = 0.0;
  if (ok)
#pragma unroll 4
    for (int r = grp; r < m; r += kBnGroups) {
      const long long i = (long long)r * c + ch;
      const double gv = (double)gval(i);
      sg += gv;
      sgx = fma(gv, ((double)x[i] - (double)mean) * (double)invstd, sgx);
    }
  const double tg = bn_group_sum(sg, red);
  const double tgx = bn_group_sum(sgx, red);
  if (!ok) return;
  if (grp == 0) {
    dgamma[ch] = (float)tgx;
    dbeta[ch] = (float)tg;
  }
  if (!dx) return;
  const double k = (double)gamma[ch] * (double)invstd, mg = tg / (double)m, mgx = tgx / (double)m;
  for (int r = grp; r < m; r += kBnGroups) {
    const long long i = (long long)r * c + ch;
    float v = (float)(k * ((double)gval(i) - mg - ((double)x[i] - (double)mean) * (double)invstd * mgx));
    if (DR && p.relu_x && !(x[i] > 0.f)) v = 0.f;
    dx[i] = v;
  }
}

int ew_grid(long long work) {
  long long b = cdiv64(work, 256);
  if (b > 4096) b = 4096;
  return (int)(b < 1 ? 1 : b);
}

// ------------------------------------------------------------------------------------------------
// MultimodalPooling (models/pooling.py:6-127): u = [proj_a(x_a) | proj_b(x_b)] [n, 2d] (+ bias, from
// the small GEMM), a | b = dropout(tanh(u)) (one Dropout module, two draws: keep [n, 2d]), then
// kind 0 max / 1 avg / 2 sum / 3 attention / 4 gated.  Attention and gated run their scoring MLP's
// first Linear (+ bias) on the small GEMM into hpre [n, hd]; tanh, the second Linear (hd -> 2 / 1 +
// bias), softmax / sigmoid and the mix run here, one workgroup per row, fixed-order block sums.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pool_act_fwd(long long total, int d2, const float* __restrict__ u, int ldu,
                                                      const uint8_t* __restrict__ keep, float scale,
                                                      float* __restrict__ tu, float* __restrict__ ab) {
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    const long long r = e / d2;
    const int j = (int)(e - r * d2);
    const float t = tanhf(u[r * ldu + j]);
    tu[e] = t;
    ab[e] = keep ? t * (keep[e] ? scale : 0.f) : t;
  }
}

__global__ __launch_bounds__(kRowThreads) void k_pool_mix_fwd(int d, int hd, int kind, const float* __restrict__ ab,
                                                              const float* __restrict__ hpre, float* __restrict__ hh,
                                                              const float* __restrict__ w2, const float* __restrict__ b2,
                                                              float* __restrict__ wts, float* __restrict__ z, int ldz) {
  __shared__ float red[kRowThreads / 64];
  const long long r = blockIdx.x;
  const float* a = ab + r * 2 * d;
  const float* b = a + d;
  float* zr = z + r * ldz;
  if (kind <= 2) {
    for (int j = threadIdx.x; j < d; j += kRowThreads) {
      const float x = a[j], y = b[j];
      zr[j] = kind == 0 ? ((x > y || x != x) ? x : y) : (kind == 1 ? (x + y) / 2.f : x + y);
    }
    return;
  }
  const float* hp = hpre + r * hd;
  float* hr = hh + r * hd;
  float s0 = 0.f, s1 = 0.f;
  for (int j = threadIdx.x; j < hd; j += kRowThreads) {
    const float t = tanhf(hp[j]);
    hr[j] = t;
    s0 = fmaf(w2[j], t, s0);
    if (kind == 3) s1 = fmaf(w2[hd + j], t, s1);
  }
  s0 = block_sum(s0, red) + b2[0];
  float wa, wb;
  if (kind == 3) {
    s1 = block_sum(s1, red) + b2[1];
    const float m = fmaxf(s0, s1);
    const float e0 = expf(s0 - m), e1 = expf(s1 - m);
    const float inv = 1.f / (e0 + e1);
    wa = e0 * inv;
    wb = e1 * inv;
  } else {
    wa = 1.f / (1.f + expf(-s0));
    wb = 1.f - wa;
  }
  if (threadIdx.x == 0) {
    wts[2 * r] = wa;
    wts[2 * r + 1] = wb;
  }
  for (int j = threadIdx.x; j < d; j += kRowThreads) zr[j] = wa * a[j] + wb * b[j];
}

// dz -> dab [n, 2d] through the mix; attention / gated also: ds [n, k] (scores' gradient, for the
// second Linear's weight gradient ds^T @ hh) and dhpre [n, hd] (through that Linear and the tanh).
__global__ __launch_bounds__(kRowThreads) void k_pool_mix_bwd(int d, int hd, int kind, const float* __restrict__ dz,
                                                              int lddz, const float* __restrict__ ab,
                                                              const float* __restrict__ hh, const float* __restrict__ w2,
                                                              const float* __restrict__ wts, float* __restrict__ dab,
                                                              float* __restrict__ ds, float* __restrict__ dhpre) {
  __shared__ float red[kRowThreads / 64];
  const long long r = blockIdx.x;
  const float* a = ab + r * 2 * d;
  const float* b = a + d;
  const float* g = dz + r * lddz;
  float* da = dab + r * 2 * d;
  float* db = da + d;
  if (kind <= 2) {
    for (int j = threadIdx.x; j < d; j += kRowThreads) {
      const float gv = g[j];
      if (kind == 0) {  // torch.maximum's derivative: ties split the gradient in half
        const float x = a[j], y = b[j];
        const float h = gv / 2.f;
        da[j] = x == y ? h : (x > y ? gv : 0.f);
        db[j] = x == y ? h : (y > x ? gv : 0.f);
      } else {
        const float v = kind == 1 ? gv / 2.f : gv;
        da[j] = v;
        db[j] = v;
      }
    }
    return;
  }
  const float wa = wts[2 * r], wb = wts[2 * r + 1];
  float pa = 0.f, pb = 0.f;
  for (int j = threadIdx.x; j < d; j += kRowThreads) {
    const float gv = g[j];
    pa = fmaf(gv, a[j], pa);
    pb = fmaf(gv, b[j], pb);
    da[j] = wa * gv;
    db[j] = wb * gv;
  }
  pa = block_sum(pa, red);
  pb = block_sum(pb, red);
  float d0, d1 = 0.f;
  if (kind == 3) {  // softmax backward over the two scores
    const float dot = wa * pa + wb * pb;
    d0 = wa * (pa - dot);
    d1 = wb * (pb - dot);
  } else {          // z = g a + (1 - g) b: dg = sum dz (a - b); sigmoid backward
    d0 = (pa - pb) * wa * (1.f - wa);
  }
  if (threadIdx.x == 0) {
    ds[r * (kind == 3 ? 2 : 1)] = d0;
    if (kind == 3) ds[r * 2 + 1] = d1;
  }
  const float* hr = hh + r * hd;
  float* dh = dhpre + r * hd;
  for (int j = threadIdx.x; j < hd; j += kRowThreads) {
    float v = d0 * w2[j];
    if (kind == 3) v = fmaf(d1, w2[hd + j], v);
    const float t = hr[j];
    dh[j] = v * (1.f - t * t);
  }
}

// du = (dab [+ dab2]) * keep * scale * (1 - tanh(u)^2)
__global__ __launch_bounds__(256) void k_pool_act_bwd(long long total, const float* __restrict__ dab,
                                                      const float* __restrict__ dab2, const float* __restrict__ tu,
                                                      const uint8_t* __restrict__ keep, float scale,
                                                      float* __restrict__ du) {
  for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
    float v = dab[e];
    if (dab2) v += dab2[e];
    if (keep) v = v * (keep[e] ? scale : 0.f);
    const float t = tu[e];
    du[e] = v * (1.f - t * t);
  }
}

}  // namespace

extern "C" int tspm_gmu_fwd(int32_t n, int32_t d, const float* u, int32_t ldu, const float* wz, float* h,
                            int32_t ldh, float* gate, float* z, int32_t ldz, tspm_stream_t stream) {
  if (n <= 0 || d <= 0 || ldu < 2 * d || ldh < 2 * d || ldz < d || !u || !wz || !h || !gate || !z)
    return TSPM_ERR_INVALID;
  hipLaunchKernelGGL(k_gmu_fwd, dim3(n), dim3(kRowThreads), 0, static_cast<hipStream_t>(stream), d, u, ldu, wz, h,
                     ldh, gate, z, ldz);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_gmu_bwd(int32_t n, int32_t d, const float* dz, int32_t lddz, const float* h, int32_t ldh,
                            const float* gate, const float* wz, float* du, int32_t lddu, float* ds,
                            tspm_stream_t stream) {
  if (n <= 0 || d <= 0 || lddz < d || ldh < 2 * d || lddu < 2 * d || !dz || !h || !gate || !wz || !du || !ds)
    return TSPM_ERR_INVALID;
  hipLaunchKernelGGL(k_gmu_bwd, dim3(n), dim3(kRowThreads), 0, static_cast<hipStream_t>(stream), d, dz, lddz, h, ldh,
                     gate, wz, du, lddu, ds);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_maxout_fwd(int32_t n, int32_t d, const float* a, int32_t lda, const uint8_t* keep,
                               float keep_scale, float* y, int32_t ldy, tspm_stream_t stream) {
  if (n <= 0 || d <= 0 || lda < 2 * d || ldy < d || !a || !y) return TSPM_ERR_INVALID;
  hipLaunchKernelGGL(k_maxout_fwd, dim3(ew_grid((long long)n * d)), dim3(256), 0, static_cast<hipStream_t>(stream), n,
                     d, a, lda, keep, keep_scale, y, ldy);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_maxout_bwd(int32_t n, int32_t d, const float* dy, int32_t lddy, const float* a, int32_t lda,
                               const uint8_t* keep, float keep_scale, float* da, int32_t ldda, tspm_stream_t stream) {
  if (n <= 0 || d <= 0 || lddy < d || lda < 2 * d || ldda < 2 * d || !dy || !a || !da) return TSPM_ERR_INVALID;
  hipLaunchKernelGGL(k_maxout_bwd, dim3(ew_grid((long long)n * d)), dim3(256), 0, static_cast<hipStream_t>(stream), n,
                     d, dy, lddy, a, lda, keep, keep_scale, da, ldda);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_bce_logits(int32_t n, int32_t classes, const float* logits, const float* targets, float* loss,
                               float* dlogits, float grad_scale, float threshold, float* stats, tspm_stream_t stream) {
  if (n <= 0 || classes <= 0 || !logits || !targets || !loss) return TSPM_ERR_INVALID;
  hipLaunchKernelGGL(k_bce_logits, dim3(1), dim3(kLossThreads), 0, static_cast<hipStream_t>(stream), n, classes, logits,
                     targets, loss, dlogits, grad_scale, threshold, stats);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_bn1d_fwd(int32_t m, int32_t c, const float* x, const float* gamma, const float* beta,
                             float* running_mean, float* running_var, float momentum, float eps, float* save_mean,
                             float* save_invstd, float* y, tspm_stream_t stream) {
  if (m <= 0 || c <= 0 || !x || !gamma || !beta || !save_mean || !save_invstd || !y) return TSPM_ERR_INVALID;
  const Bn1dFwd p{c, x, gamma, beta, running_mean, running_var, momentum, eps, save_mean, save_invstd, y};
  hipLaunchKernelGGL(k_bn1d_fwd<false>, dim3(cdiv(c, kBnCh)), dim3(kBnCh * kBnGroups), 0, static_cast<hipStream_t>(stream),
                     m, p);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_bn1d_bwd(int32_t m, int32_t c, const float* g, const float* x, const float* mean,
                             const float* invstd, const float* gamma, float* dgamma, float* dbeta, float* dx,
                             tspm_stream_t stream) {
  if (m <= 0 || c <= 0 || !g || !x || !mean || !invstd || !gamma || !dgamma || !dbeta) return TSPM_ERR_INVALID;
  const Bn1dBwd p{c, g, x, mean, invstd, gamma, dgamma, dbeta, dx};
  hipLaunchKernelGGL(k_bn1d_bwd<false>, dim3(cdiv(c, kBnCh)), dim3(kBnCh * kBnGroups), 0, static_cast<hipStream_t>(stream),
                     m, p);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_bn1d_fwd_drop(int32_t m, int32_t c, const float* x, const float* gamma, const float* beta,
                                  float* running_mean, float* running_var, float momentum, float eps, float* save_mean,
                                  float* save_invstd, const uint8_t* keep, float keep_scale, float* y,
                                  tspm_stream_t stream) {
  if (m <= 0 || c <= 0 || !x || !gamma || !beta || !save_mean || !save_invstd || !y) return TSPM_ERR_INVALID;
  const Bn1dFwd p{c, x, gamma, beta, running_mean, running_var, momentum, eps, save_mean, save_invstd, y, keep, keep_scale};
  hipLaunchKernelGGL(k_bn1d_fwd<true>, dim3(cdiv(c, kBnCh)), dim3(kBnCh * kBnGroups), 0, static_cast<hipStream_t>(stream),
                     m, p);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_bn1d_bwd_drop_relu(int32_t m, int32_t c, const float* g, const uint8_t* g_keep, float g_scale,
                                       const float* x, const float* mean, const float* invstd, const float* gamma,
                                       float* dgamma, float* dbeta, float* dx, tspm_stream_t stream) {
  if (m <= 0 || c <= 0 || !g || !x || !mean || !invstd || !gamma || !dgamma || !dbeta) return TSPM_ERR_INVALID;
  const Bn1dBwd p{c, g, x, mean, invstd, gamma, dgamma, dbeta, dx, g_keep, g_scale, 1};
  hipLaunchKernelGGL(k_bn1d_bwd<true>, dim3(cdiv(c, kBnCh)), dim3(kBnCh * kBnGroups), 0, static_cast<hipStream_t>(stream),
                     m, p);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_bn1d_fwd_pair(int32_t m, int32_t c0, const float* x0, const float* gamma0, const float* beta0,
                                  float* running_mean0, float* running_var0, float momentum0, float eps0,
                                  float* save_mean0, float* save_invstd0, float* y0, int32_t c1, const float* x1,
                                  const float* gamma1, const float* beta1, float* running_mean1, float* running_var1,
                                  float momentum1, float eps1, float* save_mean1, float* save_invstd1, float* y1,
                                  tspm_stream_t stream) {
  if (m <= 0 || c0 <= 0 || c1 <= 0 || !x0 || !gamma0 || !beta0 || !save_mean0 || !save_invstd0 || !y0 || !x1 ||
      !gamma1 || !beta1 || !save_mean1 || !save_invstd1 || !y1)
    return TSPM_ERR_INVALID;
  const Bn1dFwd p0{c0, x0, gamma0, beta0, running_mean0, running_var0, momentum0, eps0, save_mean0, save_invstd0, y0};
  const Bn1dFwd p1{c1, x1, gamma1, beta1, running_mean1, running_var1, momentum1, eps1, save_mean1, save_invstd1, y1};
  const int nb0 = cdiv(c0, kBnCh);
  hipLaunchKernelGGL(k_bn1d_fwd2, dim3(nb0 + cdiv(c1, kBnCh)), dim3(kBnCh * kBnGroups), 0,
                     static_cast<hipStream_t>(stream), m, p0, p1, nb0);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_bn1d_bwd_pair(int32_t m, int32_t c0, const float* g0, const float* x0, const float* mean0,
                                  const float* invstd0, const float* gamma0, float* dgamma0, float* dbeta0, float* dx0,
                                  int32_t c1, const float* g1, const float* x1, const float* mean1,
                                  const float* invstd1, const float* gamma1, float* dgamma1, float* dbeta1, float* dx1,
                                  tspm_stream_t stream) {
  if (m <= 0 || c0 <= 0 || c1 <= 0 || !g0 || !x0 || !mean0 || !invstd0 || !gamma0 || !dgamma0 || !dbeta0 || !g1 ||
      !x1 || !mean1 || !invstd1 || !gamma1 || !dgamma1 || !dbeta1)
    return TSPM_ERR_INVALID;
  const Bn1dBwd p0{c0, g0, x0, mean0, invstd0, gamma0, dgamma0, dbeta0, dx0};
  const Bn1dBwd p1{c1, g1, x1, mean1, invstd1, gamma1, dgamma1, dbeta1, dx1};
  const int nb0 = cdiv(c0, kBnCh);
  hipLaunchKernelGGL(k_bn1d_bwd2, dim3(nb0 + cdiv(c1, kBnCh)), dim3(kBnCh * kBnGroups), 0,
                     static_cast<hipStream_t>(stream), m, p0, p1, nb0);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_maxout_fwd_rng(int32_t n, int32_t d, const float* a, int32_t lda, float p, uint64_t seed,
                                   const uint64_t* counter, int64_t index_offset, uint8_t* keep, float keep_scale,
                                   float* y, int32_t ldy, tspm_stream_t stream) {
  if (n <= 0 || d <= 0 || lda < 2 * d || ldy < d || !a || !keep || !y || p < 0.f || p >= 1.f || index_offset < 0)
    return TSPM_ERR_INVALID;
  hipLaunchKernelGGL(k_maxout_fwd_rng, dim3(ew_grid((long long)n * d)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     n, d, a, lda, p, (unsigned long long)seed, counter, (long long)index_offset, keep, keep_scale, y,
                     ldy);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_pool_act_fwd(int32_t n, int32_t d, const float* u, int32_t ldu, const uint8_t* keep, float keep_scale,
                                 float* tu, float* ab, tspm_stream_t stream) {
  if (n <= 0 || d <= 0 || ldu < 2 * d || !u || !tu || !ab) return TSPM_ERR_INVALID;
  const long long total = (long long)n * 2 * d;
  hipLaunchKernelGGL(k_pool_act_fwd, dim3(ew_grid(total)), dim3(256), 0, static_cast<hipStream_t>(stream), total, 2 * d,
                     u, ldu, keep, keep_scale, tu, ab);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_pool_mix_fwd(int32_t n, int32_t d, int32_t hd, int32_t kind, const float* ab, const float* hpre,
                                 float* hh, const float* w2, const float* b2, float* wts, float* z, int32_t ldz,
                                 tspm_stream_t stream) {
  if (n <= 0 || d <= 0 || kind < 0 || kind > 4 || ldz < d || !ab || !z) return TSPM_ERR_INVALID;
  if (kind >= 3 && (hd <= 0 || !hpre || !hh || !w2 || !b2 || !wts)) return TSPM_ERR_INVALID;
  hipLaunchKernelGGL(k_pool_mix_fwd, dim3(n), dim3(kRowThreads), 0, static_cast<hipStream_t>(stream), d, hd, kind, ab,
                     hpre, hh, w2, b2, wts, z, ldz);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_pool_mix_bwd(int32_t n, int32_t d, int32_t hd, int32_t kind, const float* dz, int32_t lddz,
                                 const float* ab, const float* hh, const float* w2, const float* wts, float* dab,
                                 float* ds, float* dhpre, tspm_stream_t stream) {
  if (n <= 0 || d <= 0 || kind < 0 || kind > 4 || lddz < d || !dz || !ab || !dab) return TSPM_ERR_INVALID;
  if (kind >= 3 && (hd <= 0 || !hh || !w2 || !wts || !ds || !dhpre)) return TSPM_ERR_INVALID;
  hipLaunchKernelGGL(k_pool_mix_bwd, dim3(n), dim3(kRowThreads), 0, static_cast<hipStream_t>(stream), d, hd, kind, dz,
                     lddz, ab, hh, w2, wts, dab, ds, dhpre);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_pool_act_bwd(int32_t n, int32_t d, const float* dab, const float* dab2, const float* tu,
                                 const uint8_t* keep, float keep_scale, float* du, tspm_stream_t stream) {
  if (n <= 0 || d <= 0 || !dab || !tu || !du) return TSPM_ERR_INVALID;
  const long long total = (long long)n * 2 * d;
  hipLaunchKernelGGL(k_pool_act_bwd, dim3(ew_grid(total)), dim3(256), 0, static_cast<hipStream_t>(stream), total, dab,
                     dab2, tu, keep, keep_scale, du);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}
