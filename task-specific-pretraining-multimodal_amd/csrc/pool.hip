// Max pooling (nn.MaxPool2d(3, 2, 1), MML_Suite/models/msa/networks/resnet.py:140,208) and global
// average pooling (nn.AdaptiveAvgPool2d((1,1)) + flatten, resnet.py:149,215-216) on HWNC tensors.
// HBM-bound; one thread per 4 channels of one output element, 16-byte loads/stores.
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void k_maxpool_fwd(int N, int H, int W, int C, int k, int st, int pad, int P,
                                                     int Q, const float* __restrict__ x, float* __restrict__ y,
                                                     uint8_t* __restrict__ idx) {
  const int L = C >> 2;
  const long long total = (long long)P * Q * N * L;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c4 = (int)(i % L);
    long long row = i / L;  // (p, q, n)
    const int n = (int)(row % N);
    const int pos = (int)(row / N);
    const int p = pos / Q, q = pos - p * Q;
    f32x4 best = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    int bi[4] = {0, 0, 0, 0};
    if (k == 3) {
      // the ResNet stem pool: all nine window loads in flight before the compares (a load per `continue`d
      // iteration waited for each tap in turn); out-of-range taps re-read a clamped element, then skipped
      f32x4 v[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int h = min(max(p * st - pad + t / 3, 0), H - 1), w = min(max(q * st - pad + t % 3, 0), W - 1);
        v[t] = ld4(x + (((long long)h * W + w) * N + n) * C + 4 * c4);
      }
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int h = p * st - pad + t / 3, w = q * st - pad + t % 3;
        if (h < 0 || h >= H || w < 0 || w >= W) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (v[t][j] > best[j] || isnan(v[t][j])) { best[j] = v[t][j]; bi[j] = t; }
      }
    } else {
      for (int kh = 0; kh < k; ++kh) {
        const int h = p * st - pad + kh;
        if (h < 0 || h >= H) continue;
        for (int kw = 0; kw < k; ++kw) {
          const int w = q * st - pad + kw;
          if (w < 0 || w >= W) continue;
          const f32x4 v = ld4(x + (((long long)h * W + w) * N + n) * C + 4 * c4);
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (v[j] > best[j] || isnan(v[j])) { best[j] = v[j]; bi[j] = kh * k + kw; }
        }
      }
    }
    st4(y + row * C + 4 * c4, best);
    uchar4 u;
    u.x = (uint8_t)bi[0]; u.y = (uint8_t)bi[1]; u.z = (uint8_t)bi[2]; u.w = (uint8_t)bi[3];
    *reinterpret_cast<uchar4*>(idx + row * C + 4 * c4) = u;
  }
}

// Tiled variant for the transposed copy: [64 rows x 64 channels] per workgroup, y and idx as
// above plus y_t[c][ld_t] (rows contiguous: the wgrad operand layout) through an LDS transpose.
__global__ __launch_bounds__(256) void k_maxpool_fwd_t(int N, int H, int W, int C, int k, int st, int pad, int P,
                                                       int Q, const float* __restrict__ x, float* __restrict__ y,
                                                       uint8_t* __restrict__ idx, float* __restrict__ y_t,
                                                       long long ld_t) {
  __shared__ float tile[64][65];
  const int t = threadIdx.x, l16 = t & 15, rg = t >> 4;
  const int c4 = blockIdx.y * 16 + l16;
  const bool cok = 4 * c4 < C;
  const long long M = (long long)P * Q * N;
  const long long r0 = (long long)blockIdx.x * 64;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int rl = rg + 16 * i;
    const long long row = r0 + rl;
    f32x4 best = {0.f, 0.f, 0.f, 0.f};
    if (cok && row < M) {
      const int n = (int)(row % N);
      const int pos = (int)(row / N);
      const int p = pos / Q, q = pos - p * Q;
      best = f32x4{-INFINITY, -INFINITY, -INFINITY, -INFINITY};
      int bi[4] = {0, 0, 0, 0};
      for (int kh = 0; kh < k; ++kh) {
        const int h = p * st - pad + kh;
        if (h < 0 || h >= H) continue;
        for (int kw = 0; kw < k; ++kw) {
          const int w = q * st - pad + kw;
          if (w < 0 || w >= W) continue;
          const f32x4 v = ld4(x + (((long long)h * W + w) * N + n) * C + 4 * c4);
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (v[j] > best[j] || isnan(v[j])) { best[j] = v[j]; bi[j] = kh * k + kw; }
        }
      }
      st4(y + row * C + 4 * c4, best);
      uchar4 u;
      u.x = (uint8_t)bi[0]; u.y = (uint8_t)bi[1]; u.z = (uint8_t)bi[2]; u.w = (uint8_t)bi[3];
      *reinterpret_cast<uchar4*>(idx + row * C + 4 * c4) = u;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) tile[rl][4 * l16 + j] = best[j];
  }
  __syncthreads();
  const int cl = t >> 2, qq = t & 3;
  const int c = blockIdx.y * 64 + cl;
  if (c < C) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      const int rl = qq * 16 + 4 * kk;
      if (r0 + rl < M) {
        const f32x4 v = {tile[rl][cl], tile[rl + 1][cl], tile[rl + 2][cl], tile[rl + 3][cl]};
        st4(y_t + (long long)c * ld_t + r0 + rl, v);
      }
    }
  }
}

// gather form: every input element sums dy over the windows that picked it (deterministic order)
__global__ __launch_bounds__(256) void k_maxpool_bwd(int N, int H, int W, int C, int k, int st, int pad, int P,
                                                     int Q, const float* __restrict__ dy,
                                                     const uint8_t* __restrict__ idx, float* __restrict__ dx) {
  const int L = C >> 2;
  const long long total = (long long)H * W * N * L;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c4 = (int)(i % L);
    long long row = i / L;
    const int n = (int)(row % N);
    const int pos = (int)(row / N);
    const int h = pos / W, w = pos - h * W;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    // p such that 0 <= h - (p*st - pad) < k
    const int p_lo = max(0, (h + pad - k + st) / st), p_hi = min(P - 1, (h + pad) / st);
    const int q_lo = max(0, (w + pad - k + st) / st), q_hi = min(Q - 1, (w + pad) / st);
    if (k == 3 && st == 2) {
      // the ResNet stem pool: an input element sits in at most 2 x 2 windows; all their loads in flight
      // before the sums (same window order: p, then q, ascending)
      uchar4 u4[4];
      f32x4 g4[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int pc = min(p_lo + (t >> 1), P - 1), qc = min(q_lo + (t & 1), Q - 1);
        const long long o = (((long long)pc * Q + qc) * N + n) * C + 4 * c4;
        u4[t] = *reinterpret_cast<const uchar4*>(idx + o);
        g4[t] = ld4(dy + o);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int p = p_lo + (t >> 1), q = q_lo + (t & 1);
        const int kh = h - (p * st - pad), kw = w - (q * st - pad);
        if (p > p_hi || q > q_hi || kh < 0 || kh >= k || kw < 0 || kw >= k) continue;
        const int tap = kh * k + kw;
        if (u4[t].x == tap) acc[0] += g4[t][0];
        if (u4[t].y == tap) acc[1] += g4[t][1];
        if (u4[t].z == tap) acc[2] += g4[t][2];
        if (u4[t].w == tap) acc[3] += g4[t][3];
      }
      st4(dx + row * C + 4 * c4, acc);
      continue;
    }
    for (int p = p_lo; p <= p_hi; ++p) {
      const int kh = h - (p * st - pad);
      if (kh < 0 || kh >= k) continue;
      for (int q = q_lo; q <= q_hi; ++q) {
        const int kw = w - (q * st - pad);
        if (kw < 0 || kw >= k) continue;
        const long long o = (((long long)p * Q + q) * N + n) * C + 4 * c4;
        const uchar4 u = *reinterpret_cast<const uchar4*>(idx + o);
        const f32x4 g = ld4(dy + o);
        const int tap = kh * k + kw;
        if (u.x == tap) acc[0] += g[0];
        if (u.y == tap) acc[1] += g[1];
        if (u.z == tap) acc[2] += g[2];
        if (u.w == tap) acc[3] += g[3];
      }
    }
    st4(dx + row * C + 4 * c4, acc);
  }
}

__global__ __launch_bounds__(256) void k_avgpool_fwd(int npos, int N, int C, const float* __restrict__ x,
                                                     float* __restrict__ y) {
  const int L = C >> 2;
  const long long total = (long long)N * L;
  const float inv = 1.0f / (float)npos;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    f32x4 s = {0.f, 0.f, 0.f, 0.f};
    for (int p = 0; p < npos; ++p) s += ld4(x + (long long)p * N * C + 4 * i);
    // ATen's CPU adaptive_avg_pool2d: sum over the window then divide by its size
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = s[j] / (float)npos;
    (void)inv;
    st4(y + 4 * i, o);
  }
}

__global__ __launch_bounds__(256) void k_avgpool_bwd(int npos, int N, int C, const float* __restrict__ dy, int ldy,
                                                     float* __restrict__ dx) {
  const int L = C >> 2;
  const long long total = (long long)npos * N * L;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < total; i += (long long)gridDim.x * 256) {
    const int c4 = (int)(i % L);
    const long long row = i / L;
    const int n = (int)(row % N);
    f32x4 g = ld4(dy + (long long)n * ldy + 4 * c4);
    f32x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = g[j] / (float)npos;
    st4(dx + row * C + 4 * c4, o);
  }
}

int grid_for(long long work) {
  long long b = cdiv64(work, 256);
  if (b > 4096) b = 4096;
  return (int)(b < 1 ? 1 : b);
}

}  // namespace

extern "C" int tspm_maxpool_fwd(int32_t n, int32_t h, int32_t w, int32_t c, int32_t k, int32_t stride, int32_t pad,
                                int32_t p, int32_t q, const float* x, float* y, uint8_t* idx, float* y_t,
                                int64_t ld_t, tspm_stream_t stream) {
  if (n <= 0 || h <= 0 || w <= 0 || c <= 0 || c % 4 || k <= 0 || k > 15 || stride <= 0 || pad < 0 || !x || !y || !idx)
    return TSPM_ERR_INVALID;
  if (p != (h + 2 * pad - k) / stride + 1 || q != (w + 2 * pad - k) / stride + 1 || p <= 0 || q <= 0)
    return TSPM_ERR_INVALID;
  if (y_t) {
    const long long M = (long long)p * q * n;
    if (M % 4 || ld_t < M || ld_t % 4 || (reinterpret_cast<uintptr_t>(y_t) & 15)) return TSPM_ERR_INVALID;
    hipLaunchKernelGGL(k_maxpool_fwd_t, dim3((unsigned)cdiv64(M, 64), cdiv(c, 64)), dim3(256), 0,
                       static_cast<hipStream_t>(stream), n, h, w, c, k, stride, pad, p, q, x, y, idx, y_t,
                       (long long)ld_t);
    TSPM_LAUNCH_CHECK();
    return TSPM_OK;
  }
  hipLaunchKernelGGL(k_maxpool_fwd, dim3((unsigned)cdiv64((long long)p * q * n * c / 4, 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), n, h, w, c, k, stride, pad, p, q, x, y, idx);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_maxpool_bwd(int32_t n, int32_t h, int32_t w, int32_t c, int32_t k, int32_t stride, int32_t pad,
                                int32_t p, int32_t q, const float* dy, const uint8_t* idx, float* dx,
                                tspm_stream_t stream) {
  if (n <= 0 || h <= 0 || w <= 0 || c <= 0 || c % 4 || k <= 0 || k > 15 || stride <= 0 || pad < 0 || !dy || !idx || !dx)
    return TSPM_ERR_INVALID;
  if (p != (h + 2 * pad - k) / stride + 1 || q != (w + 2 * pad - k) / stride + 1) return TSPM_ERR_INVALID;
  hipLaunchKernelGGL(k_maxpool_bwd, dim3((unsigned)cdiv64((long long)h * w * n * c / 4, 256)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), n, h, w, c, k, stride, pad, p, q, dy, idx, dx);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_avgpool_fwd(int32_t npos, int32_t n, int32_t c, const float* x, float* y, tspm_stream_t stream) {
  if (npos <= 0 || n <= 0 || c <= 0 || c % 4 || !x || !y) return TSPM_ERR_INVALID;
  hipLaunchKernelGGL(k_avgpool_fwd, dim3(grid_for((long long)n * c / 4)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), npos, n, c, x, y);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_avgpool_bwd(int32_t npos, int32_t n, int32_t c, const float* dy, int32_t ldy, float* dx,
                                tspm_stream_t stream) {
  if (npos <= 0 || n <= 0 || c <= 0 || c % 4 || ldy < c || ldy % 4 || !dy || !dx) return TSPM_ERR_INVALID;
  hipLaunchKernelGGL(k_avgpool_bwd, dim3(grid_for((long long)npos * n * c / 4)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), npos, n, c, dy, ldy, dx);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}
