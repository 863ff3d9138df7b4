#include <chrono>
#include <cstdio>
// Fusion head (Linear/ReLU/Dropout, MML_Suite/models/avmnist.py:219-230,267), encoder fc
// (resnet.py:150,217), cross-entropy (experiment_utils/loss.py:123-148), Adam (torch.optim.Adam as
// built at config/optimizer_config.py:199-226) and the image colormap LUT (data/avmnist.py:186-191).
#include "common.h"

#ifdef TSPM_STAMPS
// Diagnostic build only: phase stamps of k_head_rows (read back by scripts/head_bench.py --stamps)
__device__ unsigned long long tspm_g_stamps_misc[TSPM_STAMP_WAVES * TSPM_STAMP_SLOTS];
extern "C" int tspm_debug_stamps_misc(void* host_dst, size_t bytes) {
  if (bytes > sizeof(tspm_g_stamps_misc)) bytes = sizeof(tspm_g_stamps_misc);
  return hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(tspm_g_stamps_misc), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? 0 : 2;
}
extern "C" int tspm_debug_stamps_misc_clear(void) {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(tspm_g_stamps_misc)) != hipSuccess) return 2;
  return hipMemset(p, 0, sizeof(tspm_g_stamps_misc)) == hipSuccess ? 0 : 2;
}
#endif

namespace {

int grid_for(long long work) {
  long long b = cdiv64(work, 256);
  if (b > 4096) b = 4096;
  return (int)(b < 1 ? 1 : b);
}

// Small fp32 GEMM on MFMA for the encoder fc and the fusion head (at batch 128 the largest is
// 128x512x128): C[m,n] = epi(sum_k A(m,k) B(k,n)) with arbitrary element strides, so the three
// products of nn.Linear (forward, input grad, weight grad) are one kernel without transposes.
// One workgroup per 32x32 tile; WK waves split K and combine through LDS in fixed order
// (deterministic).  Optional epilogue: + bias[n], ReLU, dropout keep mask (keep[m*N+n] ? x*scale : 0),
// and rowsum[m] = sum_k A(m,k) (the bias gradient of the weight-grad product).
struct GemmArgs {
  int M, N, K;
  const float* A; long long sam, sak;
  const float* B; long long sbk, sbn;
  float* C; long long ldc;
  const float* bias;
  int relu;
  const uint8_t* keep;
  float kscale;
  float* rowsum;
  int vec;  // set by gemm_small: a K-contiguous operand with 16-byte aligned rows (see the main loop)
  int kslice;   // split-K across workgroups (gridDim.y slices of kslice, multiple of 32); 0 = whole K
  float* slab;  // split-K: raw partial products to slab[blockIdx.y][M][N] (epilogue in k_splitk_reduce)
  int quad;     // set by gemm_small: 64x64 tiles, one quadrant per wave (see k_gemm_small)
  int wkeff;    // pair launches: the product's own wave count (K split as in its own launch; extra waves idle)
  float* slab_rs;  // split-K with rowsum: per-slice row sums to slab_rs[blockIdx.y][M] (summed in k_splitk_reduce)
};

// One round of UU*8 reduction steps for the K-contiguous path of k_gemm_small: lane half kh covers
// k = kk .. kk+4*UU-1 (kk = k0 + 4*UU*kh) and MFMA (u, j) pairs k0+4u+j (kh 0) with k0+4*UU+4u+j (kh 1).
template <int UU>
TSPM_DEV void vec_round(const float* Ap, const float* Bp, long long sak, long long sbk, bool av, bool bv, bool mok,
                        bool nok, int kk, f32x16& acc, float& rs) {
  float a[UU][4], b[UU][4];
#pragma unroll
  for (int u = 0; u < UU; ++u) {
    if (av) {
      const float4 v = mok ? *reinterpret_cast<const float4*>(Ap + kk + 4 * u) : make_float4(0.f, 0.f, 0.f, 0.f);
      a[u][0] = v.x; a[u][1] = v.y; a[u][2] = v.z; a[u][3] = v.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) a[u][j] = mok ? Ap[(long long)(kk + 4 * u + j) * sak] : 0.f;
    }
    if (bv) {
      const float4 v = nok ? *reinterpret_cast<const float4*>(Bp + kk + 4 * u) : make_float4(0.f, 0.f, 0.f, 0.f);
      b[u][0] = v.x; b[u][1] = v.y; b[u][2] = v.z; b[u][3] = v.w;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) b[u][j] = nok ? Bp[(long long)(kk + 4 * u + j) * sbk] : 0.f;
    }
  }
#pragma unroll
  for (int u = 0; u < UU; ++u)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc = mfma32(a[u][j], b[u][j], acc);
      rs += a[u][j];
    }
}

template <int WK>
TSPM_DEV void gemm_body(const GemmArgs& g, int bid, float* lds) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // quad mode (g.quad, WK == 4): a 64x64 output tile per workgroup, one 32x32 quadrant per wave over
  // the whole K — the waves sharing A rows / B columns hit each other's lines in the CU's L1 instead
  // of re-reading them from L2 (large weight-grad / data-grad products with >= 1024 32x32 tiles).
  const bool quad = WK == 4 && g.quad;
  const int ts = quad ? 64 : 32;
  const int tiles_n = cdiv_dev(g.N, ts);
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int row = lane & 31, kh = lane >> 5;
  const int row0 = tm * ts + (quad ? (wave >> 1) * 32 : 0), col0 = tn * ts + (quad ? (wave & 1) * 32 : 0);
  const int m = row0 + row, col = col0 + row;
  const int kq = g.vec ? 32 : 8;  // wave K-chunks stay multiples of the main loop's round
  const int kbase = g.kslice ? blockIdx.y * g.kslice : 0;
  const int kend = g.kslice ? min(g.K, kbase + g.kslice) : g.K;
  const int wks = g.wkeff > 0 ? g.wkeff : WK;
  const int kchunk = quad ? kend - kbase : ((cdiv_dev(kend - kbase, wks) + kq - 1) / kq) * kq;
  const int kb = kbase + (quad ? 0 : wave * kchunk), ke = min(kend, kb + kchunk);
  const bool mok = m < g.M, nok = col < g.N;
  const float* Ap = g.A + (mok ? (long long)m * g.sam : 0);
  const float* Bp = g.B + (nok ? (long long)col * g.sbn : 0);
  const bool want_rs = g.rowsum != nullptr && col0 == 0;
  f32x16 acc = {};
  float rs = 0.f;
  // 4 reduction steps per round with all their loads issued before the MFMAs (the operands come from
  // L2 with ~0.5-1 us latency; one step per round left every round waiting on its own loads).  Same
  // MFMA / row-sum order as the one-step loop below, so results are bitwise unchanged.
  int k0 = kb;
  constexpr int U = 4;
  // K-contiguous operands (sak == 1 / sbk == 1: the nn.Linear forward x and w, the data-grad dy):
  // 32 reduction steps per round in a permuted order — lane half kh loads 16 consecutive k
  // (k0 + 16*kh .. +15) as four 16-byte loads, and MFMA (u, j) pairs k0+4u+j (kh 0) with
  // k0+16+4u+j (kh 1).  Both operands use the same permutation, so every k is summed exactly once;
  // each row's 128-byte line is fetched by one instruction group instead of 16 scalar loads.
  // The uneven-K tail falls through to the loops below (whose k sets are disjoint from these).
  if (g.vec) {
    const bool av = g.sak == 1, bv = g.sbk == 1;
    // (64-step rounds, vec_round<8>, measured no faster on the MMIMDb shapes: 64 vs 62 us for the
    // 256x512x4096 product — the 32x32 tile's operand re-reads bound it, not load latency)
    for (; k0 + 32 <= ke; k0 += 32) vec_round<4>(Ap, Bp, g.sak, g.sbk, av, bv, mok, nok, k0 + 16 * kh, acc, rs);
  }
  for (; k0 + 8 * U <= ke; k0 += 8 * U) {
    float a[U][4], b[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = k0 + 8 * u + 2 * j + kh;
        a[u][j] = mok ? Ap[(long long)k * g.sak] : 0.f;
        b[u][j] = nok ? Bp[(long long)k * g.sbk] : 0.f;
      }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc = mfma32(a[u][j], b[u][j], acc);
        rs += a[u][j];
      }
  }
  for (; k0 < ke; k0 += 8) {
    float a[4], b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + 2 * j + kh;
      const bool kok = k < ke;
      a[j] = (mok && kok) ? Ap[(long long)k * g.sak] : 0.f;
      b[j] = (nok && kok) ? Bp[(long long)k * g.sbk] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      acc = mfma32(a[j], b[j], acc);
      rs += a[j];
    }
  }
  if (want_rs) rs += __shfl_xor(rs, 32, 64);
  if (WK > 1 && !quad) {
    if (wave > 0) {
      float* dst = lds + (wave - 1) * (16 * 64 + 32);
#pragma unroll
      for (int r = 0; r < 16; ++r) dst[r * 64 + lane] = acc[r];
      if (lane < 32) dst[16 * 64 + lane] = rs;
    }
    __syncthreads();
    if (wave > 0) return;
#pragma unroll
    for (int w = 1; w < WK; ++w) {
      const float* src = lds + (w - 1) * (16 * 64 + 32);
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] += src[r * 64 + lane];
      rs += src[16 * 64 + row];
    }
  }
  const int ccol = col0 + (lane & 31);
  if (g.slab) {
    if (ccol < g.N) {
      float* sl = g.slab + (long long)blockIdx.y * g.M * g.N;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int cm = row0 + acc_row(r, lane);
        if (cm < g.M) sl[(long long)cm * g.N + ccol] = acc[r];
      }
    }
    if (want_rs && g.slab_rs && lane < 32 && mok) g.slab_rs[(long long)blockIdx.y * g.M + m] = rs;
    return;
  }
  if (ccol < g.N) {
    const float bv = g.bias ? g.bias[ccol] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int cm = row0 + acc_row(r, lane);
      if (cm >= g.M) continue;
      float v = acc[r] + bv;
      if (g.relu) v = relu_f(v);
      if (g.keep) v *= g.keep[(long long)cm * g.N + ccol] ? g.kscale : 0.f;  // x * mask (NaN stays NaN)
      g.C[(long long)cm * g.ldc + ccol] = v;
    }
  }
  if (want_rs && lane < 32 && mok) g.rowsum[m] = rs;
}

template <int WK>
__global__ __launch_bounds__(64 * WK) void k_gemm_small(GemmArgs g) {
  extern __shared__ float lds[];
  gemm_body<WK>(g, blockIdx.x, lds);
}

// Two independent products in one launch (the weight-grad and data-grad of one nn.Linear): blocks
// [0, tiles_a) run `a`, the rest run `b` — a workgroup-uniform branch, same body, same results as two
// launches.
template <int WK>
__global__ __launch_bounds__(64 * WK) void k_gemm_pair(GemmArgs a, GemmArgs b, int tiles_a) {
  extern __shared__ float lds[];
  if ((int)blockIdx.x < tiles_a)
    gemm_body<WK>(a, blockIdx.x, lds);
  else
    gemm_body<WK>(b, blockIdx.x - tiles_a, lds);
}

// Quad tiles (64x64, one quadrant per wave) measured on the MMIMDb image-encoder products at batch 256 did
// not pay — weight-grad 25.4 us (25.0 with 32x32 tiles), data-grad 36.8 us (25-31): the L1 sharing between
// a workgroup's waves does not materialise for these strides.  Off (not reachable).
constexpr bool quad_tiles_enabled() { return false; }

// Split-K combine: C = epi(sum over slices in order of slab[s]) with gemm_small's epilogue.
__global__ __launch_bounds__(256) void k_splitk_reduce(GemmArgs g, int splits) {
  const long long total = (long long)g.M * g.N;
  for (long long t = blockIdx.x * 256LL + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const int cm = (int)(t / g.N), ccol = (int)(t % g.N);
    float v = 0.f;
#pragma unroll 8
    for (int sidx = 0; sidx < splits; ++sidx) v += g.slab[(long long)sidx * total + t];  // loads in flight together
    if (g.bias) v += g.bias[ccol];
    if (g.relu) v = relu_f(v);
    if (g.keep) v *= g.keep[t] ? g.kscale : 0.f;
    g.C[(long long)cm * g.ldc + ccol] = v;
  }
  if (g.rowsum && g.slab_rs) {
    for (long long t = blockIdx.x * 256LL + threadIdx.x; t < g.M; t += (long long)gridDim.x * 256) {
      float v = 0.f;
#pragma unroll 8
      for (int sidx = 0; sidx < splits; ++sidx) v += g.slab_rs[(long long)sidx * g.M + t];
      g.rowsum[t] = v;
    }
  }
}

int gemm_small(const GemmArgs& g0, hipStream_t st, int splits = 1);

int gemm_small(const GemmArgs& g0, hipStream_t st, int splits) {
  GemmArgs g = g0;
  auto rows16 = [](const float* p, long long ld) {
    return (reinterpret_cast<uintptr_t>(p) & 15) == 0 && ld % 4 == 0;
  };
  const bool av = g.sak == 1 && rows16(g.A, g.sam), bv = g.sbk == 1 && rows16(g.B, g.sbn);
  g.vec = (av || bv) && (g.sak == 1 || g.sbk == 1) && g.K >= 128 ? 1 : 0;  // >= 32 k per wave
  if (g.vec && ((g.sak == 1 && !av) || (g.sbk == 1 && !bv))) g.vec = 0;
  const int tiles = cdiv(g.M, 32) * cdiv(g.N, 32);
  const GemmArgs gf = g;  // the final epilogue's arguments
  int kk = g.K;
  if (splits > 1) {
    g.kslice = ((cdiv(g.K, splits) + 31) / 32) * 32;
    splits = cdiv(g.K, g.kslice);
    kk = g.kslice;
  } else {
    g.slab = nullptr;
  }
  int wk = 1;
  // <= 256 threads: co-resides with conv work on other streams.  (8 waves per tile for the few-tile encoder fc
  // products, K = 512: step 2.584-2.590 vs 2.584-2.589 ms, no gain — profiles/r4/r4j_gemm_wk8_*.json)
  while (wk < 4 && kk / (wk * 2) >= 32) wk *= 2;
  // quad tiles where 32x32 tiles are plentiful (>= 1024) and K is short enough for one wave
  g.quad = (splits <= 1 && tiles >= 1024 && g.K <= 1024 && quad_tiles_enabled()) ? 1 : 0;
  if (g.quad) wk = 4;
  const size_t lds = g.quad ? 0 : (size_t)(wk - 1) * (16 * 64 + 32) * sizeof(float);
  const dim3 grid(g.quad ? cdiv(g.M, 64) * cdiv(g.N, 64) : tiles, splits > 1 ? splits : 1);
  switch (wk) {
    case 1: hipLaunchKernelGGL(k_gemm_small<1>, grid, dim3(64), lds, st, g); break;
    case 2: hipLaunchKernelGGL(k_gemm_small<2>, grid, dim3(128), lds, st, g); break;
    default: hipLaunchKernelGGL(k_gemm_small<4>, grid, dim3(256), lds, st, g); break;
  }
  TSPM_LAUNCH_CHECK();
  if (splits > 1) {
    hipLaunchKernelGGL(k_splitk_reduce, dim3(grid_for((long long)g.M * g.N)), dim3(256), 0, st, gf, splits);
    TSPM_LAUNCH_CHECK();
  }
  return TSPM_OK;
}

__global__ __launch_bounds__(256) void k_act_bwd(int N, int COLS, float* __restrict__ g, int ldg,
                                                 const float* __restrict__ y, int ldy, float scale) {
  const long long total = (long long)N * COLS;
  for (long long t = blockIdx.x * 256LL + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const int c = (int)(t % COLS), n = (int)(t / COLS);
    float* gp = g + (long long)n * ldg + c;
    *gp = y[(long long)n * ldy + c] > 0.f ? *gp * scale : 0.f;
  }
}

// counter-based RNG (tspm_dropout_* in common.h)
__global__ __launch_bounds__(256) void k_dropout_mask(long long count, float p, uint64_t seed,
                                                      const uint64_t* __restrict__ ctr, uint8_t* __restrict__ keep) {
  const uint64_t base = tspm_dropout_base(seed, ctr ? *ctr : 0ULL);
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < count; i += (long long)gridDim.x * 256)
    keep[i] = tspm_dropout_keep(base, i, p) ? 1 : 0;
}

// one workgroup; rows strided over threads; deterministic tree reduction in double
__global__ __launch_bounds__(256) void k_cross_entropy(int N, int K, const float* __restrict__ logits,
                                                       const int64_t* __restrict__ labels, float* __restrict__ loss,
                                                       float* __restrict__ dlogits, float gscale,
                                                       float* __restrict__ stats) {
  __shared__ double sl[256];
  __shared__ int sc[256];
  double lsum = 0.0;
  int correct = 0;
  const float invn = 1.0f / (float)N;
  for (int n = threadIdx.x; n < N; n += 256) {
    const float* z = logits + (long long)n * K;
    float mx = z[0];
    int am = 0;
    for (int k = 1; k < K; ++k)
      if (z[k] > mx) { mx = z[k]; am = k; }
    float se = 0.f;
    for (int k = 0; k < K; ++k) se += expf(z[k] - mx);
    const float lse = logf(se);
    const long long lab64 = labels[n];
    const bool lok = lab64 >= 0 && lab64 < K;  // out-of-range label: NaN loss/grad, no OOB read
    const int lab = lok ? (int)lab64 : 0;
    lsum += lok ? (double)(lse - (z[lab] - mx)) : (double)__builtin_nanf("");
    correct += (am == lab) ? 1 : 0;
    if (dlogits) {
      float* d = dlogits + (long long)n * K;
      for (int k = 0; k < K; ++k) {
        const float pk = expf(z[k] - mx) / se;
        d[k] = lok ? (pk - (k == lab ? 1.f : 0.f)) * invn * gscale : __builtin_nanf("");
      }
    }
  }
  sl[threadIdx.x] = lsum;
  sc[threadIdx.x] = correct;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) { sl[threadIdx.x] += sl[threadIdx.x + s]; sc[threadIdx.x] += sc[threadIdx.x + s]; }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float l = (float)(sl[0] / (double)N);
    if (loss) loss[0] = l * gscale;  // LossFunctionGroup total = weight * CE (weight 1.0: exact)
    if (stats) {
      stats[0] += (float)sl[0];
      stats[1] += (float)sc[0];
      stats[2] += (float)N;
    }
  }
}

__global__ void k_adam_begin(tspm_adam_hyper* h) { h->step += 1; }

// num_batches_tracked += value for every BatchNorm of a model (one shared int64 vector)
__global__ __launch_bounds__(64) void k_counters_add(long long n, int64_t* __restrict__ c, long long v) {
  for (long long i = blockIdx.x * 64LL + threadIdx.x; i < n; i += (long long)gridDim.x * 64) c[i] += v;
}

__global__ __launch_bounds__(256) void k_adam(long long count, float* __restrict__ p, const float* __restrict__ g,
                                              float* __restrict__ m, float* __restrict__ v,
                                              const tspm_adam_hyper* __restrict__ hp,
                                              const float* __restrict__ clip) {
  __shared__ AdamConsts sh;
  if (threadIdx.x == 0) sh = adam_consts(hp);
  __syncthreads();
  const AdamConsts c = sh;
  const float cc = clip ? clip[0] : 1.f;
  auto upd = [&](float& pp, float gg, float& mm, float& vv) { adam_update(pp, gg, mm, vv, c, clip != nullptr, cc); };
  const long long n4 = count >> 2;
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    f32x4 pp = ld4(p + 4 * i), gg = ld4(g + 4 * i), mm = ld4(m + 4 * i), vv = ld4(v + 4 * i);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float a = pp[j], b = mm[j], c = vv[j];
      upd(a, gg[j], b, c);
      pp[j] = a; mm[j] = b; vv[j] = c;
    }
    st4(p + 4 * i, pp);
    st4(m + 4 * i, mm);
    st4(v + 4 * i, vv);
  }
  if (blockIdx.x == 0 && threadIdx.x < (count & 3)) {
    const long long i = (n4 << 2) + threadIdx.x;
    float a = p[i], b = m[i], c = v[i];
    upd(a, g[i], b, c);
    p[i] = a; m[i] = b; v[i] = c;
  }
}

__global__ __launch_bounds__(256) void k_image_lut(long long count, const uint8_t* __restrict__ u8,
                                                   const uint8_t* __restrict__ lut, float* __restrict__ out) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < count; i += (long long)gridDim.x * 256)
    out[i] = (float)lut[u8[i]] * (1.0f / 255.0f);
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

extern "C" int tspm_linear_fwd(int32_t n, int32_t in, int32_t out, const float* x, int32_t ldx, const float* w,
                               const float* b, int32_t relu, const uint8_t* keep, float keep_scale, float* y,
                               int32_t ldy, tspm_stream_t stream) {
  if (n <= 0 || in <= 0 || out <= 0 || ldx < in || ldy < out || !x || !w || !y) return TSPM_ERR_INVALID;
  // y[n,o] = sum_i x[n,i] w[o,i]:  A = x (m=n, k=i), B(k=i, n=o) = w[o,i]
  GemmArgs g{n, out, in, x, ldx, 1, w, 1, in, y, ldy, b, relu, keep, keep_scale, nullptr};
  return gemm_small(g, static_cast<hipStream_t>(stream));
}

extern "C" size_t tspm_linear_fwd_splitk_workspace(int32_t n, int32_t in, int32_t out, int32_t splits) {
  if (n <= 0 || in <= 0 || out <= 0 || splits <= 1) return 0;
  const int ks = ((cdiv(in, splits) + 31) / 32) * 32;
  return (size_t)cdiv(in, ks) * n * out * sizeof(float);
}

extern "C" int tspm_linear_fwd_splitk(int32_t n, int32_t in, int32_t out, const float* x, int32_t ldx, const float* w,
                                      const float* b, int32_t relu, const uint8_t* keep, float keep_scale, float* y,
                                      int32_t ldy, int32_t splits, void* workspace, size_t workspace_bytes,
                                      tspm_stream_t stream) {
  if (n <= 0 || in <= 0 || out <= 0 || ldx < in || ldy < out || !x || !w || !y || splits < 1) return TSPM_ERR_INVALID;
  const size_t need = tspm_linear_fwd_splitk_workspace(n, in, out, splits);
  if (need > 0 && (!workspace || workspace_bytes < need)) return TSPM_ERR_WORKSPACE;
  GemmArgs g{n, out, in, x, ldx, 1, w, 1, in, y, ldy, b, relu, keep, keep_scale, nullptr};
  g.slab = static_cast<float*>(workspace);
  return gemm_small(g, static_cast<hipStream_t>(stream), need > 0 ? splits : 1);
}

extern "C" int tspm_linear_bwd_data(int32_t n, int32_t in, int32_t out, const float* dy, int32_t ldy, const float* w,
                                    float* dx, int32_t ldx, tspm_stream_t stream) {
  if (n <= 0 || in <= 0 || out <= 0 || ldx < in || ldy < out || !dy || !w || !dx) return TSPM_ERR_INVALID;
  // dx[n,i] = sum_o dy[n,o] w[o,i]
  GemmArgs g{n, in, out, dy, ldy, 1, w, in, 1, dx, ldx, nullptr, 0, nullptr, 1.f, nullptr};
  return gemm_small(g, static_cast<hipStream_t>(stream));
}

extern "C" int tspm_linear_bwd_weight(int32_t n, int32_t in, int32_t out, const float* x, int32_t ldx, const float* dy,
                                      int32_t ldy, float* dw, float* db, tspm_stream_t stream) {
  if (n <= 0 || in <= 0 || out <= 0 || ldx < in || ldy < out || !x || !dy || !dw) return TSPM_ERR_INVALID;
  // dw[o,i] = sum_n dy[n,o] x[n,i]  (A(m=o, k=n) = dy[n,o]);  db[o] = sum_n dy[n,o]
  GemmArgs g{out, in, n, dy, 1, ldy, x, ldx, 1, dw, in, nullptr, 0, nullptr, 1.f, db};
  return gemm_small(g, static_cast<hipStream_t>(stream));
}

extern "C" size_t tspm_linear_bwd_weight_splitk_workspace(int32_t n, int32_t in, int32_t out, int32_t splits) {
  if (n <= 0 || in <= 0 || out <= 0 || splits <= 1) return 0;
  const int ks = ((cdiv(n, splits) + 31) / 32) * 32;
  const long long sl = cdiv(n, ks);
  return (size_t)sl * ((long long)out * in + out) * sizeof(float);
}

extern "C" int tspm_linear_bwd_weight_splitk(int32_t n, int32_t in, int32_t out, const float* x, int32_t ldx,
                                             const float* dy, int32_t ldy, float* dw, float* db, int32_t splits,
                                             void* workspace, size_t workspace_bytes, tspm_stream_t stream) {
  if (n <= 0 || in <= 0 || out <= 0 || ldx < in || ldy < out || !x || !dy || !dw || splits < 1) return TSPM_ERR_INVALID;
  const size_t need = tspm_linear_bwd_weight_splitk_workspace(n, in, out, splits);
  if (need > 0 && (!workspace || workspace_bytes < need)) return TSPM_ERR_WORKSPACE;
  GemmArgs g{out, in, n, dy, 1, ldy, x, ldx, 1, dw, in, nullptr, 0, nullptr, 1.f, db};
  if (need > 0) {
    const int ks = ((cdiv(n, splits) + 31) / 32) * 32;
    g.slab = static_cast<float*>(workspace);
    g.slab_rs = g.slab + (long long)cdiv(n, ks) * out * in;
  }
  return gemm_small(g, static_cast<hipStream_t>(stream), need > 0 ? splits : 1);
}

// Up to 4 independent products in one launch: blocks are dealt out to the problems in order.
struct GemmMulti {
  GemmArgs p[4];
  int start[5];  // start[i] = first block of problem i, start[count] = total
  int count;
};

template <int WK>
__global__ __launch_bounds__(64 * WK) void k_gemm_multi(GemmMulti mp) {
  extern __shared__ float lds[];
  const int b = blockIdx.x;
  int i = 0;
  while (i + 1 < mp.count && b >= mp.start[i + 1]) ++i;  // workgroup-uniform
  gemm_body<WK>(mp.p[i], b - mp.start[i], lds);
}

// K-contiguity / vector decision and wave count of gemm_small, for a pair launch (no split, no quad).
int gemm_wk(GemmArgs& g) {
  auto rows16 = [](const float* p, long long ld) {
    return (reinterpret_cast<uintptr_t>(p) & 15) == 0 && ld % 4 == 0;
  };
  const bool av = g.sak == 1 && rows16(g.A, g.sam), bv = g.sbk == 1 && rows16(g.B, g.sbn);
  g.vec = (av || bv) && (g.sak == 1 || g.sbk == 1) && g.K >= 128 ? 1 : 0;
  if (g.vec && ((g.sak == 1 && !av) || (g.sbk == 1 && !bv))) g.vec = 0;
  g.kslice = 0;
  g.slab = nullptr;
  g.quad = 0;
  int wk = 1;
  while (wk < 4 && g.K / (wk * 2) >= 32) wk *= 2;
  g.wkeff = wk;
  return wk;
}

extern "C" int tspm_linear_bwd(int32_t n, int32_t in, int32_t out, const float* x, int32_t ldx, const float* dy,
                               int32_t ldy, const float* w, float* dw, float* db, float* dx, int32_t lddx,
                               tspm_stream_t stream) {
  if (n <= 0 || in <= 0 || out <= 0 || ldx < in || ldy < out || !x || !dy || !dw) return TSPM_ERR_INVALID;
  if (dx && (!w || lddx < in)) return TSPM_ERR_INVALID;
  hipStream_t st = static_cast<hipStream_t>(stream);
  // dw[o,i] = sum_n dy[n,o] x[n,i] (+ db = row sums);  dx[n,i] = sum_o dy[n,o] w[o,i]
  GemmArgs a{out, in, n, dy, 1, ldy, x, ldx, 1, dw, in, nullptr, 0, nullptr, 1.f, db};
  if (!dx) return gemm_small(a, st);
  GemmArgs b{n, in, out, dy, ldy, 1, w, in, 1, dx, lddx, nullptr, 0, nullptr, 1.f, nullptr};
  const int wa = gemm_wk(a), wb = gemm_wk(b);
  const int wk = wa > wb ? wa : wb;  // a product with fewer waves of its own leaves the extra ones idle
  // (empty K range, zero partials in the fixed-order combine): bitwise the two separate launches
  const int ta = cdiv(a.M, 32) * cdiv(a.N, 32), tb = cdiv(b.M, 32) * cdiv(b.N, 32);
  const size_t lds = (size_t)(wk - 1) * (16 * 64 + 32) * sizeof(float);
  switch (wk) {
    case 1: hipLaunchKernelGGL(k_gemm_pair<1>, dim3(ta + tb), dim3(64), lds, st, a, b, ta); break;
    case 2: hipLaunchKernelGGL(k_gemm_pair<2>, dim3(ta + tb), dim3(128), lds, st, a, b, ta); break;
    default: hipLaunchKernelGGL(k_gemm_pair<4>, dim3(ta + tb), dim3(256), lds, st, a, b, ta); break;
  }
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_linear_fwd_pair(int32_t n, int32_t in, int32_t out, const float* x0, int32_t ldx0, const float* w0,
                                    float* y0, int32_t ldy0, const float* x1, int32_t ldx1, const float* w1, float* y1,
                                    int32_t ldy1, tspm_stream_t stream) {
  if (n <= 0 || in <= 0 || out <= 0 || ldx0 < in || ldy0 < out || ldx1 < in || ldy1 < out || !x0 || !w0 || !y0 ||
      !x1 || !w1 || !y1)
    return TSPM_ERR_INVALID;
  hipStream_t st = static_cast<hipStream_t>(stream);
  GemmArgs a{n, out, in, x0, ldx0, 1, w0, 1, in, y0, ldy0, nullptr, 0, nullptr, 1.f, nullptr};
  GemmArgs b{n, out, in, x1, ldx1, 1, w1, 1, in, y1, ldy1, nullptr, 0, nullptr, 1.f, nullptr};
  const int wa = gemm_wk(a), wb = gemm_wk(b);
  const int wk = wa > wb ? wa : wb;
  const int ta = cdiv(a.M, 32) * cdiv(a.N, 32), tb = cdiv(b.M, 32) * cdiv(b.N, 32);
  const size_t lds = (size_t)(wk - 1) * (16 * 64 + 32) * sizeof(float);
  switch (wk) {
    case 1: hipLaunchKernelGGL(k_gemm_pair<1>, dim3(ta + tb), dim3(64), lds, st, a, b, ta); break;
    case 2: hipLaunchKernelGGL(k_gemm_pair<2>, dim3(ta + tb), dim3(128), lds, st, a, b, ta); break;
    default: hipLaunchKernelGGL(k_gemm_pair<4>, dim3(ta + tb), dim3(256), lds, st, a, b, ta); break;
  }
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_linear_bwd_multi(int32_t count, const tspm_linear_bwd_desc* descs, tspm_stream_t stream) {
  if (count < 1 || count > 2 || !descs) return TSPM_ERR_INVALID;
  GemmMulti mp{};
  int np = 0, wk = 1;
  for (int i = 0; i < count; ++i) {
    const tspm_linear_bwd_desc& d = descs[i];
    if (d.n <= 0 || d.in <= 0 || d.out <= 0 || d.ldx < d.in || d.ldy < d.out || !d.x || !d.dy || !d.dw)
      return TSPM_ERR_INVALID;
    if (d.dx && (!d.w || d.lddx < d.in)) return TSPM_ERR_INVALID;
    mp.p[np++] = GemmArgs{d.out, d.in, d.n, d.dy, 1, d.ldy, d.x, d.ldx, 1, d.dw, d.in, nullptr, 0, nullptr, 1.f, d.db};
    if (d.dx)
      mp.p[np++] = GemmArgs{d.n, d.in, d.out, d.dy, d.ldy, 1, d.w, d.in, 1, d.dx, d.lddx, nullptr, 0, nullptr, 1.f,
                            nullptr};
  }
  int total = 0;
  for (int i = 0; i < np; ++i) {
    const int w = gemm_wk(mp.p[i]);
    wk = w > wk ? w : wk;
    mp.start[i] = total;
    total += cdiv(mp.p[i].M, 32) * cdiv(mp.p[i].N, 32);
  }
  mp.start[np] = total;
  mp.count = np;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const size_t lds = (size_t)(wk - 1) * (16 * 64 + 32) * sizeof(float);
  switch (wk) {
    case 1: hipLaunchKernelGGL(k_gemm_multi<1>, dim3(total), dim3(64), lds, st, mp); break;
    case 2: hipLaunchKernelGGL(k_gemm_multi<2>, dim3(total), dim3(128), lds, st, mp); break;
    default: hipLaunchKernelGGL(k_gemm_multi<4>, dim3(total), dim3(256), lds, st, mp); break;
  }
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_act_bwd(int32_t n, int32_t cols, float* g, int32_t ldg, const float* y, int32_t ldy, float scale,
                            tspm_stream_t stream) {
  if (n <= 0 || cols <= 0 || ldg < cols || ldy < cols || !g || !y) return TSPM_ERR_INVALID;
  hipLaunchKernelGGL(k_act_bwd, dim3(grid_for((long long)n * cols)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     n, cols, g, ldg, y, ldy, scale);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_dropout_mask(int64_t count, float p, uint64_t seed, const uint64_t* counter, uint8_t* keep,
                                 tspm_stream_t stream) {
  if (count < 0 || !keep || p < 0.f || p >= 1.f) return TSPM_ERR_INVALID;
  if (count == 0) return TSPM_OK;
  hipLaunchKernelGGL(k_dropout_mask, dim3(grid_for(count)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     (long long)count, p, (unsigned long long)seed, counter, keep);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_cross_entropy(int32_t n, int32_t classes, const float* logits, const int64_t* labels, float* loss,
                                  float* dlogits, float grad_scale, float* stats, tspm_stream_t stream) {
  if (n <= 0 || classes <= 0 || !logits || !labels) return TSPM_ERR_INVALID;
  hipLaunchKernelGGL(k_cross_entropy, dim3(1), dim3(256), 0, static_cast<hipStream_t>(stream), n, classes, logits,
                     labels, loss, dlogits, grad_scale, stats);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_counters_add(int64_t* counters, int64_t count, int64_t value, tspm_stream_t stream) {
  if (count < 0 || (count > 0 && !counters)) return TSPM_ERR_INVALID;
  if (count == 0) return TSPM_OK;
  const long long blocks = cdiv64(count, 64) > 64 ? 64 : cdiv64(count, 64);
  hipLaunchKernelGGL(k_counters_add, dim3((unsigned)blocks), dim3(64), 0, static_cast<hipStream_t>(stream),
                     (long long)count, counters, (long long)value);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_adam_begin(tspm_adam_hyper* hyper, tspm_stream_t stream) {
  if (!hyper) return TSPM_ERR_INVALID;
  hipLaunchKernelGGL(k_adam_begin, dim3(1), dim3(1), 0, static_cast<hipStream_t>(stream), hyper);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_adam_step(int64_t count, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                              const tspm_adam_hyper* hyper, tspm_stream_t stream) {
  if (count < 0 || !param || !grad || !exp_avg || !exp_avg_sq || !hyper) return TSPM_ERR_INVALID;
  if (!aligned16(param) || !aligned16(grad) || !aligned16(exp_avg) || !aligned16(exp_avg_sq)) return TSPM_ERR_INVALID;
  if (count == 0) return TSPM_OK;
  long long blocks = cdiv64(count / 4 + 1, 256);
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(k_adam, dim3((int)blocks), dim3(256), 0, static_cast<hipStream_t>(stream), (long long)count, param,
                     grad, exp_avg, exp_avg_sq, hyper, nullptr);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_adam_step_clip(int64_t count, float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                                   const tspm_adam_hyper* hyper, const float* clip_coef, tspm_stream_t stream) {
  if (count < 0 || !param || !grad || !exp_avg || !exp_avg_sq || !hyper || !clip_coef) return TSPM_ERR_INVALID;
  if (!aligned16(param) || !aligned16(grad) || !aligned16(exp_avg) || !aligned16(exp_avg_sq)) return TSPM_ERR_INVALID;
  if (count == 0) return TSPM_OK;
  long long blocks = cdiv64(count / 4 + 1, 256);
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(k_adam, dim3((int)blocks), dim3(256), 0, static_cast<hipStream_t>(stream), (long long)count, param,
                     grad, exp_avg, exp_avg_sq, hyper, clip_coef);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

extern "C" int tspm_image_lut(int64_t count, const uint8_t* u8, const uint8_t* lut, float* out, tspm_stream_t stream) {
  if (count < 0 || !u8 || !lut || !out) return TSPM_ERR_INVALID;
  if (count == 0) return TSPM_OK;
  hipLaunchKernelGGL(k_image_lut, dim3(grid_for(count)), dim3(256), 0, static_cast<hipStream_t>(stream),
                     (long long)count, u8, lut, out);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

struct tspm_flag {
  unsigned long long* dev;   // device counter (only the bump kernel touches it)
  unsigned long long* host;  // coherent pinned host word the bump kernel publishes to
};
namespace {
__global__ void k_flag_bump(unsigned long long* dev, unsigned long long* host) {
  const unsigned long long v = dev[0] + 1;
  dev[0] = v;
  __hip_atomic_store(host, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
}  // namespace

extern "C" int tspm_flag_create(tspm_flag** flag) {
  if (!flag) return TSPM_ERR_INVALID;
  tspm_flag* f = new tspm_flag{nullptr, nullptr};
  if (hipMalloc(&f->dev, 64) != hipSuccess || hipMemset(f->dev, 0, 64) != hipSuccess ||
      hipHostMalloc(&f->host, 64, hipHostMallocCoherent) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
    if (f->dev) (void)hipFree(f->dev);
    if (f->host) (void)hipHostFree(f->host);
    delete f;
    return TSPM_ERR_LAUNCH;
  }
  __atomic_store_n(f->host, 0ull, __ATOMIC_SEQ_CST);
  *flag = f;
  return TSPM_OK;
}
extern "C" int tspm_flag_destroy(tspm_flag* f) {
  if (!f) return TSPM_ERR_INVALID;
  // every bump kernel that may still be queued has finished before the words go away
  const bool synced = hipDeviceSynchronize() == hipSuccess;
  const bool freed = hipFree(f->dev) == hipSuccess;
  const bool hfreed = hipHostFree(f->host) == hipSuccess;
  delete f;
  return synced && freed && hfreed ? TSPM_OK : TSPM_ERR_LAUNCH;
}
extern "C" int tspm_flag_bump(tspm_flag* f, tspm_stream_t stream) {
  if (!f) return TSPM_ERR_INVALID;
  hipLaunchKernelGGL(k_flag_bump, dim3(1), dim3(1), 0, static_cast<hipStream_t>(stream), f->dev, f->host);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}
extern "C" int tspm_flag_host_wait(tspm_flag* f, uint64_t value, int32_t timeout_ms) {
  if (!f) return TSPM_ERR_INVALID;
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned spin = 0;; ++spin) {
    if (__atomic_load_n(f->host, __ATOMIC_ACQUIRE) >= value) return TSPM_OK;
    if ((spin & 1023) == 1023) {
      const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0);
      if (ms.count() > timeout_ms) return TSPM_ERR_LAUNCH;
    }
    __builtin_ia32_pause();
  }
}

extern "C" int tspm_abi_version(void) { return TSPM_ABI_VERSION; }

extern "C" const char* tspm_status_string(int status) {
  switch (status) {
    case TSPM_OK: return "ok";
    case TSPM_ERR_INVALID: return "invalid argument";
    case TSPM_ERR_LAUNCH: return "kernel launch failed";
    case TSPM_ERR_WORKSPACE: return "workspace too small";
    default: return "unknown status";
  }
}

namespace {

// ---- fusion head train step (tspm_head_train_step) ---------------------------------------------------
// Launch 1: one workgroup per RB samples runs the head's whole row-local chain with the three weight
// matrices staged in LDS (w0 + w3 + w5 = 134 KB at 192 -> 128 -> 64 -> 10; read once per workgroup with
// 16-byte loads, so the six dependent products below see LDS latency, not L2 latency):
//   h1 = relu(x w0^T + b0) * keep/(1-p),  hh = relu(h1 w3^T + b3),  logits = hh w5^T + b5,  CE per row,
//   dlogits,  dz3 = (dlogits w5) * (hh > 0),  dz0 = (dz3 w3) * (h1 > 0 ? 1/(1-p) : 0),  dx = dz0 w0.
// A thread owns one output column for RPT rows: forward products read a weight row as 16-byte LDS loads
// (row pitch = 4 mod 64 words: the 16 lanes of a ds_read_b128 group hit distinct banks), transposed
// backward products read consecutive columns across lanes; the row values are LDS broadcasts.
// Launch 2 (k_head_wgrad): the weight gradients on the small-GEMM tiles + one workgroup reducing the
// per-row losses in row order.
// Row block per workgroup (RB) and threads: RB = 1 with 512 threads by default (round 5: 128 workgroups at batch
// 128 instead of 32 — the head sits on the critical path where the image stream idles); TSPM_HEAD_RB=4 keeps the
// round-4 shape (4 rows, 256 threads) for A/B.
constexpr int HEAD_MAXIN = 256, HEAD_MAXH = 256, HEAD_MAXH2 = 128, HEAD_MAXC = 16;
constexpr int head_ldc(int C) { return ((C + 3) & ~3) + 4; }  // logits rows 16-B aligned (ld4 reads of dlogits)

struct HeadArgs {
  tspm_head_desc d;
  float scale;  // 1/(1-p), or 1
};

// LDS floats of k_head_rows for a shape (weights + row blocks, every row padded by 4 floats; logits rows to 4)
size_t head_lds_floats(int F, int H, int H2, int C, int RB) {
  return (size_t)H * (F + 4) + (size_t)H2 * (H + 4) + (size_t)C * (H2 + 4) +
         (size_t)RB * ((F + 4) + (H + 4) + (H2 + 4) + head_ldc(C)) + (size_t)(H + H2 + C + RB);
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its global
// stores (__syncthreads' workgroup fence waits vmcnt(0) — a full write round trip per phase of the head's
// chain; no thread of k_head_rows reads another thread's global stores)
TSPM_DEV void head_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Y[r][o] = sum_k X[r][k] W[o][k] (W in LDS [O][ldw], K % 4 == 0; X in LDS, ld ldx) for rows [0, RB) in
// groups of RPT rows; epi(r, o, acc) consumes each result.
template <int RB, int RPT, class Epi>
TSPM_DEV void head_xwT(const float* X, int ldx, const float* W, int ldw, int K, int O, Epi epi) {
  static_assert(RB % RPT == 0, "rows per thread divide the row block");
  constexpr int G = RB / RPT;
  for (int item = threadIdx.x; item < O * G; item += blockDim.x) {
    const int o = item % O, rg = item / O;
    const float* wp = W + o * ldw;
    const float* xp = X + rg * RPT * ldx;
    // two partial sums per row (even / odd 4-element chunks of k): twice the independent FMA chains
    float acc[RPT][2];
#pragma unroll
    for (int r = 0; r < RPT; ++r) acc[r][0] = acc[r][1] = 0.f;
    int k = 0;
#pragma unroll 2
    for (; k + 8 <= K; k += 8) {
      const f32x4 w0 = ld4(wp + k), w1 = ld4(wp + k + 4);
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        const f32x4 x0 = ld4(xp + r * ldx + k), x1 = ld4(xp + r * ldx + k + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          acc[r][0] = fmaf(x0[j], w0[j], acc[r][0]);
          acc[r][1] = fmaf(x1[j], w1[j], acc[r][1]);
        }
      }
    }
    if (k < K) {  // K % 8 == 4
      const f32x4 w0 = ld4(wp + k);
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        const f32x4 x0 = ld4(xp + r * ldx + k);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[r][0] = fmaf(x0[j], w0[j], acc[r][0]);
      }
    }
#pragma unroll
    for (int r = 0; r < RPT; ++r) epi(rg * RPT + r, o, acc[r][0] + acc[r][1]);
  }
}

// Y[r][o] = sum_k X[r][k] W[k][o] (W in LDS [K][ldw]: consecutive o across lanes), rows in groups of RPT.
template <int RB, int RPT, class Epi>
TSPM_DEV void head_xW(const float* X, int ldx, const float* W, int ldw, int K, int O, Epi epi) {
  static_assert(RB % RPT == 0, "rows per thread divide the row block");
  constexpr int G = RB / RPT;
  for (int item = threadIdx.x; item < O * G; item += blockDim.x) {
    const int o = item % O, rg = item / O;
    const float* xp = X + rg * RPT * ldx;
    float acc[RPT];
#pragma unroll
    for (int r = 0; r < RPT; ++r) acc[r] = 0.f;
    int k = 0;
#pragma unroll 2
    for (; k + 4 <= K; k += 4) {
      float w[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = W[(k + j) * ldw + o];
#pragma unroll
      for (int r = 0; r < RPT; ++r) {
        const f32x4 x = ld4(xp + r * ldx + k);
        acc[r] = fmaf(x[0], w[0], acc[r]);
        acc[r] = fmaf(x[1], w[1], acc[r]);
        acc[r] = fmaf(x[2], w[2], acc[r]);
        acc[r] = fmaf(x[3], w[3], acc[r]);
      }
    }
    for (; k < K; ++k) {
      const float w = W[k * ldw + o];
#pragma unroll
      for (int r = 0; r < RPT; ++r) acc[r] = fmaf(xp[r * ldx + k], w, acc[r]);
    }
#pragma unroll
    for (int r = 0; r < RPT; ++r) epi(rg * RPT + r, o, acc[r]);
  }
}

// Staging of k_head_rows: the row block's inputs and the three weight matrices, global -> LDS (LDS rows
// padded by 4 floats).  The first U float4 of every thread of each segment are loaded for ALL segments
// before any LDS store, so the 134 KB of the 192 -> 128 -> 64 -> 10 head arrive in one memory round trip
// (one load at a time left every iteration waiting a full L2 round trip: 32 us for the head; 8 at a
// time: 20 us); larger shapes finish in further rounds.
struct HeadSeg {
  const float* src;
  float* dst;
  int rows, c4, srows;  // rows to write, float4 per row, rows present in src (the rest are zeros)
  long long ld;          // src row pitch (floats)
  TSPM_DEV int total() const { return rows * c4; }
  // i / c4 without an integer division (~40 instructions each: the staging's index math, not its loads, was
  // what made it slow — 9 us for 134 KB): a float reciprocal estimate corrected by one step either way
  TSPM_DEV int row_of(int i) const {
    int r = (int)((float)i * (1.0f / (float)c4));
    r -= r * c4 > i ? 1 : 0;
    r += (r + 1) * c4 <= i ? 1 : 0;
    return r;
  }
  // unconditional (clamped) load, so a round's loads are all in flight before the first LDS store
  TSPM_DEV f32x4 load(int i) const {
    const int ic = min(i, total() - 1), r = row_of(ic), k = ic - r * c4;
    const f32x4 v = ld4(src + (long long)min(r, srows - 1) * ld + 4 * k);
    return r < srows ? v : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  TSPM_DEV void store(int i, f32x4 v) const {
    const int r = row_of(i), k = i - r * c4;
    st4(dst + r * (4 * c4 + 4) + 4 * k, v);
  }
};
template <int U>
TSPM_DEV void head_load(const HeadSeg& g, f32x4 (&v)[U]) {
#pragma unroll
  for (int u = 0; u < U; ++u) v[u] = g.load(u * (int)blockDim.x + (int)threadIdx.x);
}
template <int U>
TSPM_DEV void head_store(const HeadSeg& g, const f32x4 (&v)[U]) {
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int i = u * (int)blockDim.x + (int)threadIdx.x;
    if (i < g.total()) g.store(i, v[u]);
  }
  for (int i = U * (int)blockDim.x + (int)threadIdx.x; i < g.total(); i += blockDim.x) g.store(i, g.load(i));
}

template <int RB, int THREADS>
__global__ __launch_bounds__(THREADS) void k_head_rows(HeadArgs a) {
  constexpr int R2 = RB < 2 ? RB : 2, R4 = RB < 4 ? RB : 4;  // rows per thread of the fc0 / dz0 / dx products
  const tspm_head_desc& d = a.d;
  extern __shared__ float lds[];
  const int F = d.in, H = d.hidden, H2 = d.hidden2, C = d.classes;
  const int ldx = F + 4, ldh = H + 4, ldh2 = H2 + 4, ldc = head_ldc(C);
  float* sw0 = lds;                      // [H][F + 4]
  float* sw3 = sw0 + H * ldx;            // [H2][H + 4]
  float* sw5 = sw3 + H2 * ldh;           // [C][H2 + 4]
  float* sx = sw5 + C * ldh2;            // [RB][F + 4]
  float* sh1 = sx + RB * ldx;       // [RB][H + 4]
  float* shh = sh1 + RB * ldh;      // [RB][H2 + 4]
  float* sz = shh + RB * ldh2;      // [RB][C + 4]
  float* sb0 = sz + RB * ldc;       // biases [H], [H2], [C]; labels of the row block [RB] (as int)
  float* sb3 = sb0 + H;
  float* sb5 = sb3 + H2;
  int* slab = reinterpret_cast<int*>(sb5 + C);
  const int n0 = blockIdx.x * RB;
  const int rows = min(RB, d.n - n0);
  const int t = threadIdx.x;
  TSPM_STAMP(tspm_g_stamps_misc, 0);
  TSPM_STAMP_CLK(tspm_g_stamps_misc, 6);
  // stage the row block's inputs (rows past n: zeros, never stored), the weights, biases and labels: every
  // global load is issued first (one memory round trip); x, w0, the biases and labels are stored before fc0,
  // w3 / w5 behind it (their loads land while fc0 runs)
  const HeadSeg g3{d.w3, sw3, H2, H / 4, H2, H}, g5{d.w5, sw5, C, H2 / 4, C, H2};
  // the default head's weights in one round: 128 x 64 (2048 float4: 8 per thread at 256), 64 x 10 (160: 1)
  constexpr int U0 = (128 * 192 / 4 + THREADS - 1) / THREADS, U3 = (64 * 128 / 4 + THREADS - 1) / THREADS;
  f32x4 v3[U3], v5[1];
  uint64_t base = 0;
  {
    const HeadSeg gx{d.x + (long long)n0 * d.ldx, sx, RB, F / 4, rows, d.ldx};
    const HeadSeg g0{d.w0, sw0, H, F / 4, H, F};
    f32x4 vx[(RB * 256 / 4 + THREADS - 1) / THREADS], v0[U0];  // x rows (F <= 256); 192 x 128
    const uint64_t ctr = (d.p > 0.f && d.gen_keep && d.counter) ? *d.counter : 0ULL;
    head_load(gx, vx);
    head_load(g0, v0);
    head_load(g3, v3);
    head_load(g5, v5);
    // biases [H], [H2], [C] and the row block's labels: element i = t, t + blockDim (unconditional loads)
    const int NB = H + H2 + C + RB;
    float bv[2];
    long long lv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = t + u * (int)blockDim.x;
      const float* bp = i < H ? d.b0 + i : i < H + H2 ? d.b3 + (i - H) : i < H + H2 + C ? d.b5 + (i - H - H2) : d.b0;
      bv[u] = *bp;
      const int r = min(max(i - (H + H2 + C), 0), rows - 1);
      lv[u] = d.labels[n0 + r];
    }
    head_store(gx, vx);
    head_store(g0, v0);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int i = t + u * (int)blockDim.x;
      if (i < H) sb0[i] = bv[u];
      else if (i < H + H2) sb3[i - H] = bv[u];
      else if (i < H + H2 + C) sb5[i - H - H2] = bv[u];
      else if (i < NB) {  // label of row r; out-of-range labels (int64) clamp to -1 (the CE below turns them into NaN)
        const int r = i - H - H2 - C;
        const long long l = r < rows ? lv[u] : 0;
        slab[r] = (l >= 0 && l < C) ? (int)l : -1;
      }
    }
    for (int i = t + 2 * (int)blockDim.x; i < NB; i += blockDim.x) {  // larger heads than the default
      if (i < H) sb0[i] = d.b0[i];
      else if (i < H + H2) sb3[i - H] = d.b3[i - H];
      else if (i < H + H2 + C) sb5[i - H - H2] = d.b5[i - H - H2];
      else {
        const int r = i - H - H2 - C;
        const long long l = r < rows ? d.labels[n0 + r] : 0;
        slab[r] = (l >= 0 && l < C) ? (int)l : -1;
      }
    }
    if (d.p > 0.f && d.gen_keep) base = tspm_dropout_base(d.seed, ctr);
  }
  head_sync();
  TSPM_STAMP(tspm_g_stamps_misc, 1);
  // fc0 + ReLU + dropout (tspm_linear_fwd's epilogue order: + bias, relu, * keep*scale)
  head_xwT<RB, R2>(sx, ldx, sw0, ldx, F, H, [&](int r, int o, float acc) {
    float v = relu_f(acc + sb0[o]);
    if (d.p > 0.f) {
      const long long i = (long long)(n0 + r) * H + o;
      bool kp;
      if (d.gen_keep) {
        kp = tspm_dropout_keep(base, i, d.p);
        if (r < rows) d.keep[i] = kp ? 1 : 0;
      } else {
        kp = r < rows ? d.keep[i] != 0 : false;
      }
      v *= kp ? a.scale : 0.f;
    }
    sh1[r * ldh + o] = v;
    if (r < rows) d.h1[(long long)(n0 + r) * H + o] = v;
  });
  head_store(g3, v3);
  head_store(g5, v5);
  head_sync();
  TSPM_STAMP(tspm_g_stamps_misc, 2);
  head_xwT<RB, 1>(sh1, ldh, sw3, ldh, H, H2, [&](int r, int o, float acc) {
    const float v = relu_f(acc + sb3[o]);
    shh[r * ldh2 + o] = v;
    if (r < rows) d.hh[(long long)(n0 + r) * H2 + o] = v;
  });
  head_sync();
  head_xwT<RB, 1>(shh, ldh2, sw5, ldh2, H2, C, [&](int r, int o, float acc) {
    const float v = acc + sb5[o];
    sz[r * ldc + o] = v;
    if (r < rows) d.logits[(long long)(n0 + r) * C + o] = v;
  });
  head_sync();
  TSPM_STAMP(tspm_g_stamps_misc, 3);
  // cross-entropy per row (tspm_cross_entropy's arithmetic); sz becomes dlogits.  Wave 0: 16 lanes per row,
  // lane k owns class k — the exponentials in parallel, the max scan and the sum of exponentials in class
  // order by every lane of the row (the same operations and order as one thread per row)
  if (t < 16 * RB) {
    const int r = t >> 4, k = t & 15;
    float* z = sz + r * ldc;
    const bool kv = k < C;
    if (r < rows) {
      float mx = z[0];
      int am = 0;
      for (int j = 1; j < C; ++j)
        if (z[j] > mx) { mx = z[j]; am = j; }
      const float e = kv ? expf(z[k] - mx) : 0.f;
      float se = 0.f;
      for (int j = 0; j < C; ++j) se += __shfl(e, (t & ~15) + j, 64);
      const bool lok = slab[r] >= 0;
      const int lab = lok ? slab[r] : 0;
      if (k == 0) {
        const float lse = logf(se);
        d.row_ws[n0 + r] = lok ? lse - (z[lab] - mx) : __builtin_nanf("");
        d.row_ws[d.n + n0 + r] = (am == lab) ? 1.f : 0.f;
      }
      const float invn = 1.0f / (float)d.n;
      const float pk = e / se;
      const float g = lok ? (pk - (k == lab ? 1.f : 0.f)) * invn * d.loss_weight : __builtin_nanf("");
      if (kv) {  // after every lane of the row has read z (one wave: program order)
        z[k] = g;
        d.dlogits[(long long)(n0 + r) * C + k] = g;
      }
    } else if (kv) {
      z[k] = 0.f;
    }
  }
  head_sync();
  TSPM_STAMP(tspm_g_stamps_misc, 4);
  // dz3 = (dlogits w5) * (hh > 0)   (w5 is [C][H2]: the transposed product) -> shh; item (r, o)'s hh value
  // is read and overwritten by its own thread only
  head_xW<RB, 1>(sz, ldc, sw5, ldh2, C, H2, [&](int r, int o, float acc) {
    const float v = shh[r * ldh2 + o] > 0.f ? acc : 0.f;
    if (r < rows) d.dz3[(long long)(n0 + r) * H2 + o] = v;
    shh[r * ldh2 + o] = v;
  });
  head_sync();
  // dz0 = (dz3 w3) * (h1 > 0 ? scale : 0)   (w3 is [H2][H]) -> sh1
  head_xW<RB, R2>(shh, ldh2, sw3, ldh, H2, H, [&](int r, int o, float acc) {
    const float v = sh1[r * ldh + o] > 0.f ? acc * a.scale : 0.f;
    if (r < rows) d.dz0[(long long)(n0 + r) * H + o] = v;
    sh1[r * ldh + o] = v;
  });
  head_sync();
  // dx = dz0 w0   (w0 is [H][F])
  head_xW<RB, R4>(sh1, ldh, sw0, ldx, H, F, [&](int r, int o, float acc) {
    if (r < rows) d.dx[(long long)(n0 + r) * d.lddx + o] = acc;
  });
  TSPM_STAMP(tspm_g_stamps_misc, 5);
  TSPM_STAMP_CLK(tspm_g_stamps_misc, 7);
}

template <int WK>
__global__ __launch_bounds__(64 * WK) void k_head_wgrad(GemmMulti mp, int total, HeadArgs a) {
  extern __shared__ float lds[];
  const int b = blockIdx.x;
  if (b < total) {
    int i = 0;
    while (i + 1 < mp.count && b >= mp.start[i + 1]) ++i;  // workgroup-uniform
    gemm_body<WK>(mp.p[i], b - mp.start[i], lds);
    return;
  }
  // the loss: fixed-order sums of the per-row losses / correct flags, in double
  const tspm_head_desc& d = a.d;
  double* red = reinterpret_cast<double*>(lds);
  const int T = 64 * WK;
  double ls = 0.0, cs = 0.0;
  for (int n = threadIdx.x; n < d.n; n += T) {
    ls += (double)d.row_ws[n];
    cs += (double)d.row_ws[d.n + n];
  }
  red[threadIdx.x] = ls;
  red[T + threadIdx.x] = cs;
  __syncthreads();
  for (int s = T / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      red[threadIdx.x] += red[threadIdx.x + s];
      red[T + threadIdx.x] += red[T + threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float l = (float)(red[0] / (double)d.n);
    d.loss[0] = l * d.loss_weight;
    if (d.adam_step) d.adam_step[0] += 1;  // after launch 1 read the step counter (dropout), before any Adam launch
    if (d.stats) {
      d.stats[0] += (float)red[0];
      d.stats[1] += (float)red[T];
      d.stats[2] += (float)d.n;
    }
  }
}

}  // namespace

extern "C" int tspm_head_train_step(const tspm_head_desc* desc, tspm_stream_t stream) {
  if (!desc) return TSPM_ERR_INVALID;
  const tspm_head_desc& d = *desc;
  if (d.rows_per_block != 0 && d.rows_per_block != 1 && d.rows_per_block != 4) return TSPM_ERR_INVALID;
  if (d.n <= 0 || d.in <= 0 || d.hidden <= 0 || d.hidden2 <= 0 || d.classes <= 0) return TSPM_ERR_INVALID;
  if (d.in > HEAD_MAXIN || d.hidden > HEAD_MAXH || d.hidden2 > HEAD_MAXH2 || d.classes > HEAD_MAXC)
    return TSPM_ERR_INVALID;
  if (d.in % 4 || d.hidden % 4 || d.hidden2 % 4 || d.ldx < d.in || d.ldx % 4 || d.lddx < d.in) return TSPM_ERR_INVALID;
  if (!d.x || !d.w0 || !d.b0 || !d.w3 || !d.b3 || !d.w5 || !d.b5 || !d.labels || !d.h1 || !d.hh || !d.logits ||
      !d.dlogits || !d.dz3 || !d.dz0 || !d.dx || !d.row_ws || !d.gw0 || !d.gb0 || !d.gw3 || !d.gb3 || !d.gw5 ||
      !d.gb5 || !d.loss)
    return TSPM_ERR_INVALID;
  if (!aligned16(d.x) || !aligned16(d.w0) || !aligned16(d.w3) || !aligned16(d.w5)) return TSPM_ERR_INVALID;
  if (d.p < 0.f || d.p >= 1.f || (d.p > 0.f && !d.keep)) return TSPM_ERR_INVALID;
  hipStream_t st = static_cast<hipStream_t>(stream);
  HeadArgs a{d, d.p > 0.f ? 1.0f / (1.0f - d.p) : 1.0f};
  // one sample per workgroup up to 256 rows (batch 128: 21.2 vs 26.7 us graph-timed, step -9 us); blocks of 4
  // beyond (batch 1024: 1,024 workgroups each staging the 134 KB of weights took 52.9 vs 21.1 us,
  // gpurun_out/r5b_head*.txt); tspm_head_desc.rows_per_block = 1 / 4 forces one (ABI 21; 0 = this default)
  const int rb = d.rows_per_block ? d.rows_per_block : (d.n <= 256 ? 1 : 4);
  const size_t lds_rows = head_lds_floats(d.in, d.hidden, d.hidden2, d.classes, rb) * sizeof(float);
  if (lds_rows > 160 * 1024) return TSPM_ERR_INVALID;
  if (rb == 4) hipLaunchKernelGGL((k_head_rows<4, 256>), dim3(cdiv(d.n, 4)), dim3(256), lds_rows, st, a);
  else hipLaunchKernelGGL((k_head_rows<1, 512>), dim3(d.n), dim3(512), lds_rows, st, a);
  TSPM_LAUNCH_CHECK();
  // weight gradients: dw[o,i] = sum_n dz[n,o] in[n,i], db[o] = sum_n dz[n,o] (tspm_linear_bwd_weight's
  // operands), plus the loss workgroup
  GemmMulti mp{};
  mp.p[0] = GemmArgs{d.classes, d.hidden2, d.n, d.dlogits, 1, d.classes, d.hh, d.hidden2, 1, d.gw5, d.hidden2,
                     nullptr, 0, nullptr, 1.f, d.gb5};
  mp.p[1] = GemmArgs{d.hidden2, d.hidden, d.n, d.dz3, 1, d.hidden2, d.h1, d.hidden, 1, d.gw3, d.hidden, nullptr, 0,
                     nullptr, 1.f, d.gb3};
  mp.p[2] = GemmArgs{d.hidden, d.in, d.n, d.dz0, 1, d.hidden, d.x, d.ldx, 1, d.gw0, d.in, nullptr, 0, nullptr, 1.f,
                     d.gb0};
  mp.count = 3;
  int total = 0, wk = 1;
  for (int i = 0; i < 3; ++i) {
    const int w = gemm_wk(mp.p[i]);
    wk = w > wk ? w : wk;
    mp.start[i] = total;
    total += cdiv(mp.p[i].M, 32) * cdiv(mp.p[i].N, 32);
  }
  mp.start[3] = total;
  // LDS: the small-GEMM combine, or 2 x threads doubles for the loss workgroup
  const size_t lds_gemm = (size_t)(wk - 1) * (16 * 64 + 32) * sizeof(float);
  const size_t lds_loss = (size_t)2 * 64 * wk * sizeof(double);
  const size_t lds = lds_gemm > lds_loss ? lds_gemm : lds_loss;
  switch (wk) {
    case 1: hipLaunchKernelGGL(k_head_wgrad<1>, dim3(total + 1), dim3(64), lds, st, mp, total, a); break;
    case 2: hipLaunchKernelGGL(k_head_wgrad<2>, dim3(total + 1), dim3(128), lds, st, mp, total, a); break;
    default: hipLaunchKernelGGL(k_head_wgrad<4>, dim3(total + 1), dim3(256), lds, st, mp, total, a); break;
  }
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}
