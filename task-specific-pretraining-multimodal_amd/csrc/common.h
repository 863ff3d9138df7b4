// Shared definitions for the tspm gfx950 kernels.
//
// Activation layout everywhere: "HWNC" — rows ordered (h, w, n), C contiguous floats per row.
// Position-major rows make the set of non-padding 3x3 taps uniform across a wave whose rows share
// one (h, w) (true whenever the batch is a multiple of the wave's row count), so padding taps are
// skipped instead of multiplied by zero (61 % of nominal conv MACs are valid taps).
// Weight layout: OHWI (= the channels_last view of the reference's OIHW nn.Conv2d weight).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/tspm.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

#define TSPM_DEV __device__ __forceinline__

TSPM_DEV f32x16 mfma32(float a, float b, f32x16 c) {
  // v_mfma_f32_32x32x2_f32: lane l supplies A[l&31][l>>5], B[l>>5][l&31];
  // D reg r of lane l = C[(r&3) + 8*(r>>2) + 4*(l>>5)][l&31]
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

TSPM_DEV int acc_row(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

// Counter-based dropout RNG (splitmix64 finaliser over seed / device counter / element index), shared by
// tspm_dropout_mask and the MMIMDb MaxOut forward that draws its mask in-launch (same keep bits).
TSPM_DEV uint64_t tspm_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
TSPM_DEV uint64_t tspm_dropout_base(uint64_t seed, uint64_t c) { return tspm_mix64(seed ^ tspm_mix64(c + 0x9e3779b97f4a7c15ULL)); }
TSPM_DEV bool tspm_dropout_keep(uint64_t base, long long i, float p) {
  const uint64_t h = tspm_mix64(base + (uint64_t)i * 0x9e3779b97f4a7c15ULL);
  return (float)(h >> 40) * (1.0f / 16777216.0f) >= p;
}

// nn.ReLU / F.relu: clamp_min(x, 0), which propagates NaN (fmaxf would return 0 for a NaN input)
// Adam (torch.optim.Adam, L2 weight decay folded into the gradient): the per-launch constants and the element
// update, shared by k_adam (misc.hip) and the weight-gradient epilogues that apply it (conv_lds.hip), so both
// forms give bitwise the same parameters and moments.  1-beta2 and the bias corrections are formed in double and
// rounded to fp32 once, as ATen does.
struct AdamConsts {
  float step_size, bc2s, w1, b2, omb2, eps, wd, gs;
};
TSPM_DEV AdamConsts adam_consts(const tspm_adam_hyper* hp) {
  const tspm_adam_hyper h = *hp;
  const double bc1 = 1.0 - pow(h.beta1, (double)h.step);
  const double bc2 = 1.0 - pow(h.beta2, (double)h.step);
  AdamConsts c;
  c.step_size = (float)(h.lr / bc1);
  c.bc2s = (float)sqrt(bc2);
  c.w1 = (float)(1.0 - h.beta1);
  c.b2 = (float)h.beta2;
  c.omb2 = (float)(1.0 - h.beta2);
  c.eps = (float)h.eps;
  c.wd = (float)h.weight_decay;
  c.gs = (float)h.grad_scale;
  return c;
}
// adam_consts held in scalar registers (every lane computes the same values)
TSPM_DEV AdamConsts adam_consts_uniform(const tspm_adam_hyper* hp) {
  AdamConsts c = adam_consts(hp);
  auto u = [](float f) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(f))); };
  c.step_size = u(c.step_size); c.bc2s = u(c.bc2s); c.w1 = u(c.w1); c.b2 = u(c.b2);
  c.omb2 = u(c.omb2); c.eps = u(c.eps); c.wd = u(c.wd); c.gs = u(c.gs);
  return c;
}
// g' = g * grad_scale [* clip]; g' += wd * p; m = lerp(m, g', 1-beta1); v = beta2 v + (1-beta2) g'^2;
// p -= step_size * m / (sqrt(v) / sqrt(bc2) + eps)
TSPM_DEV void adam_update(float& pp, float gg, float& mm, float& vv, const AdamConsts& c, bool clip, float cc) {
  gg = gg * c.gs;
  if (clip) gg = gg * cc;
  if (c.wd != 0.f) gg = gg + c.wd * pp;
  mm = mm + c.w1 * (gg - mm);
  vv = vv * c.b2;
  vv = vv + c.omb2 * gg * gg;
  const float denom = sqrtf(vv) / c.bc2s + c.eps;
  pp = pp + (-c.step_size) * (mm / denom);
}

TSPM_DEV float relu_f(float v) { return v > 0.f ? v : (v != v ? v : 0.f); }
TSPM_DEV f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
TSPM_DEV void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }

TSPM_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

TSPM_DEV int cdiv_dev(int a, int b) { return (a + b - 1) / b; }

static inline int cdiv(int a, int b) { return (a + b - 1) / b; }
static inline int64_t cdiv64(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Diagnostic build only (-DTSPM_STAMPS, `make stamps` → libtspm_stamps.so): lane 0 of every wave
// records s_memrealtime (100 MHz, chip-global) at numbered points of a kernel into a per-TU device
// buffer read back by tspm_debug_stamps().  The product build compiles these to nothing.
#ifdef TSPM_STAMPS
#define TSPM_STAMP_SLOTS 12  // 0-7 phase stamps, 8-11 conv_lds.hip LoopClock
#define TSPM_STAMP_WAVES (1 << 18)
#define TSPM_STAMP(buf, slot)                                                                             \
  do {                                                                                                    \
    const unsigned long long t__ = __builtin_amdgcn_s_memrealtime();                                     \
    const unsigned long long w__ = ((unsigned long long)blockIdx.x +                                     \
                                    (unsigned long long)gridDim.x * (blockIdx.y + (unsigned long long)gridDim.y * blockIdx.z)) * \
                                       (blockDim.x >> 6) + (threadIdx.x >> 6);                           \
    if ((threadIdx.x & 63) == 0 && w__ < TSPM_STAMP_WAVES) buf[w__ * TSPM_STAMP_SLOTS + (slot)] = t__;  \
  } while (0)
// slot 6 / 7: s_memtime (shader clock) at entry / exit, for the in-kernel clock
#define TSPM_STAMP_CLK(buf, slot)                                                                         \
  do {                                                                                                    \
    const unsigned long long t__ = __builtin_amdgcn_s_memtime();                                         \
    const unsigned long long w__ = ((unsigned long long)blockIdx.x +                                     \
                                    (unsigned long long)gridDim.x * (blockIdx.y + (unsigned long long)gridDim.y * blockIdx.z)) * \
                                       (blockDim.x >> 6) + (threadIdx.x >> 6);                           \
    if ((threadIdx.x & 63) == 0 && w__ < TSPM_STAMP_WAVES) buf[w__ * TSPM_STAMP_SLOTS + (slot)] = t__;  \
  } while (0)
#else
#define TSPM_STAMP_CLK(buf, slot) \
  do {                            \
  } while (0)
#define TSPM_STAMP(buf, slot) \
  do {                        \
  } while (0)
#endif

#define TSPM_LAUNCH_CHECK()                               \
  do {                                                    \
    hipError_t e__ = hipGetLastError();                   \
    if (e__ != hipSuccess) return TSPM_ERR_LAUNCH;        \
  } while (0)

// Write-through (sc1) store: visible at agent scope once the storing wave drains vmcnt, without
// a release fence (whose buffer_wbl2 writes back the whole XCD L2).
TSPM_DEV void st_sc1(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
// L1-bypassing (sc1) global load of hand-off payload: `global_load_dword … sc1` (global address
// space, never flat).  Used for EVERY load of bytes another workgroup published with st_sc1 in
// the same launch, so the reader needs no agent-scope acquire (MI355X_MICROARCH.md, "Valid forms",
// first row of the sc1 hand-off table: one lane's relaxed agent add after every storing wave's
// vmcnt(0) wait and a workgroup barrier; the last adder's workgroup loads behind a barrier).
TSPM_DEV float ld_sc1(const float* p) {
  return __hip_atomic_load((__attribute__((address_space(1))) float*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// In-launch hand-off to the LAST arriving workgroup of a group (cdna_hip_programming.md §5 and
// §6 Guideline 16, the sc1 form): every wave has stored its share of the payload with st_sc1 and
// drains vmcnt, the workgroup draws a ticket (relaxed agent-scope add); the workgroup that draws
// total-1 acquires at agent scope (drops this CU's stale L1 lines), re-arms the counter to 0 for the
// next launch and returns true in every thread.  `flag` is one int of the kernel's LDS.  Every
// thread of the workgroup must call this (it contains barriers).  Counters must be zero before the
// first launch that uses them.
//
// acquire == false: the caller reads every byte of the payload with ld_sc1 (L1 bypassed), so the
// ≈1.7 µs agent acquire (buffer_inv sc1 + its wait) is skipped — the payload's visibility then rests
// on the sc1 stores and loads alone (MI355X_MICROARCH.md, sc1 hand-off table, first row).
TSPM_DEV bool last_arriver(unsigned* cnt, unsigned total, int* flag, bool acquire = true) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == total - 1;
    if (last) {
      if (acquire) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    *flag = last;
  }
  __syncthreads();
  const bool last = *flag != 0;
  __syncthreads();
  return last;
}

// Per-channel merge of BatchNorm partial statistics {K, mean-K, M2} of G row tiles (tile t holds
// min(rpt, M - t*rpt) rows) for channels [c0, c0+CB), in double with a fixed-order reduction, by
// ONE workgroup whose size is a power-of-two multiple of CB.  Writes save_mean / save_invstd and
// updates the running statistics (momentum, unbiased variance) like nn.BatchNorm2d.
// `red` must hold blockDim.x doubles, `smu` CB doubles (LDS).
//
// bn_merge_range is the merge itself over tiles [g_lo, g_hi) of a partial array with G_all tiles:
// returns (in the threads with t < CB) the range's mean and sum of squared deviations in double.
// Fixed-order sum of v over the GG = T / CB threads that share channel slot t % CB (CB a power of two);
// the result is valid in threads t < CB.  Within a wave the slots' copies are folded by xor butterflies
// (CB < 64: lanes l and l ^ o, o = CB .. 32, hold the same slot), then the waves' (or, for CB >= 64, the
// threads') partials are added in index order through `red` — one barrier instead of log2(GG).
TSPM_DEV double bn_group_sum(double v, int t, int CB, int T, double* red) {
  int parts;
  if (CB < 64) {
    for (int o = CB; o < 64; o <<= 1) v += __shfl_xor(v, o, 64);
    if ((t & 63) < CB) red[(t >> 6) * CB + (t & 63)] = v;
    parts = T >> 6;
  } else {
    red[t] = v;
    parts = T / CB;
  }
  __syncthreads();
  double r = 0.0;
  if (t < CB)
    for (int j = 0; j < parts; ++j) r += red[j * CB + t];
  return r;
}

template <bool SC1 = false>  // SC1: the partials are an in-launch hand-off read with ld_sc1
TSPM_DEV void bn_merge_range(long long M, int C, int G_all, long long rpt, const float* part, int g_lo, int g_hi,
                             int c0, int CB, double* red, double* smu, double& mean_out, double& m2_out,
                             int nthreads = 0) {
  auto ld = [](const float* p) -> float {
    if constexpr (SC1) return ld_sc1(p);
    else return *p;
  };
  // nthreads: the threads taking part (0 = the whole workgroup); the LDS conv kernels' loader waves
  // have left by the time their compute threads merge
  const int t = threadIdx.x, T = nthreads > 0 ? nthreads : (int)blockDim.x;
  const int GG = T / CB, cl = t % CB, gg = t / CB;
  const int c = c0 + cl;
  const bool cok = c < C;
  const long long plane = (long long)G_all * C;
  const long long n_rows = min((long long)g_hi * rpt, M) - (long long)g_lo * rpt;
  // tiles g_lo+gg, g_lo+gg+GG, ... in batches of 8 independent loads (the reads follow an acquire:
  // they miss in cache, so issue them together).  The loads are unconditional — tiles past g_hi re-read
  // tile g_hi-1 and get weight 0 — because a load under `if (g < g_hi)` made the compiler wait for each
  // tile's loads before issuing the next (vmcnt(0)/(1) after every tile: 11.9 us for the audio stem's
  // 3,008-tile merge).  When the whole range is one batch per thread (every layer but the audio stem's),
  // the three planes are loaded once and the second pass runs from registers.
  const bool one = g_hi - g_lo <= 8 * GG;
  float k0[8], k1[8], k2[8];
  auto load = [&](int g0, bool m2) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const long long o = (long long)min(g0 + u * GG, g_hi - 1) * C + c;
      k0[u] = ld(part + o);
      k1[u] = ld(part + plane + o);
      if (m2) k2[u] = ld(part + 2 * plane + o);
    }
  };
  auto nb_of = [&](int g) -> double { return g < g_hi ? (double)min(rpt, M - (long long)g * rpt) : 0.0; };
  double s = 0.0;
  if (cok)
    for (int g0 = g_lo + gg; g0 < g_hi; g0 += 8 * GG) {
      load(g0, one);
#pragma unroll
      for (int u = 0; u < 8; ++u) s += nb_of(g0 + u * GG) * ((double)k0[u] + (double)k1[u]);
    }
  s = bn_group_sum(s, t, CB, T, red);
  if (t < CB) smu[cl] = s / (double)n_rows;
  __syncthreads();
  const double mean = smu[cl];
  double q = 0.0;
  if (cok)
    for (int g0 = g_lo + gg; g0 < g_hi; g0 += 8 * GG) {
      if (!one) load(g0, true);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int g = g0 + u * GG;
        if (g < g_hi) {
          const double nb = nb_of(g);
          const double mb = (double)k0[u] + (double)k1[u];
          q += (double)k2[u] + nb * (mb - mean) * (mb - mean);
        }
      }
    }
  q = bn_group_sum(q, t, CB, T, red);
  mean_out = mean;
  m2_out = q;  // valid in threads t < CB
  __syncthreads();  // red is reused by the caller's next merge
}

// First level of a two-level merge: tiles [g_lo, g_hi) of `part` (G_all tiles) into ONE tile
// `g_out` of `part1` (G1 tiles) in the same {K, mean-K, M2} format (K = mean rounded to float, so
// mean-K carries the rounding residual), written through (sc1) for the second-level merger.
template <bool SC1 = false>
TSPM_DEV void bn_merge_level1(long long M, int C, int G_all, long long rpt, const float* part, int g_lo, int g_hi,
                              int c0, int CB, float* part1, int G1, int g_out, double* red, double* smu,
                              int nthreads = 0) {
  double mean, m2;
  bn_merge_range<SC1>(M, C, G_all, rpt, part, g_lo, g_hi, c0, CB, red, smu, mean, m2, nthreads);
  const int t = threadIdx.x, c = c0 + t;
  if (t < CB && c < C) {
    const long long plane1 = (long long)G1 * C, o = (long long)g_out * C + c;
    const float K = (float)mean;
    __hip_atomic_store(part1 + o, K, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(part1 + plane1 + o, (float)(mean - (double)K), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(part1 + 2 * plane1 + o, (float)m2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

template <bool SC1 = false>
TSPM_DEV void bn_merge_block(long long M, int C, int G, long long rpt, const float* part, int c0, int CB,
                             float* rmean, float* rvar, float momentum, float eps, float* smean, float* sinv,
                             double* red, double* smu, int nthreads = 0) {
  double mean, m2;
  bn_merge_range<SC1>(M, C, G, rpt, part, 0, G, c0, CB, red, smu, mean, m2, nthreads);
  const int cl = threadIdx.x, c = c0 + cl;
  if (cl < CB && c < C) {
    const double n = (double)M;
    double var = m2 / n;
    if (var < 0.0) var = 0.0;
    const float fmean = (float)mean, fvar = (float)var;
    smean[c] = fmean;
    sinv[c] = 1.0f / sqrtf(fvar + eps);
    if (rmean) rmean[c] = momentum * fmean + (1.f - momentum) * rmean[c];
    if (rvar) {
      const float unb = M > 1 ? (float)(m2 / (n - 1.0)) : fvar;
      rvar[c] = momentum * unb + (1.f - momentum) * rvar[c];
    }
  }
}
