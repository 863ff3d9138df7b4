// Diagnostic microbenchmark (not part of the product): dependent-load latency of one wave over a
// buffer, by working-set size and stride, timed with s_memrealtime (100 MHz).  Built by
// scripts/membench.py into build/membench.so.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void k_chase(const uint32_t* __restrict__ next, int hops, uint32_t start, unsigned long long* out) {
  uint32_t i = start;
  // warm pass
  for (int h = 0; h < hops; ++h) i = next[i];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int h = 0; h < hops; ++h) i = next[i];
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[0] = t1 - t0;
    out[1] = i;
  }
}

// Cold variant: no warm pass (first touch of every line / page).
__global__ void k_chase_cold(const uint32_t* __restrict__ next, int hops, uint32_t start, unsigned long long* out) {
  uint32_t i = start;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int h = 0; h < hops; ++h) i = next[i];
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    out[0] = t1 - t0;
    out[1] = i;
  }
}

extern "C" int mb_chase(const uint32_t* next, int hops, uint32_t start, unsigned long long* out, int cold) {
  if (cold) hipLaunchKernelGGL(k_chase_cold, dim3(1), dim3(64), 0, 0, next, hops, start, out);
  else hipLaunchKernelGGL(k_chase, dim3(1), dim3(64), 0, 0, next, hops, start, out);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

// Load-shape throughput: every wave issues `iters` x (8 independent 16-B loads per lane) over an
// L2-resident buffer.  pattern 0: lane l reads row (l & 31), 16-B chunk (l >> 5) of a row of
// `row_bytes` (32 rows x 32 B per instruction, the conv kernels' fragment-shaped A/B loads);
// pattern 1: lane l reads row (l >> 3), chunk (l & 7) (8 rows x 128 B per instruction: full lines).
__global__ void k_shape(const float* __restrict__ buf, long long nfloats, int row_bytes, int iters, int pattern,
                        float* out) {
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int rf = row_bytes / 4;
  int row, col;
  if (pattern == 0) { row = lane & 31; col = (lane >> 5) * 4; }
  else { row = lane >> 3; col = (lane & 7) * 4; }
  typedef float f4 __attribute__((ext_vector_type(4)));
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const long long rows_total = nfloats / rf;
  long long base_row = ((long long)wave * 97) % (rows_total - 64);
  for (int it = 0; it < iters; ++it) {
    f4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      // 8 consecutive 32-byte column steps of the same rows (pattern 0) / 8 row blocks (pattern 1)
      long long r = base_row + row + (pattern == 1 ? u * 8 : 0);
      int c = col + (pattern == 0 ? u * 8 : 0);
      if (c >= rf) c -= rf;
      v[u] = *reinterpret_cast<const f4*>(buf + r * rf + c);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) acc += v[u];
    base_row += 64;
    if (base_row + 64 >= rows_total) base_row = 0;
  }
  if (acc.x == 12345.f) out[0] = acc.y + acc.z + acc.w;
}

extern "C" int mb_shape(const float* buf, long long nfloats, int row_bytes, int iters, int pattern, float* out,
                        int blocks, int threads) {
  hipLaunchKernelGGL(k_shape, dim3(blocks), dim3(threads), 0, 0, buf, nfloats, row_bytes, iters, pattern, out);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
