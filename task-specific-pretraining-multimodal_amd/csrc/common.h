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

#define TSPM_LAUNCH_CHECK()                               \
  do {                                                    \
    hipError_t e__ = hipGetLastError();                   \
    if (e__ != hipSuccess) return TSPM_ERR_LAUNCH;        \
  } while (0)
