// LDS-staged implicit-GEMM convolution (tspm_conv_algo.variant == 1) on v_mfma_f32_32x32x2_f32.
//
// Replaces nn.Conv2d fwd / dgrad / wgrad of MML_Suite/models/msa/networks/resnet.py:25,30,176
// (3x3 s1/s2 p1 and 1x1 s2 convolutions; the Cin=1 stem stays on conv.hip's gather kernels).
//
// Why a second family: operands fetched straight into MFMA fragments are "fragment-shaped" loads,
// 32 rows x 32 B per wave instruction.  Measured on MI355X (scripts/membench.py) such loads stream
// at ~9.6 TB/s chip-wide against ~34 TB/s for full 128-B lines, and the register-direct kernels
// (conv.hip) sit under that ceiling.  Here every operand stage is fetched in full lines (8 lanes
// per 128-B row segment), staged through LDS and read back in fragment order:
//   * workgroup = 4 waves = WM x WN x WK; tile BM x BN = (WM*TM*32) x (WN*TN*32); the WK waves split
//     each 32-deep stage between them (8*4/WK reduction elements each) and combine their
//     accumulators through LDS in fixed order at the end;
//   * an LDS ring of 2-4 stage slots filled by LDS-DMA (global_load_lds, 16 B per lane): the loads
//     of the next D-1 stages are in flight while one stage is multiplied; one barrier per stage;
//   * operands whose fragments run along a 128-B row (the gathered activation rows of fwd / dgrad
//     and the fwd weights) are stored as 32-float rows with the 16-B chunk q of row r at position
//     q ^ ((r >> 1) & 7): the ds_read_b128 of one chunk column by 32 rows is bank-conflict-free;
//     operands whose fragments run down a column (dgrad weights, both wgrad operands) are read with
//     ds_read_b32 from plain rows (conflict-free: 32 consecutive floats per lane half);
//   * split-K over `splits` workgroups (grid.z): fp32 slabs written through (sc1), reduced in slab
//     order by the last arriving workgroup of each tile, which then runs the epilogue (results do
//     not depend on arrival order).
// Row blocks never straddle an output position (N % BM == 0 with the HWNC row order), so the set
// of non-padding taps is uniform per workgroup and padding taps are skipped, not multiplied.
#include "conv_common.h"

// This file is compiled twice (Makefile): as is (variant 1, register-staged loader waves) and with
// TSPM_LOADER_WAVES=0 TSPM_LDS_NS=tspm_lds_dma TSPM_LDS_IMPL=lds_impl_dma TSPM_LDS_SECONDARY (variant 2).
#ifndef TSPM_LDS_NS
#define TSPM_LDS_NS tspm_lds_reg
#endif
#ifndef TSPM_LDS_IMPL
#define TSPM_LDS_IMPL lds_impl_reg
#endif

#if defined(TSPM_STAMPS) && defined(TSPM_LDS_SECONDARY)
// the second build of this file (variant 2) records no stamps: its kernels cannot reach the first build's
// buffer without -fgpu-rdc (a separate buffer + readback would be needed to stamp variant 2)
#undef TSPM_STAMP
#define TSPM_STAMP(buf, slot) \
  do {                        \
  } while (0)
#undef TSPM_STAMP_CLK
#define TSPM_STAMP_CLK(buf, slot) \
  do {                            \
  } while (0)
#endif
#if defined(TSPM_STAMPS) && !defined(TSPM_LDS_SECONDARY)
__device__ unsigned long long tspm_g_stamps_lds[TSPM_STAMP_WAVES * TSPM_STAMP_SLOTS];
extern "C" int tspm_debug_stamps_lds(void* host_dst, size_t bytes) {
  if (bytes > sizeof(tspm_g_stamps_lds)) bytes = sizeof(tspm_g_stamps_lds);
  return hipMemcpyFromSymbol(host_dst, HIP_SYMBOL(tspm_g_stamps_lds), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : 2;
}
extern "C" int tspm_debug_stamps_lds_clear(void) {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(tspm_g_stamps_lds)) != hipSuccess) return 2;
  return hipMemset(p, 0, sizeof(tspm_g_stamps_lds)) == hipSuccess ? 0 : 2;
}
#endif

namespace {

constexpr int kThreads = 256;  // compute (MFMA) threads: 4 waves, one per SIMD

// Loader waves (variant 1, TSPM_LOADER_WAVES=2, the default build): 4 more waves per workgroup that only move
// operands — full-line 16-B global loads RS stages ahead into registers, then ds_write_b128 to the stage's LDS
// slot (lane-linear per 1-KiB piece).  Measured on MI355X (stamped builds, round 2): a global_load_lds blocks
// its wave ~170 cycles at issue, and with one wave per SIMD doing both, the load issue path and the MFMA path
// of a stage added up (one stage of a 32x64 tile: 0.36 + 0.45 us).  With a loader wave beside each compute
// wave on the same SIMD, the compute wave's MFMA stream no longer stops at the load issues.  The loader waves
// leave after the ring loop (s_barrier then counts only the surviving waves, as the ISA defines), so the
// epilogues, split-K hand-offs and BN merges run on the 256 compute threads: results are bitwise those of the
// single-role kernel (same MFMA order).  TSPM_LOADER_WAVES=0 (variant 2, the second build of this file):
// single-role waves issuing their own LDS-DMA (global_load_lds) into a 2-4-slot ring.
#ifndef TSPM_LOADER_WAVES
#define TSPM_LOADER_WAVES 2
#endif
static_assert(TSPM_LOADER_WAVES == 0 || TSPM_LOADER_WAVES == 2, "variant 1 (2) or variant 2 (0)");
constexpr int kLoaderThreads = TSPM_LOADER_WAVES == 2 ? 256 : 0;
constexpr bool kRegStage = TSPM_LOADER_WAVES == 2;
// TSPM_LDS_SPLIT (variant 4, the third build of this file): the variant-1 kernels with every fp32 product formed
// on the bf16 matrix cores.  The loader waves split each fp32 operand exactly into three bf16 pieces
// (x = h + m + l: h = x truncated to bf16, m = the remainder truncated, l = what is left — at most 8 significant
// bits each, so the sum is exact) and stage the three planes in LDS; each 16-deep reduction step of a 32x32 tile
// is the 9 v_mfma_f32_32x32x16_bf16 of all piece pairs.  Every piece product is exact in the fp32 accumulator
// (8 x 8 significant bits), so each x*w is formed exactly as the sum of its 9 parts; only the grouping of the
// fp32 additions differs from the f32 MFMA's fmaf chain.  9 x 32 cycles per 16-deep step against 8 x 64 for
// v_mfma_f32_32x32x2_f32 (MI355X_MICROARCH.md: bf16 MFMA 1/16 the cycles per FLOP of f32).
#ifdef TSPM_LDS_SPLIT
constexpr bool kSplit = true;
// wk == 1 tiles: stages per sign block of the bias-cancelling sign alternation (ring_loop)
#ifndef TSPM_SPLIT_SIGN_EVERY
#define TSPM_SPLIT_SIGN_EVERY 1
#endif
constexpr int kSignEvery = TSPM_SPLIT_SIGN_EVERY;
// Stage pairs (A/B switch): a 4-slot LDS ring with one loader -> compute barrier per two stages, for tiles whose four
// stage images fit TSPM_PAIR_MAX_BYTES (so two workgroups still share a CU); other tiles keep 2 slots, 1 barrier per stage
#ifndef TSPM_SPLIT_PAIR
#define TSPM_SPLIT_PAIR 0
#endif
#ifndef TSPM_PAIR_MAX_BYTES
#define TSPM_PAIR_MAX_BYTES (80 * 1024)
#endif
constexpr bool kPairBuild = TSPM_SPLIT_PAIR != 0;
static_assert(TSPM_LOADER_WAVES == 2, "the split build stages through the register loader waves");
// the split build's kernels carry their own names (k_fwd_x9, ...) so that traces tell the two builds apart
#define k_fwd_lds k_fwd_x9
#define k_fwd_pair_lds k_fwd_pair_x9
#define k_dgrad_lds k_dgrad_x9
#define k_wgrad_lds k_wgrad_x9
#define k_bwd_lds k_bwd_x9
#define k_bwd_quad_lds k_bwd_quad_x9
#else
constexpr bool kSplit = false;
constexpr int kSignEvery = 1;
constexpr bool kPairBuild = false;
#define TSPM_PAIR_MAX_BYTES (80 * 1024)
#endif
// minimum waves per SIMD the register allocation must allow (__launch_bounds__ second argument): with
// loader waves, 4 (two 512-thread workgroups per CU, so the two encoder streams' conv launches can share
// CUs) for the one-block-per-wave tiles, 2 for the larger wave tiles (128 VGPRs would spill them)
#ifndef TSPM_LDS_WAVES_SMALL
#define TSPM_LDS_WAVES_SMALL (TSPM_LOADER_WAVES ? 4 : 1)
#endif
// The 2-block wave tiles (TM * TN == 2) with at most 6 loader pieces per stage (BM + BN <= 192): 4 waves per SIMD
// as well (round 5) once the split-K epilogue keeps 32-bit offsets (no spill at 128 VGPRs), so two workgroups
// share a CU.  Measured (library A/B, alternating processes, gpurun_out/r5c_ab_*.json): batch 128 2.6160 vs
// 2.6165 ms (neutral), batch 1024 conv 8.71 vs 8.84 ms per step (frac 0.479 vs 0.472), step 9.80 vs 9.83 ms.
// TSPM_LDS_WAVES_LARGE=2 (variant 1) / 1 (variant 2) restores one workgroup per CU; the larger tiles
// (9 pieces: 108 loader VGPRs) stay at 2 / 1.
#ifndef TSPM_LDS_WAVES_LARGE
#define TSPM_LDS_WAVES_LARGE 4
#endif
template <class C>
constexpr int min_waves() {
  return C::TM * C::TN == 1 ? TSPM_LDS_WAVES_SMALL
                            : (C::BM + C::BN <= 192 ? TSPM_LDS_WAVES_LARGE : (kLoaderThreads ? 2 : 1));
}
template <class C1, class C2>
constexpr int min_waves2() { return min_waves<C1>() < min_waves<C2>() ? min_waves<C1>() : min_waves<C2>(); }
constexpr int kBlock = kThreads + kLoaderThreads;
TSPM_DEV bool is_loader_wave() {
  return kLoaderThreads > 0 && __builtin_amdgcn_readfirstlane((int)threadIdx.x) >= kThreads;
}

TSPM_DEV int swz(int row) { return (row >> 1) & 7; }

// 4 consecutive k (chunk q) of `row` in a swizzled 32-float-row image
TSPM_DEV f32x4 frag_row(const float* img, int row, int q) {
  return *reinterpret_cast<const f32x4*>(img + row * 32 + ((q ^ swz(row)) << 2));
}
// img[k0 + j][col], j < 4, of a plain image with row length ld
TSPM_DEV f32x4 frag_col(const float* img, int ld, int k0, int col) {
  f32x4 v;
  v[0] = img[k0 * ld + col];
  v[1] = img[(k0 + 1) * ld + col];
  v[2] = img[(k0 + 2) * ld + col];
  v[3] = img[(k0 + 3) * ld + col];
  return v;
}

// wave -> (wm, wn, wk); wk slowest so that the WM*WN waves of one k-slice are contiguous
template <class C>
struct WaveId {
  int wm, wn, wk;
  TSPM_DEV WaveId() {
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    wm = w % C::WM;
    wn = (w / C::WM) % C::WN;
    wk = w / (C::WM * C::WN);
  }
};

// one 16-B-per-lane LDS-DMA: lane l's bytes land at dst + 16*l (dst wave-uniform)
TSPM_DEV void glds16(const float* src, float* dst) {
#ifndef TSPM_EXP_NOGLDS  // diagnostic ablation (stamped build only): skip the operand DMA
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
#endif
}

// ring depth for a stage image of `stage_floats`: as deep as fits 64 KiB (two workgroups per CU
// keep 128 KiB of rings), at least double-buffered
#ifndef TSPM_RING_MAX
#define TSPM_RING_MAX 4
#endif
#ifndef TSPM_RING_BYTES
#define TSPM_RING_BYTES (64 * 1024)
#endif
// register-staged operand stages in flight per loader thread (variant 1).  Measured in the
// batch-128 step (A/B, 2 runs each, same box): 2 stages 2.684-2.691 ms (2.697-2.706 with the previous loop,
// which drained every load at each trip), 3 stages 2.677-2.681, 4 stages (3 for the large tiles)
// 2.705-2.707; TSPM_REG_STAGES overrides (A/B builds)
template <int NI>
constexpr int reg_stages() {
#ifdef TSPM_REG_STAGES
  return TSPM_REG_STAGES;
#else
  return 3;
#endif
}
template <int STAGE>
constexpr int ring_depth() {
  // register staging: the loads in flight sit in registers (split build with stage pairs: 4 slots when they fit)
  if (kRegStage) return (kPairBuild && STAGE * 4 * 4 <= TSPM_PAIR_MAX_BYTES) ? 4 : 2;
  int d = TSPM_RING_MAX;
  while (d > 2 && STAGE * 4 * d > TSPM_RING_BYTES) --d;
  return d;
}

template <int TM_, int TN_, int WM_, int WN_, int WK_>
struct Cfg {
  static constexpr int TM = TM_, TN = TN_, WM = WM_, WN = WN_, WK = WK_;
  static constexpr int BM = WM * TM * 32, BN = WN * TN * 32;
  static constexpr int KGW = 4 / WK;                     // 8-k groups per wave per stage
  // floats per stage image (A then B): 32 fp32 per row, or (split build) three planes of 32 bf16 per row
  static constexpr int STAGE = (BM + BN) * (kSplit ? 48 : 32);
  static constexpr int D = ring_depth<STAGE>();          // LDS ring slots
  static constexpr int NI = (BM + BN) / 32;              // LDS-DMA instructions per thread per stage
  static_assert(WM * WN * WK == 4, "4 waves per workgroup");
};

// Per-stage operand offsets returned by a kernel's prep(stage) (A and B operand base offsets).
struct Off {
  long long a, b;
};

// Workgroup coordinates of a GEMM tile: the launch's own blockIdx / gridDim.x, or virtual ones when
// two GEMMs share one launch (k_bwd_lds).
struct Blk {
  int x, y, z, gx;
};
TSPM_DEV Blk hw_blk() { return Blk{(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z, (int)gridDim.x}; }

// XCD-aware tile order.  The dispatcher deals workgroups round-robin to the 8 XCDs (linear id L goes
// to XCD L % 8), each with its own L2.  Logical tiles are ordered row block fastest, and neighbouring
// row blocks read overlapping input rows (the filter taps of adjacent output positions, HWNC row
// order), so each XCD is given a CONTIGUOUS range of logical tiles: XCD k runs tiles
// [start_k, start_k + count_k) in dispatch order — the shared rows then hit that XCD's L2 instead of
// being fetched once per XCD.  A bijection for any grid size (the first W % 8 XCDs take one more).
constexpr int kXcds = 8;
TSPM_DEV int xcd_swizzle(int L, int W) {
  const int q = W / kXcds, r = W % kXcds;
  const int xcd = L % kXcds, idx = L / kXcds;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}
TSPM_DEV Blk grid_blk(int xcd) {
  if (!xcd) return hw_blk();
  const int gx = gridDim.x, gy = gridDim.y;
  if (xcd == 2) {  // within each split-K plane only: every XCD keeps a share of every plane
    const int T = xcd_swizzle(blockIdx.x + gx * blockIdx.y, gx * gy);
    return Blk{T % gx, T / gx, (int)blockIdx.z, gx};
  }
  const int L = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const int T = xcd_swizzle(L, gx * gy * gridDim.z);
  const int x = T % gx, yz = T / gx;
  return Blk{x, yz % gy, yz / gy, gx};
}

// One stage's MFMAs with the next stage's LDS-DMA issues interleaved between them.  Measured
// (scripts/stamp_conv.py ablations): a global_load_lds blocks its wave ~170 cycles at issue, and
// with one wave per SIMD issuing them all before the MFMAs serialised DMA issue and matrix work
// (per stage: DMA path 0.56 us + MFMA path 0.65 us = 1.13 us).  Issued between MFMAs (64-cycle
// f32 MFMAs keep the matrix pipe busy meanwhile) the issue cost hides under the matrix work.
// MFMA order (kk, j, a, b) equals Acc::mma4's, so results are bitwise unchanged.
template <class C, int NI, class IssueI>
TSPM_DEV void mma_interleaved(Acc<C::TM, C::TN>& acc, const f32x4 (&A)[C::KGW][C::TM],
                              const f32x4 (&B)[C::KGW][C::TN], IssueI&& issue_i) {
  constexpr int NF = C::KGW * 4 * C::TM * C::TN;
#pragma unroll
  for (int f = 0; f < NF; ++f) {
    const int b = f % C::TN, a = (f / C::TN) % C::TM, j = (f / (C::TN * C::TM)) % 4, kk = f / (C::TN * C::TM * 4);
    acc.v[a][b] = mfma32(A[kk][a][j], B[kk][b][j], acc.v[a][b]);
#pragma unroll
    for (int i = 0; i < NI; ++i)
      if ((i * NF) / NI == f) issue_i(i);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// One stage's MFMAs without DMA issues (compute waves when loader waves carry the DMA); same MFMA order.
template <class C>
TSPM_DEV void mma_plain(Acc<C::TM, C::TN>& acc, const f32x4 (&A)[C::KGW][C::TM], const f32x4 (&B)[C::KGW][C::TN]) {
#pragma unroll
  for (int kk = 0; kk < C::KGW; ++kk)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int a = 0; a < C::TM; ++a)
#pragma unroll
        for (int b = 0; b < C::TN; ++b) acc.v[a][b] = mfma32(A[kk][a][j], B[kk][b][j], acc.v[a][b]);
}

// ---- split build (variant 4): the three-plane bf16 stage image ------------------------------------------------
// Plane p of an operand with R rows (A: R = BM, B: R = BN) holds 32 bf16 per GEMM row or column, R * 64 bytes; the
// A planes come first, then the B planes.  Two layouts, by how the operand sits in memory:
//  * row operands (the reduction index runs along a memory row: fwd x and w, dgrad dy): [row][32 k], 64-B rows of
//    four 16-B chunks, chunk c of row r at c ^ ((r >> 2) & 3) — the ds_read_b128 fragment reads (32 rows of one
//    chunk per lane half) then cover all 64 banks in each 16-lane group;
//  * column operands (the reduction index runs down memory rows: dgrad w, wgrad dy and x): [32 k][R], read with
//    ds_read_b64_tr_b16 (4 k-rows x 16 columns per 16-lane group, delivered per column); rows of 128 B swap their
//    64-B halves on k-rows with bit 1 set and rows of >= 256 B rotate their 64-B quarters by k & 3, so the four
//    k-rows of a transposed read land on distinct banks.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef short i16x8 __attribute__((ext_vector_type(8)));

// Exact split of 4 fp32 values into three bf16 pieces, packed 2 per dword (element 2i in the low half).
// h = x truncated to bf16; r = x - h is exact (same sign and binade); m = r truncated; l = r - m (<= 8 significant
// bits: exact in bf16).  Non-finite inputs stay non-finite (a NaN keeps a NaN piece; an infinity gives inf - inf).
TSPM_DEV void split3(const f32x4& v, uint2& H, uint2& M, uint2& L) {
  unsigned hb[4], mb[4], lb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const unsigned xb = __float_as_uint(v[j]);
    const float r = v[j] - __uint_as_float(xb & 0xffff0000u);
    const unsigned rb = __float_as_uint(r);
    hb[j] = xb;
    mb[j] = rb;
    lb[j] = __float_as_uint(r - __uint_as_float(rb & 0xffff0000u));
  }
  // v_perm_b32: the high halves of (lo, hi) -> one dword
  H = make_uint2(__builtin_amdgcn_perm(hb[1], hb[0], 0x07060302u), __builtin_amdgcn_perm(hb[3], hb[2], 0x07060302u));
  M = make_uint2(__builtin_amdgcn_perm(mb[1], mb[0], 0x07060302u), __builtin_amdgcn_perm(mb[3], mb[2], 0x07060302u));
  L = make_uint2(__builtin_amdgcn_perm(lb[1], lb[0], 0x07060302u), __builtin_amdgcn_perm(lb[3], lb[2], 0x07060302u));
}
// byte offset of (k-row k, column col) in a column plane of CC columns
template <int CC>
TSPM_DEV int col_off(int k, int col) {
  constexpr int RB = CC * 2;
  const int t = RB <= 64 ? 0 : (RB == 128 ? ((k >> 1) & 1) : (k & 3));
  return k * RB + ((col * 2) ^ (t << 6));
}
// byte offset of 4 consecutive k (fp32 chunk q of the stage, k = 4q..4q+3) of row `row` in a row plane
TSPM_DEV int row_off(int row, int q) { return row * 64 + ((((q >> 1) ^ ((row >> 2) & 3))) << 4) + ((q & 1) << 3); }
// the 32x32x16 operand fragment (lane: GEMM row/column lane & 31, k = 16 s + 8 (lane >> 5) + j) of a row plane
TSPM_DEV bf16x8 frag_row16(const char* plane, int row0, int s, int lane) {
  const int row = row0 + (lane & 31), c = 2 * s + (lane >> 5);
  return *reinterpret_cast<const bf16x8*>(plane + row * 64 + ((c ^ ((row >> 2) & 3)) << 4));
}
// ... of a column plane: two transposed reads, k-rows 16 s + 8 h + [0, 4) and [4, 8); lane 4q+p of each 16-lane group
// addresses k-row q, columns 4p..4p+3 of the group's 16 columns
template <int CC>
TSPM_DEV bf16x8 frag_col16(const char* plane, int col0, int s, int lane) {
  const int g = (lane >> 4) & 3, i = lane & 15;
  const int col = col0 + 16 * (g & 1) + 4 * (i & 3);
  const int k = 16 * s + 8 * (g >> 1) + (i >> 2);
  typedef __attribute__((address_space(3))) i16x4 lds_i16x4;
  const i16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(plane + col_off<CC>(k, col)));
  const i16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_i16x4*)(plane + col_off<CC>(k + 4, col)));
  const i16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}
// a stage piece's byte offset (plane 0 of its operand, relative to the operand's first plane): the loader's lane
// mapping of the row operands (row (i*4+wv)*8 + lane/8, fp32 chunk (lane & 7) ^ swz(row) — the bodies pre-swizzle
// the global address) and of the column operands (element e = (i*4+wv)*64 + lane: k-row e / (CC/4), 4 columns)
template <int CC, bool COL>
TSPM_DEV int split_piece_off(int i, int wv, int lane) {
  if constexpr (COL) {
    const int e = (i * 4 + wv) * 64 + lane;
    return col_off<CC>(e / (CC / 4), (e % (CC / 4)) * 4);
  } else {
    const int row = (i * 4 + wv) * 8 + (lane >> 3);
    return row_off(row, (lane & 7) ^ swz(row));
  }
}
// the 16-deep step (0 or 1) of the stage a loader piece belongs to (same lane mapping as split_piece_off)
template <int CC, bool COL>
TSPM_DEV int split_piece_step(int i, int wv, int lane) {
  if constexpr (COL) {
    return ((i * 4 + wv) * 64 + lane) / (CC / 4) >> 4;
  } else {
    const int row = (i * 4 + wv) * 8 + (lane >> 3);
    return ((lane & 7) ^ swz(row)) >> 2;
  }
}
template <int CC, bool COL>
TSPM_DEV bf16x8 split_frag(const char* plane, int blk0, int s, int lane) {
  if constexpr (COL) return frag_col16<CC>(plane, blk0, s, lane);
  else return frag_row16(plane, blk0, s, lane);
}

// LDS-DMA ring over stages [st0, st1): C::D stage slots of C::STAGE floats.  prep(st) returns the
// operand offsets of stage st, issue_i(off, slot, i) issues this thread's i-th of C::NI
// global_load_lds (16 B per lane, lane-linear destination) of that stage into the slot,
// frags(slot, A, B) reads one stage's MFMA fragments from LDS.  Loads run D-1 stages ahead of the
// multiply.  Ordering: a slot is read only after the issuing threads' counted `s_waitcnt vmcnt`
// and a barrier; a slot is refilled only after the barrier that follows every wave's multiply of
// its previous stage (the MFMAs consumed the ds_reads).  Past the end the ring re-loads stage
// st1-1 into slots that are never read again, so the vmcnt count is the same in every iteration.
// Raw s_barrier, not __syncthreads(): the latter waits vmcnt(0) and would drain the ring.  Every
// thread of the workgroup must call this with the same st0/st1; the ring is drained on return.
// Returns true in loader waves, which must then leave the kernel (they take no part in what follows).
// With loader waves the roles split: the loaders issue every DMA and wait for it (counted vmcnt) before
// each stage barrier; the compute waves only pass the barriers, read fragments and multiply.
// With loader waves the loader's per-stage path is: LDS write of the stage, lgkmcnt(0), barrier, next loads.
// Per-stage loop diagnostics (stamped build only, TSPM_STAMPS): the compute waves accumulate shader cycles
// (s_memtime) spent waiting at the stage barrier, reading + waiting for the stage's fragments and issuing
// its MFMAs, into stamp slots 8-10 (slot 11: stages).  The reads of the clock add waits of their own (an
// s_memtime result is counted in lgkmcnt), so these profile a perturbed loop, not the product.
#if defined(TSPM_STAMPS) && !defined(TSPM_LDS_SECONDARY)
struct LoopClock {
  unsigned long long bar = 0, lds = 0, mma = 0, t = 0;
  int n = 0;
  TSPM_DEV void start() { t = __builtin_amdgcn_s_memtime(); }
  TSPM_DEV void lap(unsigned long long& acc) {
    const unsigned long long u = __builtin_amdgcn_s_memtime();
    acc += u - t;
    t = u;
  }
  TSPM_DEV void flush() {
    const unsigned long long w = ((unsigned long long)blockIdx.x +
                                  (unsigned long long)gridDim.x * (blockIdx.y + (unsigned long long)gridDim.y * blockIdx.z)) *
                                     (blockDim.x >> 6) + (threadIdx.x >> 6);
    if ((threadIdx.x & 63) == 0 && w < TSPM_STAMP_WAVES) {
      tspm_g_stamps_lds[w * TSPM_STAMP_SLOTS + 8] = bar;
      tspm_g_stamps_lds[w * TSPM_STAMP_SLOTS + 9] = lds;
      tspm_g_stamps_lds[w * TSPM_STAMP_SLOTS + 10] = mma;
      tspm_g_stamps_lds[w * TSPM_STAMP_SLOTS + 11] = n;
    }
  }
};
#define TSPM_LOOP_CLOCK_DECL LoopClock lc__; lc__.start()
#define TSPM_LOOP_LAP(field) do { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); lc__.lap(lc__.field); } while (0)
#define TSPM_LOOP_STAGE() (++lc__.n)
#define TSPM_LOOP_FLUSH() lc__.flush()
#else
#define TSPM_LOOP_CLOCK_DECL do {} while (0)
#define TSPM_LOOP_LAP(field) do {} while (0)
#define TSPM_LOOP_STAGE() do {} while (0)
#define TSPM_LOOP_FLUSH() do {} while (0)
#endif

// ACOL / BCOL (split build only): the A / B operand is a column operand (see the split image above); the split
// build ignores dst_i and frags and places / reads the three planes itself.
template <class C, bool ACOL = false, bool BCOL = false, class Prep, class Src, class Dst, class Frags>
TSPM_DEV bool ring_loop(Acc<C::TM, C::TN>& acc, float* lds, int st0, int st1, Prep&& prep, Src&& src_i, Dst&& dst_i,
                        Frags&& frags) {
  constexpr int D = C::D, NI = C::NI, SF = C::STAGE;
  constexpr int NA = C::BM / 32;                          // loader pieces of the A operand
  constexpr int PA = C::BM * 64, PB = C::BN * 64;         // split build: bytes per bf16 plane of A / B
  const int n = st1 - st0;
  const bool loader = is_loader_wave();
  if (n <= 0) return loader;
  if constexpr (kSplit) {
    const int lane = threadIdx.x & 63;
    if (loader) {
      const int wv = (threadIdx.x >> 6) & 3;
#ifdef TSPM_SPLIT_REG_STAGES  // A/B builds: the split loader's register stages alone
      constexpr int RS = TSPM_SPLIT_REG_STAGES;
#else
      constexpr int RS = reg_stages<NI>();
#endif
      f32x4 R[RS][NI];
      int doff[NI];
      unsigned nstep[NI];  // wk == 2: the sign flip of the A pieces of step 1 (the second wave's half of each stage)
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        doff[i] = i < NA ? split_piece_off<C::BM, ACOL>(i, wv, lane)
                         : 3 * PA + split_piece_off<C::BN, BCOL>(i - NA, wv, lane);
        nstep[i] = (C::WK == 2 && i < NA && split_piece_step<C::BM, ACOL>(i, wv, lane) == 1) ? 0x80008000u : 0u;
      }
      auto load = [&](int st, f32x4 (&Rb)[NI]) {
        const Off off = prep(st);
#pragma unroll
        for (int i = 0; i < NI; ++i) Rb[i] = *reinterpret_cast<const f32x4*>(src_i(off, i));
      };
      auto store = [&](int it, f32x4 (&Rb)[NI]) {
        char* slot = reinterpret_cast<char*>(lds + (it % D) * SF);
        // wk == 1: the A pieces of every other block of kSignEvery stages are staged negated (see the compute loop)
        const unsigned neg = (C::WK == 1 && ((it / kSignEvery) & 1)) ? 0x80008000u : 0u;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          uint2 h, m, l;
          split3(Rb[i], h, m, l);
          if (i < NA) {
            const unsigned ng = neg ^ nstep[i];
            h.x ^= ng; h.y ^= ng; m.x ^= ng; m.y ^= ng; l.x ^= ng; l.y ^= ng;
          }
          const int ps = i < NA ? PA : PB;
          *reinterpret_cast<uint2*>(slot + doff[i]) = h;
          *reinterpret_cast<uint2*>(slot + doff[i] + ps) = m;
          *reinterpret_cast<uint2*>(slot + doff[i] + 2 * ps) = l;
        }
        if (D == 2 || (it & 1) || it == n - 1) {  // stage pairs: one barrier per two stages (and after the last)
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
        }
      };
      // the variant-1 loader loop (unconditional loads, full trips one basic block): see below
      const int last = st1 - 1;
#pragma unroll
      for (int j = 0; j < RS; ++j) load(min(st0 + j, last), R[j]);
      int it = 0;
      for (; it + RS <= n; it += RS) {
#pragma unroll
        for (int j = 0; j < RS; ++j) {
          store(it + j, R[j]);
          load(min(st0 + it + j + RS, last), R[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < RS - 1; ++j)
        if (it + j < n) store(it + j, R[j]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      return true;
    }
    static_assert(C::WK <= 2, "split build: each wave takes whole 16-deep steps");
    const WaveId<C> id;
    constexpr int NS = 2 / C::WK;  // 16-deep steps per wave per stage
    // Sign alternation.  The bf16 MFMA's accumulation is not an unbiased rounding: measured against fp64
    // (scripts/split_bias.py) its error has a mean of about -3e-8 of the mean |result| whatever the signs of the
    // data (a two's-complement truncation toward -inf), which a long reduction turns into a drift (-2.9e-6 over the
    // 49k rows of an audio layer1 weight gradient, against +1.5e-8 for the f32 MFMA).  So half of every reduction
    // runs negated, and the truncation pushes the true sum down in one half and up in the other:
    //  * wk == 2: the second wave's steps (k 16..31 of each stage) are staged as -A (the loader flips the pieces'
    //    sign bits); that wave accumulates -S1 and negates its accumulator once before the k-slice combine — no
    //    per-stage cost;
    //  * wk == 1: blocks of kSignEvery stages alternate: the loader stages -A on odd blocks and the accumulator,
    //    which holds sigma * S (sigma = the block's sign), is negated between blocks (a wait for the MFMA chain).
    // Negations are exact; the products are unchanged.
    auto negate = [&]() {
#pragma unroll
      for (int a = 0; a < C::TM; ++a)
#pragma unroll
        for (int b = 0; b < C::TN; ++b)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc.v[a][b][r] = -acc.v[a][b][r];
    };
    for (int it = 0; it < n; ++it) {
      if (C::WK == 1 && it > 0 && it % kSignEvery == 0) negate();
      if (D == 2 || !(it & 1)) {
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
      }
      const char* img = reinterpret_cast<const char*>(lds + (it % D) * SF);
#pragma unroll
      for (int ss = 0; ss < NS; ++ss) {
        const int s = id.wk * NS + ss;
        bf16x8 A[3][C::TM], B[3][C::TN];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
#pragma unroll
          for (int a = 0; a < C::TM; ++a)
            A[p][a] = split_frag<C::BM, ACOL>(img + p * PA, (id.wm * C::TM + a) * 32, s, lane);
#pragma unroll
          for (int b = 0; b < C::TN; ++b)
            B[p][b] = split_frag<C::BN, BCOL>(img + 3 * PA + p * PB, (id.wn * C::TN + b) * 32, s, lane);
        }
        // the 9 piece products, smallest first
        constexpr int PQ[9][2] = {{2, 2}, {1, 2}, {2, 1}, {0, 2}, {1, 1}, {2, 0}, {0, 1}, {1, 0}, {0, 0}};
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
          for (int a = 0; a < C::TM; ++a)
#pragma unroll
            for (int b = 0; b < C::TN; ++b)
              acc.v[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[PQ[t][0]][a], B[PQ[t][1]][b], acc.v[a][b], 0, 0, 0);
      }
    }
    if (C::WK == 1 ? (((n - 1) / kSignEvery) & 1) : id.wk == 1) negate();  // back to +S
    __builtin_amdgcn_s_barrier();
    return false;
  }
  if constexpr (kLoaderThreads > 0) {
    if (loader) {
      const int lane4 = (threadIdx.x & 63) * 4;
      // RS stages of operand loads in flight in registers (two LDS slots): a stage's loads are issued RS
      // stages before its LDS write, which covers more of the memory latency than two stages of MFMA work
      constexpr int RS = reg_stages<NI>();
      f32x4 R[RS][NI];
      auto load = [&](int st, f32x4 (&Rb)[NI]) {
#if defined(TSPM_EXP_SAMEADDR)  // diagnostic ablation (A/B builds only): every stage re-reads stage st0's operands
        const Off off = prep(st0 + 0 * st);
#else
        const Off off = prep(st);
#endif
#pragma unroll
        for (int i = 0; i < NI; ++i) {
#if defined(TSPM_EXP_NOLOAD)  // diagnostic ablation (A/B builds only): no operand traffic, address-dependent values
          const float v = (float)(reinterpret_cast<uintptr_t>(src_i(off, i)) & 7);
          Rb[i] = f32x4{v, v, v, v};
#else
          Rb[i] = *reinterpret_cast<const f32x4*>(src_i(off, i));
#endif
        }
      };
      auto store = [&](int it, f32x4 (&Rb)[NI]) {
#pragma unroll
        for (int i = 0; i < NI; ++i) *reinterpret_cast<f32x4*>(dst_i(lds + (it & 1) * SF, i) + lane4) = Rb[i];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the stage is in LDS before the barrier
        __builtin_amdgcn_s_barrier();
      };
      // Every load group is issued unconditionally (past the end the loader re-loads stage st1-1 into
      // buffers that are never stored), so the vmcnt scoreboard is the same on every path through the
      // loop: the compiler's wait before a stage's LDS write is then vmcnt((RS-1)*NI) — the RS-1 later
      // stages stay in flight.  (With the loads conditional it merged the paths conservatively and
      // drained ALL loads at every trip: one exposed memory latency per trip.)
      const int last = st1 - 1;
#pragma unroll
      for (int j = 0; j < RS; ++j) load(min(st0 + j, last), R[j]);
      // RS stages per trip, buffers indexed statically; (D = 2: slot it % 2 was last read before barrier it-1).
      // Full trips are one basic block (each buffer keeps its registers across the back-edge — a copy of a
      // buffer whose loads are in flight would force a wait for them), the last partial trip stores only.
      int it = 0;
      for (; it + RS <= n; it += RS) {
#pragma unroll
        for (int j = 0; j < RS; ++j) {
          store(it + j, R[j]);
          load(min(st0 + it + j + RS, last), R[j]);
        }
      }
#pragma unroll
      for (int j = 0; j < RS - 1; ++j)
        if (it + j < n) store(it + j, R[j]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      return true;
    }
    f32x4 A[C::KGW][C::TM], B[C::KGW][C::TN];
    TSPM_LOOP_CLOCK_DECL;
    for (int it = 0; it < n; ++it) {
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      TSPM_LOOP_LAP(bar);
      if (it == 0) TSPM_STAMP(tspm_g_stamps_lds, 1);
      frags(lds + (it % D) * SF, A, B);
      TSPM_LOOP_LAP(lds);
#if defined(TSPM_EXP_NOMFMA)  // diagnostic ablation (A/B builds only): fragments read, no matrix work
      acc.v[0][0][0] += A[0][0][0] + B[0][0][0];
#else
      mma_plain<C>(acc, A, B);
#endif
      TSPM_LOOP_LAP(mma);
      TSPM_LOOP_STAGE();
    }
    TSPM_LOOP_FLUSH();
    __builtin_amdgcn_s_barrier();
    return false;
  }
#pragma unroll
  for (int d = 0; d < D - 1; ++d) {
    const Off off = prep(min(st0 + d, st1 - 1));
#pragma unroll
    for (int i = 0; i < NI; ++i) glds16(src_i(off, i), dst_i(lds + d * SF, i));
  }
  f32x4 A[C::KGW][C::TM], B[C::KGW][C::TN];
  for (int it = 0; it < n; ++it) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 2) * NI) : "memory");
    __builtin_amdgcn_s_barrier();
    if (it == 0) TSPM_STAMP(tspm_g_stamps_lds, 1);
    const Off off = prep(min(st0 + it + D - 1, st1 - 1));
    float* nslot = lds + ((it + D - 1) % D) * SF;
    frags(lds + (it % D) * SF, A, B);
    mma_interleaved<C, NI>(acc, A, B, [&](int i) { glds16(src_i(off, i), dst_i(nslot, i)); });
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  return false;
}

// Combine the WK k-slices of each (wm, wn) tile through LDS, in k-slice order (deterministic).
// Afterwards waves with wk == 0 hold the tile.  All waves must call (barriers).
template <class C>
TSPM_DEV void combine_k(Acc<C::TM, C::TN>& acc, float* lds, const WaveId<C>& id, int lane) {
  if constexpr (C::WK > 1) {
    constexpr int TILE = C::TM * C::TN * 16 * 64;
    const int mn = id.wm * C::WN + id.wn;
    __syncthreads();  // the stage images may still be read by slower waves
    if (id.wk > 0) {
      float* dst = lds + ((id.wk - 1) * C::WM * C::WN + mn) * TILE;
#pragma unroll
      for (int a = 0; a < C::TM; ++a)
#pragma unroll
        for (int b = 0; b < C::TN; ++b)
#pragma unroll
          for (int i = 0; i < 16; ++i) dst[((a * C::TN + b) * 16 + i) * 64 + lane] = acc.v[a][b][i];
    }
    __syncthreads();
    if (id.wk == 0) {
      for (int k = 1; k < C::WK; ++k) {
        const float* src = lds + ((k - 1) * C::WM * C::WN + mn) * TILE;
#pragma unroll
        for (int a = 0; a < C::TM; ++a)
#pragma unroll
          for (int b = 0; b < C::TN; ++b)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc.v[a][b][i] += src[((a * C::TN + b) * 16 + i) * 64 + lane];
      }
    }
    __syncthreads();
  }
}

// Split-K over workgroups: every workgroup writes its (combined) tile to slab z; the last arriver
// of the tile re-reads all slabs in slab order into the waves that hold the tile.  Returns false in
// the workgroups that are done.  slab = rows*ld floats; tile origin (row0, col0) per wave.
template <class C>
TSPM_DEV bool splitk_reduce(Acc<C::TM, C::TN>& acc, const WaveId<C>& id, int lane, float* slabs, long long slab,
                            int splits, unsigned* cnt, int row0, int col0, int rows, int cols, long long ld,
                            float* lds, const Blk& bk, bool acquire) {
  if (splits <= 1) return true;
  if (id.wk == 0) acc.store(slabs + (long long)bk.z * slab, row0, col0, rows, cols, ld, lane, false, true);
  if (!last_arriver(cnt + (bk.y * bk.gx + bk.x), (unsigned)splits, reinterpret_cast<int*>(lds), acquire))
    return false;
  TSPM_STAMP(tspm_g_stamps_lds, 6);
  if (id.wk == 0) {
    // Every slab's TM*TN*16 loads are issued together before its in-order adds (the summation order is
    // unchanged: slab z is added after slab z-1), so one slab costs one memory round trip instead of a
    // chain of them (phase stamps: the R34 layer3 forward's slab read took 7-15 us as a load-add chain).
    // 32-bit offsets (a slab is rows * ld < 2^31 floats: checked on the host) and one 32x32 fragment's loads
    // in flight at a time: the epilogue sets the kernel's VGPR count, and at <= 128 VGPRs the 2-block wave
    // tiles fit two workgroups per CU (round 5)
    acc.zero();
    int off[C::TM][C::TN][16];
#pragma unroll
    for (int a = 0; a < C::TM; ++a)
#pragma unroll
      for (int b = 0; b < C::TN; ++b) {
        const int col = min(col0 + b * 32 + (lane & 31), cols - 1);
#pragma unroll
        for (int i = 0; i < 16; ++i) off[a][b][i] = min(row0 + a * 32 + acc_row(i, lane), rows - 1) * (int)ld + col;
      }
    for (int z = 0; z < splits; ++z) {
      const float* src = slabs + (long long)z * slab;
#pragma unroll
      for (int a = 0; a < C::TM; ++a)
#pragma unroll
        for (int b = 0; b < C::TN; ++b) {
          float v[16];
#pragma unroll
          for (int i = 0; i < 16; ++i) v[i] = ld_sc1(src + off[a][b][i]);
#pragma unroll
          for (int i = 0; i < 16; ++i) acc.v[a][b][i] += v[i];
        }
    }
  }
  return true;
}

// =============================================================================================
// Forward: y[(p,q,n), k] = sum_{valid (r,s), c} x[(p*st-pad+r, q*st-pad+s, n), c] w[k, r, s, c]
// A image: BM rows (n) x 32 channels (swizzled); B image: BN rows (output channel) x 32 channels.
// =============================================================================================
// bk: the tile's coordinates and the row-block count (gx) of this GEMM; gy its column-block count (the launch's own
// grid for k_fwd_lds, virtual ones when two forwards share a launch — k_fwd_pair_lds)
template <class C>
TSPM_DEV void fwd_body(const ConvArgs& g, const float* __restrict__ x, const float* __restrict__ w,
                       float* __restrict__ y, const tspm_bn_fuse& bf, float* __restrict__ slabs, int gw, int ng,
                       float* lds, const Blk& bk, int gy) {
  TSPM_STAMP(tspm_g_stamps_lds, 0);
  const int tid = threadIdx.x, lane = tid & 63;
  const WaveId<C> id;
  const int N = g.n, Cc = g.c, K = g.k, RSC = g.r * g.s * Cc;
  const int m0 = bk.x * C::BM, n0col = bk.y * C::BN;
  const int pos = m0 / N, nb0 = m0 - pos * N;
  const int pp = pos / g.q, qq = pos - pp * g.q;
  const int h0 = pp * g.st - g.pad, w0 = qq * g.st - g.pad;
  const int r_lo = max(0, -h0), r_hi = min(g.r - 1, g.h - 1 - h0);
  const int s_lo = max(0, -w0), s_hi = min(g.s - 1, g.w - 1 - w0);
  const int nr = r_hi - r_lo + 1, ns = s_hi - s_lo + 1;
  const int cb = Cc >> 5;
  const int T = (nr > 0 && ns > 0) ? nr * ns * cb : 0;
  const int st0 = split_lo(T, bk.z, g.splits), st1 = split_lo(T, bk.z + 1, g.splits);

  constexpr int NA = C::BM / 32, NB = C::BN / 32;
  const int wv = (tid >> 6) & 3;
  const float* xa[NA];
  const float* wb[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int row = (i * 4 + wv) * 8 + (lane >> 3);
    xa[i] = x + (long long)(nb0 + row) * Cc + (((lane & 7) ^ swz(row)) << 2);
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int row = (i * 4 + wv) * 8 + (lane >> 3);
    wb[i] = w + (long long)min(n0col + row, K - 1) * RSC + (((lane & 7) ^ swz(row)) << 2);
  }
  Acc<C::TM, C::TN> acc;
  acc.zero();
  auto prep = [&](int st) -> Off {
    const int tap = st / cb, cc = (st - tap * cb) << 5;
    const int tr = tap / ns;
    const int r = r_lo + tr, s = s_lo + (tap - tr * ns);
    return Off{((long long)(h0 + r) * g.w + (w0 + s)) * N * Cc + cc, (long long)(r * g.s + s) * Cc + cc};
  };
  if (ring_loop<C>(
      acc, lds, st0, st1, prep,
      [&](const Off& off, int i) -> const float* { return i < NA ? xa[i] + off.a : wb[i - NA] + off.b; },
      [&](float* slot, int i) -> float* {
        return i < NA ? slot + (i * 4 + wv) * 256 : slot + C::BM * 32 + ((i - NA) * 4 + wv) * 256;
      },
      [&](const float* img, f32x4 (&A)[C::KGW][C::TM], f32x4 (&B)[C::KGW][C::TN]) {
#pragma unroll
        for (int kk = 0; kk < C::KGW; ++kk) {
          const int q = (id.wk * C::KGW + kk) * 2 + (lane >> 5);
#pragma unroll
          for (int a = 0; a < C::TM; ++a) A[kk][a] = frag_row(img, (id.wm * C::TM + a) * 32 + (lane & 31), q);
#pragma unroll
          for (int b = 0; b < C::TN; ++b)
            B[kk][b] = frag_row(img + C::BM * 32, (id.wn * C::TN + b) * 32 + (lane & 31), q);
        }
      }))
    return;
  TSPM_STAMP(tspm_g_stamps_lds, 2);
  combine_k<C>(acc, lds, id, lane);
  TSPM_STAMP(tspm_g_stamps_lds, 3);
  const int row0 = m0 + id.wm * C::TM * 32, col0 = n0col + id.wn * C::TN * 32;
  if (!splitk_reduce<C>(acc, id, lane, slabs, (long long)g.m * K, g.splits, g.cnt, row0, col0, g.m, K, K, lds, bk, g.acq != 0))
    return;
  TSPM_STAMP(tspm_g_stamps_lds, 4);
  const bool active = id.wk == 0 && col0 < K;
  if (active) {
    acc.store(y, row0, col0, g.m, K, K, lane, false);
    if (bf.partial)
      acc.bn_partials(bf.partial, (long long)bk.gx * C::WM * K, bk.x * C::WM + id.wm, row0, col0, g.m, K,
                      lane, bf.counters != nullptr);
  }
  TSPM_STAMP(tspm_g_stamps_lds, 5);
  if (bf.counters) {
    int* flag = reinterpret_cast<int*>(lds);
    double* red = reinterpret_cast<double*>(lds) + 2;
    double* smu = red + kThreads;
    const int T = bk.gx * C::WM;
    const float* part = bf.partial;
    int G = T;
    long long rpt = C::TM * 32;
    if (ng > 0) {
      // two levels: the last workgroup of each group of gw row blocks merges the group's tiles into
      // one tile of the second array; the last group merges those
      const int grp = bk.x / gw;
      const int x0 = grp * gw, x1 = min(bk.gx, x0 + gw);
      if (!last_arriver(bf.counters + gy + bk.y * ng + grp, (unsigned)(x1 - x0), flag, g.acq != 0)) return;
      float* part1 = bf.partial + 3LL * T * K;
      bn_merge_level1<true>(g.m, K, T, rpt, bf.partial, x0 * C::WM, x1 * C::WM, n0col, C::BN, part1, ng, grp, red, smu,
                            kThreads);
      if (!last_arriver(bf.counters + bk.y, (unsigned)ng, flag, g.acq != 0)) return;
      part = part1;
      G = ng;
      rpt = (long long)gw * C::WM * C::TM * 32;
    } else if (!last_arriver(bf.counters + bk.y, (unsigned)bk.gx, flag, g.acq != 0)) {
      return;
    }
    bn_merge_block<true>(g.m, K, G, rpt, part, n0col, C::BN, bf.running_mean, bf.running_var, bf.momentum, bf.eps,
                   bf.save_mean, bf.save_invstd, red, smu, kThreads);
  }
}
template <class C>
__global__ __launch_bounds__(kBlock, min_waves<C>()) void k_fwd_lds(ConvArgs g, const float* __restrict__ x,
                                                     const float* __restrict__ w, float* __restrict__ y,
                                                     tspm_bn_fuse bf, float* __restrict__ slabs, int gw, int ng) {
  extern __shared__ float lds[];
  fwd_body<C>(g, x, w, y, bf, slabs, gw, ng, lds, grid_blk(g.xcd), (int)gridDim.y);
}

// Two independent forwards in ONE launch (round 6): the first conv of a downsampling BasicBlock and its 1x1
// downsample read the same block input and are independent (resnet.py:41,50-51), so their tiles share a grid —
// workgroups [0, n1) run the first GEMM's tiles, the rest the second's; each body is k_fwd_lds's, so every output,
// BN partial and in-launch merge is bitwise that of the separate launch.  Same tile configuration, own splits.
struct FwdJob {
  ConvArgs g;
  const float* x;
  const float* w;
  float* y;
  tspm_bn_fuse bf;
  float* slabs;
  int gw, ng, gx, gy;
};
template <class C>
__global__ __launch_bounds__(kBlock, min_waves<C>()) void k_fwd_pair_lds(FwdJob j1, FwdJob j2) {
  extern __shared__ float lds[];
  int b = (int)blockIdx.x;
  const int n1 = j1.gx * j1.gy * j1.g.splits;
  const FwdJob& j = b < n1 ? j1 : j2;
  if (b >= n1) b -= n1;
  const int z = b / (j.gx * j.gy);
  b -= z * j.gx * j.gy;
  const int yb = b / j.gx;
  fwd_body<C>(j.g, j.x, j.w, j.y, j.bf, j.slabs, j.gw, j.ng, lds, Blk{b - yb * j.gx, yb, z, j.gx}, j.gy);
}

// =============================================================================================
// Data gradient: dx[(h,w,n), ci] = sum_{valid (r,s), co} dy[((h+pad-r)/st, (w+pad-s)/st, n), co] w[co,r,s,ci]
// A image: BM rows (n) x 32 output channels (swizzled); B image: 32 rows (co) x BN input channels.
// =============================================================================================
// Round 6: the BatchNorm backward of one dgrad column block [c0, c0 + CB), run by the block's last-finishing tile
// (ConvArgs.bnx_*): the channels' partial tiles are merged in tspm_bn_bwd_apply_part's order (per channel, 16 row
// groups each summing tiles rg, rg + 16, ... in double, then the groups in order), the coefficients are formed as
// k_bn_bwd_apply_m forms them, and dy [, dy2] [, dres] are written over all M rows — tspm_bn_bwd_apply_part's
// values without its launch.  dx and the partials were published with st_sc1 (write-through); the ticket takes an
// agent-scope acquire, so they are read with plain (vector) loads.
__host__ __device__ inline size_t bnx_lds_bytes(int CB) { return 16 + (size_t)16 * CB * 3 * sizeof(double) + (size_t)CB * 8 * sizeof(float); }
TSPM_DEV void bnx_tail(const ConvArgs& g, const float* __restrict__ dx, int c0, int CB, float* lds) {
  const int t = threadIdx.x;
  const int M = g.m, C = g.c, G = M >> 5;
  const long long plane = (long long)G * C;
  const bool two = g.bnb_y2 != nullptr;
  double* acc = reinterpret_cast<double*>(lds + 4);              // [16][CB][3]
  float* coef = reinterpret_cast<float*>(acc + 16 * CB * 3);      // [8][CB]: ca cb cm ca2 cb2 cm2
  for (int i = t; i < 16 * CB; i += kThreads) {
    const int rg = i / CB, cl = i - rg * CB, c = c0 + cl;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0;
    if (c < C)
      for (int tile = rg; tile < G; tile += 16) {  // (behind the ticket's agent acquire: plain loads)
        const long long o = (long long)tile * C + c;
        a0 += (double)g.bnb_part[o];
        a1 += (double)g.bnb_part[plane + o];
        if (two) a2 += (double)g.bnb_part[2 * plane + o];
      }
    acc[(rg * CB + cl) * 3 + 0] = a0;
    acc[(rg * CB + cl) * 3 + 1] = a1;
    acc[(rg * CB + cl) * 3 + 2] = a2;
  }
  __syncthreads();
  for (int cl = t; cl < CB; cl += kThreads) {
    const int c = c0 + cl;
    if (c >= C) continue;
    double sg = acc[cl * 3 + 0], sx = acc[cl * 3 + 1], sx2 = acc[cl * 3 + 2];
    for (int k = 1; k < 16; ++k) {
      sg += acc[(k * CB + cl) * 3 + 0];
      sx += acc[(k * CB + cl) * 3 + 1];
      sx2 += acc[(k * CB + cl) * 3 + 2];
    }
    const double n = (double)M;
    const double iv = g.bnx_inv[c], ga = g.bnx_gamma[c];
    const double dg = sx * iv;
    const double a_ = ga * iv;
    coef[0 * CB + cl] = (float)a_;
    coef[1 * CB + cl] = (float)(a_ * iv * dg / n);
    coef[2 * CB + cl] = (float)(a_ * sg / n);
    g.bnx_dgamma[c] = (float)dg;
    g.bnx_dbeta[c] = (float)sg;
    if (two) {
      const double iv2 = g.bnx_inv2[c], ga2 = g.bnx_gamma2[c];
      const double dg2 = sx2 * iv2;
      const double a2 = ga2 * iv2;
      coef[3 * CB + cl] = (float)a2;
      coef[4 * CB + cl] = (float)(a2 * iv2 * dg2 / n);
      coef[5 * CB + cl] = (float)(a2 * sg / n);
      g.bnx_dgamma2[c] = (float)dg2;
      g.bnx_dbeta2[c] = (float)sg;
    }
  }
  __syncthreads();
  // apply: thread = (row group, 4 channels)
  const int L4 = CB >> 2, nrg = kThreads / L4;
  const int q = t % L4, rg = t / L4;
  const int c = c0 + 4 * q;
  if (rg >= nrg || c >= C) return;
  f32x4 ca, cb, cm, ca2 = {0.f, 0.f, 0.f, 0.f}, cb2 = ca2, cm2 = ca2;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    ca[j] = coef[0 * CB + 4 * q + j];
    cb[j] = coef[1 * CB + 4 * q + j];
    cm[j] = coef[2 * CB + 4 * q + j];
    if (two) {
      ca2[j] = coef[3 * CB + 4 * q + j];
      cb2[j] = coef[4 * CB + 4 * q + j];
      cm2[j] = coef[5 * CB + 4 * q + j];
    }
  }
  const f32x4 mu = ld4(g.bnb_mean + c);
  const f32x4 mu2 = two ? ld4(g.bnb_mean2 + c) : f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int U = 4;  // rows per batch: their loads in flight together (clamped rows re-read, never stored)
  for (int rb = rg; rb < M; rb += U * nrg) {
    f32x4 gv[U], ov[U], yv[U], y2v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long off = (long long)min(rb + u * nrg, M - 1) * C + c;
      gv[u] = ld4(dx + off);
      ov[u] = ld4(g.bnb_out + off);
      yv[u] = ld4(g.bnb_y + off);
      if (two) y2v[u] = ld4(g.bnb_y2 + off);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int row = rb + u * nrg;
      if (row >= M) continue;
      const long long off = (long long)row * C + c;
#pragma unroll
      for (int j = 0; j < 4; ++j) gv[u][j] = ov[u][j] > 0.f ? gv[u][j] : 0.f;
      st4(g.bnx_dy + off, ca * gv[u] - cm - cb * (yv[u] - mu));
      if (two) st4(g.bnx_dy2 + off, ca2 * gv[u] - cm2 - cb2 * (y2v[u] - mu2));
      if (g.bnx_dres) st4(g.bnx_dres + off, gv[u]);
    }
  }
}

template <class C>
TSPM_DEV void dgrad_body(const ConvArgs& g, const float* __restrict__ dy, const float* __restrict__ w,
                         float* __restrict__ dx, float* __restrict__ slabs, float* lds, const Blk& bk) {
  TSPM_STAMP(tspm_g_stamps_lds, 0);
  const int tid = threadIdx.x, lane = tid & 63;
  const WaveId<C> id;
  const int N = g.n, Cc = g.c, K = g.k, RSC = g.r * g.s * Cc;
  const int m0 = bk.x * C::BM, c0col = bk.y * C::BN;
  const int pos = m0 / N, nb0 = m0 - pos * N;
  const int hi = pos / g.w, wi = pos - hi * g.w;
  unsigned rmask = 0, smask = 0;
  for (int r = 0; r < g.r; ++r) {
    const int t = hi + g.pad - r;
    if (t >= 0 && t % g.st == 0 && t / g.st < g.p) rmask |= 1u << r;
  }
  for (int s = 0; s < g.s; ++s) {
    const int t = wi + g.pad - s;
    if (t >= 0 && t % g.st == 0 && t / g.st < g.q) smask |= 1u << s;
  }
  const int nr = __builtin_popcount(rmask), ns = __builtin_popcount(smask);
  const int kb = K >> 5;
  const int T = nr * ns * kb;
  const int st0 = split_lo(T, bk.z, g.splits), st1 = split_lo(T, bk.z + 1, g.splits);

  constexpr int NA = C::BM / 32;
  constexpr int BCH = C::BN / 4;            // 16-B chunks per B row
  constexpr int NB = C::BN / 32;            // = 32 rows * BCH chunks / 256 threads
  const int wv = (tid >> 6) & 3;
  const float* da[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int row = (i * 4 + wv) * 8 + (lane >> 3);
    da[i] = dy + (long long)(nb0 + row) * K + (((lane & 7) ^ swz(row)) << 2);
  }
  const float* wb[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int e = (i * 4 + wv) * 64 + lane;
    const int brow = e / BCH, bcol = (e - brow * BCH) * 4;
    wb[i] = w + (long long)brow * RSC + min(c0col + bcol, Cc - 4);
  }
  Acc<C::TM, C::TN> acc;
  acc.zero();
  if (ring_loop<C, false, true>(
      acc, lds, st0, st1,
      [&](int st) -> Off {
        const int t = st / kb, k0 = (st - t * kb) << 5;
        const int ri = t / ns, si = t - ri * ns;
        unsigned rm = rmask, sm = smask;
        for (int i = 0; i < ri; ++i) rm &= rm - 1;
        for (int i = 0; i < si; ++i) sm &= sm - 1;
        const int r = __builtin_ctz(rm), s = __builtin_ctz(sm);
        const int pp = (hi + g.pad - r) / g.st, qq = (wi + g.pad - s) / g.st;
        return Off{((long long)pp * g.q + qq) * N * K + k0, (long long)k0 * RSC + (r * g.s + s) * Cc};
      },
      [&](const Off& off, int i) -> const float* { return i < NA ? da[i] + off.a : wb[i - NA] + off.b; },
      [&](float* slot, int i) -> float* {
        return i < NA ? slot + (i * 4 + wv) * 256 : slot + C::BM * 32 + ((i - NA) * 4 + wv) * 256;
      },
      [&](const float* img, f32x4 (&A)[C::KGW][C::TM], f32x4 (&B)[C::KGW][C::TN]) {
#pragma unroll
        for (int kk = 0; kk < C::KGW; ++kk) {
          const int q = (id.wk * C::KGW + kk) * 2 + (lane >> 5);
#pragma unroll
          for (int a = 0; a < C::TM; ++a) A[kk][a] = frag_row(img, (id.wm * C::TM + a) * 32 + (lane & 31), q);
#pragma unroll
          for (int b = 0; b < C::TN; ++b)
            B[kk][b] = frag_col(img + C::BM * 32, C::BN, q * 4, (id.wn * C::TN + b) * 32 + (lane & 31));
        }
      }))
    return;
  TSPM_STAMP(tspm_g_stamps_lds, 2);
  combine_k<C>(acc, lds, id, lane);
  TSPM_STAMP(tspm_g_stamps_lds, 3);
  const int row0 = m0 + id.wm * C::TM * 32, col0 = c0col + id.wn * C::TN * 32;
  if (!splitk_reduce<C>(acc, id, lane, slabs, (long long)g.m * Cc, g.splits, g.cnt, row0, col0, g.m, Cc, Cc, lds, bk, g.acq != 0))
    return;
  TSPM_STAMP(tspm_g_stamps_lds, 4);
  if (id.wk == 0 && col0 < Cc) {
    if (g.bnb_part) acc.store_bnb(dx, row0, col0, g.m, Cc, Cc, lane, g.beta != 0, g);
    else acc.store(dx, row0, col0, g.m, Cc, Cc, lane, g.beta != 0);
  }
  TSPM_STAMP(tspm_g_stamps_lds, 5);
  if (g.bnx_dy) {  // the column block's last tile runs its BN backward (round 6)
    if (!last_arriver(g.bnx_cnt + bk.y, (unsigned)bk.gx, reinterpret_cast<int*>(lds), true)) return;
    bnx_tail(g, dx, c0col, C::BN, lds);
  }
}
template <class C>
__global__ __launch_bounds__(kBlock, min_waves<C>()) void k_dgrad_lds(ConvArgs g, const float* __restrict__ dy,
                                                       const float* __restrict__ w, float* __restrict__ dx,
                                                       float* __restrict__ slabs) {
  extern __shared__ float lds[];
  dgrad_body<C>(g, dy, w, dx, slabs, lds, grid_blk(g.xcd));
}

// =============================================================================================
// Weight gradient: dw[co, (r,s,ci)] = sum_m dy[m, co] x[in(m, r, s), ci], one tap per workgroup
// column block (C % BN == 0).  Stage = 32 rows m (32 samples of one output position inside the
// tap's valid rectangle).  A image: 32 rows (m) x BM output channels; B image: 32 rows x BN inputs.
// =============================================================================================
template <class C>
TSPM_DEV void wgrad_body(const ConvArgs& g, const float* __restrict__ x, const float* __restrict__ dy,
                         float* __restrict__ dw, float* __restrict__ slabs, float* lds, const Blk& bk) {
  const int tid = threadIdx.x, lane = tid & 63;
  const WaveId<C> id;
  const int N = g.n, Cc = g.c, K = g.k, RSC = g.r * g.s * Cc;
  const int co0 = bk.x * C::BM, col0b = bk.y * C::BN;
  const int tap = col0b / Cc, ci0 = col0b - tap * Cc;
  const int r = tap / g.s, s = tap - r * g.s;
  const int pp_lo = max(0, cdiv_dev(g.pad - r, g.st)), pp_hi = min(g.p - 1, (g.h - 1 + g.pad - r) / g.st);
  const int qq_lo = max(0, cdiv_dev(g.pad - s, g.st)), qq_hi = min(g.q - 1, (g.w - 1 + g.pad - s) / g.st);
  const int npp = max(0, pp_hi - pp_lo + 1), nqq = max(0, qq_hi - qq_lo + 1), n32 = N >> 5;
  const int T = npp * nqq * n32;
  const int st0 = split_lo(T, bk.z, g.splits), st1 = split_lo(T, bk.z + 1, g.splits);

  constexpr int ACH = C::BM / 4, BCH = C::BN / 4;
  constexpr int NA = C::BM / 32, NB = C::BN / 32;
  const int wv = (tid >> 6) & 3;
  const float* ap[NA];
  const float* bp[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int e = (i * 4 + wv) * 64 + lane;
    const int arow = e / ACH, acol = (e - arow * ACH) * 4;
    ap[i] = dy + (long long)arow * K + min(co0 + acol, K - 4);
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int e = (i * 4 + wv) * 64 + lane;
    const int brow = e / BCH, bcol = (e - brow * BCH) * 4;
    bp[i] = x + (long long)brow * Cc + ci0 + bcol;
  }
  Acc<C::TM, C::TN> acc;
  acc.zero();
  if (ring_loop<C, true, true>(
      acc, lds, st0, st1,
      [&](int st) -> Off {
        const int pc = st / n32, nc = st - pc * n32;
        const int ip = pc / nqq, iq = pc - ip * nqq;
        const int pp = pp_lo + ip, qq = qq_lo + iq;
        const long long mrow = ((long long)pp * g.q + qq) * N + nc * 32;
        const long long xrow = ((long long)(pp * g.st - g.pad + r) * g.w + (qq * g.st - g.pad + s)) * N + nc * 32;
        return Off{mrow * K, xrow * Cc};
      },
      [&](const Off& off, int i) -> const float* { return i < NA ? ap[i] + off.a : bp[i - NA] + off.b; },
      [&](float* slot, int i) -> float* {
        return i < NA ? slot + (i * 4 + wv) * 256 : slot + 32 * C::BM + ((i - NA) * 4 + wv) * 256;
      },
      [&](const float* img, f32x4 (&A)[C::KGW][C::TM], f32x4 (&B)[C::KGW][C::TN]) {
#pragma unroll
        for (int kk = 0; kk < C::KGW; ++kk) {
          const int k0 = (id.wk * C::KGW + kk) * 8 + 4 * (lane >> 5);
#pragma unroll
          for (int a = 0; a < C::TM; ++a) A[kk][a] = frag_col(img, C::BM, k0, (id.wm * C::TM + a) * 32 + (lane & 31));
#pragma unroll
          for (int b = 0; b < C::TN; ++b)
            B[kk][b] = frag_col(img + 32 * C::BM, C::BN, k0, (id.wn * C::TN + b) * 32 + (lane & 31));
        }
      }))
    return;
  combine_k<C>(acc, lds, id, lane);
  const int row0 = co0 + id.wm * C::TM * 32, col0 = col0b + id.wn * C::TN * 32;
  if (!splitk_reduce<C>(acc, id, lane, slabs, (long long)K * RSC, g.splits, g.cnt, row0, col0, K, RSC, RSC, lds, bk, g.acq != 0))
    return;
  if (id.wk == 0 && row0 < K) acc.store(dw, row0, col0, K, RSC, RSC, lane, false);
}
template <class C>
__global__ __launch_bounds__(kBlock, min_waves<C>()) void k_wgrad_lds(ConvArgs g, const float* __restrict__ x,
                                                       const float* __restrict__ dy, float* __restrict__ dw,
                                                       float* __restrict__ slabs) {
  extern __shared__ float lds[];
  wgrad_body<C>(g, x, dy, dw, slabs, lds, grid_blk(g.xcd));
}

// =============================================================================================
// Input AND weight gradient of one convolution in ONE launch (tspm_conv_bwd).  Both implicit GEMMs
// read the same dy and are independent, and at batch 128 either alone leaves most of the 256 CUs
// idle, so they share one grid: workgroups [0, nw) run the weight-gradient tiles (virtual grid
// wgx x wgy x splits), the rest the data-gradient tiles.  The branch is workgroup-uniform; each
// body is the standalone kernel's, so results are bitwise those of the two separate launches.
// =============================================================================================
// An Adam update carried by a backward launch (tspm_conv_bwd_adam, ABI 20): `blocks` extra workgroups of the grid
// run k_adam's element loop (adam_consts / adam_update: bitwise tspm_adam_step) over `count` elements of the flat
// buffers — parameters an earlier backward launch finished — beside the launch's latency-bound GEMM tiles.
struct AdamJobArgs {
  float* p;
  const float* g;
  float *m, *v;
  long long count;
  const tspm_adam_hyper* h;
};
TSPM_DEV void adam_job_body(const AdamJobArgs& a, int blk, int blocks) {
  const AdamConsts c = adam_consts_uniform(a.h);
  const long long n4 = a.count >> 2;
  for (long long i = (long long)blk * kBlock + threadIdx.x; i < n4; i += (long long)blocks * kBlock) {
    f32x4 pp = ld4(a.p + 4 * i), gg = ld4(a.g + 4 * i), mm = ld4(a.m + 4 * i), vv = ld4(a.v + 4 * i);
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // element copies, as k_adam
      float a = pp[j], b = mm[j], cc = vv[j];
      adam_update(a, gg[j], b, cc, c, false, 1.f);
      pp[j] = a; mm[j] = b; vv[j] = cc;
    }
    st4(a.p + 4 * i, pp);
    st4(a.m + 4 * i, mm);
    st4(a.v + 4 * i, vv);
  }
  if (blk == 0 && threadIdx.x < (a.count & 3)) {
    const long long i = (n4 << 2) + threadIdx.x;
    float pp = a.p[i], mm = a.m[i], vv = a.v[i];
    adam_update(pp, a.g[i], mm, vv, c, false, 1.f);
    a.p[i] = pp;
    a.m[i] = mm;
    a.v[i] = vv;
  }
}

template <class CD, class CW>
__global__ __launch_bounds__(kBlock, (min_waves2<CD, CW>())) void k_bwd_lds(ConvArgs gd, const float* __restrict__ dy,
                                                     const float* __restrict__ w, float* __restrict__ dx,
                                                     float* __restrict__ slabs_d, int dgx, int dgy, ConvArgs gw,
                                                     const float* __restrict__ x, float* __restrict__ dw,
                                                     float* __restrict__ slabs_w, int wgx, int wgy, AdamJobArgs aj,
                                                     int naj) {
  extern __shared__ float lds[];
  const int nconv = (int)gridDim.x - naj;
  if ((int)blockIdx.x < naj) {  // the carried Adam update: the first naj workgroups, dispatched ahead of the tiles
    adam_job_body(aj, (int)blockIdx.x, naj);
    return;
  }
  const int b0 = (int)blockIdx.x - naj;
  int b = gd.xcd == 1 ? xcd_swizzle(b0, nconv) : b0;
  const int nw = wgx * wgy * gw.splits;
  if (b < nw) {
    const int z = b / (wgx * wgy);
    b -= z * wgx * wgy;
    const int y = b / wgx;
    wgrad_body<CW>(gw, x, dy, dw, slabs_w, lds, Blk{b - y * wgx, y, z, wgx});
  } else {
    b -= nw;
    const int z = b / (dgx * dgy);
    b -= z * dgx * dgy;
    const int y = b / dgx;
    dgrad_body<CD>(gd, dy, w, dx, slabs_d, lds, Blk{b - y * dgx, y, z, dgx});
  }
}

// The backward of a downsampling block's second conv and of its 1x1 downsample in ONE launch (round 6): both read
// gradients the block's bn2 backward has just written (d_y2 and d_yd) and write disjoint tensors (conv2's input
// gradient and the block-input gradient that conv1's data gradient later accumulates onto), so their four GEMMs —
// the two weight gradients, then the two data gradients — share a grid, each body k_bwd_lds's (same tile
// configurations, own split counts); carried-Adam workgroups first, as k_bwd_lds.
struct BwdHalf {
  ConvArgs gd, gw;
  const float *dy, *w, *x;
  float *dx, *dw, *slabs_d, *slabs_w;
  int dgx, dgy, wgx, wgy;
};
template <class CD, class CW>
__global__ __launch_bounds__(kBlock, (min_waves2<CD, CW>())) void k_bwd_quad_lds(BwdHalf h1, BwdHalf h2,
                                                                                AdamJobArgs aj, int naj) {
  extern __shared__ float lds[];
  if ((int)blockIdx.x < naj) {
    adam_job_body(aj, (int)blockIdx.x, naj);
    return;
  }
  int b = (int)blockIdx.x - naj;
  const int nw1 = h1.wgx * h1.wgy * h1.gw.splits, nw2 = h2.wgx * h2.wgy * h2.gw.splits;
  const int nd1 = h1.dgx * h1.dgy * h1.gd.splits;
  if (b < nw1 + nw2) {
    const BwdHalf& h = b < nw1 ? h1 : h2;
    if (b >= nw1) b -= nw1;
    const int z = b / (h.wgx * h.wgy);
    b -= z * h.wgx * h.wgy;
    const int y = b / h.wgx;
    wgrad_body<CW>(h.gw, h.x, h.dy, h.dw, h.slabs_w, lds, Blk{b - y * h.wgx, y, z, h.wgx});
  } else {
    b -= nw1 + nw2;
    const BwdHalf& h = b < nd1 ? h1 : h2;
    if (b >= nd1) b -= nd1;
    const int z = b / (h.dgx * h.dgy);
    b -= z * h.dgx * h.dgy;
    const int y = b / h.dgx;
    dgrad_body<CD>(h.gd, h.dy, h.w, h.dx, h.slabs_d, lds, Blk{b - y * h.dgx, y, z, h.dgx});
  }
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
using tspm_detail::LdsAlgo;

bool algo_ok(const LdsAlgo& a) {
  // (tm, tn) in {(1,1), (1,2), (2,1)}: the 2x2 wave tiles spilled and no tuned table selected them (removed
  // in round 5 with the round-3 fragment-prefetch experiment that raced on them)
  if (!((a.tm == 1 && (a.tn == 1 || a.tn == 2)) || (a.tm == 2 && a.tn == 1))) return false;
  if (!(a.wm >= 1 && a.wn >= 1 && a.wk >= 1 && a.wm * a.wn * a.wk == 4)) return false;
  if (kSplit && a.wk > 2) return false;
  return a.splits >= 1 && a.splits <= 256;
}
int bm_of(const LdsAlgo& a) { return a.wm * a.tm * 32; }
int bn_of(const LdsAlgo& a) { return a.wn * a.tn * 32; }

size_t lds_bytes(const LdsAlgo& a, bool bn_tail) {
  const size_t st1 = (size_t)(bm_of(a) + bn_of(a)) * (kSplit ? 48 : 32) * sizeof(float);  // = Cfg::STAGE
  int depth = kRegStage ? ((kPairBuild && st1 * 4 <= TSPM_PAIR_MAX_BYTES) ? 4 : 2) : TSPM_RING_MAX;  // = ring_depth<>
  while (!kRegStage && depth > 2 && st1 * depth > TSPM_RING_BYTES) --depth;
  const size_t stage = depth * st1;
  const size_t comb = (size_t)(a.wk - 1) * a.wm * a.wn * a.tm * a.tn * 16 * 64 * sizeof(float);
  const size_t tail = bn_tail ? 16 + 8 * (size_t)(kThreads + bn_of(a)) : 16;
  return std::max(std::max(stage, comb), tail);
}

bool hwnc(const tspm_conv_shape* s, const tspm_strides4* st) {
  if (!st) return true;
  return st->sc == 1 && st->sn == s->c && st->sw == (long long)s->n * s->c && st->sh == (long long)s->w * s->n * s->c;
}

// XCD-aware workgroup -> tile mapping (1: over the whole grid, 2: within each split-K plane): measured
// slower in the step (2.82 -> 3.01 ms) or neutral — identity mapping.  Results are bitwise the
// same either way).  Not reachable.
constexpr int xcd_enabled() { return 0; }

// The last arriver of a split-K tile / BN merge group reads the sc1 payload with sc1 loads and takes no
// agent-scope acquire (conv 2.612 -> 2.595 ms without it; bitwise the same).  The algo flag
// TSPM_ALGO_HANDOFF_ACQUIRE restores the acquire: the reference side of the hand-off validation
// (tests/test_gpu_handoff.py), not a performance option.
ConvArgs args_of(const tspm_conv_shape* s, const LdsAlgo& a) {
  ConvArgs g{};
  g.n = s->n; g.h = s->h; g.w = s->w; g.c = s->c; g.k = s->k; g.r = s->r; g.s = s->s;
  g.st = s->stride; g.pad = s->pad; g.p = s->p; g.q = s->q;
  g.sn = s->c; g.sh = (long long)s->w * s->n * s->c; g.sw = (long long)s->n * s->c; g.sc = 1;
  g.m = 0; g.splits = 1; g.slab = 0; g.beta = 0; g.cnt = nullptr;
  g.xcd = xcd_enabled();
  g.acq = a.acq;
  return g;
}

size_t splitk_ws(int splits, long long rows, long long cols) {
  return splits > 1 ? TSPM_COUNTER_BYTES + (size_t)splits * rows * cols * sizeof(float) : 0;
}
// the split-K reduction addresses one slab with 32-bit offsets
bool slab_fits(int splits, long long rows, long long cols) { return splits <= 1 || rows * cols < (1LL << 31); }

// dispatch over the supported (tm, tn, wm, wn, wk) combinations
#define TSPM_LDS_CASE(TM_, TN_, WM_, WN_, WK_, FN)                                      \
  if (a.tm == TM_ && a.tn == TN_ && a.wm == WM_ && a.wn == WN_ && a.wk == WK_) {      \
    using CF = Cfg<TM_, TN_, WM_, WN_, WK_>;                                          \
    FN(CF);                                                                           \
    return TSPM_OK;                                                                   \
  }
#define TSPM_LDS_WAVES(TM_, TN_, FN)      \
  TSPM_LDS_CASE(TM_, TN_, 4, 1, 1, FN)    \
  TSPM_LDS_CASE(TM_, TN_, 2, 2, 1, FN)    \
  TSPM_LDS_CASE(TM_, TN_, 1, 4, 1, FN)    \
  TSPM_LDS_CASE(TM_, TN_, 2, 1, 2, FN)    \
  TSPM_LDS_CASE(TM_, TN_, 1, 2, 2, FN)    \
  TSPM_LDS_CASE_WK4(TM_, TN_, FN)
// wk == 4 (8-deep slices of a stage per wave): not in the split build, whose waves take whole 16-deep steps
#ifdef TSPM_LDS_SPLIT
#define TSPM_LDS_CASE_WK4(TM_, TN_, FN)
#else
#define TSPM_LDS_CASE_WK4(TM_, TN_, FN) TSPM_LDS_CASE(TM_, TN_, 1, 1, 4, FN)
#endif
#define TSPM_LDS_DISPATCH(FN)   \
  TSPM_LDS_WAVES(1, 1, FN)      \
  TSPM_LDS_WAVES(1, 2, FN)      \
  TSPM_LDS_WAVES(2, 1, FN)      \
  return TSPM_ERR_INVALID;

// BN merge plan of a forward launch: ng == 0 one level (<= 16 tiles per merging thread); ng > 0
// two levels, first-level groups of gw row blocks (<= 8 tiles per merging thread) and ng groups
// (<= 16 per thread); ng < 0 none fits (tspm_bn_finalize).
struct BnLevels {
  int gw, ng;
};
BnLevels bn_levels(const tspm_conv_shape* s, const LdsAlgo& a) {
  const int bnn = bn_of(a), groups = kThreads / bnn;
  const int gx = (s->p * s->q * s->n) / bm_of(a);
  if (cdiv(gx * a.wm, groups) <= 16) return BnLevels{0, 0};
  const int gw = std::max(1, 8 * groups / a.wm);
  const int ng = cdiv(gx, gw);
  if (cdiv(ng, groups) > 16) return BnLevels{0, -1};
  return BnLevels{gw, ng};
}

}  // namespace

namespace TSPM_LDS_NS {
using tspm_detail::LdsAlgo;

bool lds_fwd_supported(const tspm_conv_shape* s, const tspm_strides4* xs, const LdsAlgo& a) {
  if (!algo_ok(a) || !hwnc(s, xs)) return false;
  if (s->c % 32 != 0 || s->r > 31 || s->s > 31) return false;
  const int bm = bm_of(a);
  return s->n % bm == 0 && lds_bytes(a, true) <= 160 * 1024;
}
bool lds_dgrad_supported(const tspm_conv_shape* s, const LdsAlgo& a) {
  if (!algo_ok(a)) return false;
  if (s->k % 32 != 0 || s->c % 4 != 0 || s->r > 31 || s->s > 31) return false;
  return s->n % bm_of(a) == 0 && lds_bytes(a, false) <= 160 * 1024;
}
bool lds_wgrad_supported(const tspm_conv_shape* s, const tspm_strides4* xs, const LdsAlgo& a) {
  if (!algo_ok(a) || !hwnc(s, xs)) return false;
  if (s->n % 32 != 0 || s->k % 4 != 0 || s->c % bn_of(a) != 0) return false;
  return lds_bytes(a, false) <= 160 * 1024;
}
size_t lds_fwd_workspace(const tspm_conv_shape* s, const LdsAlgo& a) {
  return splitk_ws(a.splits, (long long)s->p * s->q * s->n, s->k);
}
int lds_fwd_bn_inlaunch(const tspm_conv_shape* s, const LdsAlgo& a) { return bn_levels(s, a).ng == 0 ? 1 : 0; }
int lds_fwd_bn_counters(const tspm_conv_shape* s, const LdsAlgo& a) {
  const BnLevels lv = bn_levels(s, a);
  return cdiv(s->k, bn_of(a)) * (1 + std::max(lv.ng, 0));
}
long long lds_fwd_bn_partial_floats(const tspm_conv_shape* s, const LdsAlgo& a) {
  const BnLevels lv = bn_levels(s, a);
  const long long tiles = (long long)(s->p * s->q * s->n) / (a.tm * 32);
  return 3LL * (tiles + std::max(lv.ng, 0)) * s->k;
}
size_t lds_dgrad_workspace(const tspm_conv_shape* s, const LdsAlgo& a) {
  return splitk_ws(a.splits, (long long)s->h * s->w * s->n, s->c);
}
size_t lds_wgrad_workspace(const tspm_conv_shape* s, const LdsAlgo& a) {
  return splitk_ws(a.splits, s->k, (long long)s->r * s->s * s->c);
}

// A forward launch's arguments (split-K workspace, BN merge plan); `want` keeps the caller's BN request when the
// merge cannot run in-launch (then tspm_bn_finalize follows the launch)
int fwd_job(const tspm_conv_shape* s, const LdsAlgo& a, const float* x, const float* w, float* y,
            const tspm_bn_fuse* bn, void* ws, size_t ws_bytes, FwdJob& j, tspm_bn_fuse& want) {
  j = FwdJob{};
  j.g = args_of(s, a);
  ConvArgs& g = j.g;
  g.m = s->p * s->q * s->n;
  g.splits = a.splits;
  if (!slab_fits(a.splits, g.m, s->k)) return TSPM_ERR_INVALID;
  if (a.splits > 1) {
    if (!ws || ws_bytes < lds_fwd_workspace(s, a)) return TSPM_ERR_WORKSPACE;
    g.cnt = static_cast<unsigned*>(ws);
    j.slabs = reinterpret_cast<float*>(static_cast<char*>(ws) + TSPM_COUNTER_BYTES);
  }
  tspm_bn_fuse bf{};
  if (bn) bf = *bn;
  j.gx = g.m / bm_of(a);
  j.gy = cdiv(s->k, bn_of(a));
  if ((size_t)j.gx * j.gy > TSPM_COUNTER_BYTES / sizeof(unsigned) && a.splits > 1) return TSPM_ERR_INVALID;
  // in-launch BN merge: one level when each merging thread reads few tiles, two levels when the
  // caller's buffers allow it (tspm_bn_fuse.counters_len / partial_floats), else tspm_bn_finalize
  const int tiles = j.gx * a.wm;
  const BnLevels lv = bn_levels(s, a);
  want = bf;
  if (bf.counters && lv.ng != 0) {
    const bool room = lv.ng > 0 && bf.counters_len >= (long long)j.gy * (1 + lv.ng) &&
                      bf.partial_floats >= 3LL * (tiles + lv.ng) * s->k;
    if (!room) bf.counters = nullptr;
  }
  j.gw = bf.counters ? lv.gw : 0;
  j.ng = bf.counters ? lv.ng : 0;
  j.bf = bf;
  j.x = x; j.w = w; j.y = y;
  return TSPM_OK;
}
int fwd_finalize(const tspm_conv_shape* s, const LdsAlgo& a, const FwdJob& j, const tspm_bn_fuse& want,
                 hipStream_t st) {
  if (want.counters && !j.bf.counters)
    return tspm_bn_finalize(j.g.m, s->k, j.gx * a.wm, a.tm * 32, want.partial, want.running_mean, want.running_var,
                            want.momentum, want.eps, want.save_mean, want.save_invstd, st);
  return TSPM_OK;
}

int lds_fwd(const tspm_conv_shape* s, const LdsAlgo& a, const float* x, const float* w, float* y,
            const tspm_bn_fuse* bn, void* ws, size_t ws_bytes, hipStream_t st) {
  FwdJob j;
  tspm_bn_fuse want;
  const int e = fwd_job(s, a, x, w, y, bn, ws, ws_bytes, j, want);
  if (e != TSPM_OK) return e;
  const dim3 grid(j.gx, j.gy, a.splits);
  const size_t lds = tspm_detail::lds_with_floor(lds_bytes(a, j.bf.counters != nullptr), a);
#define TSPM_FWD(CFG) \
  hipLaunchKernelGGL(k_fwd_lds<CFG>, grid, dim3(kBlock), lds, st, j.g, x, w, y, j.bf, j.slabs, j.gw, j.ng)
  const int rc = [&]() -> int { TSPM_LDS_DISPATCH(TSPM_FWD) }();
#undef TSPM_FWD
  if (rc != TSPM_OK) return rc;
  TSPM_LAUNCH_CHECK();
  return fwd_finalize(s, a, j, want, st);
}

// two forwards of the same tile configuration in one launch (k_fwd_pair_lds); the caller checked support
int lds_fwd_pair(const tspm_conv_shape* s1, const LdsAlgo& a1, const float* x1, const float* w1, float* y1,
                 const tspm_bn_fuse* bn1, void* ws1, size_t ws1_bytes, const tspm_conv_shape* s2, const LdsAlgo& a2,
                 const float* x2, const float* w2, float* y2, const tspm_bn_fuse* bn2, void* ws2, size_t ws2_bytes,
                 hipStream_t st) {
  if (a1.tm != a2.tm || a1.tn != a2.tn || a1.wm != a2.wm || a1.wn != a2.wn || a1.wk != a2.wk) return TSPM_ERR_INVALID;
  if (a1.splits > 1 && a2.splits > 1 && ws1 == ws2) return TSPM_ERR_INVALID;  // counters / slabs would collide
  FwdJob j1, j2;
  tspm_bn_fuse want1, want2;
  int e = fwd_job(s1, a1, x1, w1, y1, bn1, ws1, ws1_bytes, j1, want1);
  if (e != TSPM_OK) return e;
  e = fwd_job(s2, a2, x2, w2, y2, bn2, ws2, ws2_bytes, j2, want2);
  if (e != TSPM_OK) return e;
  if (j1.bf.counters && j2.bf.counters && j1.bf.counters == j2.bf.counters) return TSPM_ERR_INVALID;
  if (j1.bf.partial && j1.bf.partial == j2.bf.partial) return TSPM_ERR_INVALID;
  const long long nblk = (long long)j1.gx * j1.gy * a1.splits + (long long)j2.gx * j2.gy * a2.splits;
  LdsAlgo af = a1;
  af.floor = std::max(a1.floor, a2.floor);
  const size_t lds = tspm_detail::lds_with_floor(
      std::max(lds_bytes(a1, j1.bf.counters != nullptr), lds_bytes(a2, j2.bf.counters != nullptr)), af);
  const LdsAlgo& a = a1;
#define TSPM_FWD2(CFG) hipLaunchKernelGGL(k_fwd_pair_lds<CFG>, dim3((unsigned)nblk), dim3(kBlock), lds, st, j1, j2)
  const int rc = [&]() -> int { TSPM_LDS_DISPATCH(TSPM_FWD2) }();
#undef TSPM_FWD2
  if (rc != TSPM_OK) return rc;
  TSPM_LAUNCH_CHECK();
  e = fwd_finalize(s1, a1, j1, want1, st);
  if (e != TSPM_OK) return e;
  return fwd_finalize(s2, a2, j2, want2, st);
}

int lds_dgrad(const tspm_conv_shape* s, const LdsAlgo& a, const float* dy, const float* w, float* dx, int beta,
              void* ws, size_t ws_bytes, hipStream_t st) {
  ConvArgs g = args_of(s, a);
  g.m = s->h * s->w * s->n;
  g.splits = a.splits;
  g.beta = beta ? 1 : 0;
  if (!slab_fits(a.splits, g.m, s->c)) return TSPM_ERR_INVALID;
  float* slabs = nullptr;
  if (a.splits > 1) {
    if (!ws || ws_bytes < lds_dgrad_workspace(s, a)) return TSPM_ERR_WORKSPACE;
    g.cnt = static_cast<unsigned*>(ws);
    slabs = reinterpret_cast<float*>(static_cast<char*>(ws) + TSPM_COUNTER_BYTES);
  }
  const dim3 grid(g.m / bm_of(a), cdiv(s->c, bn_of(a)), a.splits);
  if ((size_t)grid.x * grid.y > TSPM_COUNTER_BYTES / sizeof(unsigned) && a.splits > 1) return TSPM_ERR_INVALID;
  const size_t lds = tspm_detail::lds_with_floor(lds_bytes(a, false), a);
#define TSPM_DG(CFG) hipLaunchKernelGGL(k_dgrad_lds<CFG>, grid, dim3(kBlock), lds, st, g, dy, w, dx, slabs)
  const int rc = [&]() -> int { TSPM_LDS_DISPATCH(TSPM_DG) }();
#undef TSPM_DG
  if (rc != TSPM_OK) return rc;
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

int lds_wgrad(const tspm_conv_shape* s, const LdsAlgo& a, const float* x, const float* dy, float* dw, void* ws,
              size_t ws_bytes, hipStream_t st) {
  ConvArgs g = args_of(s, a);
  g.m = s->k;
  g.splits = a.splits;
  if (!slab_fits(a.splits, s->k, (long long)s->r * s->s * s->c)) return TSPM_ERR_INVALID;
  float* slabs = nullptr;
  if (a.splits > 1) {
    if (!ws || ws_bytes < lds_wgrad_workspace(s, a)) return TSPM_ERR_WORKSPACE;
    g.cnt = static_cast<unsigned*>(ws);
    slabs = reinterpret_cast<float*>(static_cast<char*>(ws) + TSPM_COUNTER_BYTES);
  }
  const int RSC = s->r * s->s * s->c;
  const dim3 grid(cdiv(s->k, bm_of(a)), RSC / bn_of(a), a.splits);
  if ((size_t)grid.x * grid.y > TSPM_COUNTER_BYTES / sizeof(unsigned) && a.splits > 1) return TSPM_ERR_INVALID;
  const size_t lds = tspm_detail::lds_with_floor(lds_bytes(a, false), a);
#define TSPM_WG(CFG) hipLaunchKernelGGL(k_wgrad_lds<CFG>, grid, dim3(kBlock), lds, st, g, x, dy, dw, slabs)
  const int rc = [&]() -> int { TSPM_LDS_DISPATCH(TSPM_WG) }();
#undef TSPM_WG
  if (rc != TSPM_OK) return rc;
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

// ---- fused dgrad + wgrad (k_bwd_lds): the (dgrad, wgrad) tile pairs built into the library are the
// configurations the batch-128/256 tuning picks most (tuned/*.json): 5 for dgrad x 5 for wgrad
struct BwdLaunch {
  ConvArgs gd, gw;
  const float *dy, *w, *x;
  float *dx, *dw, *slabs_d, *slabs_w;
  int dgx, dgy, wgx, wgy;
  size_t lds;
  hipStream_t st;
  AdamJobArgs aj;
  int naj;
  const BwdHalf* second;  // k_bwd_quad_lds: the downsample's backward in the same launch (nullptr: k_bwd_lds)
};
template <class CD, class CW>
void bwd_go(const BwdLaunch& L) {
  if (L.second) {
    const BwdHalf h1{L.gd, L.gw, L.dy, L.w, L.x, L.dx, L.dw, L.slabs_d, L.slabs_w, L.dgx, L.dgy, L.wgx, L.wgy};
    const BwdHalf& h2 = *L.second;
    const int nblk = h1.wgx * h1.wgy * h1.gw.splits + h2.wgx * h2.wgy * h2.gw.splits + h1.dgx * h1.dgy * h1.gd.splits +
                     h2.dgx * h2.dgy * h2.gd.splits + L.naj;
    hipLaunchKernelGGL((k_bwd_quad_lds<CD, CW>), dim3(nblk), dim3(kBlock), L.lds, L.st, h1, h2, L.aj, L.naj);
    return;
  }
  const int nblk = L.wgx * L.wgy * L.gw.splits + L.dgx * L.dgy * L.gd.splits + L.naj;
  hipLaunchKernelGGL((k_bwd_lds<CD, CW>), dim3(nblk), dim3(kBlock), L.lds, L.st, L.gd, L.dy, L.w, L.dx, L.slabs_d,
                     L.dgx, L.dgy, L.gw, L.x, L.dw, L.slabs_w, L.wgx, L.wgy, L.aj, L.naj);
}
bool is_cfg(const LdsAlgo& a, int tm, int wm, int wn, int wk) {
  return a.tm == tm && a.tn == 1 && a.wm == wm && a.wn == wn && a.wk == wk;
}
template <class CD>
bool bwd_w(const LdsAlgo& aw, const BwdLaunch* L) {  // L == nullptr: query only
#define TSPM_BW(TM_, WM_, WN_, WK_)                             \
  if (is_cfg(aw, TM_, WM_, WN_, WK_)) {                         \
    if (L) bwd_go<CD, Cfg<TM_, 1, WM_, WN_, WK_>>(*L);          \
    return true;                                                \
  }
  TSPM_BW(1, 2, 2, 1)
#ifndef TSPM_LDS_SPLIT
  TSPM_BW(1, 1, 1, 4)
#endif
  TSPM_BW(1, 1, 2, 2)
  TSPM_BW(1, 2, 1, 2)
  TSPM_BW(2, 2, 2, 1)
#undef TSPM_BW
  return false;
}
bool bwd_dispatch(const LdsAlgo& ad, const LdsAlgo& aw, const BwdLaunch* L) {
#define TSPM_BD(TM_, WM_, WN_, WK_) \
  if (is_cfg(ad, TM_, WM_, WN_, WK_)) return bwd_w<Cfg<TM_, 1, WM_, WN_, WK_>>(aw, L);
  TSPM_BD(1, 1, 2, 2)
  TSPM_BD(1, 1, 4, 1)
#ifndef TSPM_LDS_SPLIT
  TSPM_BD(1, 1, 1, 4)
#endif
  TSPM_BD(2, 2, 2, 1)
  TSPM_BD(2, 1, 4, 1)
#undef TSPM_BD
  return false;
}

bool lds_bwd_built(const LdsAlgo& ad, const LdsAlgo& aw) { return bwd_dispatch(ad, aw, nullptr); }

// one conv's dgrad + wgrad arguments (split-K workspaces, grid) for k_bwd_lds / k_bwd_quad_lds
int bwd_half(const tspm_conv_shape* s, const LdsAlgo& ad, const LdsAlgo& aw, const float* x, const float* dy,
             const float* w, float* dx, int beta, float* dw, const tspm_bn_bwd_part* bnp, void* wsd, size_t wsd_bytes,
             void* wsw, size_t wsw_bytes, BwdHalf& h) {
  if (!slab_fits(ad.splits, (long long)s->h * s->w * s->n, s->c) ||
      !slab_fits(aw.splits, s->k, (long long)s->r * s->s * s->c))
    return TSPM_ERR_INVALID;
  h = BwdHalf{};
  h.gd = args_of(s, ad);
  h.gd.m = s->h * s->w * s->n;
  h.gd.splits = ad.splits;
  h.gd.beta = beta ? 1 : 0;
  if (bnp) {  // the BN-backward partial sums of dx in the dgrad epilogue (round 6)
    if (h.gd.m % 32 != 0 || !bnp->out || !bnp->y || !bnp->mean || !bnp->part || (bnp->y2 && !bnp->mean2))
      return TSPM_ERR_INVALID;
    h.gd.bnb_out = bnp->out; h.gd.bnb_y = bnp->y; h.gd.bnb_mean = bnp->mean;
    h.gd.bnb_y2 = bnp->y2; h.gd.bnb_mean2 = bnp->mean2; h.gd.bnb_part = bnp->part;
    if (bnp->idx) {  // max-pool gather: dx is the 3x3/2/1 pool's output gradient over a pool_h x pool_w map
      if (bnp->y2 || bnp->pool_h <= 0 || bnp->pool_w <= 0 || (bnp->pool_h - 1) / 2 + 1 != s->h ||
          (bnp->pool_w - 1) / 2 + 1 != s->w)
        return TSPM_ERR_INVALID;
      h.gd.bnb_idx = bnp->idx; h.gd.bnb_H = bnp->pool_h; h.gd.bnb_W = bnp->pool_w;
    }
    if (bnp->dy) {  // the whole BN backward in the epilogue (round 6)
      if (bnp->idx || !bnp->invstd || !bnp->gamma || !bnp->dgamma || !bnp->dbeta || !bnp->counters ||
          (bnp->y2 && (!bnp->invstd2 || !bnp->gamma2 || !bnp->dgamma2 || !bnp->dbeta2 || !bnp->dy2)) || s->c % 4)
        return TSPM_ERR_INVALID;
      h.gd.bnx_inv = bnp->invstd; h.gd.bnx_gamma = bnp->gamma; h.gd.bnx_dgamma = bnp->dgamma;
      h.gd.bnx_dbeta = bnp->dbeta; h.gd.bnx_dy = bnp->dy; h.gd.bnx_inv2 = bnp->invstd2; h.gd.bnx_gamma2 = bnp->gamma2;
      h.gd.bnx_dgamma2 = bnp->dgamma2; h.gd.bnx_dbeta2 = bnp->dbeta2; h.gd.bnx_dy2 = bnp->dy2;
      h.gd.bnx_dres = bnp->dres; h.gd.bnx_cnt = bnp->counters;
    }
  }
  if (ad.splits > 1) {
    if (!wsd || wsd_bytes < lds_dgrad_workspace(s, ad)) return TSPM_ERR_WORKSPACE;
    h.gd.cnt = static_cast<unsigned*>(wsd);
    h.slabs_d = reinterpret_cast<float*>(static_cast<char*>(wsd) + TSPM_COUNTER_BYTES);
  }
  h.gw = args_of(s, aw);
  h.gw.m = s->k;
  h.gw.splits = aw.splits;
  if (aw.splits > 1) {
    if (!wsw || wsw_bytes < lds_wgrad_workspace(s, aw)) return TSPM_ERR_WORKSPACE;
    h.gw.cnt = static_cast<unsigned*>(wsw);
    h.slabs_w = reinterpret_cast<float*>(static_cast<char*>(wsw) + TSPM_COUNTER_BYTES);
  }
  if (ad.splits > 1 && aw.splits > 1 && wsd == wsw) return TSPM_ERR_INVALID;  // counters / slabs would collide
  h.dgx = h.gd.m / bm_of(ad);
  h.dgy = cdiv(s->c, bn_of(ad));
  h.wgx = cdiv(s->k, bm_of(aw));
  h.wgy = s->r * s->s * s->c / bn_of(aw);
  const size_t cmax = TSPM_COUNTER_BYTES / sizeof(unsigned);
  if ((ad.splits > 1 && (size_t)h.dgx * h.dgy > cmax) || (aw.splits > 1 && (size_t)h.wgx * h.wgy > cmax))
    return TSPM_ERR_INVALID;
  h.dy = dy; h.w = w; h.x = x; h.dx = dx; h.dw = dw;
  return TSPM_OK;
}

int lds_bwd(const tspm_conv_shape* s, const LdsAlgo& ad, const LdsAlgo& aw, const float* x, const float* dy,
            const float* w, float* dx, int beta, float* dw, const tspm_adam_job* adam, const tspm_bn_bwd_part* bnp,
            void* wsd, size_t wsd_bytes, void* wsw, size_t wsw_bytes, hipStream_t st) {
  if (!bwd_dispatch(ad, aw, nullptr)) return TSPM_ERR_INVALID;
  BwdHalf h;
  const int e = bwd_half(s, ad, aw, x, dy, w, dx, beta, dw, bnp, wsd, wsd_bytes, wsw, wsw_bytes, h);
  if (e != TSPM_OK) return e;
  BwdLaunch L{};
  L.gd = h.gd; L.gw = h.gw; L.dy = h.dy; L.w = h.w; L.x = h.x; L.dx = h.dx; L.dw = h.dw;
  L.slabs_d = h.slabs_d; L.slabs_w = h.slabs_w; L.dgx = h.dgx; L.dgy = h.dgy; L.wgx = h.wgx; L.wgy = h.wgy;
  if (adam) {
    L.aj = AdamJobArgs{adam->param, adam->grad, adam->exp_avg, adam->exp_avg_sq, (long long)adam->count, adam->hyper};
    L.naj = adam->blocks;
  }
  LdsAlgo af = ad;  // one launch: the larger of the two halves' floors
  af.floor = std::max(ad.floor, aw.floor);
  size_t need = std::max(lds_bytes(ad, false), lds_bytes(aw, false));
  if (h.gd.bnx_dy) need = std::max(need, bnx_lds_bytes(bn_of(ad)));
  L.lds = tspm_detail::lds_with_floor(need, af);
  L.st = st;
  bwd_dispatch(ad, aw, &L);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

// conv2's backward and the downsample's in one launch (k_bwd_quad_lds): the downsample's algos take conv2's tile
// configurations (ad2 / aw2 must match ad / aw except splits and floor); workspaces pairwise distinct when split
int lds_bwd_quad(const tspm_conv_shape* s, const LdsAlgo& ad, const LdsAlgo& aw, const float* x, const float* dy,
                 const float* w, float* dx, int beta, float* dw, const tspm_bn_bwd_part* bnp, void* wsd,
                 size_t wsd_bytes, void* wsw, size_t wsw_bytes, const tspm_conv_shape* s2, const LdsAlgo& ad2,
                 const LdsAlgo& aw2, const float* x2, const float* dy2, const float* w2, float* dx2, float* dw2,
                 void* wsd2, size_t wsd2_bytes, void* wsw2, size_t wsw2_bytes, const tspm_adam_job* adam,
                 hipStream_t st) {
  if (!bwd_dispatch(ad, aw, nullptr)) return TSPM_ERR_INVALID;
  auto same = [](const LdsAlgo& a, const LdsAlgo& b) {
    return a.tm == b.tm && a.tn == b.tn && a.wm == b.wm && a.wn == b.wn && a.wk == b.wk;
  };
  if (!same(ad, ad2) || !same(aw, aw2)) return TSPM_ERR_INVALID;
  const void* wss[4] = {ad.splits > 1 ? wsd : nullptr, aw.splits > 1 ? wsw : nullptr,
                        ad2.splits > 1 ? wsd2 : nullptr, aw2.splits > 1 ? wsw2 : nullptr};
  for (int i = 0; i < 4; ++i)
    for (int j = i + 1; j < 4; ++j)
      if (wss[i] && wss[i] == wss[j]) return TSPM_ERR_INVALID;
  BwdHalf h1, h2;
  int e = bwd_half(s, ad, aw, x, dy, w, dx, beta, dw, bnp, wsd, wsd_bytes, wsw, wsw_bytes, h1);
  if (e != TSPM_OK) return e;
  e = bwd_half(s2, ad2, aw2, x2, dy2, w2, dx2, 0, dw2, nullptr, wsd2, wsd2_bytes, wsw2, wsw2_bytes, h2);
  if (e != TSPM_OK) return e;
  BwdLaunch L{};
  L.gd = h1.gd; L.gw = h1.gw; L.dy = h1.dy; L.w = h1.w; L.x = h1.x; L.dx = h1.dx; L.dw = h1.dw;
  L.slabs_d = h1.slabs_d; L.slabs_w = h1.slabs_w; L.dgx = h1.dgx; L.dgy = h1.dgy; L.wgx = h1.wgx; L.wgy = h1.wgy;
  L.second = &h2;
  if (adam) {
    L.aj = AdamJobArgs{adam->param, adam->grad, adam->exp_avg, adam->exp_avg_sq, (long long)adam->count, adam->hyper};
    L.naj = adam->blocks;
  }
  LdsAlgo af = ad;
  af.floor = std::max(std::max(ad.floor, aw.floor), std::max(ad2.floor, aw2.floor));
  size_t need = std::max(lds_bytes(ad, false), lds_bytes(aw, false));
  if (h1.gd.bnx_dy) need = std::max(need, bnx_lds_bytes(bn_of(ad)));
  L.lds = tspm_detail::lds_with_floor(need, af);
  L.st = st;
  bwd_dispatch(ad, aw, &L);
  TSPM_LAUNCH_CHECK();
  return TSPM_OK;
}

}  // namespace TSPM_LDS_NS

namespace tspm_detail {
const LdsImpl& TSPM_LDS_IMPL() {
  namespace v = TSPM_LDS_NS;
  static const LdsImpl t{&v::lds_fwd_supported, &v::lds_dgrad_supported, &v::lds_wgrad_supported,
                         &v::lds_fwd_workspace, &v::lds_fwd_bn_counters, &v::lds_fwd_bn_partial_floats,
                         &v::lds_dgrad_workspace, &v::lds_wgrad_workspace, &v::lds_fwd,
                         &v::lds_dgrad, &v::lds_wgrad, &v::lds_bwd_built, &v::lds_bwd, &v::lds_fwd_pair,
                         &v::lds_fwd_bn_inlaunch, &v::lds_bwd_quad};
  return t;
}
}  // namespace tspm_detail
